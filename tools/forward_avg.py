"""Per-dispatch averages of bench.py's roofline kernels from a rocprofv3 kernel trace of the same
bench command, to check bench.py's live figures against rocprof:

  * corr_lookup_kernel<4,4,false>, B=1 grid (1760 x 256 threads) and B=8 grid (14080 x 256), split into
      - rotated: the dispatches of bench.py's cache-cold rotation graphs (runs of >= 16 consecutive
        lookups with no other kernel between them)  -> compare with roofline / lookup_b8 launch_us
      - in-forward: every other lookup dispatch (the 32 per forward of the timed graph replays)
  * conv_halo_kernel<3,3,64,1> at B=1 in the update loop (the convc2 | convf2 pair and the flow-head
    conv1, 224 work-groups each)                            -> compare with dominant_kernel launch_us

    python tools/forward_avg.py gpurun_out/prof_<tag>/run_kernel_trace.csv [out.json]
"""
import csv
import json
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))


def dur(r):
    return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0


def is_lookup(r):  # the lookup-only kernel, either window form (<4, 4, false> / <4, 4, false, SCAL>)
    n = r["Kernel_Name"]
    return "corr_lookup_kernel<4, 4, false>" in n or "corr_lookup_kernel<4, 4, false," in n


# runs of consecutive lookup dispatches
runs, cur = [], []
for r in rows:
    if is_lookup(r):
        cur.append(r)
    else:
        if cur:
            runs.append(cur)
        cur = []
if cur:
    runs.append(cur)
res = {}
for grid, tag in ((1760 * 256, "B=1"), (14080 * 256, "B=8")):
    rot = [dur(r) for run in runs if len(run) >= 16 for r in run if int(r["Grid_Size_X"]) == grid]
    fwd = [dur(r) for run in runs if len(run) < 16 for r in run if int(r["Grid_Size_X"]) == grid]
    for name, v in (("rotated", rot), ("in-forward", fwd)):
        if v:
            res[f"corr_lookup {tag} {name}"] = {"dispatches": len(v), "mean_us": round(statistics.mean(v), 3),
                                                 "median_us": round(statistics.median(v), 3)}
# the B=1 update-loop launches of conv_halo_kernel<3,3,64,1> (the convc2 | convf2 pair and the flow
# head's conv1: 224 work-groups each): dispatches between a forward's first lookup and the end of that
# forward (prep_images starts the next one), so the encoder's 1/8-res 3x3 convs do not count
fz, in_fwd = [], False
for r in rows:
    if "prep_images" in r["Kernel_Name"]:
        in_fwd = True
    elif "flow_from_coords" in r["Kernel_Name"]:
        in_fwd = False
    elif in_fwd and ("corr_lookup_kernel<4, 4, true>" in r["Kernel_Name"] or
                     "corr_lookup_kernel<4, 4, true," in r["Kernel_Name"]):
        fz.append(dur(r))
if fz:
    res["corr_lookup + convf1 B=1 in-forward"] = {"dispatches": len(fz), "mean_us": round(statistics.mean(fz), 3),
                                                   "median_us": round(statistics.median(fz), 3)}
h, in_fwd, in_loop = [], False, False
for r in rows:
    name = r["Kernel_Name"]
    if "prep_images" in name:  # a forward starts
        in_fwd, in_loop = True, False
    elif "flow_from_coords" in name:  # ... and ends (the bench's per-kernel replays come after)
        in_fwd = in_loop = False
    elif in_fwd and ("corr_lookup_kernel<4, 4, true" in name or
                     ("corr_lookup_kernel<4, 4" in name and int(r["Grid_Size_X"]) == 1760 * 256)):
        in_loop = True  # a B=1 lookup of the forward (lookup-only, or the lookup + convf1 launch)
    elif in_loop and "conv_halo_kernel<3, 3, 64, 1>" in name and int(r["Grid_Size_X"]) in (168 * 512, 224 * 512):
        h.append(dur(r))
if h:
    res["conv_halo_kernel<3,3,64,1> B=1 update loop (pair + fh1)"] = {
        "dispatches": len(h), "mean_us": round(statistics.mean(h), 3), "median_us": round(statistics.median(h), 3)}
for k, v in res.items():
    print(f"{k:50s} {v['dispatches']:6d} dispatches  mean {v['mean_us']:8.2f} us  median {v['median_us']:8.2f} us")
if len(sys.argv) > 2:
    json.dump(res, open(sys.argv[2], "w"), indent=1)
