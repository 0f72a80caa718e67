"""Summarise tools/pmc_forward.sh into profiles/r02_lookup_pmc.json and profiles/r02_halo_pmc.json.

Only the dispatches of the LAST forward count (from the last prep_images dispatch on).
FETCH_SIZE / WRITE_SIZE are KiB per dispatch; on gfx950 FETCH_SIZE under-reports reads
(MI355X_MICROARCH.md, HBM section), so reads are scaled by the calibration copy's
true/reported ratio measured in the same process (64 MiB, 4-B accesses).
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs): the share of
the chip's SIMD-cycles with the MFMA pipe busy while the kernel ran.
Each JSON carries source_sha = sha1 of the kernel's .hip file; bench.py reads a summary only
while the source it was taken on is unchanged.
"""
import csv
import glob
import hashlib
import json
import os
import re
import statistics
import sys

base = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RND = os.environ.get("PMC_ROUND", "r05")  # <out>/<round>_*_pmc.json
OUTD = os.environ.get("PMC_OUT", os.path.join(ROOT, "profiles"))  # (on a GPU box: gpurun_out, then copy)


def sha(name):
    return hashlib.sha1(open(os.path.join(ROOT, "raft_optical_flow_amd", "csrc", name), "rb").read()).hexdigest()


def short(name):
    n = name.replace("raft::(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*", "", n).strip()


def last_forward(rows):
    """{dispatch: (kernel, {counter: value})} of the last forward."""
    disp = {}
    for r in rows:
        d = int(r["Dispatch_Id"])
        disp.setdefault(d, [short(r["Kernel_Name"]), {}])[1][r["Counter_Name"]] = float(r["Counter_Value"])
    order = sorted(disp)
    starts = [d for d in order if disp[d][0].startswith("prep_images")]
    calib = [d for d in order if disp[d][0].startswith("nhwc_to_nchw")]
    fwd = [d for d in order if d >= starts[-1]]
    return [disp[d] for d in fwd], (disp[calib[0]] if calib else None)


passes = {}
for f in sorted(glob.glob(os.path.join(base, "p*", "run_counter_collection.csv"))):
    passes[os.path.basename(os.path.dirname(f))] = last_forward(list(csv.DictReader(open(f))))

fwd_f, cal_f = passes["p1"]
fwd_w, cal_w = passes["p2"]
calib_bytes = 64 * 1024 * 1024
read_scale = calib_bytes / (cal_f[1]["FETCH_SIZE"] * 1024.0)
write_scale = calib_bytes / (cal_w[1]["WRITE_SIZE"] * 1024.0)
lk_f = [c["FETCH_SIZE"] for k, c in fwd_f if k.startswith("corr_lookup")]
lk_w = [c["WRITE_SIZE"] for k, c in fwd_w if k.startswith("corr_lookup")]
hit = [c for k, c in passes["p4"][0] if k.startswith("corr_lookup")]
P = B * 55 * 128
alg_read, alg_write = P * (4 * 100 * 4 + 8), P * 4 * 81 * 4
res = {} if not lk_f else {
    "kernel": "corr_lookup_kernel<4, 4, false, SCAL> (B=1: the scalar-interval window form)", "source_sha": sha("corr_pyramid.hip"), "shape_bhw": [B, 440, 1024],
    "workload": f"bench.py config-2 forward, B={B}, 436x1024 padded to 440x1024, iters=32, f16x3; "
                f"the {len(lk_f)} lookups of the last of two eager forwards (tools/pmc_forward.py)",
    "fetch_size_kib_raw_avg": statistics.mean(lk_f), "write_size_kib_raw_avg": statistics.mean(lk_w),
    "calibration": {"kernel": "nhwc_to_nchw (C=1) 64 MiB copy", "fetch_kib": cal_f[1]["FETCH_SIZE"],
                    "write_kib": cal_w[1]["WRITE_SIZE"], "read_scale": round(read_scale, 4),
                    "write_scale": round(write_scale, 4)},
    "hbm_read_bytes_per_launch": round(statistics.mean(lk_f) * 1024 * read_scale),
    "hbm_write_bytes_per_launch": round(statistics.mean(lk_w) * 1024 * write_scale),
    "algorithmic_read_bytes": alg_read, "algorithmic_write_bytes": alg_write,
    "l2_hit_rate": round(sum(c["TCC_HIT_sum"] for c in hit) / sum(c["TCC_HIT_sum"] + c["TCC_MISS_sum"] for c in hit), 4),
}
if lk_f:
    res["hbm_bytes_per_launch"] = res["hbm_read_bytes_per_launch"] + res["hbm_write_bytes_per_launch"]
    res["traffic_over_algorithmic"] = round(res["hbm_bytes_per_launch"] / (alg_read + alg_write), 3)
sfx = "" if B == 1 else f"_b{B}"
# (the standalone lookup kernel only runs in the forward without the fused launch: RAFT_FUSE_CONVC1=0)
if lk_f:
    json.dump(res, open(os.path.join(OUTD, f"{RND}_lookup_pmc{sfx}.json"), "w"), indent=1)
print(json.dumps(res, indent=1))

halo = {"source_sha": sha("conv_halo.hip"),
        "workload": f"bench.py config-2 forward, B={B}, f16x3: every conv kernel dispatch of the last forward",
        "definition": "mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 * GRBM_GUI_ACTIVE / 8), mean over dispatches"}
per = {}
for k, c in passes["p3"][0]:
    if "conv" in k and "SQ_VALU_MFMA_BUSY_CYCLES" in c and c.get("GRBM_GUI_ACTIVE"):
        per.setdefault(k, []).append((c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * c["GRBM_GUI_ACTIVE"] / 8),
                                      c["SQ_VALU_MFMA_BUSY_CYCLES"], c["GRBM_GUI_ACTIVE"] / 8))
for k, v in per.items():
    halo[k] = {"dispatches": len(v), "mfma_busy": round(statistics.mean(x[0] for x in v), 4),
               "mfma_busy_cycles_avg": round(statistics.mean(x[1] for x in v)),
               "gui_active_cycles_avg": round(statistics.mean(x[2] for x in v))}
json.dump(halo, open(os.path.join(OUTD, f"{RND}_halo_pmc{sfx}.json"), "w"), indent=1)
print(json.dumps(halo, indent=1))

# the forward's fused lookup launch (raft_corr_lookup_conv): window reads + coords + flow in,
# convc1 (256) and convf1 (128) output rows out (bench.py fused_lookup_bytes_per_pixel)
lc_f = [c["FETCH_SIZE"] for k, c in fwd_f if k.startswith("lookup_conv")]
lc_w = [c["WRITE_SIZE"] for k, c in fwd_w if k.startswith("lookup_conv")]
if lc_f:
    lhit = [c for k, c in passes["p4"][0] if k.startswith("lookup_conv")]
    a_r, a_w = P * (4 * 100 * 4 + 8), P * (4 * (256 + 128) + 8)
    lc = {"kernel": "lookup_conv_kernel (raft_corr_lookup_conv: lookup + convc1 + convf1)", "source_sha": sha("lookup_conv.hip"),
          "shape_bhw": [B, 440, 1024],
          "workload": f"bench.py config-2 forward, B={B}, f16x3; the {len(lc_f)} fused lookups of the last forward",
          "hbm_read_bytes_per_launch": round(statistics.mean(lc_f) * 1024 * read_scale),
          "hbm_write_bytes_per_launch": round(statistics.mean(lc_w) * 1024 * write_scale),
          "algorithmic_read_bytes": a_r, "algorithmic_write_bytes": a_w,
          "l2_hit_rate": round(sum(c["TCC_HIT_sum"] for c in lhit) / max(1.0, sum(c["TCC_HIT_sum"] + c["TCC_MISS_sum"] for c in lhit)), 4)}
    lc["hbm_bytes_per_launch"] = lc["hbm_read_bytes_per_launch"] + lc["hbm_write_bytes_per_launch"]
    lc["traffic_over_algorithmic"] = round(lc["hbm_bytes_per_launch"] / (a_r + a_w), 3)
    json.dump(lc, open(os.path.join(OUTD, f"{RND}_lookup_conv_pmc{sfx}.json"), "w"), indent=1)
    print(json.dumps(lc, indent=1))
