"""The bench's roofline launch under rocprof: splits the dispatches of one kernel in a
rocprofv3 kernel trace of `python bench.py` into the back-to-back ones (the bench's own roofline
graph: 4 x 32 launches of the forward's fused lookup with nothing between them) and the rest (the
forwards), and prints their means next to the bench line's live figure.

    python tools/roofline_rocprof.py <run_kernel_trace.csv> <bench.json> [kernel-substring]"""
import csv
import json
import statistics
import sys

trace, bench = sys.argv[1], sys.argv[2]
kname = sys.argv[3] if len(sys.argv) > 3 else "lookup_conv_kernel"
rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"] for r in rows]
b2b, rest = [], []
for i, r in enumerate(rows):
    if kname not in r["Kernel_Name"]:
        continue
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    near = (i > 0 and kname in names[i - 1]) or (i + 1 < len(rows) and kname in names[i + 1])
    (b2b if near else rest).append(d)
live = json.load(open(bench))["roofline"]["launch_us"]
out = {
    "kernel": kname,
    "bench_live_launch_us": live,
    "rocprof_back_to_back": {"dispatches": len(b2b), "mean_us": round(statistics.mean(b2b), 3),
                             "median_us": round(statistics.median(b2b), 3)},
    "rocprof_in_forward": {"dispatches": len(rest), "mean_us": round(statistics.mean(rest), 3),
                           "median_us": round(statistics.median(rest), 3)},
}
out["live_vs_rocprof_back_to_back"] = round(live / out["rocprof_back_to_back"]["mean_us"] - 1, 4)
# (round 4: the live figure is the in-forward launch span, so it is checked against the in-forward mean)
out["live_vs_rocprof_in_forward"] = round(live / out["rocprof_in_forward"]["mean_us"] - 1, 4)
out["in_forward_vs_back_to_back"] = round(out["rocprof_in_forward"]["mean_us"] / out["rocprof_back_to_back"]["mean_us"] - 1, 4)
print(json.dumps(out, indent=1))
