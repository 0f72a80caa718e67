"""Timeline of the last forward's encoder phase in a rocprofv3 kernel trace (tools/fwd_profile.py):
per kernel its queue, start and end (us from the forward's first kernel) and duration, so the critical
path across the two streams can be read off.

    python tools/timeline.py gpurun_out/fp/run_kernel_trace.csv [max_rows]
"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
lim = int(sys.argv[2]) if len(sys.argv) > 2 else 200


def name(r):
    n = r["Kernel_Name"].replace("raft::(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0]


starts = [i for i, r in enumerate(rows) if name(r).startswith("prep_images")]
s = starts[-1]
end = next(i for i in range(s, len(rows)) if name(rows[i]).startswith("init_coords")) + 1
t0 = int(rows[s]["Start_Timestamp"])
for r in rows[s:end][:lim]:
    a, b = (int(r["Start_Timestamp"]) - t0) / 1000, (int(r["End_Timestamp"]) - t0) / 1000
    print(f"q{r['Queue_Id']:>2} {a:9.1f} {b:9.1f} {b - a:8.1f}  {name(r)[:60]}  grid {int(r['Grid_Size_X']) // max(1, int(r['Workgroup_Size_X']))}")
