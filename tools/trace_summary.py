"""Summarise a rocprofv3 kernel trace: per-kernel time of one forward (the last one)."""
import csv
import sys
from collections import OrderedDict

rows = list(csv.DictReader(open(sys.argv[1])))
ks = [(r["Kernel_Name"].replace("raft::(anonymous namespace)::", "").replace("void ", "").split("(")[0],
       int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])), int(r["Grid_Size_Y"]),
       (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0) for r in rows]
idx = [i for i, k in enumerate(ks) if k[0].startswith("prep_images")]
s = idx[-2] if len(idx) > 1 else idx[-1]
e = idx[-1] if len(idx) > 1 else len(ks)
fwd = ks[s:e]
tot = OrderedDict()
for name, gx, gy, us in fwd:
    tot.setdefault(name, [0, 0.0])
    tot[name][0] += 1
    tot[name][1] += us
total = sum(v[1] for v in tot.values())
print(f"one forward: {len(fwd)} kernels, {total/1000:.2f} ms of kernel time")
for k, (n, us) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
    print(f"  {k:40s} {n:5d} calls {us/1000:8.3f} ms  {100*us/total:5.1f}%")
if len(sys.argv) > 2:
    # print one iteration of the loop: from the 2nd corr_lookup to the 3rd
    li = [i for i, k in enumerate(fwd) if "lookup" in k[0]]
    for k in fwd[li[1]:li[2]]:
        print("   ", k)
