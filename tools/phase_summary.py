"""Phase breakdown of the last forward in a rocprofv3 kernel trace (tools/fwd_profile.py):
encoder phase (prep_images .. init_coords), the update loop per iteration (mean per launch slot),
and the tail.  Times are kernel busy spans (first start .. last end) plus per-kernel sums.

    python tools/phase_summary.py gpurun_out/fp/run_kernel_trace.csv
"""
import csv
import statistics
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))


def name(r):
    n = r["Kernel_Name"].replace("raft::(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0]


ks = [(name(r), int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])))
      for r in rows]
starts = [i for i, k in enumerate(ks) if k[0].startswith("prep_images")]
s = starts[-1]
end = next(i for i in range(s, len(ks)) if ks[i][0].startswith("flow_from_coords")) + 1
fwd = ks[s:end]
ic = next(i for i, k in enumerate(fwd) if k[0].startswith("init_coords"))
enc = fwd[: ic + 1]
loop = fwd[ic + 1:]
span = lambda ks_: (ks_[-1][2] - ks_[0][1]) / 1000.0  # noqa: E731
print(f"forward span {span(fwd):.1f} us, {len(fwd)} kernels")
print(f"encoder phase span {span(enc):.1f} us ({len(enc)} kernels), busy sum {sum(k[2]-k[1] for k in enc)/1000:.1f} us")
agg = defaultdict(lambda: [0, 0.0])
for k in enc:
    agg[k[0]][0] += 1
    agg[k[0]][1] += (k[2] - k[1]) / 1000.0
for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"   {n:60s} {c:4d} {t:8.1f} us")
print("encoder phase in order (name, grid, us, gap-before us):")
prev = None
for k in enc:
    gap = (k[1] - prev) / 1000.0 if prev else 0.0
    print(f"   {k[0][:60]:60s} {k[3]:6d} {(k[2]-k[1])/1000:7.1f} {gap:6.1f}")
    prev = k[2]
# iterations: split at each lookup-type kernel
li = [i for i, k in enumerate(loop) if "lookup" in k[0]]
its = [loop[li[j]:li[j + 1]] for j in range(len(li) - 1)]
print(f"loop span {span(loop):.1f} us, {len(li)} iterations, mean iteration span "
      f"{statistics.mean([(its[j+1][0][1]-its[j][0][1])/1000 for j in range(len(its)-1)]):.1f} us")
if its:
    mid = its[1:-1] or its
    n = min(len(t) for t in mid)
    print("mean per launch slot (iterations 2..n-1):")
    tot = 0.0
    for j in range(n):
        d = [(t[j][2] - t[j][1]) / 1000 for t in mid]
        g = [(t[j][1] - t[j - 1][2]) / 1000 for t in mid] if j else [0]
        tot += statistics.mean(d)
        print(f"   {mid[0][j][0][:60]:60s} {mid[0][j][3]:6d} {statistics.mean(d):7.2f} us  gap {statistics.mean(g):5.2f}")
    print(f"   sum {tot:.1f} us")
tail = its[-1] if its else []
print("last iteration:", [(k[0][:40], round((k[2] - k[1]) / 1000, 1)) for k in tail])
