"""Per-kernel instruction mix of the first loop of a kernel in a hipcc -save-temps .s file.

    python tools/asm_stats.py file.s SYMBOL_SUBSTRING
"""
import re
import sys
from collections import Counter

path, pat = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and pat in l)
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
body = lines[start:end]
meta = [l for l in lines[end:end + 400] if re.search(r"\.(vgpr_count|agpr_count|sgpr_count|vgpr_spill_count|private_segment_fixed_size|group_segment_fixed_size):", l)]
print(body[0].split(":")[0])
for m in meta[:6]:
    print("  ", m.strip())
hdr = [i for i, l in enumerate(body) if "Loop Header" in l]
print("loop headers at", hdr)
if hdr:
    h = hdr[0]
    # the loop body ends at the last backward branch to a label at/after the header
    lab = body[h].split(":")[0]
    tail = max(i for i, l in enumerate(body) if re.search(r"s_cbranch\w* " + re.escape(lab) + r"\b|s_branch " + re.escape(lab) + r"\b", l))
    loop = body[h:tail + 1]
    c = Counter()
    for l in loop:
        m = re.match(r"^\s+([sv]_\w+|ds_\w+|buffer_\w+|global_\w+|scratch_\w+)", l)
        if m:
            op = m.group(1)
            c[op] += 1
    cls = Counter()
    for op, n in c.items():
        k = ("mfma" if "mfma" in op else "ds" if op.startswith("ds_") else "vmem" if op.startswith(("buffer", "global", "scratch"))
             else "smem" if op.startswith("s_load") or op.startswith("s_buffer") else "salu" if op.startswith("s_") else "valu")
        cls[k] += n
    print(f"loop lines {h}-{tail}: ", dict(cls))
    for op, n in c.most_common(40):
        print(f"  {n:4d} {op}")
