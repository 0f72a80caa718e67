#!/bin/bash
# Multi-tile rule knobs on one box: the K-padding limit (fnet layer 2's 3 chunks) and the later-tile
# cost, on the encoder conv shapes and the configs' forwards.  Each GPU step time-limited.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${TAG:-r04i}
O=gpurun_out/exp_${TAG}.txt
mkdir -p gpurun_out
: > $O
run() { echo "== $*" >> $O; timeout -k 10 200 "$@" >> $O 2>&1 || { echo "failed: $*"; tail -30 $O; exit 1; }; }
for pad in 0.125 0.5; do
  run env RAFT_HALO_MT_PAD=$pad SHAPESET=enc python tools/conv_bench.py 1
done
for a in "--batch 8 --height 540 --width 960" "--batch 1 --height 1080 --width 1920 --precision bf16" ""; do
  for v in "RAFT_HALO_MT_COST=0.8" "RAFT_HALO_MT_COST=0.6" "RAFT_HALO_MT_COST=1.0" "RAFT_HALO_MT_PAD=0.5"; do
    echo "== $v bench $a" >> $O
    env $v timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-fp32-exact $a >> $O 2>> gpurun_out/exp_${TAG}.err || { echo failed; tail -20 gpurun_out/exp_${TAG}.err; exit 1; }
  done
done
python - "$O" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("=="): tag = line.strip()
    elif line.startswith("{"):
        d = json.loads(line); print(tag, d["value"], "upd", d["update_gemm"]["convs_us"], "it", d["iteration"]["iteration_us"])
    elif " us " in line and "TF/s" in line: print("  ", line.rstrip())
PY
