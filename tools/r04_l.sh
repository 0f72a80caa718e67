#!/bin/bash
# Config 5 (bf16, B=1) on the final tree, interleaved on one box: default vs no big tiles
# (RAFT_HALO_BIG_MIN=0) vs one tile per work-group (RAFT_HALO_MT=0).
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${TAG:-r04l}
O=gpurun_out/exp_${TAG}.txt
mkdir -p gpurun_out
: > $O
for r in 1 2; do
  for v in "X=0" "RAFT_HALO_BIG_MIN=0" "RAFT_HALO_MT=0"; do
    echo "== $v bench config5" >> $O
    env $v timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-fp32-exact --batch 1 --height 1080 --width 1920 --precision bf16 >> $O 2>> gpurun_out/exp_${TAG}.err || { echo failed; tail -20 gpurun_out/exp_${TAG}.err; exit 1; }
  done
done
python - "$O" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("=="): tag = line.strip()
    elif line.startswith("{"):
        d = json.loads(line); print(tag, d["value"], "upd", d["update_gemm"]["convs_us"], "it", d["iteration"]["iteration_us"])
PY
