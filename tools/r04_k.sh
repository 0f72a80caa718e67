#!/bin/bash
# The flow head's 256 -> 2 conv at config 5: 4x16 tiles (RAFT_SN_TH4_MIN=256: 510 work-groups) vs
# 2x16 (default below 512 4x16 tiles), interleaved on one box; the small-n conv parity tests first.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${TAG:-r04k}
O=gpurun_out/exp_${TAG}.txt
mkdir -p gpurun_out
: > $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "conv2d_vs_torch or flow_head or update_block" -x -q --timeout 240 --timeout-method thread > gpurun_out/t_${TAG}.log 2>&1
rc=$?; tail -2 gpurun_out/t_${TAG}.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in "X=0" "RAFT_SN_TH4_MIN=256"; do
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
