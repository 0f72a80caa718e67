#!/bin/bash
# corr_build4 with coalesced level-0 stores (tests, stamps, alone vs corr_build2) and the configs with
# the one-product 3x3 multi-tile rule, one box.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${TAG:-r04mt4}
O=gpurun_out/exp_${TAG}.txt
mkdir -p gpurun_out
: > $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_halo_mt.py tests/test_gpu_corr_build.py -q --timeout 240 --timeout-method thread > gpurun_out/t_${TAG}_first.log 2>&1
rc=$?; tail -4 gpurun_out/t_${TAG}_first.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc  # (1: test failures only)
run() { echo "== $*" >> $O; timeout -k 10 200 "$@" >> $O 2>&1 || { echo "failed: $*"; tail -30 $O; exit 1; }; }
run env RAFT_HIP_LIB=variants/cb4st/libraft_hip.so python tools/cb4_stamps.py 1 135 240
run python tools/corr4_bench.py 1 55 128
run python tools/corr4_bench.py 1 135 240
run python tools/corr4_bench.py 8 68 120
for a in "--batch 1 --height 1080 --width 1920 --precision bf16" "--batch 8 --height 540 --width 960" ""; do
  for v in "RAFT_CORR_BUILD4=1" "RAFT_CORR_BUILD4=0"; do
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
    elif "cyc" in line or "stamps" in line or "corr build" in line: print("  ", line.rstrip())
PY
