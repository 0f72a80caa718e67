#!/bin/bash
# Round 5, step P: the correlation build as two 4-wave work-groups per CU (RAFT_CB4_W4=1, default) vs one
# 8-wave work-group (0): corr-build tests under both, the build alone at configs 2 / 5 / 4 maps, configs 2 and 5.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for E in 1 0; do
  RAFT_CB4_W4=$E timeout -k 10 200 python -u -m pytest tests/test_gpu_corr_build.py tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread 2>&1 | tail -1 || exit 1
done
for E in 1 0 1 0; do
  for shp in "1 55 128" "1 135 240" "8 68 120"; do
    echo -n "CB4_W4=$E: "
    RAFT_CB4_W4=$E timeout -k 10 120 python tools/corr4_bench.py $shp 2>&1 | grep "corr build" || exit 1
  done
done
run() {
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-exact "$@" > gpurun_out/p_line.json 2> gpurun_out/p_line.err || { tail -20 gpurun_out/p_line.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/p_line.json')); print('CB4_W4=$RAFT_CB4_W4', d['value'], d['config']['workload'][:28], 'iter', d['iteration']['iteration_us'])"
}
for rep in 1 2; do
  for E in 1 0; do
    export RAFT_CB4_W4=$E
    run --steps 20 --warmup 3 || exit 1
    run --batch 1 --height 1080 --width 1920 --precision bf16 --steps 5 --warmup 1 || exit 1
  done
done
