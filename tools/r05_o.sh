#!/bin/bash
# Round 5, step O: level 2 of the pyramid pooled in corr_build4's registers (RAFT_CB4_L2=1, default)
# vs the pool2 pass over level 1 (RAFT_CB4_L2=0): GPU suite, configs 2 and 5 interleaved.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/t_r05o.log 2>&1 || { tail -30 gpurun_out/t_r05o.log; exit 1; }
tail -1 gpurun_out/t_r05o.log
run() {
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-exact "$@" > gpurun_out/o_line.json 2> gpurun_out/o_line.err || { tail -20 gpurun_out/o_line.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/o_line.json')); print('CB4_L2=$RAFT_CB4_L2', d['value'], d['config']['workload'][:28], 'iter', d['iteration']['iteration_us'])"
}
for rep in 1 2; do
  for E in 1 0; do
    export RAFT_CB4_L2=$E
    run --steps 20 --warmup 3 || exit 1
    run --batch 1 --height 1080 --width 1920 --precision bf16 --steps 5 --warmup 1 || exit 1
  done
done
