#!/bin/bash
# Round 5, step J: persistent fused-lookup work-groups (RAFT_LC_PERSIST): GPU suite, configs 5 / 4 A/B,
# stamps at config 5.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/t_r05j.log 2>&1 || { tail -30 gpurun_out/t_r05j.log; exit 1; }
tail -2 gpurun_out/t_r05j.log
run() {
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-fp32-exact "$@" > gpurun_out/j_line.json 2> gpurun_out/j_line.err || { tail -20 gpurun_out/j_line.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/j_line.json')); r=d.get('roofline') or {}; print('PERSIST=$RAFT_LC_PERSIST', d['value'], d['config']['workload'][:40], 'iter', d['iteration']['iteration_us'], 'convs', d['update_gemm']['convs_us'], 'lookup', r.get('launch_us') or r.get('iteration_us'), r.get('inforward_span_us'))"
}
for rep in 1 2; do
  for E in 1 0; do
    export RAFT_LC_PERSIST=$E
    run --batch 1 --height 1080 --width 1920 --precision bf16 || exit 1
    run --batch 8 --height 540 --width 960 || exit 1
  done
done
unset RAFT_LC_PERSIST
for E in 1 0; do
  echo "== stamps config 5 PERSIST=$E"
  RAFT_LC_PERSIST=$E RAFT_SKIP_SRC_CHECK=1 RAFT_HIP_LIB=ab/lcst/libraft_hip.so timeout -k 10 200 python tools/lc_stamps.py --h 1080 --w 1920 --precision bf16 2>&1 | grep -v amdgpu.ids | tail -12 || exit 1
done
