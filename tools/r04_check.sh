#!/bin/bash
# Round-4 GPU round trip: targeted tests, the full GPU suite, the config-2 bench line, configs 4 / 5,
# and a kernel trace of a config-2 forward with its phase summary.  Every GPU step has its own time
# limit and the chain stops at the first failure.
#   TAG        output name suffix (default r04);  FIRST / FIRST_K: test files / -k expression run first
#   TESTS=0    skip the full suite;  SWEEP=0 skip configs 4 / 5;  TRACE=0 skip the trace
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${TAG:-r04}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$FIRST" ]; then
  timeout -k 10 400 python -u -m pytest $FIRST ${FIRST_K:+-k "$FIRST_K"} -x -q --timeout 240 --timeout-method thread > gpurun_out/t_${TAG}_first.log 2>&1
  rc=$?; tail -4 gpurun_out/t_${TAG}_first.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "${TESTS:-1}" != 0 ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t_${TAG}.log 2>&1
  rc=$?; tail -4 gpurun_out/t_${TAG}.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench_${TAG}.json'))
print('config2', d['value'], 'ms', d['ms_per_step'], 'lookup', d['roofline']['launch_us'], d['roofline']['frac'], 'upd', d['update_gemm']['convs_us'], d['update_gemm']['frac'], 'it', d['iteration']['iteration_us'])"
if [ "${SWEEP:-1}" != 0 ]; then
  for a in "--batch 8 --height 540 --width 960" "--batch 1 --height 1080 --width 1920 --precision bf16"; do
    timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-fp32-exact $a >> gpurun_out/sweep_${TAG}.jsonl 2>> gpurun_out/sweep_${TAG}.err || { tail -20 gpurun_out/sweep_${TAG}.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/sweep_${TAG}.jsonl').readlines()[-1])
print('$a', d['value'], 'upd', d['update_gemm']['convs_us'], d['update_gemm']['frac'], 'it', d['iteration']['iteration_us'])"
  done
fi
if [ "${TRACE:-1}" != 0 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fp_${TAG} -o run --output-format csv -- python tools/fwd_profile.py 1 440 1024 f16x3 > gpurun_out/fp_${TAG}.log 2>&1 || { tail -20 gpurun_out/fp_${TAG}.log; exit 1; }
  python tools/phase_summary.py gpurun_out/fp_${TAG}/run_kernel_trace.csv > gpurun_out/phase_${TAG}.txt 2>&1
  grep -E "forward span|encoder phase span|loop span" gpurun_out/phase_${TAG}.txt
fi
