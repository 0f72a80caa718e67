#!/bin/bash
# Round-3 development round trip: focused GPU tests, an A/B bench of an env knob, a forward trace.
#   TESTS="tests/test_gpu_lookup_conv.py ..."  pytest targets (default: the fused lookup tests)
#   AB="RAFT_FUSE_CONVC1=0"                     env of the A side of the bench A/B (B = default)
#   TRACE=1                                     rocprofv3 kernel trace of tools/fwd_profile.py + phase summary
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-dev}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${TESTS}" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS} -x -q --timeout 240 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/t_$TAG.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
BARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-fp32-exact ${BENCH_ARGS}"
if [ -n "${AB}" ]; then
  for side in A B A B; do
    if [ $side = A ]; then E="${AB}"; else E=""; fi
    env $E timeout -k 10 300 python bench.py $BARGS > gpurun_out/ab_${TAG}_$side.json 2> gpurun_out/ab_${TAG}_$side.err || { echo "bench $side failed"; tail -20 gpurun_out/ab_${TAG}_$side.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_${TAG}_$side.json')); print('$side', d['value'], 'iter', d['iteration']['iteration_us'], 'convs', d['update_gemm']['convs_us'], 'lookup', d['roofline']['launch_us'], d['roofline']['frac'])"
  done
else
  timeout -k 10 300 python bench.py $BARGS > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo bench failed; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
  cat gpurun_out/bench_$TAG.json
fi
if [ -n "${TRACE}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fp_$TAG -o run --output-format csv -- python tools/fwd_profile.py > gpurun_out/fp_$TAG.log 2>&1
  rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python tools/phase_summary.py gpurun_out/fp_$TAG/run_kernel_trace.csv > gpurun_out/phase_$TAG.txt 2>&1
  head -60 gpurun_out/phase_$TAG.txt
fi
