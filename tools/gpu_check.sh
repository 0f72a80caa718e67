#!/bin/bash
# GPU round trip used during development: parity tests, bench, kernel-trace profile.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-dev}
timeout -k 10 500 python -m pytest tests/test_gpu_parity.py -q -m gpu -x -s > gpurun_out/gpu_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/gpu_$TAG.log
# a crash / abort / timeout ends the GPU work of this call (plain test failures do not)
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 20 --warmup 3 ${BENCH_ARGS} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo bench failed; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
if [ -n "$PROFILE" ]; then
  export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-fp32-exact ${BENCH_ARGS} > gpurun_out/prof_$TAG.log 2>&1
  echo "prof rc=$?"
fi
