#!/bin/bash
# GPU round trip used during development: parity tests, bench, kernel-trace profile, in-forward PMC.
#   PROFILE=1  rocprofv3 --kernel-trace --stats of a short bench run
#   PMC=1      tools/pmc_forward.sh (lookup HBM bytes, conv MFMA busy) -> profiles/r02_*_pmc.json
#   TESTS=0    skip the pytest run
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-dev}
mkdir -p gpurun_out
if [ "${TESTS:-1}" != 0 ]; then
  timeout -k 10 500 python -u -m pytest tests/ -q -m gpu -x -s --timeout 240 --timeout-method thread > gpurun_out/gpu_$TAG.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/gpu_$TAG.log
  # a crash / abort / timeout ends the GPU work of this call (plain test failures do not)
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
timeout -k 10 400 python bench.py --steps 20 --warmup 3 ${BENCH_ARGS} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo bench failed; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
if [ -n "$PROFILE" ]; then
  export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-fp32-exact ${BENCH_ARGS} > gpurun_out/prof_$TAG.log 2>&1
  rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$PMC" ]; then
  ./tools/pmc_forward.sh 1 || exit 1
fi
