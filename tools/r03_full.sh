#!/bin/bash
# Round-3 full check on one box: GPU suite, smoke, default bench line, rocprof kernel stats of the bench.
#   TAG=<name>   output tag (default full)
#   SKIP_TESTS=1 bench + profile only
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${TAG:-full}
mkdir -p gpurun_out
if [ -z "${SKIP_TESTS}" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/smoke_$TAG.log | tail -2; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_$TAG.err; exit $rc; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --no-cpu-baseline --no-fp32-exact > gpurun_out/bench_${TAG}_rocprof.json 2> gpurun_out/bench_${TAG}_rocprof.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
if [ -n "${TRACE}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fp_$TAG -o run --output-format csv -- python tools/fwd_profile.py > gpurun_out/fp_$TAG.log 2>&1
  rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python tools/phase_summary.py gpurun_out/fp_$TAG/run_kernel_trace.csv > gpurun_out/phase_$TAG.txt 2>&1
  head -40 gpurun_out/phase_$TAG.txt
fi
