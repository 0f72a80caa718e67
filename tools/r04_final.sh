#!/bin/bash
# Round-4 end-of-round evidence on one box.  PART=a: the GPU suite, smoke, the default bench line and
# a rocprofv3 --kernel-trace --stats of that same bench command.  PART=b: the in-forward PMC passes
# (tools/pmc_forward.sh -> gpurun_out/r04_*_pmc.json) and the configs 3-5 sweep.  Each GPU step
# time-limited; the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${PART:-a}" = a ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t_r04f.log 2>&1
  rc=$?; tail -3 gpurun_out/t_r04f.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
  timeout -k 10 300 python bench.py > gpurun_out/bench_r04f.json 2> gpurun_out/bench_r04f.err || { tail -20 gpurun_out/bench_r04f.err; exit 1; }
  cat gpurun_out/bench_r04f.json
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04f -o run --output-format csv -- python bench.py > gpurun_out/bench_r04f_rocprof.json 2> gpurun_out/bench_r04f_rocprof.err || { tail -20 gpurun_out/bench_r04f_rocprof.err; exit 1; }
  ls gpurun_out/prof_r04f
  python tools/roofline_rocprof.py gpurun_out/prof_r04f/run_kernel_trace.csv gpurun_out/bench_r04f_rocprof.json > gpurun_out/r04_final_roofline_rocprof.json
  cat gpurun_out/r04_final_roofline_rocprof.json
else
  PMC_OUT=gpurun_out PMC_ROUND=r04 timeout -k 10 600 bash tools/pmc_forward.sh 1 > gpurun_out/pmc_r04f.log 2>&1 || { tail -20 gpurun_out/pmc_r04f.log; exit 1; }
  tail -5 gpurun_out/pmc_r04f.log
  # the bench's forward (the fused lookup launch): r04_lookup_conv_pmc.json and its conv counters
  mkdir -p gpurun_out/pmc_unfused && cp gpurun_out/r04_halo_pmc.json gpurun_out/pmc_unfused/
  RAFT_FUSE_CONVF1=1 PMC_OUT=gpurun_out PMC_ROUND=r04 timeout -k 10 600 bash tools/pmc_forward.sh 1 > gpurun_out/pmc2_r04f.log 2>&1 || { tail -20 gpurun_out/pmc2_r04f.log; exit 1; }
  [ -n "$PMC_ONLY" ] && exit 0
  timeout -k 10 900 bash tools/config_sweep.sh r04f || exit 1
fi
