#!/bin/bash
# End-of-round evidence on one box (TAG names the round, e.g. r05).  PART=a: the GPU suite, smoke, the
# default bench line and a rocprofv3 --kernel-trace --stats of that same bench command (+ the fused lookup's
# in-forward vs back-to-back means, tools/roofline_rocprof.py) and a config-2 forward trace.  PART=b: the
# in-forward PMC passes (tools/pmc_forward.sh -> gpurun_out/<TAG>_*_pmc.json) and the configs 3-5 lines.
# Each GPU step time-limited; the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05}
if [ "${PART:-a}" = a ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_${TAG}_ev.log 2>&1
  rc=$?; tail -3 gpurun_out/t_${TAG}_ev.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
  timeout -k 10 300 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
  cat gpurun_out/bench_${TAG}.json
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}_rocprof.json 2> gpurun_out/bench_${TAG}_rocprof.err || { tail -20 gpurun_out/bench_${TAG}_rocprof.err; exit 1; }
  python tools/roofline_rocprof.py gpurun_out/prof_${TAG}/run_kernel_trace.csv gpurun_out/bench_${TAG}_rocprof.json > gpurun_out/${TAG}_roofline_rocprof.json
  cat gpurun_out/${TAG}_roofline_rocprof.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fwd_${TAG} -o run --output-format csv -- python tools/fwd_profile.py 1 440 1024 f16x3 > gpurun_out/fwd_${TAG}.log 2>&1 || { tail -20 gpurun_out/fwd_${TAG}.log; exit 1; }
  python tools/phase_summary.py gpurun_out/fwd_${TAG}/run_kernel_trace.csv > gpurun_out/${TAG}_forward_phases_config2.txt 2>&1
  grep -E "forward span|encoder phase span|loop span" gpurun_out/${TAG}_forward_phases_config2.txt
else
  # the lookup-only forward (RAFT_FUSE_CONVF1=0, pmc_forward.py's default): <TAG>_lookup_pmc.json
  PMC_OUT=gpurun_out PMC_ROUND=$TAG timeout -k 10 600 bash tools/pmc_forward.sh 1 > gpurun_out/pmc_${TAG}.log 2>&1 || { tail -20 gpurun_out/pmc_${TAG}.log; exit 1; }
  mkdir -p gpurun_out/pmc_unfused && cp gpurun_out/${TAG}_halo_pmc.json gpurun_out/pmc_unfused/
  # the bench's forward (the fused lookup launch): <TAG>_lookup_conv_pmc.json and its conv counters
  RAFT_FUSE_CONVF1=1 PMC_OUT=gpurun_out PMC_ROUND=$TAG timeout -k 10 600 bash tools/pmc_forward.sh 1 > gpurun_out/pmc2_${TAG}.log 2>&1 || { tail -20 gpurun_out/pmc2_${TAG}.log; exit 1; }
  tail -5 gpurun_out/pmc2_${TAG}.log
  [ -n "$PMC_ONLY" ] && exit 0
  timeout -k 10 900 bash tools/config_sweep.sh $TAG || exit 1
fi
