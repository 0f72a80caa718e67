#!/bin/bash
# Round-4 final tree (after the wide-tile threshold change): GPU suite, smoke, the default bench line,
# the in-forward PMC passes (unfused + fused forward) and the configs 3-5 sweep, one box.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t_r04f2.log 2>&1
rc=$?; tail -3 gpurun_out/t_r04f2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_r04f2.json 2> gpurun_out/bench_r04f2.err || { tail -20 gpurun_out/bench_r04f2.err; exit 1; }
cat gpurun_out/bench_r04f2.json
PMC_OUT=gpurun_out PMC_ROUND=r04 timeout -k 10 600 bash tools/pmc_forward.sh 1 > gpurun_out/pmc_r04f2.log 2>&1 || { tail -20 gpurun_out/pmc_r04f2.log; exit 1; }
mkdir -p gpurun_out/pmc_unfused && cp gpurun_out/r04_halo_pmc.json gpurun_out/pmc_unfused/
RAFT_FUSE_CONVF1=1 PMC_OUT=gpurun_out PMC_ROUND=r04 timeout -k 10 600 bash tools/pmc_forward.sh 1 > gpurun_out/pmc2_r04f2.log 2>&1 || { tail -20 gpurun_out/pmc2_r04f2.log; exit 1; }
timeout -k 10 900 bash tools/config_sweep.sh r04f2 || exit 1
