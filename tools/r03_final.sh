#!/bin/bash
# Round-3 end-of-round evidence on one box (part A): GPU suite, smoke, bench (graph + eager),
# rocprof kernel stats of the bench, in-forward kernel trace + phase summary, in-forward PMC.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r03}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_$T.log 2>&1; rc=$?; tail -2 gpurun_out/t_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -5 gpurun_out/${T}_bench.err; exit 1; }
timeout -k 10 300 python bench.py --no-graph --no-cpu-baseline --no-fp32-exact --steps 10 > gpurun_out/${T}_bench_eager.json 2> gpurun_out/${T}_bench_eager.err || exit 1
python -c "
import json
for f in ('gpurun_out/${T}_bench.json','gpurun_out/${T}_bench_eager.json'):
    d=json.load(open(f)); print(f, d['value'], d['roofline']['launch_us'], d['roofline']['frac'], (d.get('lookup_b8') or {}).get('frac'), d['update_gemm']['frac'], (d.get('cpu_baseline') or {}).get('value'))
"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- python bench.py --no-cpu-baseline --no-fp32-exact > gpurun_out/${T}_bench_under_rocprof.json 2> gpurun_out/${T}_rocprof.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fp_$T -o run --output-format csv -- python tools/fwd_profile.py > gpurun_out/fp_$T.log 2>&1 || exit 1
python tools/phase_summary.py gpurun_out/fp_$T/run_kernel_trace.csv > gpurun_out/phase_$T.txt 2>&1
grep -E "forward span|encoder phase span|loop span" gpurun_out/phase_$T.txt
./tools/pmc_forward.sh 1 > gpurun_out/pmc_$T.log 2>&1 || { tail -5 gpurun_out/pmc_$T.log; exit 1; }
RAFT_FUSE_CONVF1=1 ./tools/pmc_forward.sh 1 > gpurun_out/pmc2_$T.log 2>&1 || { tail -5 gpurun_out/pmc2_$T.log; exit 1; }
cp profiles/r03_*pmc*.json gpurun_out/ 2>/dev/null; ls profiles/r03_* 
