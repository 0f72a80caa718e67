#!/bin/bash
# r06: GPU suite + smoke + default bench line on the current tree
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r06c}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench_$TAG.json'))
print('value', d['value'], 'dropin', d['drop_in_forward']['value'], 'roof', d['roofline']['frac'], d['roofline']['launch_us'], 'b8', d['lookup_b8']['frac'], 'iter', d['iteration']['iteration_us'], 'convs', d['update_gemm']['convs_us'], d['update_gemm']['frac'], 'dom', d['dominant_kernel']['frac'], 'exact', d['fp32_exact']['value'])"
