#!/bin/bash
# r06: the GPU suite, then BASELINE configs 3-5 on the current tree (tools/config_sweep.sh)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t_r06sw.log 2>&1
rc=$?; tail -3 gpurun_out/t_r06sw.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_r06sw.json 2> gpurun_out/bench_r06sw.err || { tail -20 gpurun_out/bench_r06sw.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench_r06sw.json'))
print('value', d['value'], 'dropin', d['drop_in_forward']['value'], 'roof', d['roofline']['frac'], d['roofline']['launch_us'], 'b8', d['lookup_b8']['frac'], 'iter', d['iteration']['iteration_us'], 'convs', d['update_gemm']['convs_us'], d['update_gemm']['frac'], 'dom', d['dominant_kernel']['frac'], 'exact', d['fp32_exact']['value'])"
timeout -k 10 900 bash tools/config_sweep.sh r06 || exit 1
