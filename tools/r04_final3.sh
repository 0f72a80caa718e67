#!/bin/bash
# Last check of the final tree: the GPU suite, smoke, the default bench line and config 5 (B=1).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t_r04f3.log 2>&1
rc=$?; tail -3 gpurun_out/t_r04f3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_r04f3.json 2> gpurun_out/bench_r04f3.err || { tail -20 gpurun_out/bench_r04f3.err; exit 1; }
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-fp32-exact --batch 1 --height 1080 --width 1920 --precision bf16 > gpurun_out/bench_r04f3_c5.json 2>> gpurun_out/bench_r04f3.err || exit 1
python -c "
import json
for f in ('gpurun_out/bench_r04f3.json', 'gpurun_out/bench_r04f3_c5.json'):
    d=json.load(open(f)); print(f, d['value'], d['roofline']['launch_us'], d['roofline']['frac'], d['update_gemm']['frac'], d['dominant_kernel'].get('mfma_busy'))"
