#!/bin/bash
# Round-end check on one box: full GPU suite, smoke, the default bench line, and the eager (no hipGraph) bench.
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_final2.log 2>&1; rc=$?; tail -2 gpurun_out/t_final2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || exit 1
timeout -k 10 300 python bench.py --no-graph --no-cpu-baseline --no-fp32-exact --steps 10 > gpurun_out/bench_eager.json 2> gpurun_out/bench_eager.err || exit 1
python -c "
import json
for f in ('gpurun_out/bench_final.json','gpurun_out/bench_eager.json'):
    d=json.load(open(f)); print(f, d['value'], d['config']['workload'][-12:], d['roofline']['frac'], (d.get('lookup_b8') or {}).get('frac'), d['update_gemm']['frac'], (d.get('cpu_baseline') or {}).get('value'))
"
