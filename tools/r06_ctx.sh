#!/bin/bash
# r06: context-branch enqueue order (RAFT_CTX_ORDER late / early / mix): bench.py interleaved on one box,
# then one rocprof forward trace per order (same method for all three)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for o in late early mix; do
    RAFT_CTX_ORDER=$o timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/ctx_$o.json 2> gpurun_out/ctx_$o.err || { tail -20 gpurun_out/ctx_$o.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/ctx_$o.json'))
print('$o', d['value'], 'dropin', d['drop_in_forward']['value'], 'iter', d['iteration']['iteration_us'])"
  done
done
for o in late early mix; do
  export RAFT_CTX_ORDER=$o
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/fwdctx_$o -o run --output-format csv -- python tools/fwd_profile.py 1 440 1024 f16x3 > gpurun_out/fwdctx_$o.log 2>&1 || { tail -20 gpurun_out/fwdctx_$o.log; exit 1; }
  python tools/phase_summary.py gpurun_out/fwdctx_$o/run_kernel_trace.csv > gpurun_out/ctx_${o}_phases.txt 2>&1
  echo "== $o"; grep -E "forward span|encoder phase span|loop span" gpurun_out/ctx_${o}_phases.txt
done
