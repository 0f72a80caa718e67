#!/bin/bash
# bench line per library variant (ab/<name>/libraft_hip.so; "base" = the in-tree build), twice interleaved
#   tools/ab_variants.sh "base nowait noacq" [extra bench args]
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for V in $1; do
    if [ "$V" = base ]; then LIB=raft_optical_flow_amd/libraft_hip.so; else LIB=ab/$V/libraft_hip.so; fi
    RAFT_SKIP_SRC_CHECK=1 RAFT_HIP_LIB=$LIB timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-fp32-exact $2 > gpurun_out/abv_$V.json 2> gpurun_out/abv_$V.err || { echo "bench $V failed"; tail -20 gpurun_out/abv_$V.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/abv_$V.json')); dk=d.get('dominant_kernel') or {}; r=d.get('roofline') or {}; print('$V', d['value'], 'iter', d['iteration']['iteration_us'], 'convs', d['update_gemm']['convs_us'], 'dom', dk.get('launch_us'), dk.get('frac'), 'lookup', r.get('launch_us'), r.get('frac'), r.get('inforward_span_us'))"
  done
done
