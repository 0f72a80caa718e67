#!/bin/bash
# Same-box A/B of whole trees: this tree ("cur") vs trees built by tools/tree_from_rev.sh under ab/<name>,
# interleaved, config-2 bench lines (no CPU / exact-fp32 legs).
#   tools/ab_tree.sh "r3 cur" [reps] [extra bench args]
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
REPS=${2:-2}
for rep in $(seq 1 $REPS); do
  for V in $1; do
    if [ "$V" = cur ]; then D=.; else D=ab/$V; fi
    OUT=$(pwd)/gpurun_out/ab_${V}_$rep
    (cd $D && timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-fp32-exact $3) > $OUT.json 2> $OUT.err || { echo "bench $V failed"; tail -20 $OUT.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT.json')); dk=d.get('dominant_kernel') or {}; r=d.get('roofline') or {}; print('$V', d['value'], 'iter', d['iteration']['iteration_us'], 'convs', d['update_gemm']['convs_us'], 'dom', dk.get('launch_us'), dk.get('frac'), 'lookup', r.get('launch_us'), r.get('frac'))"
  done
done
