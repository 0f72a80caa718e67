#!/bin/bash
# A/B of environment knobs on one box: tools/ab_env.sh "ENV=A" "ENV=B" ...  (bench, 3 runs each, interleaved)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "$@"; do
    env $cfg timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-exact ${BENCH_ARGS} > gpurun_out/ab.json 2>gpurun_out/ab.err || { echo "failed: $cfg"; tail -5 gpurun_out/ab.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); print('$cfg', d['value'], d['ms_per_step'])"
  done
done
