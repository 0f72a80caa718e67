#!/bin/bash
# corr build with / without non-temporal pyramid stores: config 5 and config 4, A/B on one box
set -o pipefail
cd "$(dirname "$0")/.."
for rep in 1 2; do
for E in RAFT_CORR_NT=0 RAFT_CORR_NT=1; do
  for A in "--height 1080 --width 1920 --precision bf16" "--batch 8 --height 540 --width 960"; do
    env $E timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-fp32-exact $A > gpurun_out/nt.json 2>gpurun_out/nt.err || { tail -5 gpurun_out/nt.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/nt.json')); print('$E', '$A', d['value'], d['ms_per_step'], 'lookup', d['roofline']['launch_us'])"
  done
done
done
