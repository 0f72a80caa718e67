#!/bin/bash
# Configs 2-5 on one GPU with RAFT_CHAIN on / off (A/B on the same box); one bench JSON line each.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-sweep}
OUT=gpurun_out/sweep_$TAG.jsonl
mkdir -p gpurun_out
: > $OUT
run() {
  local E=$1; shift
  env $E timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-fp32-exact "$@" > gpurun_out/sw.json 2>> gpurun_out/sweep_$TAG.err || { echo "failed: $E $*"; tail -20 gpurun_out/sweep_$TAG.err; exit 1; }
  python -c "
import json,sys; d=json.load(open('gpurun_out/sw.json')); d['env']='$E'; d['args']='$*'
open('$OUT','a').write(json.dumps(d)+'\n')
r=d['roofline']; u=d['update_gemm']
print('$E', '$*', d['value'], 'iter', d['iteration']['iteration_us'], 'convs', u['convs_us'], u['frac'], 'roof', r.get('launch_us', r.get('iteration_us')), r['frac'])"
}
for E in RAFT_CHAIN=0 RAFT_CHAIN=1; do run $E --steps 20; done
for E in RAFT_CHAIN=0 RAFT_CHAIN=1; do run $E --batch 8 --height 540 --width 960; done   # config 4 (per GPU)
for E in RAFT_CHAIN=0 RAFT_CHAIN=1; do run $E --batch 8 --alternate-corr; done            # config 3
run RAFT_X=0 --batch 1 --height 1080 --width 1920 --precision bf16                       # config 5
