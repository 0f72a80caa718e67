#!/bin/bash
# BASELINE.json configs 3-5 on one GPU (config 2 is bench.py's default line; config 4's 64 pairs over
# 8 GPUs = 8 pairs per GPU, so its per-GPU workload is measured here at --batch 8).
# Each line is bench.py's JSON; the sweep stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-sweep}
OUT=gpurun_out/sweep_$TAG.jsonl
mkdir -p gpurun_out
: > $OUT
run() {
  echo "== $*" >&2
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-fp32-exact "$@" >> $OUT 2>> gpurun_out/sweep_$TAG.err || { echo "failed: $*"; tail -20 gpurun_out/sweep_$TAG.err; exit 1; }
  tail -1 $OUT
}
run --batch 8 --alternate-corr                                   # config 3
run --batch 8 --height 540 --width 960                           # config 4 (per GPU)
run --batch 1 --height 1080 --width 1920 --precision bf16        # config 5 (bf16 mixed precision)
run --batch 4 --height 1080 --width 1920 --precision bf16        # config 5, 4 pairs per GPU
run --batch 1 --height 1080 --width 1920 --precision f16         # config 5 geometry, the reference's fp16 autocast
run --batch 1 --height 1080 --width 1920                         # config 5 geometry, fp32-accurate convs
