#!/bin/bash
# Tile-choice knobs for config 5 (bf16) and config 4 on one box: the wide 128-column tiles from one
# round of them (RAFT_HALO_WIDE_MIN=256) and a lower big-tile cost (RAFT_HALO_BIG_COST=1.4).
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${TAG:-r04j}
O=gpurun_out/exp_${TAG}.txt
mkdir -p gpurun_out
: > $O
run() { echo "== $*" >> $O; timeout -k 10 200 "$@" >> $O 2>&1 || { echo "failed: $*"; tail -30 $O; exit 1; }; }
for v in "X=0" "RAFT_HALO_WIDE_MIN=256"; do
  run env $v PREC=bf16 CB_H=135 CB_W=240 python tools/conv_bench.py 1 convc1,convc2,conv,zr_split,q_split,fh1
done
for r in 1 2; do
  for v in "X=0" "RAFT_HALO_WIDE_MIN=256" "RAFT_HALO_BIG_COST=1.4" "RAFT_HALO_WIDE_MIN=256 RAFT_HALO_BIG_COST=1.4"; do
    echo "== $v bench config5" >> $O
    env $v timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-fp32-exact --batch 1 --height 1080 --width 1920 --precision bf16 >> $O 2>> gpurun_out/exp_${TAG}.err || { echo failed; tail -20 gpurun_out/exp_${TAG}.err; exit 1; }
  done
done
for v in "X=0" "RAFT_FUSE_CONVC1=0"; do
  echo "== $v bench config5" >> $O
  env $v timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-fp32-exact --batch 1 --height 1080 --width 1920 --precision bf16 >> $O 2>> gpurun_out/exp_${TAG}.err || { echo failed; tail -20 gpurun_out/exp_${TAG}.err; exit 1; }
done
for v in "X=0" "RAFT_HALO_BIG_COST=1.4" "RAFT_FUSE_CONVC1=0"; do
  echo "== $v bench config4" >> $O
  env $v timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-fp32-exact --batch 8 --height 540 --width 960 >> $O 2>> gpurun_out/exp_${TAG}.err || { echo failed; tail -20 gpurun_out/exp_${TAG}.err; exit 1; }
done
python - "$O" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("=="): tag = line.strip()
    elif line.startswith("{"):
        d = json.loads(line); print(tag, d["value"], "upd", d["update_gemm"]["convs_us"], "it", d["iteration"]["iteration_us"])
    elif " us " in line and "TF/s" in line: print("  ", line.rstrip())
PY
