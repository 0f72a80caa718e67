#!/bin/bash
# Round-4 kernel experiments on one box (each step time-limited, the chain stops at a failure):
#   the update convs at B=1 and B=8 and the encoder convs, big tiles on / off (RAFT_HALO_BIG_MIN=0);
#   halo phase stamps (variants/hst, -DSTAMPS) and fused-lookup stamps (variants/lcst, -DLC_STAMPS).
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${TAG:-r04}
O=gpurun_out/exp_${TAG}.txt
mkdir -p gpurun_out
: > $O
run() { echo "== $*" >> $O; timeout -k 10 200 "$@" >> $O 2>&1 || { echo "failed: $*"; tail -30 $O; exit 1; }; }
for big in 0 512; do
  run env RAFT_HALO_BIG_MIN=$big SHAPESET=enc python tools/conv_bench.py 1
  run env RAFT_HALO_BIG_MIN=$big python tools/conv_bench.py 8 convc2,conv,zr_split,q_split,fh1
done
run python tools/conv_bench.py 1
run env RAFT_HIP_LIB=variants/hst/libraft_hip.so HSTAMPS=1 python tools/conv_bench.py 1 convc2,conv,zr_split,q_split,fh1
run env RAFT_HIP_LIB=variants/hst/libraft_hip.so HSTAMPS=1 SHAPESET=enc python tools/conv_bench.py 1
run env RAFT_HIP_LIB=variants/lcst/libraft_hip.so python tools/lc_stamps.py
cat $O
