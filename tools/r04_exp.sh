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
if [ "${CONV:-1}" != 0 ]; then
for big in 0 1; do
  run env RAFT_HALO_BIG_MIN=$big SHAPESET=enc python tools/conv_bench.py 1
  run env RAFT_HALO_BIG_MIN=$big python tools/conv_bench.py 8 convc2,conv,zr_split,q_split,fh1
done
run python tools/conv_bench.py 1
fi
if [ "${STAMPS:-1}" != 0 ]; then
run env RAFT_HIP_LIB=variants/hst/libraft_hip.so HSTAMPS=1 python tools/conv_bench.py 1 convc2,conv,zr_split,q_split,fh1
run env RAFT_HIP_LIB=variants/hst/libraft_hip.so HSTAMPS=1 SHAPESET=enc python tools/conv_bench.py 1
run env RAFT_HIP_LIB=variants/lcst/libraft_hip.so python tools/lc_stamps.py
fi
if [ "${ALT:-0}" != 0 ]; then  # config 3's alternate lookup: MFMA box GEMM vs the VALU tile kernel, and its phase stamps
  for sp in 0 1; do
    run python tools/alt_bench.py 8 $sp
    run env RAFT_ALT_MFMA=0 python tools/alt_bench.py 8 $sp
  done
  run env RAFT_HIP_LIB=variants/altst/libraft_hip.so python tools/alt_stamps.py 8 1
fi
if [ -n "$AB_CONFIGS" ]; then  # the forward with the big tiles off, same box (A/B against r04_check's sweep)
  for a in "--batch 8 --height 540 --width 960" "--batch 1 --height 1080 --width 1920 --precision bf16" ""; do
    echo "== RAFT_HALO_BIG_MIN=0 bench $a" >> $O
    RAFT_HALO_BIG_MIN=0 timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-fp32-exact $a >> $O 2>> gpurun_out/exp_${TAG}.err || { echo failed; exit 1; }
  done
fi
if [ -n "$TRACE5" ]; then  # kernel trace + phase summary of a config-5 forward (1080x1920 bf16, B=1)
  export TMPDIR=/tmp
  ALT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fp5_${TAG} -o run --output-format csv -- python tools/fwd_profile.py 1 1080 1920 bf16 > gpurun_out/fp5_${TAG}.log 2>&1 || { echo trace5 failed; exit 1; }
  python tools/phase_summary.py gpurun_out/fp5_${TAG}/run_kernel_trace.csv > gpurun_out/phase5_${TAG}.txt 2>&1
fi
cat $O
