#!/bin/bash
# Round 5, step L: the alternate lookup's MFMAs on all 8 waves (16x16 blocks, ALT_MFMA16) vs 6 waves of
# 32x32 blocks (am32): alt tests, alt_bench sigma 0 / 1, config 3 bench, interleaved.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x -k "alt or config3" --timeout 120 --timeout-method thread 2>&1 | tail -2 || exit 1
for rep in 1 2; do
  for V in base am32; do
    if [ "$V" = base ]; then LIB=raft_optical_flow_amd/libraft_hip.so; else LIB=ab/$V/libraft_hip.so; fi
    for sg in 0 1; do
      echo -n "$V sigma $sg: "
      RAFT_SKIP_SRC_CHECK=1 RAFT_HIP_LIB=$LIB timeout -k 10 200 python tools/alt_bench.py 8 $sg 2>&1 | grep "alt lookup" || exit 1
    done
  done
done
./tools/ab_variants.sh "base am32" "--batch 8 --alternate-corr --steps 5 --warmup 1" || exit 1
