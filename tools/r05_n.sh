#!/bin/bash
# Round 5, step N: the alternate lookup's box GEMM on 4 waves of 32x48 (m16x2, ALT_MFMA16=2) vs 8 waves
# of 16x48 (base): alt tests on the variant, alt_bench sigma 0 / 1 interleaved, MFMA-phase stamps.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
RAFT_SKIP_SRC_CHECK=1 RAFT_HIP_LIB=ab/m16x2/libraft_hip.so timeout -k 10 300 python -u -m pytest tests -m gpu -q -x -k "alt or config3" --timeout 120 --timeout-method thread 2>&1 | tail -2 || exit 1
for rep in 1 2; do
  for V in base m16x2; do
    if [ "$V" = base ]; then LIB=raft_optical_flow_amd/libraft_hip.so; else LIB=ab/$V/libraft_hip.so; fi
    for sg in 0 1; do
      echo -n "$V sigma $sg: "
      RAFT_SKIP_SRC_CHECK=1 RAFT_HIP_LIB=$LIB timeout -k 10 200 python tools/alt_bench.py 8 $sg 2>&1 | grep "alt lookup" || exit 1
    done
  done
done
for V in altst altst2; do
  echo "== stamps $V"
  RAFT_SKIP_SRC_CHECK=1 RAFT_HIP_LIB=ab/$V/libraft_hip.so timeout -k 10 200 python tools/alt_stamps.py 8 1 2>&1 | grep -E "wave|MFMAs|sync 2|total" || exit 1
done
