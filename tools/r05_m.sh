#!/bin/bash
# Round 5, step M: the alternate lookup's band split as an ablation (nosplit: the band stored as loaded,
# wrong results) - the bound on what maps split once per forward could give; stamps of both.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for V in base nosplit; do
    if [ "$V" = base ]; then LIB=raft_optical_flow_amd/libraft_hip.so; else LIB=ab/$V/libraft_hip.so; fi
    for sg in 0 1; do
      echo -n "$V sigma $sg: "
      RAFT_SKIP_SRC_CHECK=1 RAFT_HIP_LIB=$LIB timeout -k 10 200 python tools/alt_bench.py 8 $sg 2>&1 | grep "alt lookup" || exit 1
    done
  done
done
for V in altst altst_ns; do
  echo "== stamps $V"
  RAFT_SKIP_SRC_CHECK=1 RAFT_HIP_LIB=ab/$V/libraft_hip.so timeout -k 10 200 python tools/alt_stamps.py 8 1 2>&1 | grep -v amdgpu.ids | head -40 || exit 1
done
