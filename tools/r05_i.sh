#!/bin/bash
# Round 5, step I: the fused lookup's 32-bit-offset tile issue, more reps + stamps of both forms
# at configs 2 and 5.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for V in lcst lcst0; do
  echo "== stamps $V config 2"
  RAFT_SKIP_SRC_CHECK=1 RAFT_HIP_LIB=ab/$V/libraft_hip.so timeout -k 10 200 python tools/lc_stamps.py 2>&1 | grep -v amdgpu.ids | tail -12 || exit 1
  echo "== stamps $V config 5"
  RAFT_SKIP_SRC_CHECK=1 RAFT_HIP_LIB=ab/$V/libraft_hip.so timeout -k 10 200 python tools/lc_stamps.py --h 1080 --w 1920 --precision bf16 2>&1 | grep -v amdgpu.ids | tail -12 || exit 1
done
./tools/ab_variants.sh "o32off base" || exit 1
