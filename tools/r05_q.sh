#!/bin/bash
# Round 5, step Q: the fused lookup's window parameters as a per-lane table read back by v_readlane
# (LC_TAB=1, base) vs the per-load scalar chain (lt0): lookup tests, stamps at configs 2 / 5, configs 2 / 5.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_lookup_conv.py tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread 2>&1 | tail -1 || exit 1
for V in lcst lcst0; do
  echo "== stamps $V config 2"
  RAFT_SKIP_SRC_CHECK=1 RAFT_HIP_LIB=ab/$V/libraft_hip.so timeout -k 10 200 python tools/lc_stamps.py 2>&1 | grep -v amdgpu.ids | grep -v "wave starts" | tail -10 || exit 1
  echo "== stamps $V config 5"
  RAFT_SKIP_SRC_CHECK=1 RAFT_HIP_LIB=ab/$V/libraft_hip.so timeout -k 10 200 python tools/lc_stamps.py --h 1080 --w 1920 --precision bf16 2>&1 | grep -v amdgpu.ids | grep -v "wave starts" | tail -10 || exit 1
done
./tools/ab_variants.sh "base lt0" || exit 1
./tools/ab_variants.sh "base lt0" "--batch 1 --height 1080 --width 1920 --precision bf16 --steps 5 --warmup 1" || exit 1
