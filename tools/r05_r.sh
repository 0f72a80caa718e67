#!/bin/bash
# Round 5, step R: the window-parameter table on the 64-bit (large-pyramid) path too: lookup tests (incl.
# the 135x240 large-pyramid case), config-5 stamps, config 5 A/B vs the per-load scalar chain (lt0).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_lookup_conv.py -q -x --timeout 200 --timeout-method thread 2>&1 | tail -1 || exit 1
for V in lcst lcst0; do
  echo "== stamps $V config 5"
  RAFT_SKIP_SRC_CHECK=1 RAFT_HIP_LIB=ab/$V/libraft_hip.so timeout -k 10 200 python tools/lc_stamps.py --h 1080 --w 1920 --precision bf16 2>&1 | grep -v amdgpu.ids | grep -v "wave starts" | tail -10 || exit 1
done
./tools/ab_variants.sh "base lt0" "--batch 1 --height 1080 --width 1920 --precision bf16 --steps 5 --warmup 1" || exit 1
