#!/bin/bash
# Round 5, step F: GPU suite (8 loaders default, convf1 A early); fused-lookup variants A/B + stamps.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/t_r05f.log 2>&1; rc=$?; tail -3 gpurun_out/t_r05f.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
./tools/ab_variants.sh "base a1off pf6" || exit 1
for V in lcst lcst0; do
  echo "== stamps $V"
  RAFT_SKIP_SRC_CHECK=1 RAFT_HIP_LIB=ab/$V/libraft_hip.so timeout -k 10 200 python tools/lc_stamps.py 2>&1 | grep -v amdgpu.ids || exit 1
done
