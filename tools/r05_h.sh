#!/bin/bash
# Round 5, step H: GPU suite; the fused lookup's 32-bit-offset tile issue A/B + stamps.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/t_r05h.log 2>&1; rc=$?; tail -3 gpurun_out/t_r05h.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
./tools/ab_variants.sh "base o32off" || exit 1
echo "== stamps lcst"
RAFT_SKIP_SRC_CHECK=1 RAFT_HIP_LIB=ab/lcst/libraft_hip.so timeout -k 10 200 python tools/lc_stamps.py 2>&1 | grep -v amdgpu.ids || exit 1
