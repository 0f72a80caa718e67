#!/bin/bash
# Round 5, step G: evidence part a on the current tree (tests, smoke, bench, rocprof of the bench, forward
# trace), then the fused lookup's stamps with the coords-arrival split.
set -o pipefail
cd "$(dirname "$0")/.."
./tools/evidence.sh r05 || exit 1
echo "== stamps lcst"
RAFT_SKIP_SRC_CHECK=1 RAFT_HIP_LIB=ab/lcst/libraft_hip.so timeout -k 10 200 python tools/lc_stamps.py 2>&1 | grep -v amdgpu.ids || exit 1
