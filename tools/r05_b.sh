#!/bin/bash
# Round 5, step B: halo conv phase stamps, this tree (ab/hst, ab/hstwx) vs the round-3 head (ab/r3 + its STAMPS build), interleaved.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
SH=convc2,conv,zr_split,q_split,fh1
for rep in 1 2; do
  echo "== cur hst $rep"
  HSTAMPS=1 RAFT_SKIP_SRC_CHECK=1 RAFT_HIP_LIB=ab/hst/libraft_hip.so timeout -k 10 200 python tools/conv_bench.py 1 $SH 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== r3 r3st $rep"
  (cd ab/r3 && HSTAMPS=1 RAFT_SKIP_SRC_CHECK=1 RAFT_HIP_LIB=variants/r3st/libraft_hip.so timeout -k 10 200 python tools/conv_bench.py 1 $SH 2>&1 | grep -v amdgpu.ids) || exit 1
done
echo "== cur hstwx"
HSTAMPS=1 RAFT_SKIP_SRC_CHECK=1 RAFT_HIP_LIB=ab/hstwx/libraft_hip.so timeout -k 10 200 python tools/conv_bench.py 1 $SH 2>&1 | grep -v amdgpu.ids || exit 1
