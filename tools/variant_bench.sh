#!/bin/bash
# conv_bench over library variants (ab/<name>/libraft_hip.so; "base" = the in-tree build)
# usage: tools/variant_bench.sh "base ns4" "f16x3 f16" [B] [shapes]
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
B=${3:-1}; SH=${4:-}
for V in $1; do
  for P in $2; do
    if [ "$V" = base ]; then LIB=raft_optical_flow_amd/libraft_hip.so; else LIB=ab/$V/libraft_hip.so; fi
    echo "== $V $P"
    RAFT_SKIP_SRC_CHECK=1 RAFT_HIP_LIB=$LIB PREC=$P timeout -k 10 120 python tools/conv_bench.py $B $SH 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
