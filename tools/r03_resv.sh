#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
for V in ${VARS:-base noload nomfma noepi}; do
  if [ "$V" = base ]; then LIB=raft_optical_flow_amd/libraft_hip.so; else LIB=variants/$V/libraft_hip.so; fi
  for N in plain norm; do echo -n "$V "; RAFT_SKIP_SRC_CHECK=1 RAFT_HIP_LIB=$LIB timeout -k 10 120 python tools/res_bench.py $N 2>&1 | grep -v amdgpu.ids || exit 1; done
done
