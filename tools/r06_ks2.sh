#!/bin/bash
# r06: the K-split halo form (RAFT_HALO_KS2=1) -- parity subset, conv_bench, stamps, forward A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
RAFT_HALO_KS2=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t_r06ks2.log 2>&1
rc=$?; tail -3 gpurun_out/t_r06ks2.log; [ $rc -eq 0 ] || exit $rc
for KS in 0 1; do echo "## KS2=$KS"; RAFT_HALO_KS2=$KS timeout -k 10 200 python tools/conv_bench.py 1 convc2,zr_split,fh1 || exit 1; done
for KS in 0 1; do echo "## stamps KS2=$KS"; RAFT_HALO_KS2=$KS HSTAMPS=1 RAFT_SKIP_SRC_CHECK=1 RAFT_HIP_LIB=ab/stamps/libraft_hip.so timeout -k 10 200 python tools/conv_bench.py 1 convc2,zr_split,fh1 || exit 1; done
bash tools/ab_env.sh "RAFT_HALO_KS2=0" "RAFT_HALO_KS2=1" || exit 1
bash tools/ab_env.sh "RAFT_HALO_NL8_ENC=1" "RAFT_HALO_NL8_ENC=0" || exit 1
