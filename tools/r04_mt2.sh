#!/bin/bash
# Multi-tile halo work-groups, config-5 shapes: the update convs at 135x240 (B=1) in bf16 and f16x3
# with RAFT_HALO_MT off / on, and their phase stamps (variants/hst).
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${TAG:-r04mt2}
O=gpurun_out/exp_${TAG}.txt
mkdir -p gpurun_out
: > $O
run() { echo "== $*" >> $O; timeout -k 10 200 "$@" >> $O 2>&1 || { echo "failed: $*"; tail -30 $O; exit 1; }; }
# the 256 x 256 correlation build first: its tests, then alone at the configs' maps
timeout -k 10 300 python -u -m pytest tests/test_gpu_corr_build.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_${TAG}_corr.log 2>&1
rc=$?; tail -4 gpurun_out/t_${TAG}_corr.log; [ $rc -eq 0 ] || exit $rc
run python tools/corr4_bench.py 1 55 128
run python tools/corr4_bench.py 1 135 240
run python tools/corr4_bench.py 8 68 120
for prec in bf16 f16x3; do
  for mt in 0 1; do
    run env RAFT_HALO_MT=$mt PREC=$prec CB_H=135 CB_W=240 python tools/conv_bench.py 1 convc1,convc2,conv,zr_split,q_split,fh1
  done
done
for mt in 0 1; do
  run env RAFT_HALO_MT=$mt PREC=bf16 CB_H=135 CB_W=240 RAFT_HIP_LIB=variants/hst/libraft_hip.so HSTAMPS=1 python tools/conv_bench.py 1 convc2,zr_split,fh1
done
grep -v amdgpu.ids $O
