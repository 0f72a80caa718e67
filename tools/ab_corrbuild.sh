#!/bin/bash
# Corr-build A/B on one box: pyramid parity subset, tools/corr_build_bench.py for ab/base vs the
# in-tree library (three interleaved pairs), then the forward (tools/ab_env.sh).
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pyramid or corr_build or full_size or config or golden" > gpurun_out/t_abcb.log 2>&1; rc=$?; tail -2 gpurun_out/t_abcb.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  RAFT_HIP_LIB=ab/base/libraft_hip.so timeout -k 10 100 python tools/corr_build_bench.py 1 | sed "s|^|base |"
  timeout -k 10 100 python tools/corr_build_bench.py 1 | sed "s|^|new  |"
done
./tools/ab_env.sh "RAFT_HIP_LIB=ab/base/libraft_hip.so" "RAFT_HIP_LIB=raft_optical_flow_amd/libraft_hip.so"
