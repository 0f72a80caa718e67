#!/bin/bash
# Lookup-kernel A/B on one box: parity subset, then tools/lookup_rot.py (cache-cold B=1 / B=8) for
# ab/base vs the in-tree library, three interleaved pairs, then the forward (tools/ab_env.sh).
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "lookup or pyramid or full_size or config or radius or guard or smoke" > gpurun_out/t_ablk.log 2>&1; rc=$?; tail -2 gpurun_out/t_ablk.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  RAFT_HIP_LIB=ab/base/libraft_hip.so timeout -k 10 100 python tools/lookup_rot.py | sed "s|^|base |"
  timeout -k 10 100 python tools/lookup_rot.py | sed "s|^|new  |"
done
./tools/ab_env.sh "RAFT_HIP_LIB=ab/base/libraft_hip.so" "RAFT_HIP_LIB=raft_optical_flow_amd/libraft_hip.so"
