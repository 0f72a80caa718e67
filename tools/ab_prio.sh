#!/bin/bash
# A/B of the halo compute waves' s_setprio (dev variants built with -DHALO_PRIO=1 / 3 into ab/)
for L in ab/prio1 ab/prio3 raft_optical_flow_amd; do
  RAFT_HIP_LIB=$L/libraft_hip.so timeout -k 10 200 python tools/fixed_cost.py 2>&1 | grep fixed | sed "s|^|$L |"
done
./tools/ab_env.sh "RAFT_HIP_LIB=raft_optical_flow_amd/libraft_hip.so" "RAFT_HIP_LIB=ab/prio1/libraft_hip.so" "RAFT_HIP_LIB=ab/prio3/libraft_hip.so"
