set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
RAFT_HIP_LIB=variants/lcfence/libraft_hip.so timeout -k 10 300 python tools/diag_e2e4.py > gpurun_out/diag7.log 2>&1; echo "diag rc=$?"; grep -v amdgpu.ids gpurun_out/diag7.log | tail -6
HIP_LAUNCH_BLOCKING=1 timeout -k 10 300 python tools/diag_e2e4.py > gpurun_out/diag7b.log 2>&1; echo "diag rc=$?"; grep -v amdgpu.ids gpurun_out/diag7b.log | tail -6
