set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
RAFT_HIP_LIB=variants/lcst/libraft_hip.so timeout -k 10 200 python tools/lc_stamps.py > gpurun_out/lcst1.log 2>&1; echo "stamps rc=$?"; cat gpurun_out/lcst1.log | grep -v amdgpu.ids
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_configs.py tests/test_capi.py -x -q --timeout 300 --timeout-method thread -k "range_guard or backward or dist or rccl or sharded or bf16 or capi or alt" > gpurun_out/t_misc1.log 2>&1; echo "tests rc=$?"; tail -25 gpurun_out/t_misc1.log
