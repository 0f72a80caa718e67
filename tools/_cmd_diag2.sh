set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/diag_e2e2.py > gpurun_out/diag2.log 2>&1; echo "diag rc=$?"; grep -v amdgpu.ids gpurun_out/diag2.log | tail -12
timeout -k 10 300 python -u -m pytest tests/test_gpu_lookup_conv.py -q -rw --timeout 200 --timeout-method thread > gpurun_out/t_lc5.log 2>&1; echo "tests rc=$?"; tail -15 gpurun_out/t_lc5.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_lookup_conv.py -q -rw -k matches_unfused --timeout 200 --timeout-method thread > gpurun_out/t_lc6.log 2>&1; echo "tests rc=$?"; tail -5 gpurun_out/t_lc6.log
RAFT_HIP_LIB=variants/altst/libraft_hip.so timeout -k 10 120 python tools/alt_stamps.py 8 0.5 > gpurun_out/altst1.log 2>&1; echo "altst rc=$?"; grep -v amdgpu.ids gpurun_out/altst1.log | tail -30
