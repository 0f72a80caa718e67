set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/diag_e2e6.py > gpurun_out/diag6.log 2>&1; echo "diag rc=$?"; grep -v amdgpu.ids gpurun_out/diag6.log | tail -25
SYNC_BEFORE=1 timeout -k 10 300 python tools/diag_e2e6.py > gpurun_out/diag6s.log 2>&1; echo "diag rc=$?"; grep -v amdgpu.ids gpurun_out/diag6s.log | tail -25
