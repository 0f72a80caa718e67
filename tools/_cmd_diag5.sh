set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/diag_e2e5.py > gpurun_out/diag5.log 2>&1; echo "diag rc=$?"; grep -v amdgpu.ids gpurun_out/diag5.log | tail -25
