set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/diag_e2e4.py > gpurun_out/diag4.log 2>&1; echo "diag rc=$?"; grep -v amdgpu.ids gpurun_out/diag4.log | tail -8
