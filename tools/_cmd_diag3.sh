set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for pre in none rg all noise; do PRE=$pre timeout -k 10 200 python tools/diag_e2e3.py > gpurun_out/diag3_$pre.log 2>&1; echo "diag $pre rc=$?"; grep -v amdgpu.ids gpurun_out/diag3_$pre.log | tail -4; done
