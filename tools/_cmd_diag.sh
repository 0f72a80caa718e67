set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/diag_e2e.py > gpurun_out/diag1.log 2>&1; echo "diag rc=$?"; grep -v amdgpu.ids gpurun_out/diag1.log | tail -12
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "stem or instnorm or in_norm or encoders or wide_tiles" -q --timeout 200 --timeout-method thread > gpurun_out/t_enc1.log 2>&1; echo "tests rc=$?"; tail -15 gpurun_out/t_enc1.log
for sp in 0.5 2 8; do timeout -k 10 120 python tools/alt_bench.py 8 $sp 2>&1 | grep -v amdgpu.ids | tail -1; done
timeout -k 10 300 python tools/alt_boxes.py 8 32 > gpurun_out/altbox.log 2>&1; echo "altbox rc=$?"; grep -v amdgpu.ids gpurun_out/altbox.log | tail -8
