set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_lookup_conv.py tests/test_gpu_parity.py -k "lookup_conv or stem or conv2d_vs or instnorm or in_norm or encoders or e2e or full_size" -x -q --timeout 200 --timeout-method thread > gpurun_out/t_lc4.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/t_lc4.log; [ $rc -eq 0 ] || exit $rc
RAFT_HIP_LIB=variants/lcst/libraft_hip.so timeout -k 10 200 python tools/lc_stamps.py > gpurun_out/lcst4.log 2>&1; echo "stamps rc=$?"; grep -v amdgpu.ids gpurun_out/lcst4.log
AB="RAFT_FUSE_CONVC1=0" ./tools/r03_check.sh lc4 || exit 1
AB="RAFT_CONV_STEM=0 RAFT_EPI_STATS=0 RAFT_IN_NORM=0" TRACE=1 ./tools/r03_check.sh st1 || exit 1
timeout -k 10 300 python tools/alt_boxes.py 8 32 > gpurun_out/altbox.log 2>&1; echo "altbox rc=$?"; grep -v amdgpu.ids gpurun_out/altbox.log | tail -8
