set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/diag_e2e4.py > gpurun_out/diag10.log 2>&1; echo "diag rc=$?"; grep -v amdgpu.ids gpurun_out/diag10.log | tail -3
timeout -k 10 700 python -u -m pytest tests/test_gpu_lookup_conv.py tests/test_gpu_parity.py tests/test_gpu_configs.py -k "lookup_conv or hside or wide_tiles or e2e or encoders or in_norm or alt or config3 or graph or stem or instnorm" -x -q -rw --timeout 200 --timeout-method thread > gpurun_out/t_r3a.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -8 gpurun_out/t_r3a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/alt_bench.py 8 0.5 2>&1 | grep -v amdgpu.ids | tail -1
RAFT_HIP_LIB=variants/altst/libraft_hip.so timeout -k 10 120 python tools/alt_stamps.py 8 0.5 > gpurun_out/altst2.log 2>&1; echo "altst rc=$?"; grep -v amdgpu.ids gpurun_out/altst2.log | tail -30
AB="RAFT_FUSE_CONVC1=0" ./tools/r03_check.sh lc4 || exit 1
AB="RAFT_GRU_HSIDE=1" ./tools/r03_check.sh hs1 || exit 1
AB="RAFT_CONV_STEM=0 RAFT_EPI_STATS=0 RAFT_IN_NORM=0" TRACE=1 ./tools/r03_check.sh st1 || exit 1
AB="RAFT_HALO_WIDE=0" BENCH_ARGS="--height 1080 --width 1920 --precision bf16 --steps 5" ./tools/r03_check.sh c5w || exit 1
