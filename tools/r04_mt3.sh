#!/bin/bash
# Multi-tile halo work-groups (same N-tile, consecutive spatial tiles) and corr_build4 stamps, one box.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${TAG:-r04mt3}
O=gpurun_out/exp_${TAG}.txt
mkdir -p gpurun_out
: > $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_halo_mt.py tests/test_gpu_corr_build.py -q --timeout 240 --timeout-method thread > gpurun_out/t_${TAG}_first.log 2>&1
rc=$?; tail -4 gpurun_out/t_${TAG}_first.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc  # (1: test failures only; anything else stops)
run() { echo "== $*" >> $O; timeout -k 10 200 "$@" >> $O 2>&1 || { echo "failed: $*"; tail -30 $O; exit 1; }; }
run env RAFT_HIP_LIB=variants/cb4st/libraft_hip.so python tools/cb4_stamps.py 1 55 128
run env RAFT_HIP_LIB=variants/cb4st/libraft_hip.so python tools/cb4_stamps.py 1 135 240
for prec in bf16 f16x3; do
  for mt in 0 1; do
    run env RAFT_HALO_MT=$mt PREC=$prec CB_H=135 CB_W=240 python tools/conv_bench.py 1 convc1,convc2,conv,zr_split,q_split,fh1
  done
done
for mt in 0 1; do
  run env RAFT_HALO_MT=$mt SHAPESET=enc python tools/conv_bench.py 1
  run env RAFT_HALO_MT=$mt python tools/conv_bench.py 8 convc2,conv,zr_split,q_split,fh1
done
for a in "--batch 1 --height 1080 --width 1920 --precision bf16" "--batch 8 --height 540 --width 960" ""; do
  for mt in 1 0; do
    echo "== RAFT_HALO_MT=$mt bench $a" >> $O
    RAFT_HALO_MT=$mt timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-fp32-exact $a >> $O 2>> gpurun_out/exp_${TAG}.err || { echo failed; tail -20 gpurun_out/exp_${TAG}.err; exit 1; }
  done
done
python - "$O" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("=="): tag = line.strip()
    elif line.startswith("{"):
        d = json.loads(line); print(tag, d["value"], "upd", d["update_gemm"]["convs_us"], "it", d["iteration"]["iteration_us"])
    elif (" us " in line and "TF/s" in line) or "cyc" in line or "stamps" in line: print("  ", line.rstrip())
PY
