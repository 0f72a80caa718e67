#!/bin/bash
# Round 5, step C: GPU suite; same-box A/B vs the round-3 head (bench lines, forward traces); halo phase stamps
# of both, interleaved.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/t_r05c.log 2>&1; rc=$?; tail -3 gpurun_out/t_r05c.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
./tools/ab_tree.sh "r3 cur" 2 || exit 1
for V in cur r3; do
  if [ $V = cur ]; then T=tools; else T=ab/r3/tools; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fpc_$V -o run --output-format csv -- python $T/fwd_profile.py 1 440 1024 f16x3 > gpurun_out/fpc_$V.log 2>&1 || { tail -20 gpurun_out/fpc_$V.log; exit 1; }
  python tools/phase_summary.py gpurun_out/fpc_$V/run_kernel_trace.csv > gpurun_out/phase_r05c_$V.txt 2>&1
  grep -E "forward span|encoder phase span|loop span" gpurun_out/phase_r05c_$V.txt
done
SH=convc2,conv,zr_split,q_split,fh1
echo "== cur hst"
HSTAMPS=1 RAFT_SKIP_SRC_CHECK=1 RAFT_HIP_LIB=ab/hst/libraft_hip.so timeout -k 10 200 python tools/conv_bench.py 1 $SH 2>&1 | grep -v amdgpu.ids || exit 1
echo "== r3 r3st"
(cd ab/r3 && HSTAMPS=1 RAFT_SKIP_SRC_CHECK=1 RAFT_HIP_LIB=variants/r3st/libraft_hip.so timeout -k 10 200 python tools/conv_bench.py 1 $SH 2>&1 | grep -v amdgpu.ids) || exit 1
echo "== stamps lcst2"
RAFT_SKIP_SRC_CHECK=1 RAFT_HIP_LIB=ab/lcst2/libraft_hip.so timeout -k 10 200 python tools/lc_stamps.py 2>&1 | grep -v amdgpu.ids || exit 1
