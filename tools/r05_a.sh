#!/bin/bash
# Round 5, step A: GPU suite on this tree, then the same-box A/B against the round-3 head (ab/r3) and
# forward kernel traces of both at config 2.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/t_r05a.log 2>&1; rc=$?; tail -3 gpurun_out/t_r05a.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
./tools/ab_tree.sh "r3 cur" 2 || exit 1
for V in cur r3; do
  if [ $V = cur ]; then T=tools; else T=ab/r3/tools; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fp_$V -o run --output-format csv -- python $T/fwd_profile.py 1 440 1024 f16x3 > gpurun_out/fp_$V.log 2>&1 || { tail -20 gpurun_out/fp_$V.log; exit 1; }
  python tools/phase_summary.py gpurun_out/fp_$V/run_kernel_trace.csv > gpurun_out/phase_r05a_$V.txt 2>&1
  grep -E "forward span|encoder phase span|loop span" gpurun_out/phase_r05a_$V.txt
done
./tools/ab_variants.sh "base lce7 lct2 lct2e7 hwx1" || exit 1
for V in lcst lcst7 lcst2; do
  echo "== stamps $V"
  RAFT_SKIP_SRC_CHECK=1 RAFT_HIP_LIB=ab/$V/libraft_hip.so timeout -k 10 200 python tools/lc_stamps.py 2>&1 | grep -v amdgpu.ids || exit 1
done
./tools/variant_bench.sh "base hwx1" f16x3 1 || exit 1
for V in hst hstwx; do
  echo "== halo stamps $V"
  HSTAMPS=1 RAFT_SKIP_SRC_CHECK=1 RAFT_HIP_LIB=ab/$V/libraft_hip.so timeout -k 10 200 python tools/conv_bench.py 1 convc2,conv,zr_split,q_split,fh1 2>&1 | grep -v amdgpu.ids || exit 1
done
