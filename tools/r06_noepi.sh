#!/bin/bash
# r06: timing ablation of the conv epilogue operand loads (HALO_ABL_NOEPI, wrong results): forward A/B
# interleaved on one box (bench.py), then one rocprof in-forward trace per variant (per-slot means)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_variants.sh "base noepi" || exit 1
export RAFT_SKIP_SRC_CHECK=1
for V in base noepi; do
  if [ "$V" = base ]; then LIB=raft_optical_flow_amd/libraft_hip.so; else LIB=ab/$V/libraft_hip.so; fi
  export RAFT_HIP_LIB=$LIB
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/fwdne_$V -o run --output-format csv -- python tools/fwd_profile.py 1 440 1024 f16x3 > gpurun_out/fwdne_$V.log 2>&1 || { tail -20 gpurun_out/fwdne_$V.log; exit 1; }
  python tools/phase_summary.py gpurun_out/fwdne_$V/run_kernel_trace.csv > gpurun_out/ne_${V}_phases.txt 2>&1
  echo "== $V"; sed -n '/loop span/,/sum /p' gpurun_out/ne_${V}_phases.txt
done
