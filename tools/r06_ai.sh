#!/bin/bash
# r06: the GRU context term (add0) as the accumulators initial value (HALO_ADD0_INIT) vs in the epilogue (ai0): GPU tests on the default
# build, then forward A/B interleaved on one box (bench.py) and one rocprof in-forward trace per variant
# (per-slot means)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "halo or parity or update or conv or raft or chain or gru or golden" > gpurun_out/t_r06ai.log 2>&1
rc=$?; tail -3 gpurun_out/t_r06ai.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_variants.sh "base ai0" || exit 1
export RAFT_SKIP_SRC_CHECK=1
for V in base ai0; do
  if [ "$V" = base ]; then LIB=raft_optical_flow_amd/libraft_hip.so; else LIB=ab/$V/libraft_hip.so; fi
  export RAFT_HIP_LIB=$LIB
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/fwdai_$V -o run --output-format csv -- python tools/fwd_profile.py 1 440 1024 f16x3 > gpurun_out/fwdai_$V.log 2>&1 || { tail -20 gpurun_out/fwdai_$V.log; exit 1; }
  python tools/phase_summary.py gpurun_out/fwdai_$V/run_kernel_trace.csv > gpurun_out/ai_${V}_phases.txt 2>&1
  echo "== $V"; sed -n '/loop span/,/sum /p' gpurun_out/ai_${V}_phases.txt
done
