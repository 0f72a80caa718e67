#!/bin/bash
# Round 5, step F: GPU suite (8 loaders default, convf1 A early); fused-lookup variants A/B + stamps.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/t_r05f.log 2>&1; rc=$?; tail -3 gpurun_out/t_r05f.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
./tools/ab_variants.sh "base a1off pf6" || exit 1
for V in lcst lcst0; do
  echo "== stamps $V"
  RAFT_SKIP_SRC_CHECK=1 RAFT_HIP_LIB=ab/$V/libraft_hip.so timeout -k 10 200 python tools/lc_stamps.py 2>&1 | grep -v amdgpu.ids || exit 1
done
echo "== encoder tests with RAFT_HALO_NL8_ENC=1"
RAFT_HALO_NL8_ENC=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_halo_mt.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -q --timeout 120 --timeout-method thread -k "encoder or instnorm or in_norm or multi_tile or full_size or stem" > gpurun_out/t_r05f_enc.log 2>&1; rc=$?; tail -3 gpurun_out/t_r05f_enc.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for rep in 1 2; do
  for E in 0 1; do
    RAFT_HALO_NL8_ENC=$E timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-fp32-exact > gpurun_out/nl8e_$E.json 2> gpurun_out/nl8e_$E.err || { tail -20 gpurun_out/nl8e_$E.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/nl8e_$E.json')); print('NL8_ENC=$E', d['value'], 'ms', d['ms_per_step'])"
  done
done
RAFT_HALO_NL8_ENC=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fpf2 -o run --output-format csv -- python tools/fwd_profile.py 1 440 1024 f16x3 > gpurun_out/fpf2.log 2>&1 || { tail -20 gpurun_out/fpf2.log; exit 1; }
python tools/phase_summary.py gpurun_out/fpf2/run_kernel_trace.csv > gpurun_out/phase_r05f_config2_nl8enc.txt 2>&1
grep -E "forward span|encoder phase span|loop span" gpurun_out/phase_r05f_config2_nl8enc.txt
