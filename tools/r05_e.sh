#!/bin/bash
# Round 5, step E: GPU suite; the halo kernel's 8-loader form A/B (RAFT_HALO_NL8) at config 2, interleaved.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/t_r05e.log 2>&1; rc=$?; tail -3 gpurun_out/t_r05e.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for rep in 1 2 3; do
  for E in 0 1; do
    RAFT_HALO_NL8=$E timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-fp32-exact > gpurun_out/nl8_$E.json 2> gpurun_out/nl8_$E.err || { tail -20 gpurun_out/nl8_$E.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/nl8_$E.json')); dk=d.get('dominant_kernel') or {}; print('NL8=$E', d['value'], 'iter', d['iteration']['iteration_us'], 'convs', d['update_gemm']['convs_us'], 'dom', dk.get('launch_us'), dk.get('frac'), 'dropin', (d.get('drop_in_forward') or {}).get('value'))"
  done
done
for E in 0 1; do
  echo "== conv_bench NL8=$E"
  RAFT_HALO_NL8=$E timeout -k 10 200 python tools/conv_bench.py 1 convc2,conv,zr_split,q_split,fh1 2>&1 | grep -v amdgpu.ids || exit 1
done
