#!/bin/bash
# r06: K-split form for the 32-column update convs (conv, q): tests, conv_bench, forward A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
export RAFT_SKIP_SRC_CHECK=1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t_r06ks32.log 2>&1
rc=$?; tail -3 gpurun_out/t_r06ks32.log; [ $rc -eq 0 ] || exit $rc
bash tools/variant_bench.sh "base bn32off" f16x3 1 conv,q_split || exit 1
for rep in 1 2 3; do
  for V in base bn32off; do
    if [ "$V" = base ]; then LIB=raft_optical_flow_amd/libraft_hip.so; else LIB=ab/$V/libraft_hip.so; fi
    RAFT_HIP_LIB=$LIB timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-exact > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$V', d['value'], 'iter', d['iteration']['iteration_us'], 'convs', d['update_gemm']['convs_us'], 'dropin', d['drop_in_forward']['value'])"
  done
done
