#!/bin/bash
# r06: the K-split form's loader limit: weight lead (HALO_WX) and loader priority (HALO_LPRIO) variants
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
export RAFT_SKIP_SRC_CHECK=1
bash tools/variant_bench.sh "base wx1 wx2 lp2" f16x3 1 convc2,zr_split,fh1 || exit 1
for rep in 1 2; do
  for V in base wx1 wx2 lp2; do
    if [ "$V" = base ]; then LIB=raft_optical_flow_amd/libraft_hip.so; else LIB=ab/$V/libraft_hip.so; fi
    RAFT_HIP_LIB=$LIB timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-exact > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$V', d['value'], 'iter', d['iteration']['iteration_us'], 'convs', d['update_gemm']['convs_us'], 'dropin', d['drop_in_forward']['value'])"
  done
done
