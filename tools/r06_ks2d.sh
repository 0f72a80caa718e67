#!/bin/bash
# r06: KS2 (loaders issue weights + patches) vs KS1 -- forward A/B x3 and in-forward phase traces
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
export RAFT_SKIP_SRC_CHECK=1  # (experiment script: the in-tree library is the one built before the call)
for rep in 1 2 3; do
  for KS in 0 1; do
    RAFT_HALO_KS2=$KS timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-exact > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('KS2=$KS', d['value'], 'iter', d['iteration']['iteration_us'], 'convs', d['update_gemm']['convs_us'], 'dropin', d['drop_in_forward']['value'])"
  done
done
for KS in 0 1; do
  RAFT_HALO_KS2=$KS timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/fwd_ks$KS -o run --output-format csv -- python tools/fwd_profile.py 1 440 1024 f16x3 > gpurun_out/fwd_ks$KS.log 2>&1 || { tail -20 gpurun_out/fwd_ks$KS.log; exit 1; }
  python tools/phase_summary.py gpurun_out/fwd_ks$KS/run_kernel_trace.csv > gpurun_out/r06_phases_ks$KS.txt 2>&1
  sed -n '/loop span/,$p' gpurun_out/r06_phases_ks$KS.txt
done
echo "## conv_bench base vs nols (patches fp32 by LDS-DMA, split by the compute waves)"
bash tools/variant_bench.sh "base nols" f16x3 1 convc2,conv,zr_split,q_split,fh1 || exit 1
bash tools/ab_variants.sh "base nols" || exit 1
