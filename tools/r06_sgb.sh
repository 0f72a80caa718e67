#!/bin/bash
# r06: fragment-read scheduling variants of the halo conv (HALO_SGB = reads per MFMA gap), conv_bench
# per shape with 8 and 4 loader waves, then the forward A/B.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r06_base_bench.json 2> gpurun_out/r06_base_bench.err || { tail -20 gpurun_out/r06_base_bench.err; exit 1; }
cat gpurun_out/r06_base_bench.json
for NL in 1 0; do
  echo "#### RAFT_HALO_NL8=$NL"
  RAFT_HALO_NL8=$NL bash tools/variant_bench.sh "base sgb1 sgb2 sgb3 sgb4" f16x3 1 convc2,conv,zr_split,q_split,fh1 || exit 1
done
bash tools/ab_variants.sh "base sgb2 sgb4" || exit 1
