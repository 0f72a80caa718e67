#!/bin/bash
# r06: GPU suite on the current tree, then conv_bench + forward A/B of the halo scheduling variants
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t_r06a.log 2>&1
rc=$?; tail -3 gpurun_out/t_r06a.log; [ $rc -eq 0 ] || exit $rc
bash tools/variant_bench.sh "base sgb0 norelax" f16x3 1 convc2,conv,zr_split,q_split,fh1 || exit 1
bash tools/ab_variants.sh "base sgb0 norelax" || exit 1
