#!/bin/bash
# r06: TIMING ABLATION (wrong results): no weight DMAs after the prologue (HALO_ABL_NOW)
# -- the cost of the weight stream.  conv_bench only (random inputs), plus stamps.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
export RAFT_SKIP_SRC_CHECK=1
bash tools/variant_bench.sh "base now" f16x3 1 convc2,conv,zr_split,q_split,fh1 || exit 1
RAFT_HALO_KS2=0 bash tools/variant_bench.sh "base now" f16x3 1 convc2,zr_split,fh1 || exit 1
