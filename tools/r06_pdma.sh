#!/bin/bash
# r06: TIMING ABLATION (wrong results): the update convs' patches by LDS-DMA with no loader split (HALO_ABL_PDMA)
# -- the bound on pre-split activation rows in memory.  conv_bench only (random inputs), plus stamps.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
export RAFT_SKIP_SRC_CHECK=1
bash tools/variant_bench.sh "base pdma" f16x3 1 convc2,conv,zr_split,q_split,fh1 || exit 1
RAFT_HALO_KS2=0 bash tools/variant_bench.sh "base pdma" f16x3 1 convc2,zr_split,fh1 || exit 1
