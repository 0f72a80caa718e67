#!/bin/bash
# PMC passes on one conv shape (tools/conv_bench.py B name, PREC env): issue / stall / LDS / L2 counters.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
B=${1:-1}; NAME=${2:-zr_split}; PREC=${PREC:-f16x3}; export PREC
OUT=gpurun_out/pmcconv_${NAME}_b${B}_${PREC}
mkdir -p $OUT
i=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU" \
         "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/p$i -o run -- python tools/conv_bench.py $B $NAME > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/p$i.log; [ $i -ge 4 ] || exit 1; }
done
python tools/pmc_conv_summary.py $OUT
