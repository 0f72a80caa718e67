#!/bin/bash
# In-forward PMC passes (one counter group per pass, kernel-trace only) over tools/pmc_forward.py:
# HBM bytes of the corr lookup (FETCH_SIZE, WRITE_SIZE) and MFMA busy of the conv kernels.
#   tools/pmc_forward.sh [batch]   ->  profiles/r02_lookup_pmc.json, profiles/r02_halo_pmc.json
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
B=${1:-1}
OUT=gpurun_out/pmcfwd_b$B
mkdir -p $OUT
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES" \
         "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/p$i -o run -- python tools/pmc_forward.py $B > $OUT/p$i.log 2>&1 || { echo "pmc pass $i ($C) failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python tools/pmc_forward_summary.py $OUT $B
