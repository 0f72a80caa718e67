#!/bin/bash
# rocprofv3 PMC passes (one counter group per pass, kernel-trace only) for the lookup kernel.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  tag=$(echo $C | tr ' ' '_')
  REPS=20 timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/$tag -o run -- python tools/lookup_bench.py 1 0.7 > $OUT/$tag.log 2>&1 || { echo "pmc $C failed"; tail -5 $OUT/$tag.log; exit 1; }
done
echo pmc done
