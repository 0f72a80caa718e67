#!/bin/bash
# Conv microbench in every precision + GPU parity + bench (+ kernel-trace profile when PROFILE=1).
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-dev}
mkdir -p gpurun_out
for P in fp32 f16x3 f16; do
  PREC=$P timeout -k 10 200 python tools/conv_bench.py 1 >> gpurun_out/cb_$TAG.log 2>&1 || { echo "conv_bench $P failed"; tail -20 gpurun_out/cb_$TAG.log; exit 1; }
done
cat gpurun_out/cb_$TAG.log
./tools/gpu_check.sh $TAG
