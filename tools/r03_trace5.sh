#!/bin/bash
# kernel traces + phase summaries: config 5 (1080x1920 bf16, B=1) and config 3 (B=8 alternate)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fp_c5 -o run --output-format csv -- python tools/fwd_profile.py 1 1080 1920 bf16 > gpurun_out/fp_c5.log 2>&1 || exit 1
python tools/phase_summary.py gpurun_out/fp_c5/run_kernel_trace.csv > gpurun_out/phase_c5.txt 2>&1
ALT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fp_c3 -o run --output-format csv -- python tools/fwd_profile.py 8 440 1024 f16x3 > gpurun_out/fp_c3.log 2>&1 || exit 1
python tools/phase_summary.py gpurun_out/fp_c3/run_kernel_trace.csv > gpurun_out/phase_c3.txt 2>&1
for c in c5 c3; do grep -E "forward span|encoder phase span|loop span" gpurun_out/phase_$c.txt; sed -n '/encoder phase span/,/encoder phase in order/p' gpurun_out/phase_$c.txt | head -14; sed -n '/mean per launch slot/,/sum/p' gpurun_out/phase_$c.txt; done
