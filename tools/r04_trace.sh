#!/bin/bash
# Kernel traces + phase summaries of one config-2 forward (f16x3) and one config-5 forward (bf16,
# all-pairs) on the final tree.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fpf2 -o run --output-format csv -- python tools/fwd_profile.py 1 440 1024 f16x3 > gpurun_out/fpf2.log 2>&1 || { tail -20 gpurun_out/fpf2.log; exit 1; }
python tools/phase_summary.py gpurun_out/fpf2/run_kernel_trace.csv > gpurun_out/phase_r04_final_config2.txt 2>&1
ALT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fpf5 -o run --output-format csv -- python tools/fwd_profile.py 1 1080 1920 bf16 > gpurun_out/fpf5.log 2>&1 || { tail -20 gpurun_out/fpf5.log; exit 1; }
python tools/phase_summary.py gpurun_out/fpf5/run_kernel_trace.csv > gpurun_out/phase_r04_final_config5.txt 2>&1
grep -E "forward span|encoder phase span|loop span" gpurun_out/phase_r04_final_config2.txt gpurun_out/phase_r04_final_config5.txt
