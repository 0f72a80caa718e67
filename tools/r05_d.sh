#!/bin/bash
# Round 5, step D: config 2 A/B vs r3 (one rep), configs 3-5 bench lines, a config-5 forward trace.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
./tools/ab_tree.sh "r3 cur" 1 || exit 1
for E in 1 0 1; do
  RAFT_HALO_BIG_MT=$E timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-fp32-exact > gpurun_out/bigmt_$E.json 2> gpurun_out/bigmt_$E.err || { tail -20 gpurun_out/bigmt_$E.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bigmt_$E.json')); print('BIG_MT=$E', d['value'], 'iter', d['iteration']['iteration_us'])"
done
RAFT_HALO_BIG_MT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fpd2 -o run --output-format csv -- python tools/fwd_profile.py 1 440 1024 f16x3 > gpurun_out/fpd2.log 2>&1 || { tail -20 gpurun_out/fpd2.log; exit 1; }
python tools/phase_summary.py gpurun_out/fpd2/run_kernel_trace.csv > gpurun_out/phase_r05d_config2_bigmt.txt 2>&1
grep -E "forward span|encoder phase span|loop span" gpurun_out/phase_r05d_config2_bigmt.txt
run() {
  echo "== $*"
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-fp32-exact "$@" > gpurun_out/d_line.json 2> gpurun_out/d_line.err || { tail -20 gpurun_out/d_line.err; exit 1; }
  cat gpurun_out/d_line.json >> gpurun_out/r05d_configs.jsonl
  python -c "import json; d=json.load(open('gpurun_out/d_line.json')); r=d.get('roofline') or {}; print(d['value'], d['config']['workload'], 'iter', d['iteration']['iteration_us'], 'convs', d['update_gemm']['convs_us'], 'lookup', r.get('launch_us') or r.get('iteration_us'))"
}
: > gpurun_out/r05d_configs.jsonl
run --batch 8 --alternate-corr
run --batch 8 --height 540 --width 960
run --batch 1 --height 1080 --width 1920 --precision bf16
export RAFT_HALO_BIG_MT=1
run --batch 8 --height 540 --width 960
run --batch 1 --height 1080 --width 1920 --precision bf16
unset RAFT_HALO_BIG_MT
ALT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fpd5 -o run --output-format csv -- python tools/fwd_profile.py 1 1080 1920 bf16 > gpurun_out/fpd5.log 2>&1 || { tail -20 gpurun_out/fpd5.log; exit 1; }
python tools/phase_summary.py gpurun_out/fpd5/run_kernel_trace.csv > gpurun_out/phase_r05d_config5.txt 2>&1
grep -E "forward span|encoder phase span|loop span" gpurun_out/phase_r05d_config5.txt
