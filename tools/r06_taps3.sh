#!/bin/bash
# r06: the fused lookup's K stream pinned (LC_SGB) and the taps read once per column (LC_TAPS3) -- forward A/B,
# the bench's in-forward fused-lookup launch span (roofline.launch_us) per variant
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
export RAFT_SKIP_SRC_CHECK=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_lookup_conv.py tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -k "lookup or full_size or update or raft" > gpurun_out/t_r06t3.log 2>&1
rc=$?; tail -3 gpurun_out/t_r06t3.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for V in base taps30; do
    if [ "$V" = base ]; then LIB=raft_optical_flow_amd/libraft_hip.so; else LIB=ab/$V/libraft_hip.so; fi
    RAFT_HIP_LIB=$LIB timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-exact > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab.json')); r=d['roofline']; print('$V', d['value'], 'iter', d['iteration']['iteration_us'], 'lookup', r['launch_us'], r['frac'], 'dropin', d['drop_in_forward']['value'])"
  done
done
