#!/bin/bash
# Round 4, late: the alt-corr binning over all threads and the lookup launch-span timing on one box
# (targeted tests, alt bench + stamps, the default bench line), then the in-forward PMC passes and
# the configs 3-5 sweep (tools/r04_final.sh PART=b).  Each GPU step time-limited; stops at a failure.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${TAG:-r04g}
O=gpurun_out/exp_${TAG}.txt
mkdir -p gpurun_out
: > $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lds_nan.py tests/test_capi.py -k "alt or lds or capi or lookup_conv" -x -q --timeout 240 --timeout-method thread > gpurun_out/t_${TAG}.log 2>&1
rc=$?; tail -3 gpurun_out/t_${TAG}.log; [ $rc -eq 0 ] || exit $rc
run() { echo "== $*" >> $O; timeout -k 10 200 "$@" >> $O 2>&1 || { echo "failed: $*"; tail -30 $O; exit 1; }; }
run python tools/alt_bench.py 8 0
run python tools/alt_bench.py 8 1
run env RAFT_HIP_LIB=variants/altst/libraft_hip.so python tools/alt_stamps.py 8 1
timeout -k 10 300 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench_${TAG}.json')); r=d['roofline']; print('config2', d['value'], 'launch_us', r['launch_us'], 'span', r.get('inforward_span_us'), 'delta', r['iteration_delta_us'], 'b2b', r['back_to_back_us'], 'frac', r['frac'])"
grep -v amdgpu.ids $O
PART=b timeout -k 10 900 bash tools/r04_final.sh
