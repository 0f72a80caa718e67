#!/bin/bash
# The alt lookup with the next level's loads after the binning stores (variants/altlate) vs the
# default, interleaved on one box; then the in-forward PMC passes (unfused and the bench's fused
# forward).  Each GPU step time-limited; stops at a failure.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${TAG:-r04h}
O=gpurun_out/exp_${TAG}.txt
mkdir -p gpurun_out
: > $O
export TMPDIR=/tmp
run() { echo "== $*" >> $O; timeout -k 10 200 "$@" >> $O 2>&1 || { echo "failed: $*"; tail -30 $O; exit 1; }; }
for r in 1 2; do
  run python tools/alt_bench.py 8 1
  run env RAFT_HIP_LIB=variants/altlate/libraft_hip.so python tools/alt_bench.py 8 1
  run python tools/alt_bench.py 8 0
  run env RAFT_HIP_LIB=variants/altlate/libraft_hip.so python tools/alt_bench.py 8 0
done
grep -v amdgpu.ids $O
PART=b PMC_ONLY=1 timeout -k 10 900 bash tools/r04_final.sh
