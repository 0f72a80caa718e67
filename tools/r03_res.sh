#!/bin/bash
# resident vs halo on one encoder conv shape, then SQ PMC of the resident kernel
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for E in RAFT_RESIDENT=1 RAFT_RESIDENT=0; do
  for N in plain norm; do env $E timeout -k 10 120 python tools/res_bench.py $N 2>&1 | grep -v amdgpu.ids || exit 1; done
done
env RAFT_RESIDENT=1 timeout -k 10 120 python tools/res_bench.py plain 96 110 256 2 2>&1 | grep -v amdgpu.ids || exit 1
env RAFT_RESIDENT=0 timeout -k 10 120 python tools/res_bench.py plain 96 110 256 2 2>&1 | grep -v amdgpu.ids || exit 1
if [ -n "$PMC" ]; then ./tools/pmc_sq.sh res conv_resident python tools/res_bench.py plain; fi
