#!/bin/bash
# Lookup kernel over library variants (ab/<name>/libraft_hip.so; "base" = the in-tree build)
# usage: tools/lookup_variants.sh "base nopipe w3" "1 2 8"
set -o pipefail
cd "$(dirname "$0")/.."
for V in $1; do
  if [ "$V" = base ]; then LIB=raft_optical_flow_amd/libraft_hip.so; else LIB=ab/$V/libraft_hip.so; fi
  for B in $2; do
    echo -n "$V: "
    RAFT_HIP_LIB=$LIB timeout -k 10 120 python tools/lookup_bench.py $B 2>&1 | grep "^lookup" || exit 1
  done
done
