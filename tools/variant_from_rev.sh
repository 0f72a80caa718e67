#!/bin/bash
# Build libraft_hip.so from the kernel sources of git revision REV into variants/NAME/
# (A/B on one box: RAFT_HIP_LIB=variants/NAME/libraft_hip.so).   tools/variant_from_rev.sh REV NAME
set -e
cd "$(dirname "$0")/.."
REV=$1; NAME=$2
D=variants/$NAME
rm -rf $D && mkdir -p $D/src/raft_optical_flow_amd/csrc $D/src/include
git archive $REV raft_optical_flow_amd/csrc include | tar -x -C $D/src
make -C $D/src/raft_optical_flow_amd/csrc -j8 OUT=$(pwd)/$D/libraft_hip.so OBJDIR=$(pwd)/$D/obj > $D/build.log 2>&1
echo "built $D/libraft_hip.so from $REV"
