#!/bin/bash
# A whole tree (bench.py, package, oracle, tools) of git revision REV, built, under ab/NAME
# (for tools/ab_tree.sh: same-box A/B against an earlier round's head).   tools/tree_from_rev.sh REV NAME
set -e
cd "$(dirname "$0")/.."
REV=$1; NAME=$2
D=ab/$NAME
rm -rf $D && mkdir -p $D
git archive $REV bench.py raft_optical_flow_amd include oracle tools | tar -x -C $D
make -C $D/raft_optical_flow_amd/csrc -j8 ROOT=$(pwd)/$D OBJDIR=$(pwd)/$D/obj > $D/build.log 2>&1
rm -rf $D/obj $D/build
echo "built $D from $REV"
