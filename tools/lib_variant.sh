#!/bin/bash
# A library variant with one source file rebuilt under extra defines, linked with the in-tree objects:
#   tools/lib_variant.sh NAME "DEFS" file.hip   ->  ab/NAME/libraft_hip.so  (RAFT_HIP_LIB=ab/NAME/libraft_hip.so)
set -e
cd "$(dirname "$0")/.."
NAME=$1; DEFS=$2; SRC=$3
C=raft_optical_flow_amd/csrc
make -s -C $C -j8 > /dev/null
D=ab/$NAME; rm -rf $D; mkdir -p $D/obj
for f in $(sed -n "s/^SRCS := //p" $C/Makefile); do cp build/obj/${f%.hip}.o $D/obj/; done
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Iinclude -Wall -Wno-unused-function $DEFS -c $C/$SRC -o $D/obj/${SRC%.hip}.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $D/obj/*.o -o $D/libraft_hip.so
rm -rf $D/obj
echo "built $D ($DEFS on $SRC)"
