#!/bin/bash
# Recompile one persistent-kernel translation unit with extra defines and link a variant library.
#   bash tools/build_src_variant.sh NAME conv_wphase "-DWS_NOBAR -DWP_RING=2"
set -e
cd "$(dirname "$0")/.."
make -s -j8
NAME=$1; SRC=$2; DEFS=$3
OUT=build/variants/$NAME
mkdir -p $OUT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function \
  -mllvm -pragma-unroll-threshold=5000000 -Iinclude -Ineuralstyletransferv1_amd/csrc $DEFS \
  -c neuralstyletransferv1_amd/csrc/$SRC.hip -o $OUT/$SRC.hip.o
OBJS=$(ls build/obj/*.o | grep -v $SRC.hip.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libnst_hip.so $OUT/$SRC.hip.o $OBJS
echo "built $OUT/libnst_hip.so"
