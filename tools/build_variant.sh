#!/bin/bash
# Build a tile-shape variant of libnst_hip.so for sweeps: only conv_bf16.hip is recompiled.
#   bash tools/build_variant.sh NAME "-DNST_C2_TILE=4,16,4,1 ..."   -> build/variants/NAME/libnst_hip.so
set -e
cd "$(dirname "$0")/.."
make -s -j8
NAME=$1; DEFS=$2
OUT=build/variants/$NAME
mkdir -p $OUT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function \
  -Iinclude -Ineuralstyletransferv1_amd/csrc $DEFS -c neuralstyletransferv1_amd/csrc/conv_bf16.hip -o $OUT/conv_bf16.hip.o
OBJS=$(ls build/obj/*.o | grep -v conv_bf16.hip.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libnst_hip.so $OUT/conv_bf16.hip.o $OBJS
echo "built $OUT/libnst_hip.so"
