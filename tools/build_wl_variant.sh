#!/bin/bash
# Like build_variant.sh but recompiles conv_bf16_wl.hip (persistent residual-trunk kernels).
set -e
cd "$(dirname "$0")/.."
make -s -j8
NAME=$1; DEFS=$2
OUT=build/variants/$NAME
mkdir -p $OUT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function \
  -mllvm -pragma-unroll-threshold=200000 -Iinclude -Ineuralstyletransferv1_amd/csrc $DEFS \
  -c neuralstyletransferv1_amd/csrc/conv_bf16_wl.hip -o $OUT/conv_bf16_wl.hip.o
OBJS=$(ls build/obj/*.o | grep -v conv_bf16_wl.hip.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libnst_hip.so $OUT/conv_bf16_wl.hip.o $OBJS
echo "built $OUT/libnst_hip.so"
