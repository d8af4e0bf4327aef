#!/bin/bash
# Like build_variant.sh but recompiles conv_wstat.hip (weight-stationary residual-trunk kernels).
#   bash tools/build_ws_variant.sh NAME "-DWS_NOLOAD -DNST_WSTAT_TH=4"
set -e
cd "$(dirname "$0")/.."
make -s -j8
NAME=$1; DEFS=$2
OUT=build/variants/$NAME
mkdir -p $OUT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function \
  -mllvm -pragma-unroll-threshold=5000000 -Iinclude -Ineuralstyletransferv1_amd/csrc $DEFS \
  -c neuralstyletransferv1_amd/csrc/conv_wstat.hip -o $OUT/conv_wstat.hip.o
OBJS=$(ls build/obj/*.o | grep -v conv_wstat.hip.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libnst_hip.so $OUT/conv_wstat.hip.o $OBJS
echo "built $OUT/libnst_hip.so"
