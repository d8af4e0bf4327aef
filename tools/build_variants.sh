#!/bin/bash
# Variant builds of libnst_hip.so for A/B sweeps on the GPU (tools/*_bench.py select one with NST_HIP_LIB):
#   bash tools/build_variants.sh <source.hip> <name>=<"-D flags"> ...
# recompiles <source> with the flags and links it with the default objects into sweep/libnst_hip_<name>.so
set -e
cd "$(dirname "$0")/.."
make -j8 >/dev/null
SRC=$1; shift
base=$(basename "$SRC")
mkdir -p build/var sweep
# the Makefile's per-file flags (without them the persistent kernels' K loops stay rolled and their
# accumulators go to scratch, whose loads break the hand-counted vmcnt waits)
case "$base" in
  conv_bf16_wl.hip) extra="-mllvm -pragma-unroll-threshold=200000" ;;
  conv_wstat.hip|conv_ws2.hip|conv_ws9.hip) extra="-mllvm -pragma-unroll-threshold=5000000" ;;
  conv_wphase.hip) extra="-mllvm -pragma-unroll-threshold=5000000 -fslp-vectorize" ;;
  *) extra="" ;;
esac
for spec in "$@"; do
  name=${spec%%=*}; flags="$extra ${spec#*=}"
  objs=$(ls build/obj/*.o | grep -v "/$base.o")
  ( /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -Wall -Wno-unused-function \
    -Iinclude -Ineuralstyletransferv1_amd/csrc $flags -Rpass-analysis=kernel-resource-usage -c "$SRC" \
    -o "build/var/${base}_$name.o" 2> "build/var/${base}_$name.rem" &&
    case "$base" in  # the Makefile's scratch check for the counted-vmcnt kernels
      conv_wstat.hip|conv_wphase.hip|conv_ws9.hip|conv_gemm.hip|conv_ws2.hip) python3 tools/check_scratch.py "build/var/${base}_$name.rem" ;;
      *) true ;;
    esac || { rm -f "build/var/${base}_$name.o"; echo "variant $name failed"; exit 1; } ) &
  pids="$pids $!"
done
for p in $pids; do wait $p; done
for spec in "$@"; do
  name=${spec%%=*}
  objs=$(ls build/obj/*.o | grep -v "/$base.o")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "sweep/libnst_hip_$name.so" $objs "build/var/${base}_$name.o"
  echo "built sweep/libnst_hip_$name.so"
done
