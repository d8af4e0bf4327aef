# Build libnst_hip.so (gfx950) in-tree.  `make -j4`.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
PKG := neuralstyletransferv1_amd
CSRC := $(PKG)/csrc
BUILD := build/obj
# SLP: -fno-slp-vectorize keeps scalar f32 VALU scalar (packed f32 beside MFMAs costs extra cycles,
# conv_ws_common.h); the VALU-heavy up-conv file measured faster with packed consume math
SLP ?= -fno-slp-vectorize
CXXFLAGS = --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off $(SLP) -Wall -Wno-unused-function \
            -Iinclude -I$(CSRC)
SRCS := $(CSRC)/conv_bf16.hip $(CSRC)/conv_f16.hip $(CSRC)/conv_bf16_wl.hip $(CSRC)/conv_wstat.hip $(CSRC)/conv_wphase.hip $(CSRC)/conv_ws2.hip $(CSRC)/conv_ws9.hip $(CSRC)/conv_ws1s.hip $(CSRC)/conv_out9.hip $(CSRC)/conv_prep.hip $(CSRC)/conv_f32.hip $(CSRC)/conv_f32s.hip $(CSRC)/conv_vgg.hip $(CSRC)/nst_ops.hip $(CSRC)/vgg_ops.hip $(CSRC)/conv_gemm.hip $(CSRC)/seg_ops.hip $(CSRC)/region_ops.hip $(CSRC)/flow_ops.hip $(CSRC)/dis_ops.hip $(CSRC)/png_enc.hip $(CSRC)/nst_api.cpp $(CSRC)/vgg_gatys.cpp $(CSRC)/seg_deeplab.cpp $(CSRC)/region_api.cpp $(CSRC)/flow_api.cpp
# conv_wst16.hip (the residual trunk): nine objects from one source (NST_W16_PART: 0..7 two explicitly instantiated
# kernels each, ~2-3 min per kernel, compiled in parallel; 8 the launchers and the table).  conv_wst32.hip, its 32x32x16 variant, only for A/B
# libraries (`make wst32`: libnst_hip_wst32.so, where NST_WST16=0 selects it)
W16_OBJS := $(patsubst %,$(BUILD)/conv_wst16_p%.hip.o,0 1 2 3 4 5 6 7 8)
W32_OBJS := $(BUILD)/conv_wst32_p0.hip.o $(BUILD)/conv_wst32_p1.hip.o $(BUILD)/conv_wst32_p2.hip.o $(BUILD)/conv_wst32_p3.hip.o
OBJS := $(patsubst $(CSRC)/%,$(BUILD)/%.o,$(SRCS)) $(W16_OBJS)
LIB := $(PKG)/libnst_hip.so

all: $(LIB)

$(BUILD)/%.hip.o: $(CSRC)/%.hip $(CSRC)/conv_impl.h $(CSRC)/conv_ws_common.h $(CSRC)/conv_tab16.h $(CSRC)/conv_tab32.h $(CSRC)/nst_internal.h $(CSRC)/seg_internal.h $(CSRC)/post_common.h $(CSRC)/region_internal.h $(CSRC)/flow_internal.h include/nst_hip.h
	@mkdir -p $(BUILD)
	$(if $(NOSCRATCH),$(HIPCC) $(CXXFLAGS) -Rpass-analysis=kernel-resource-usage -c $< -o $@ 2> $@.rem && python3 tools/check_scratch.py $@.rem || { rm -f $@; exit 1; },$(HIPCC) $(CXXFLAGS) -c $< -o $@)

# kernels with hand-counted vmcnt waits: the build fails on any scratch use (tools/check_scratch.py; NST_STRICT_SCRATCH=0
# reports instead, for experiment builds)
$(BUILD)/conv_wstat.hip.o $(BUILD)/conv_wphase.hip.o $(BUILD)/conv_ws9.hip.o $(BUILD)/conv_gemm.hip.o $(BUILD)/conv_ws2.hip.o $(BUILD)/conv_ws1s.hip.o: NOSCRATCH = 1

# the persistent kernels fully unroll a long K loop (static register / LDS indices): lift the
# pragma-unroll size cap for that translation unit only
$(BUILD)/conv_bf16_wl.hip.o: CXXFLAGS += -mllvm -pragma-unroll-threshold=200000
$(BUILD)/conv_wstat.hip.o: CXXFLAGS += -mllvm -pragma-unroll-threshold=5000000
$(BUILD)/conv_wst16_p%.hip.o: $(CSRC)/conv_wst16.hip $(CSRC)/conv_impl.h $(CSRC)/conv_ws_common.h include/nst_hip.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(CXXFLAGS) -mllvm -pragma-unroll-threshold=5000000 -DNST_W16_PART=$* -Rpass-analysis=kernel-resource-usage -c $< -o $@ 2> $@.rem && python3 tools/check_scratch.py $@.rem || { rm -f $@; exit 1; }
# part 8: launchers and table only (every kernel an extern template: no kernel, no resource remarks)
$(BUILD)/conv_wst16_p8.hip.o: $(CSRC)/conv_wst16.hip $(CSRC)/conv_impl.h $(CSRC)/conv_ws_common.h include/nst_hip.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(CXXFLAGS) -DNST_W16_PART=8 -c $< -o $@
$(BUILD)/conv_wst32_p%.hip.o: $(CSRC)/conv_wst32.hip $(CSRC)/conv_impl.h $(CSRC)/conv_ws_common.h include/nst_hip.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(CXXFLAGS) -mllvm -pragma-unroll-threshold=5000000 -DNST_W32_PART=$* -Rpass-analysis=kernel-resource-usage -c $< -o $@ 2> $@.rem && python3 tools/check_scratch.py $@.rem || { rm -f $@; exit 1; }
$(BUILD)/conv_wphase.hip.o: CXXFLAGS += -mllvm -pragma-unroll-threshold=5000000
$(BUILD)/conv_wphase.hip.o: SLP =
$(BUILD)/conv_ws2.hip.o: CXXFLAGS += -mllvm -pragma-unroll-threshold=5000000
$(BUILD)/conv_ws9.hip.o: CXXFLAGS += -mllvm -pragma-unroll-threshold=5000000
$(BUILD)/conv_ws1s.hip.o: CXXFLAGS += -mllvm -pragma-unroll-threshold=5000000

$(BUILD)/%.cpp.o: $(CSRC)/%.cpp $(CSRC)/nst_internal.h $(CSRC)/seg_internal.h $(CSRC)/post_common.h $(CSRC)/region_internal.h $(CSRC)/flow_internal.h include/nst_hip.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(CXXFLAGS) -x hip -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS)

# Host-side AddressSanitizer build of the C ABI (tools/asan/nst_asan_driver.cpp): the host translation units
# with -fsanitize=address on the host side only (no device sanitizer on this pool), the kernels as built above
ASAN_HOST := nst_api.cpp vgg_gatys.cpp seg_deeplab.cpp region_api.cpp flow_api.cpp
ASAN_OBJS := $(patsubst %,build/asan/%.o,$(ASAN_HOST))
ASAN_BIN := tools/asan/nst_asan_driver
ASAN_FLAGS := -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer

build/asan/%.cpp.o: $(CSRC)/%.cpp $(CSRC)/nst_internal.h $(CSRC)/seg_internal.h $(CSRC)/post_common.h $(CSRC)/region_internal.h $(CSRC)/flow_internal.h include/nst_hip.h
	@mkdir -p build/asan
	$(HIPCC) $(CXXFLAGS) $(ASAN_FLAGS) -x hip -c $< -o $@

$(ASAN_BIN): tools/asan/nst_asan_driver.cpp $(ASAN_OBJS) $(filter-out $(patsubst %,$(BUILD)/%.o,$(ASAN_HOST)),$(OBJS))
	$(HIPCC) $(CXXFLAGS) $(ASAN_FLAGS) -x hip tools/asan/nst_asan_driver.cpp -x none $(ASAN_OBJS) \
	  $(filter-out $(patsubst %,$(BUILD)/%.o,$(ASAN_HOST)),$(OBJS)) -o $@

asan: $(ASAN_BIN)

clean:
	rm -rf $(BUILD) $(LIB) build/asan $(ASAN_BIN)

.PHONY: all clean asan stamp wst32

# diagnostic library with s_memtime stamps in the 32x32x16 trunk kernel (tools/w32_stamps.py; NST_HIP_LIB selects it)
# (STAMP_TAG / STAMP_FLAGS: variant builds for A/B, e.g. make stamp STAMP_TAG=st2 STAMP_FLAGS=-DNST_W32_ST=2)
STAMP_TAG ?= stamp
STAMP_FLAGS ?=
STAMP_LIB := $(PKG)/libnst_hip_$(STAMP_TAG).so
STAMP_SRC ?= conv_wst16
build/$(STAMP_TAG)/conv_wst32.hip.o: $(CSRC)/$(STAMP_SRC).hip $(CSRC)/conv_impl.h $(CSRC)/conv_ws_common.h include/nst_hip.h
	@mkdir -p build/$(STAMP_TAG)
	$(HIPCC) $(CXXFLAGS) -mllvm -pragma-unroll-threshold=5000000 -DNST_WST32_STAMP=1 $(STAMP_FLAGS) -Rpass-analysis=kernel-resource-usage -c $< -o $@ 2> $@.rem && python3 tools/check_scratch.py $@.rem
$(STAMP_LIB): build/$(STAMP_TAG)/conv_wst32.hip.o $(filter-out $(BUILD)/$(STAMP_SRC)_p%.hip.o,$(OBJS))
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^
stamp: $(STAMP_LIB)

$(PKG)/libnst_hip_wst32.so: $(OBJS) $(W32_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^
wst32: $(PKG)/libnst_hip_wst32.so
