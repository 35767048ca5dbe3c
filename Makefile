# Build of liblpcnet_mi355x.so (gfx950) and the CPU checker under oracle/.
#
#   make            -> lpcnet_amd/liblpcnet_mi355x.so + oracle/ libraries
#   make lib        -> the product library only
#
# Every translation unit is compiled with -ffp-contract=off: the engine is
# bit-exact with the reference x86 build only without FMA contraction.

HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
JOBS ?= 4
BUILD := build
LIB := lpcnet_amd/liblpcnet_mi355x.so
CSRC := lpcnet_amd/csrc
HDRS := include/lpcnet.h include/lpcnet_mi355x.h $(CSRC)/lpcnet_engine.h $(CSRC)/device_math.h $(CSRC)/sampler.h $(CSRC)/lds_flags.h $(CSRC)/mf_common.h $(CSRC)/l2_warm.h $(CSRC)/pow10_dd.h $(CSRC)/rcp_table_x86.inc
EXTRA ?=
COMMON := $(EXTRA) -O3 -fPIC -ffp-contract=off -fno-fast-math -std=c++17 -Iinclude -I$(CSRC) -fvisibility=hidden -Wall -Wno-unused-function
OBJS := $(BUILD)/kernels.o $(BUILD)/mf_kernel.o $(BUILD)/mf2_kernel.o $(BUILD)/fp_kernel.o $(BUILD)/selftest.o $(BUILD)/frame_kernel.o $(BUILD)/engine.o $(BUILD)/lpc_kernel.o $(BUILD)/chunk_kernel.o $(BUILD)/model_gen.o $(BUILD)/host_rcpps.o $(BUILD)/decode_kernel.o $(BUILD)/mfw_kernel.o

SYNTH := tools/lpcnet_synth
DROPIN := tools/dropin_bench

all: lib synth dropin oracle

lib: $(LIB)

# file-driven C caller of include/lpcnet.h (lpcnet_demo -synthesis equivalent):
# plain C99 against the public header only, linked to the in-tree library
synth: $(SYNTH)

$(SYNTH): tools/lpcnet_synth.c include/lpcnet.h $(LIB)
	$(CC) -std=c99 -O2 -Wall -Wextra -pedantic -Werror -Iinclude -o $@ $< -Llpcnet_amd -llpcnet_mi355x -Wl,-rpath,'$$ORIGIN/../lpcnet_amd'

# pthread C driver of the drop-in API (many handles at once) against the batch API
dropin: $(DROPIN)

$(DROPIN): tools/dropin_bench.c include/lpcnet.h include/lpcnet_mi355x.h $(LIB)
	$(CC) -std=c99 -O2 -Wall -Wextra -Werror -Iinclude -o $@ $< -Llpcnet_amd -llpcnet_mi355x -lpthread -Wl,-rpath,'$$ORIGIN/../lpcnet_amd'

$(BUILD):
	mkdir -p $(BUILD)

$(BUILD)/kernels.o: $(CSRC)/kernels.hip $(HDRS) | $(BUILD)
	$(HIPCC) -x hip --offload-arch=$(ARCH) $(COMMON) -c $< -o $@

$(BUILD)/frame_kernel.o: $(CSRC)/frame_kernel.hip $(HDRS) | $(BUILD)
	$(HIPCC) -x hip --offload-arch=$(ARCH) $(COMMON) -c $< -o $@

# no SLP vectorisation: packed f32 ops cost the shared SIMDs more than scalar pairs
$(BUILD)/mf_kernel.o: $(CSRC)/mf_kernel.hip $(HDRS) | $(BUILD)
	$(HIPCC) -x hip --offload-arch=$(ARCH) $(COMMON) -fno-slp-vectorize -c $< -o $@

$(BUILD)/mf2_kernel.o: $(CSRC)/mf2_kernel.hip $(HDRS) | $(BUILD)
	$(HIPCC) -x hip --offload-arch=$(ARCH) $(COMMON) -fno-slp-vectorize -c $< -o $@

$(BUILD)/mfw_kernel.o: $(CSRC)/mfw_kernel.hip $(HDRS) | $(BUILD)
	$(HIPCC) -x hip --offload-arch=$(ARCH) $(COMMON) -fno-slp-vectorize -c $< -o $@

# the fp32 chains schedule better under the max-ILP machine scheduler (batch-1 fp32 +0.6 %)
$(BUILD)/fp_kernel.o: $(CSRC)/fp_kernel.hip $(HDRS) | $(BUILD)
	$(HIPCC) -x hip --offload-arch=$(ARCH) $(COMMON) -mllvm -amdgpu-sched-strategy=max-ilp -c $< -o $@

$(BUILD)/selftest.o: $(CSRC)/selftest.hip $(HDRS) | $(BUILD)
	$(HIPCC) -x hip --offload-arch=$(ARCH) $(COMMON) -c $< -o $@

$(BUILD)/engine.o: $(CSRC)/engine.cpp $(HDRS) | $(BUILD)
	$(HIPCC) -x hip --offload-arch=$(ARCH) $(COMMON) -c $< -o $@

$(BUILD)/lpc_kernel.o: $(CSRC)/lpc_kernel.hip $(HDRS) | $(BUILD)
	$(HIPCC) -x hip --offload-arch=$(ARCH) $(COMMON) -c $< -o $@

$(BUILD)/chunk_kernel.o: $(CSRC)/chunk_kernel.hip $(HDRS) | $(BUILD)
	$(HIPCC) -x hip --offload-arch=$(ARCH) $(COMMON) -c $< -o $@

$(BUILD)/decode_kernel.o: $(CSRC)/decode_kernel.hip $(HDRS) | $(BUILD)
	$(HIPCC) -x hip --offload-arch=$(ARCH) $(COMMON) -c $< -o $@

$(BUILD)/model_gen.o: $(CSRC)/model_gen.cpp $(HDRS) | $(BUILD)
	$(HIPCC) -x hip --offload-arch=$(ARCH) $(COMMON) -c $< -o $@

# host-only: the CPU's own rcpps (x86 SSE), system compiler
$(BUILD)/host_rcpps.o: $(CSRC)/host_rcpps.cpp include/lpcnet_mi355x.h | $(BUILD)
	$(CXX) -O2 -fPIC -msse2 -ffp-contract=off -std=c++17 -Iinclude -fvisibility=hidden -Wall -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -lpthread

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf $(BUILD) $(LIB) $(SYNTH) $(DROPIN)
	$(MAKE) -C oracle clean

.PHONY: all lib synth dropin oracle clean
