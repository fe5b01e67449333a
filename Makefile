# Build: the HIP product library (gfx950), the CPU oracle (test infrastructure)
# and the C++ host-mirror check program.  `make -j` is safe.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
PKG := qkd_ldpc_v_amd
CSRC := $(PKG)/csrc
# -amdgpu-atomic-optimizer-strategy=None: the atomic optimizer rewrites a uniform
# atomic into a single-lane block (mbcnt + narrowed exec); with this register
# pressure LLVM (ROCm 7.2) placed a VGPR spill store inside such a block in the
# split-frame kernel, so 63 lanes reloaded an unwritten slot.
# Every atomic here is already issued by one lane on purpose.
HIPFLAGS := --offload-arch=$(ARCH) $(EXTRA_HIPFLAGS) -O3 -std=c++17 -ffp-contract=off -fPIC -Wall -Wno-unused-result \
            -mllvm -amdgpu-atomic-optimizer-strategy=None
LIB := $(PKG)/libqkdldpc_hip.so
ORACLE := oracle/libqkdldpc_oracle.so
HOSTCHK := $(PKG)/host/host_mirror_check

all: $(LIB) $(ORACLE) $(HOSTCHK)

$(CSRC)/decoder.o: $(CSRC)/decoder.hip $(CSRC)/decoder_common.hpp $(CSRC)/decoder.hpp $(CSRC)/exact_math.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/decoder_v2.o: $(CSRC)/decoder_v2.hip $(CSRC)/decoder_common.hpp $(CSRC)/decoder.hpp $(CSRC)/exact_math.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/trials.o: $(CSRC)/trials.hip $(CSRC)/decoder.hpp
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/order.o: $(CSRC)/order.hip $(CSRC)/decoder.hpp
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/capi.o: $(CSRC)/capi.hip $(CSRC)/decoder.hpp $(CSRC)/loaders.hpp include/qkd_ldpc_hip.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/loaders.o: $(CSRC)/loaders.cpp $(CSRC)/loaders.hpp
	g++ -O2 -std=c++17 -fPIC -Wall -c $< -o $@

$(LIB): $(CSRC)/decoder.o $(CSRC)/decoder_v2.o $(CSRC)/trials.o $(CSRC)/order.o $(CSRC)/capi.o $(CSRC)/loaders.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $^ -lz -o $@

# Diagnostic build with per-phase s_memtime stamps (never the product).
STAMPLIB := $(PKG)/diag/libqkdldpc_hip.so
stamps: $(STAMPLIB)
$(CSRC)/decoder_st.o: $(CSRC)/decoder.hip $(CSRC)/decoder_common.hpp $(CSRC)/decoder.hpp $(CSRC)/exact_math.h
	$(HIPCC) $(HIPFLAGS) -DQL_PHASE_STAMPS -c $< -o $@
$(CSRC)/decoder_v2_st.o: $(CSRC)/decoder_v2.hip $(CSRC)/decoder_common.hpp $(CSRC)/decoder.hpp $(CSRC)/exact_math.h
	$(HIPCC) $(HIPFLAGS) -DQL_PHASE_STAMPS -c $< -o $@
$(CSRC)/capi_st.o: $(CSRC)/capi.hip $(CSRC)/decoder.hpp $(CSRC)/loaders.hpp include/qkd_ldpc_hip.h
	$(HIPCC) $(HIPFLAGS) -DQL_PHASE_STAMPS -c $< -o $@
$(STAMPLIB): $(CSRC)/decoder_st.o $(CSRC)/decoder_v2_st.o $(CSRC)/trials.o $(CSRC)/order.o $(CSRC)/capi_st.o $(CSRC)/loaders.o
	mkdir -p $(PKG)/diag
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $^ -lz -o $@

$(ORACLE): oracle/ldpc_oracle.c oracle/ldpc_oracle.h oracle/trials_oracle.cpp
	$(MAKE) -C oracle

$(HOSTCHK): $(PKG)/host/host_mirror_check.cpp $(PKG)/host/qkd_ldpc_algorithm.hpp include/qkd_ldpc_hip.h $(LIB)
	g++ -O2 -std=c++17 -Wall -I include $< -L$(PKG) -lqkdldpc_hip -Wl,-rpath,'$$ORIGIN/..' -o $@

# FP64 VALU ceilings of the SPA edge math (tools/valu_bench.hip), run on the box.
tools/valu_bench: tools/valu_bench.hip $(CSRC)/exact_math.h
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -ffp-contract=off $< -o $@
valu_bench: tools/valu_bench

clean:
	rm -f $(CSRC)/*.o $(LIB) $(HOSTCHK) $(STAMPLIB) tools/valu_bench
	$(MAKE) -C oracle clean

.PHONY: all clean stamps valu_bench

# A/B experiment build: `make ab AB=name AB_FLAGS=-D...` -> qkd_ldpc_v_amd/ab/name/
# (selected at run time with QLDPC_AB_BUILD=name; never the product)
AB ?= x
ab:
	mkdir -p $(PKG)/ab/$(AB)
	$(HIPCC) $(HIPFLAGS) $(AB_FLAGS) -c $(CSRC)/decoder_v2.hip -o $(PKG)/ab/$(AB)/decoder_v2.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(PKG)/ab/$(AB)/decoder_v2.o $(CSRC)/decoder.o $(CSRC)/trials.o $(CSRC)/order.o $(CSRC)/capi.o $(CSRC)/loaders.o -lz -o $(PKG)/ab/$(AB)/libqkdldpc_hip.so
.PHONY: ab
