# Build: the HIP product library (gfx950), the CPU oracle (test infrastructure)
# and the C++ host-mirror check program.  `make -j` is safe.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
PKG := qkd_ldpc_v_amd
CSRC := $(PKG)/csrc
# -amdgpu-atomic-optimizer-strategy=None is a workaround for an LLVM (ROCm 7.2)
# miscompile, not a statement about the atomics: the optimizer rewrites a
# uniform atomic into a single-lane block (mbcnt + narrowed exec), and under the
# split-frame kernel's register pressure LLVM placed a VGPR spill store inside
# such a block, so 63 lanes reloaded an unwritten slot.  The
# frame claim / group barriers are single-lane, but order.hip's histogram and
# the min-sum bit gather's code-word ORs are per-lane atomics: they are merely
# not combined by the optimizer.  Regression tests for the flag: the C4
# split-frame parity tests (tests/test_gpu_parity.py::test_c4_*), which failed
# without it; tests/test_capi.py checks the flag is on every product compile line.
HIPFLAGS := --offload-arch=$(ARCH) $(EXTRA_HIPFLAGS) -O3 -std=c++17 -ffp-contract=off -fPIC -Wall -Wno-unused-result \
            -mllvm -amdgpu-atomic-optimizer-strategy=None
# The decoder kernels are scheduled with LLVM's iterative ILP strategy: same
# instructions and bits, 0.6% (C2) / 1.4% (C5) / 2.3% (C4) shorter decode
# in a same-box A/B against the default strategy (profiles/r04/sched_strategy_ab.txt).
V2FLAGS := -mllvm --amdgpu-sched-strategy=iterative-ilp
LIB := $(PKG)/libqkdldpc_hip.so
ORACLE := oracle/libqkdldpc_oracle.so
HOSTCHK := $(PKG)/host/host_mirror_check
DROPIN := tests/dropin/run_trial_check
BATCHCHK := tests/dropin/batch_check

all: $(LIB) $(ORACLE) $(HOSTCHK) $(DROPIN) $(BATCHCHK)

$(CSRC)/decoder.o: $(CSRC)/decoder.hip $(CSRC)/decoder_common.hpp $(CSRC)/decoder.hpp $(CSRC)/exact_math.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/decoder_v2.o: $(CSRC)/decoder_v2.hip $(CSRC)/decoder_common.hpp $(CSRC)/decoder.hpp $(CSRC)/exact_math.h Makefile
	$(HIPCC) $(HIPFLAGS) $(V2FLAGS) -c $< -o $@

$(CSRC)/trials.o: $(CSRC)/trials.hip $(CSRC)/decoder.hpp $(CSRC)/decoder_common.hpp $(CSRC)/exact_math.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/order.o: $(CSRC)/order.hip $(CSRC)/decoder.hpp $(CSRC)/decoder_common.hpp $(CSRC)/exact_math.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/capi.o: $(CSRC)/capi.hip $(CSRC)/decoder.hpp $(CSRC)/loaders.hpp $(CSRC)/relabel.hpp include/qkd_ldpc_hip.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CSRC)/loaders.o: $(CSRC)/loaders.cpp $(CSRC)/loaders.hpp
	g++ -O2 -std=c++17 -fPIC -Wall -c $< -o $@

$(CSRC)/relabel.o: $(CSRC)/relabel.cpp $(CSRC)/relabel.hpp
	g++ -O2 -std=c++17 -fPIC -Wall -c $< -o $@

$(LIB): $(CSRC)/decoder.o $(CSRC)/decoder_v2.o $(CSRC)/trials.o $(CSRC)/order.o $(CSRC)/capi.o $(CSRC)/loaders.o $(CSRC)/relabel.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $^ -lz -o $@

# Diagnostic build with per-phase s_memtime stamps (never the product).
STAMPLIB := $(PKG)/diag/libqkdldpc_hip.so
stamps: $(STAMPLIB)
$(CSRC)/decoder_st.o: $(CSRC)/decoder.hip $(CSRC)/decoder_common.hpp $(CSRC)/decoder.hpp $(CSRC)/exact_math.h
	$(HIPCC) $(HIPFLAGS) -DQL_PHASE_STAMPS -c $< -o $@
$(CSRC)/decoder_v2_st.o: $(CSRC)/decoder_v2.hip $(CSRC)/decoder_common.hpp $(CSRC)/decoder.hpp $(CSRC)/exact_math.h
	$(HIPCC) $(HIPFLAGS) $(V2FLAGS) -DQL_PHASE_STAMPS -c $< -o $@
$(CSRC)/capi_st.o: $(CSRC)/capi.hip $(CSRC)/decoder.hpp $(CSRC)/loaders.hpp $(CSRC)/relabel.hpp include/qkd_ldpc_hip.h
	$(HIPCC) $(HIPFLAGS) -DQL_PHASE_STAMPS -c $< -o $@
$(STAMPLIB): $(CSRC)/decoder_st.o $(CSRC)/decoder_v2_st.o $(CSRC)/trials.o $(CSRC)/order.o $(CSRC)/capi_st.o $(CSRC)/loaders.o $(CSRC)/relabel.o
	mkdir -p $(PKG)/diag
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $^ -lz -o $@

$(ORACLE): oracle/ldpc_oracle.c oracle/ldpc_oracle.h oracle/trials_oracle.cpp
	$(MAKE) -C oracle

$(HOSTCHK): $(PKG)/host/host_mirror_check.cpp $(PKG)/host/qkd_ldpc_algorithm.hpp $(PKG)/host/qkd_ldpc_impl.hpp \
            include/qkd_ldpc_hip.h $(LIB)
	g++ -O2 -std=c++17 -Wall -I include $< -L$(PKG) -lqkdldpc_hip -Wl,-rpath,'$$ORIGIN/..' -o $@

# The drop-in replacement TU for the reference's src/qkd_ldpc_algorithm.cpp,
# compiled against the reference-shaped declarations of tests/dropin/api and
# driven by a restatement of run_trial (tests/test_dropin.py).
$(DROPIN): tests/dropin/run_trial_check.cpp tests/dropin/trial_common.hpp $(PKG)/host/dropin/qkd_ldpc_algorithm.cpp \
           $(PKG)/host/qkd_ldpc_impl.hpp tests/dropin/api/qkd_ldpc_algorithm.hpp include/qkd_ldpc_hip.h $(LIB)
	g++ -O2 -std=c++20 -Wall -pthread -I tests/dropin/api -I include tests/dropin/run_trial_check.cpp \
	    $(PKG)/host/dropin/qkd_ldpc_algorithm.cpp -L$(PKG) -lqkdldpc_hip -Wl,-rpath,'$$ORIGIN/../../$(PKG)' -o $@

# The batch seam: the drop-in TU for QKD_LDPC_batch_simulation (src/simulation.cpp:693-760)
# beside the per-trial drop-in, driven by a restatement of the reference's loop pieces.
BATCH_SRCS := tests/dropin/batch_check.cpp $(PKG)/host/dropin/qkd_ldpc_algorithm.cpp $(PKG)/host/dropin/simulation_batch.cpp
$(BATCHCHK): $(BATCH_SRCS) tests/dropin/trial_common.hpp $(PKG)/host/dropin/simulation_batch.hpp \
             $(PKG)/host/qkd_ldpc_impl.hpp tests/dropin/api/qkd_ldpc_algorithm.hpp tests/dropin/api/simulation.hpp \
             include/qkd_ldpc_hip.h $(LIB)
	g++ -O2 -std=c++20 -Wall -pthread -I tests/dropin/api -I $(PKG)/host/dropin -I include $(BATCH_SRCS) \
	    -L$(PKG) -lqkdldpc_hip -Wl,-rpath,'$$ORIGIN/../../$(PKG)' -o $@

# FP64 VALU ceilings of the SPA edge math (tools/valu_bench.hip), run on the box.
tools/valu_bench: tools/valu_bench.hip $(CSRC)/exact_math.h
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -ffp-contract=off $< -o $@
valu_bench: tools/valu_bench

clean:
	rm -f $(CSRC)/*.o $(LIB) $(HOSTCHK) $(DROPIN) $(BATCHCHK) $(STAMPLIB) tools/valu_bench
	$(MAKE) -C oracle clean

.PHONY: all clean stamps valu_bench

# Sanitizer build: the host code of the product library (C ABI,
# planner, relabelling, loaders, launch code), the CPU oracle and the two C++
# drivers under ASan + UBSan (clang's runtime, the one hipcc links), into
# build/asan/.  `make asan-check` runs the CPU test suite against it
# (tools/asan_check.sh).  Device code is unchanged: GPU sanitizers are not
# available on this pool.
ASAN := build/asan
LLVM_BIN := /opt/rocm/lib/llvm/bin
SANFLAGS := -fsanitize=address -fsanitize=undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g
HIP_SAN := -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined \
           -Xarch_host -fno-omit-frame-pointer -g
ASAN_HIP_OBJS := $(ASAN)/decoder.o $(ASAN)/decoder_v2.o $(ASAN)/trials.o $(ASAN)/order.o $(ASAN)/capi.o
$(ASAN)/%.o: $(CSRC)/%.hip $(CSRC)/decoder.hpp $(CSRC)/decoder_common.hpp $(CSRC)/exact_math.h $(CSRC)/relabel.hpp $(CSRC)/loaders.hpp include/qkd_ldpc_hip.h
	mkdir -p $(ASAN)
	$(HIPCC) $(HIPFLAGS) $(HIP_SAN) -c $< -o $@
$(ASAN)/loaders.o: $(CSRC)/loaders.cpp $(CSRC)/loaders.hpp
	mkdir -p $(ASAN)
	$(LLVM_BIN)/clang++ -O1 -std=c++17 -fPIC -Wall $(SANFLAGS) -c $< -o $@
$(ASAN)/relabel.o: $(CSRC)/relabel.cpp $(CSRC)/relabel.hpp
	mkdir -p $(ASAN)
	$(LLVM_BIN)/clang++ -O1 -std=c++17 -fPIC -Wall $(SANFLAGS) -c $< -o $@
$(ASAN)/libqkdldpc_hip.so: $(ASAN_HIP_OBJS) $(ASAN)/loaders.o $(ASAN)/relabel.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -shared-libsan $(HIP_SAN) $^ -lz -o $@
$(ASAN)/libqkdldpc_oracle.so: oracle/ldpc_oracle.c oracle/ldpc_oracle.h oracle/trials_oracle.cpp
	mkdir -p $(ASAN)
	$(LLVM_BIN)/clang -O1 -std=c11 -fPIC -Wall -ffp-contract=off $(SANFLAGS) -c oracle/ldpc_oracle.c -o $(ASAN)/ldpc_oracle.o
	$(LLVM_BIN)/clang++ -O1 -std=c++17 -fPIC -Wall -ffp-contract=off $(SANFLAGS) -c oracle/trials_oracle.cpp -o $(ASAN)/trials_oracle.o
	$(LLVM_BIN)/clang++ -shared -shared-libsan $(SANFLAGS) $(ASAN)/ldpc_oracle.o $(ASAN)/trials_oracle.o -lm -lpthread -o $@
$(ASAN)/host_mirror_check: $(PKG)/host/host_mirror_check.cpp $(PKG)/host/qkd_ldpc_algorithm.hpp $(PKG)/host/qkd_ldpc_impl.hpp $(ASAN)/libqkdldpc_hip.so
	$(LLVM_BIN)/clang++ -O1 -std=c++17 -Wall $(SANFLAGS) -shared-libsan -I include $< -L$(ASAN) -lqkdldpc_hip -Wl,-rpath,'$$ORIGIN' -o $@
$(ASAN)/run_trial_check: tests/dropin/run_trial_check.cpp tests/dropin/trial_common.hpp $(PKG)/host/dropin/qkd_ldpc_algorithm.cpp $(PKG)/host/qkd_ldpc_impl.hpp $(ASAN)/libqkdldpc_hip.so
	$(LLVM_BIN)/clang++ -O1 -std=c++20 -Wall -pthread $(SANFLAGS) -shared-libsan -I tests/dropin/api -I include tests/dropin/run_trial_check.cpp \
	    $(PKG)/host/dropin/qkd_ldpc_algorithm.cpp -L$(ASAN) -lqkdldpc_hip -Wl,-rpath,'$$ORIGIN' -o $@
$(ASAN)/batch_check: $(BATCH_SRCS) tests/dropin/trial_common.hpp $(PKG)/host/dropin/simulation_batch.hpp $(PKG)/host/qkd_ldpc_impl.hpp $(ASAN)/libqkdldpc_hip.so
	$(LLVM_BIN)/clang++ -O1 -std=c++20 -Wall -pthread $(SANFLAGS) -shared-libsan -I tests/dropin/api -I $(PKG)/host/dropin -I include \
	    $(BATCH_SRCS) -L$(ASAN) -lqkdldpc_hip -Wl,-rpath,'$$ORIGIN' -o $@
asan: $(ASAN)/libqkdldpc_hip.so $(ASAN)/libqkdldpc_oracle.so $(ASAN)/host_mirror_check $(ASAN)/run_trial_check $(ASAN)/batch_check
asan-check: asan
	bash tools/asan_check.sh
.PHONY: asan asan-check

# A/B experiment build: `make ab AB=name AB_FLAGS=-D...` -> qkd_ldpc_v_amd/ab/name/
# (AB_CAPI=1: capi.hip with the same flags too, for shapes the planner shares)
# (selected at run time with QLDPC_DIAG=1 QLDPC_AB_BUILD=name; never the product)
AB ?= x
ab:
	mkdir -p $(PKG)/ab/$(AB)
	$(HIPCC) $(HIPFLAGS) $(V2FLAGS) $(AB_FLAGS) -c $(CSRC)/decoder_v2.hip -o $(PKG)/ab/$(AB)/decoder_v2.o
	if [ -n "$(AB_CAPI)" ]; then $(HIPCC) $(HIPFLAGS) $(AB_FLAGS) -c $(CSRC)/capi.hip -o $(PKG)/ab/$(AB)/capi.o; else cp $(CSRC)/capi.o $(PKG)/ab/$(AB)/capi.o; fi
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(PKG)/ab/$(AB)/decoder_v2.o $(CSRC)/decoder.o $(CSRC)/trials.o $(CSRC)/order.o $(PKG)/ab/$(AB)/capi.o $(CSRC)/loaders.o $(CSRC)/relabel.o -lz -o $(PKG)/ab/$(AB)/libqkdldpc_hip.so
.PHONY: ab
