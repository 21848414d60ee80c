# Builds libcheb_mi355.so (gfx950) in-tree (the oracle is NumPy: nothing to build for it).
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
CXXFLAGS ?= -O3 -std=c++17 -fPIC -Wall -Wno-unused-function --offload-arch=$(ARCH) $(EXTRA)
SRC_DIR  := cnn_graph_amd/csrc
OBJ_DIR  ?= build/obj
LIB      ?= cnn_graph_amd/libcheb_mi355.so
SRCS     := $(SRC_DIR)/cheb_fast.hip $(SRC_DIR)/cheb_resident.hip $(SRC_DIR)/cheb_stream.hip $(SRC_DIR)/cheb_wide.hip $(SRC_DIR)/graph_ops.hip \
            $(SRC_DIR)/lstm.hip $(SRC_DIR)/lstm_fused.hip $(SRC_DIR)/lstm_seq.hip $(SRC_DIR)/cheb_group.hip $(SRC_DIR)/epilogue.hip $(SRC_DIR)/fourier.hip \
            $(SRC_DIR)/cheb_abi.cpp $(SRC_DIR)/comm.cpp $(SRC_DIR)/coarsen.cpp \
            $(SRC_DIR)/lds_layout.cpp
# fast resident kernels: one object per instantiation of cheb_fast_kern.h
# (fastf_<Fin>_<Fout tiles>_<orders basis>, fastb_<Fin>_<fused dW: 1 rows, 2 orders basis>;
# the orders layout for Fin <= 2 only), compiled in parallel
FAST_INST := fastf_1_1_0 fastf_1_2_0 fastf_2_1_0 fastf_2_2_0 fastf_4_1_0 fastf_4_2_0 \
             fastf_1_1_1 fastf_1_2_1 fastf_2_1_1 fastf_2_2_1 \
             fastb_1_0 fastb_1_1 fastb_1_2 fastb_1_3 fastb_2_0 fastb_2_1 fastb_2_2 fastb_2_3 fastb_4_0 fastb_4_1
OBJS     := $(patsubst $(SRC_DIR)/%,$(OBJ_DIR)/%.o,$(SRCS)) $(patsubst %,$(OBJ_DIR)/%.o,$(FAST_INST))
DEPS     := $(OBJS:.o=.d)

all: $(LIB)

# header dependencies are tracked per object (-MMD), so touching the public
# header does not rebuild the (slow) resident-kernel translation units
$(OBJ_DIR)/%.o: $(SRC_DIR)/%
	@mkdir -p $(OBJ_DIR)
	$(HIPCC) $(CXXFLAGS) -MMD -MP -c $< -o $@

w1 = $(word 1,$(subst _, ,$*))
w2 = $(word 2,$(subst _, ,$*))
w3 = $(word 3,$(subst _, ,$*))
$(OBJ_DIR)/fastf_%.o: $(SRC_DIR)/cheb_fast_inst.hip
	@mkdir -p $(OBJ_DIR)
	$(HIPCC) $(CXXFLAGS) -DCG_FAST_FWD -DCG_FV=$(w1) -DCG_NT=$(w2) -DCG_OB=$(w3) -MMD -MP -c $< -o $@
$(OBJ_DIR)/fastb_%.o: $(SRC_DIR)/cheb_fast_inst.hip
	@mkdir -p $(OBJ_DIR)
	$(HIPCC) $(CXXFLAGS) -DCG_FAST_BWD -DCG_FV=$(w1) -DCG_DW=$(w2) -MMD -MP -c $< -o $@

$(LIB): $(OBJS)
	@mkdir -p $(dir $@)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $(OBJS) -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

-include $(DEPS)
# dependency files are never remade (else make's built-in `%: %.o` link rule
# would try to build fastf_1_1.d from fastf_1_1.d.o through the pattern below)
$(DEPS): ;

# Ablation build (scripts/ablate.py, via CG_LIB_PATH): the same sources with
# -DCG_DEBUG, which compiles in cg_debug_set_flags and the kernels' timing
# switches.  Never loaded by the package, the tests or the bench.
DEBUG_LIB ?= scripts/_debug/libcheb_mi355_debug.so
debug:
	$(MAKE) OBJ_DIR=build/dobj LIB=$(DEBUG_LIB) EXTRA=-DCG_DEBUG all

clean:
	rm -rf build $(LIB) $(DEBUG_LIB)

.PHONY: all clean debug
