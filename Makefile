# Builds libcheb_mi355.so (gfx950) in-tree and the oracle's reference build.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
CXXFLAGS ?= -O3 -std=c++17 -fPIC -Wall -Wno-unused-function --offload-arch=$(ARCH) $(EXTRA)
SRC_DIR  := cnn_graph_amd/csrc
OBJ_DIR  ?= build/obj
LIB      ?= cnn_graph_amd/libcheb_mi355.so
SRCS     := $(SRC_DIR)/cheb_fast.hip $(SRC_DIR)/cheb_resident.hip $(SRC_DIR)/cheb_stream.hip $(SRC_DIR)/graph_ops.hip \
            $(SRC_DIR)/lstm.hip $(SRC_DIR)/epilogue.hip $(SRC_DIR)/fourier.hip \
            $(SRC_DIR)/cheb_abi.cpp $(SRC_DIR)/comm.cpp $(SRC_DIR)/coarsen.cpp \
            $(SRC_DIR)/lds_layout.cpp
OBJS     := $(patsubst $(SRC_DIR)/%,$(OBJ_DIR)/%.o,$(SRCS))
DEPS     := $(OBJS:.o=.d)

all: $(LIB)

# header dependencies are tracked per object (-MMD), so touching the public
# header does not rebuild the (slow) resident-kernel translation units
$(OBJ_DIR)/%.o: $(SRC_DIR)/%
	@mkdir -p $(OBJ_DIR)
	$(HIPCC) $(CXXFLAGS) -MMD -MP -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $(OBJS) -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

-include $(DEPS)

clean:
	rm -rf build $(LIB)

.PHONY: all clean
