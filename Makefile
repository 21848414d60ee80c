# Builds libcheb_mi355.so (gfx950) in-tree and the oracle's reference build.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
CXXFLAGS ?= -O3 -std=c++17 -fPIC -Wall -Wno-unused-function --offload-arch=$(ARCH) $(EXTRA)
SRC_DIR  := cnn_graph_amd/csrc
OBJ_DIR  ?= build/obj
LIB      ?= cnn_graph_amd/libcheb_mi355.so
SRCS     := $(SRC_DIR)/cheb_fast.hip $(SRC_DIR)/cheb_resident.hip $(SRC_DIR)/cheb_stream.hip $(SRC_DIR)/graph_ops.hip \
            $(SRC_DIR)/cheb_abi.cpp $(SRC_DIR)/comm.cpp $(SRC_DIR)/coarsen.cpp \
            $(SRC_DIR)/lds_layout.cpp
OBJS     := $(patsubst $(SRC_DIR)/%,$(OBJ_DIR)/%.o,$(SRCS))
HDRS     := $(SRC_DIR)/cg_internal.h include/cheb_mi355.h

all: $(LIB)

$(OBJ_DIR)/%.o: $(SRC_DIR)/% $(HDRS)
	@mkdir -p $(OBJ_DIR)
	$(HIPCC) $(CXXFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $(OBJS) -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

clean:
	rm -rf build $(LIB)

.PHONY: all clean
