# Build of the MI355X runtime (libopt_amd.so) and the CPU oracle.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH  ?= gfx950
CXXFLAGS = -O3 -std=c++17 -fPIC -Wall -Wno-unused-function $(EXTRA)
SRC_DIR = opt_amd/csrc
HIP_SRCS = $(wildcard $(SRC_DIR)/*.hip)
CPP_SRCS = $(wildcard $(SRC_DIR)/*.cpp)
GEN_SRCS = $(wildcard $(SRC_DIR)/gen/*.cpp)
HDRS = $(wildcard $(SRC_DIR)/*.h) $(wildcard $(SRC_DIR)/gen/*.h) include/Opt.h include/opt_amd.h
OBJ_DIR ?= build/obj
OBJS = $(patsubst $(SRC_DIR)/%.hip,$(OBJ_DIR)/%.o,$(HIP_SRCS)) $(patsubst $(SRC_DIR)/%.cpp,$(OBJ_DIR)/%.o,$(CPP_SRCS)) \
       $(patsubst $(SRC_DIR)/gen/%.cpp,$(OBJ_DIR)/gen/%.o,$(GEN_SRCS))
# reduce_dev.h as a string literal, pasted into the sources the front end generates
GEN_DIR ?= build/gen
REDUCE_SRC = $(GEN_DIR)/reduce_dev_src.h
LIB ?= opt_amd/libopt_amd.so
RCCL_STUB = tests/rccl_stub/librccl_stub.so

all: $(LIB) oracle $(RCCL_STUB)

$(OBJ_DIR)/%.o: $(SRC_DIR)/%.hip $(HDRS)
	@mkdir -p $(OBJ_DIR)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -c $< -o $@

$(OBJ_DIR)/%.o: $(SRC_DIR)/%.cpp $(HDRS)
	@mkdir -p $(OBJ_DIR)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -c $< -o $@

$(OBJ_DIR)/gen/%.o: $(SRC_DIR)/gen/%.cpp $(HDRS) $(REDUCE_SRC)
	@mkdir -p $(OBJ_DIR)/gen
	g++ $(CXXFLAGS) -I$(GEN_DIR) -c $< -o $@

# the energies the hand-written families implement, as string literals (generic.hip:
# family_is_canonical compares a user's energy file against them)
FAMILIES = image_warping poisson_image_editing optical_flow shape_from_shading arap_mesh_deformation
FAMILY_SRC = $(GEN_DIR)/family_energies_src.h
$(FAMILY_SRC): $(patsubst %,energies/%.t,$(FAMILIES))
	@mkdir -p $(GEN_DIR)
	( for f in $(FAMILIES); do echo "{\"$$f\", R\"OPTAMDRAW("; cat energies/$$f.t; echo ')OPTAMDRAW"},'; done ) > $@

$(OBJ_DIR)/generic.o: $(SRC_DIR)/generic.hip $(HDRS) $(FAMILY_SRC)
	@mkdir -p $(OBJ_DIR)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -I$(GEN_DIR) -c $< -o $@

$(REDUCE_SRC): $(SRC_DIR)/reduce_dev.h
	@mkdir -p $(GEN_DIR)
	( echo 'static const char kReduceDevSrc[] = R"OPTAMDRAW('; cat $<; echo ')OPTAMDRAW";' ) > $@

$(LIB): $(OBJS)
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJS) -lhiprtc

oracle:
	$(MAKE) -C oracle

# test infrastructure: the multi-process RCCL stand-in (tests/rccl_stub/rccl_stub.cpp)
$(RCCL_STUB): tests/rccl_stub/rccl_stub.cpp
	$(HIPCC) -O2 -std=c++17 -fPIC -shared -Wl,-Bsymbolic -Wl,-soname,librccl_stub.so -o $@ $< -lrt
rccl_stub: $(RCCL_STUB)

clean:
	rm -rf build $(LIB) $(RCCL_STUB)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean rccl_stub
