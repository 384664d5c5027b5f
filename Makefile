# Build of the MI355X runtime (libopt_amd.so) and the CPU oracle.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH  ?= gfx950
CXXFLAGS = -O3 -std=c++17 -fPIC -Wall -Wno-unused-function
SRC_DIR = opt_amd/csrc
HIP_SRCS = $(wildcard $(SRC_DIR)/*.hip)
CPP_SRCS = $(wildcard $(SRC_DIR)/*.cpp)
GEN_SRCS = $(wildcard $(SRC_DIR)/gen/*.cpp)
HDRS = $(wildcard $(SRC_DIR)/*.h) $(wildcard $(SRC_DIR)/gen/*.h) include/Opt.h include/opt_amd.h
OBJ_DIR = build/obj
OBJS = $(patsubst $(SRC_DIR)/%.hip,$(OBJ_DIR)/%.o,$(HIP_SRCS)) $(patsubst $(SRC_DIR)/%.cpp,$(OBJ_DIR)/%.o,$(CPP_SRCS)) \
       $(patsubst $(SRC_DIR)/gen/%.cpp,$(OBJ_DIR)/gen/%.o,$(GEN_SRCS))
# reduce_dev.h as a string literal, pasted into the sources the front end generates
REDUCE_SRC = build/gen/reduce_dev_src.h
LIB = opt_amd/libopt_amd.so

all: $(LIB) oracle

$(OBJ_DIR)/%.o: $(SRC_DIR)/%.hip $(HDRS)
	@mkdir -p $(OBJ_DIR)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -c $< -o $@

$(OBJ_DIR)/%.o: $(SRC_DIR)/%.cpp $(HDRS)
	@mkdir -p $(OBJ_DIR)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -c $< -o $@

$(OBJ_DIR)/gen/%.o: $(SRC_DIR)/gen/%.cpp $(HDRS) $(REDUCE_SRC)
	@mkdir -p $(OBJ_DIR)/gen
	g++ $(CXXFLAGS) -Ibuild/gen -c $< -o $@

$(REDUCE_SRC): $(SRC_DIR)/reduce_dev.h
	@mkdir -p build/gen
	( echo 'static const char kReduceDevSrc[] = R"OPTAMDRAW('; cat $<; echo ')OPTAMDRAW";' ) > $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJS) -lhiprtc

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf build $(LIB)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean
