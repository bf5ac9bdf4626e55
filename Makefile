# miint build: HIP kernels for gfx950 + native runtime + Python extension + CLI tools.
#
#   make            -> extension + CLIs          make ext   -> Python extension only
#   make cli        -> build/bin/*               make clean
#
# Everything is compiled by hipcc for --offload-arch=gfx950 (MI355X / CDNA4) only.
# Replaces the reference Makefile (Makefile:1-9: one mpigxx target built at -O0, no rules
# for the CUDA or 4main programs, a target whose source does not exist — SURVEY C18/B17).

HIPCC    ?= /opt/rocm/bin/hipcc
HOSTCXX  ?= g++
ARCH     ?= gfx950
PYTHON   ?= python3
BUILD    := build
OBJ      := $(BUILD)/obj
BIN      := $(BUILD)/bin
PKG      := cuda_v_mpi_amd

EXT_SUFFIX := $(shell $(PYTHON) -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")
PY_INC     := $(shell $(PYTHON) -m pybind11 --includes)

COMMON   := -std=c++17 -O3 -fPIC -Icsrc/include -Wall -Wno-unused-function
# ABFLAGS: kernel variants for A/B builds (make cli BUILD=build/ab_x ABFLAGS=-D...; tools/*_ab.sh)
ABFLAGS  ?=
DEVFLAGS := $(COMMON) $(ABFLAGS) --offload-arch=$(ARCH)
HOSTFLAGS:= $(COMMON) -I/opt/rocm/include -D__HIP_PLATFORM_AMD__
LDLIBS   := -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrccl -lhiprtc -lamdhip64 -lpthread -ldl

HIP_SRC  := $(wildcard csrc/kernels/*.hip)
RT_SRC   := $(wildcard csrc/runtime/*.cpp)
HDRS     := $(wildcard csrc/include/miint/*.hpp) $(wildcard csrc/runtime/*.inc)
HIP_OBJ  := $(patsubst csrc/kernels/%.hip,$(OBJ)/k_%.o,$(HIP_SRC))
RT_OBJ   := $(patsubst csrc/runtime/%.cpp,$(OBJ)/r_%.o,$(RT_SRC))
LIB      := $(BUILD)/libmiint.a
EXT      := $(PKG)/_miint$(EXT_SUFFIX)
CLIS     := $(BIN)/riemann $(BIN)/cintegrate $(BIN)/trainscan $(BIN)/miint $(BIN)/miintrun

.PHONY: all ext cli lib clean asm
all: ext cli
ext: $(EXT)
cli: $(CLIS)
lib: $(LIB)

$(OBJ) $(BIN):
	@mkdir -p $@

$(OBJ)/k_%.o: csrc/kernels/%.hip $(HDRS) | $(OBJ)
	$(HIPCC) $(DEVFLAGS) -c $< -o $@

$(OBJ)/r_%.o: csrc/runtime/%.cpp $(HDRS) | $(OBJ)
	$(HIPCC) -x c++ $(HOSTFLAGS) -c $< -o $@

$(LIB): $(HIP_OBJ) $(RT_OBJ)
	@rm -f $@
	ar rcs $@ $^

$(OBJ)/py_module.o: csrc/python/module.cpp $(HDRS) | $(OBJ)
	$(HIPCC) -x c++ $(HOSTFLAGS) $(PY_INC) -fvisibility=hidden -c $< -o $@

$(EXT): $(OBJ)/py_module.o $(HIP_OBJ) $(RT_OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ $(LDLIBS)

$(OBJ)/cli_%.o: csrc/cli/%.cpp csrc/cli/cli_common.hpp $(HDRS) | $(OBJ)
	$(HIPCC) -x c++ $(HOSTFLAGS) -c $< -o $@

# the launcher links no HIP (it must never initialise a GPU: it forks and execs the ranks)
$(BIN)/miintrun: csrc/cli/miintrun.cpp csrc/include/miint/net.hpp | $(BIN)
	$(HOSTCXX) -std=c++17 -O2 -Wall -Icsrc/include -o $@ $<

$(BIN)/%: $(OBJ)/cli_%.o $(LIB) | $(BIN)
	$(HIPCC) -o $@ $< $(LIB) $(LDLIBS)

# Keep the gfx950 assembly of every kernel file for inspection (build/asm/*.s).
asm: | $(OBJ)
	@mkdir -p $(BUILD)/asm
	@for f in $(HIP_SRC); do b=$$(basename $$f .hip); \
	  $(HIPCC) $(DEVFLAGS) --cuda-device-only -S $$f -o $(BUILD)/asm/$$b.s; done

clean:
	rm -rf $(BUILD) $(EXT)

# Host-side sanitizers (GPU ASan / xnack+ are not available on the target pool): the CPU
# half of the runtime — oracles, parity emulation, slicing, CLI parsing, run records, the
# TCP rendezvous — under ASan+UBSan.
SAN := -fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g -O1
.PHONY: sanitize
sanitize: $(BIN)/host_selftest_asan
SAN_SRC := csrc/cli/host_selftest.cpp csrc/runtime/oracle.cpp csrc/runtime/profile_data.cpp \
           csrc/runtime/comm.cpp csrc/runtime/agree.cpp csrc/runtime/trace.cpp csrc/runtime/runtime.cpp \
           csrc/runtime/host.cpp csrc/runtime/host_comm.cpp
$(BIN)/host_selftest_asan: $(SAN_SRC) csrc/cli/cli_common.hpp $(HDRS) | $(BIN)
	$(HIPCC) -x c++ -std=c++17 -Icsrc/include -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ $(SAN) \
	  -o $@ $(SAN_SRC) \
	  -L/opt/rocm/lib -lamdhip64 -lrccl -lpthread -ldl
