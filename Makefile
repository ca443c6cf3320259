# Native build for the MI355X bidirectional-BFS framework (gfx950 only).
#
#   make -j8            -> build/lib/libbibfs.so, build/lib/libbibfs_mpi.so,
#                          build/bin/* CLI tools, bidirectional_bfs_amd/_native*.so
#   make cpu            -> host-only pieces (no hipcc needed)
#   make asan           -> host-only pieces + MPI engines with AddressSanitizer +
#                          UBSan in build-asan/ (scripts/asan_check.sh runs the
#                          CLI / MPI test subset against them)
#   make clean
#
# The reference builds each engine with its own Makefile (v1..v4/Makefile) and
# ships two of them without optimisation (v1/Makefile:2,7 typo, v4/Makefile:27);
# everything here is -O3.

ROCM      ?= /opt/rocm
MPI_HOME  ?= /opt/conda
ARCH      ?= gfx950
HIPCC     ?= $(ROCM)/bin/hipcc
CXX       ?= g++
PYTHON    ?= python3

BUILD     ?= build
OBJ       := $(BUILD)/obj
LIB       := $(BUILD)/lib
BIN       := $(BUILD)/bin
PKG       := bidirectional_bfs_amd

CXXSTD    := -std=c++17
INC       := -Icsrc/include -Icsrc/hip
OPT       ?= -O3
SANFLAGS  ?=
CXXFLAGS  += $(OPT) -fPIC $(CXXSTD) -Wall -Wextra -Wno-unused-parameter $(INC) -pthread $(SANFLAGS)
HIPFLAGS  := -O3 -fPIC $(CXXSTD) $(INC) --offload-arch=$(ARCH) -mcode-object-version=5 \
             -Wno-unused-result -munsafe-fp-atomics
MPI_INC   := -I$(MPI_HOME)/include
# system libstdc++ first: conda ships an older one
MPI_LD    := $(MPI_HOME)/lib/libmpi.so -Wl,-rpath,/usr/lib/x86_64-linux-gnu:$(MPI_HOME)/lib
HIP_LD    := -L$(ROCM)/lib -lamdhip64 -lrocprofiler-sdk-roctx -Wl,-rpath,$(ROCM)/lib
RCCL_LD   := -L$(ROCM)/lib -lrccl

PY_INC    := $(shell $(PYTHON) -c "import sysconfig; print(sysconfig.get_paths()['include'])")
PYBIND_INC:= $(shell $(PYTHON) -c "import pybind11; print(pybind11.get_include())")
PY_EXT    := $(shell $(PYTHON) -c "import sysconfig; print(sysconfig.get_config_var('EXT_SUFFIX'))")

CORE_SRC  := csrc/io/io.cpp csrc/gen/gen.cpp csrc/csr/csr.cpp csrc/cpu/serial_bibfs.cpp csrc/dist/ipc_group.cpp
HIP_SRC   := csrc/hip/csr_device.hip csrc/hip/engine_kernels.hip csrc/hip/tiny_engine.hip csrc/hip/batch_global.hip csrc/hip/hip_engine.hip \
             csrc/hip/capi.hip csrc/dist/comm.hip csrc/dist/ipc_comm.hip csrc/dist/dist_engine.hip
MPI_SRC   := csrc/cpu/mpi_bitmap_bibfs.cpp csrc/cpu/mpi_queue_bibfs.cpp

CORE_OBJ  := $(patsubst csrc/%.cpp,$(OBJ)/%.o,$(CORE_SRC))
HIP_OBJ   := $(patsubst csrc/%.hip,$(OBJ)/%.o,$(HIP_SRC))
MPI_OBJ   := $(patsubst csrc/%.cpp,$(OBJ)/%.o,$(MPI_SRC))

HEADERS   := $(wildcard csrc/include/bibfs/*.hpp csrc/include/bibfs/*.h csrc/hip/*.hpp csrc/dist/*.hpp)

CPU_TOOLS := $(BIN)/bibfs_serial $(BIN)/show_matrix $(BIN)/bibfs_gen $(BIN)/ipc_group_check
MPI_TOOLS := $(BIN)/second_try $(BIN)/mpi_queue_bibfs
GPU_TOOLS := $(BIN)/bibfs_selftest $(BIN)/bibfs_hip $(BIN)/mpi_bibfs $(BIN)/bibfs_bench

NATIVE_PY := $(PKG)/_native$(PY_EXT)

.PHONY: all cpu gpu mpi python micro clean asan
all: cpu mpi gpu python micro
cpu: $(LIB)/libbibfs_core.so $(CPU_TOOLS)
mpi: $(LIB)/libbibfs_mpi.so $(MPI_TOOLS)
gpu: $(LIB)/libbibfs.so $(GPU_TOOLS) $(BIN)/bibfs_cuda_only
python: $(NATIVE_PY)
micro: $(BIN)/lat_probe $(BIN)/mailbox_rtt $(BIN)/place_probe $(BIN)/grid_barrier

# The LDS engine's counter atomics are already issued by one lane per wave:
# the compiler's wave-reduction rewrite of them only adds instructions to the
# latency-bound rounds.
$(OBJ)/hip/engine_kernels.o $(OBJ)/hip/tiny_engine.o: HIPFLAGS += -mllvm -amdgpu-atomic-optimizer-strategy=None

$(BIN)/mailbox_rtt: benchmarks/micro/mailbox_rtt.hip
	@mkdir -p $(BIN)
	$(HIPCC) -O3 -std=c++17 --offload-arch=$(ARCH) -mcode-object-version=5 $< -o $@ -L/opt/rocm/lib -lhsa-runtime64

$(BIN)/grid_barrier: benchmarks/micro/grid_barrier.hip
	@mkdir -p $(BIN)
	$(HIPCC) -O3 -std=c++17 --offload-arch=$(ARCH) -mcode-object-version=5 $< -o $@

$(BIN)/place_probe: benchmarks/micro/place_probe.hip
	@mkdir -p $(BIN)
	$(HIPCC) -O3 -std=c++17 --offload-arch=$(ARCH) -mcode-object-version=5 $< -o $@

$(BIN)/lat_probe: benchmarks/micro/lat_probe.hip
	@mkdir -p $(BIN)
	$(HIPCC) -O3 -std=c++17 --offload-arch=$(ARCH) -mcode-object-version=5 $< -o $@

$(OBJ)/%.o: csrc/%.cpp $(HEADERS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) $(if $(findstring mpi,$<),$(MPI_INC)) -c $< -o $@

$(OBJ)/%.o: csrc/%.hip $(HEADERS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB)/libbibfs_core.so: $(CORE_OBJ)
	@mkdir -p $(LIB)
	$(CXX) -shared -o $@ $^ -pthread $(SANFLAGS)

$(LIB)/libbibfs.so: $(CORE_OBJ) $(HIP_OBJ)
	@mkdir -p $(LIB)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $^ $(HIP_LD) $(RCCL_LD) -pthread

$(LIB)/libbibfs_mpi.so: $(MPI_OBJ) $(LIB)/libbibfs_core.so
	@mkdir -p $(LIB)
	$(CXX) -shared -o $@ $(MPI_OBJ) -L$(LIB) -lbibfs_core -Wl,-rpath,'$$ORIGIN' $(MPI_LD) -pthread $(SANFLAGS)

# --- CLI tools ---------------------------------------------------------------
TOOL_CXX = $(CXX) $(CXXFLAGS)
$(BIN)/bibfs_serial: tools/bibfs_serial.cpp tools/cli_common.hpp $(LIB)/libbibfs_core.so
	@mkdir -p $(BIN)
	$(TOOL_CXX) $< -o $@ -L$(LIB) -lbibfs_core -Wl,-rpath,'$$ORIGIN/../lib'
$(BIN)/show_matrix: tools/show_matrix.cpp $(LIB)/libbibfs_core.so
	@mkdir -p $(BIN)
	$(TOOL_CXX) $< -o $@ -L$(LIB) -lbibfs_core -Wl,-rpath,'$$ORIGIN/../lib'
$(BIN)/ipc_group_check: tools/ipc_group_check.cpp csrc/dist/ipc_group.hpp $(LIB)/libbibfs_core.so
	@mkdir -p $(BIN)
	$(TOOL_CXX) $< -o $@ -L$(LIB) -lbibfs_core -Wl,-rpath,'$$ORIGIN/../lib'
$(BIN)/bibfs_gen: tools/bibfs_gen.cpp tools/cli_common.hpp $(LIB)/libbibfs_core.so
	@mkdir -p $(BIN)
	$(TOOL_CXX) $< -o $@ -L$(LIB) -lbibfs_core -Wl,-rpath,'$$ORIGIN/../lib'
$(BIN)/second_try: tools/second_try.cpp tools/cli_common.hpp $(LIB)/libbibfs_mpi.so
	@mkdir -p $(BIN)
	$(TOOL_CXX) $(MPI_INC) $< -o $@ -L$(LIB) -lbibfs_mpi -lbibfs_core -Wl,-rpath,'$$ORIGIN/../lib' $(MPI_LD)
$(BIN)/mpi_queue_bibfs: tools/mpi_queue_bibfs.cpp tools/cli_common.hpp $(LIB)/libbibfs_mpi.so
	@mkdir -p $(BIN)
	$(TOOL_CXX) $(MPI_INC) $< -o $@ -L$(LIB) -lbibfs_mpi -lbibfs_core -Wl,-rpath,'$$ORIGIN/../lib' $(MPI_LD)
$(BIN)/bibfs_hip: tools/bibfs_hip.cpp tools/cli_common.hpp $(LIB)/libbibfs.so
	@mkdir -p $(BIN)
	$(TOOL_CXX) $< -o $@ -L$(LIB) -lbibfs -Wl,-rpath,'$$ORIGIN/../lib' $(HIP_LD)
$(BIN)/bibfs_cuda_only: $(BIN)/bibfs_hip
	ln -sf bibfs_hip $@
$(BIN)/bibfs_bench: tools/bibfs_bench.cpp tools/cli_common.hpp $(LIB)/libbibfs.so
	@mkdir -p $(BIN)
	$(TOOL_CXX) $< -o $@ -L$(LIB) -lbibfs -Wl,-rpath,'$$ORIGIN/../lib' $(HIP_LD)
$(BIN)/mpi_bibfs: tools/mpi_bibfs.cpp tools/cli_common.hpp $(LIB)/libbibfs.so $(LIB)/libbibfs_mpi.so
	@mkdir -p $(BIN)
	$(TOOL_CXX) $(MPI_INC) $< -o $@ -L$(LIB) -lbibfs_mpi -lbibfs \
	  -Wl,-rpath,'$$ORIGIN/../lib' $(HIP_LD) $(RCCL_LD) $(MPI_LD)

# --- Python extension (pybind11), in-tree next to the package --------------
$(NATIVE_PY): csrc/python/bindings.cpp $(HEADERS) $(LIB)/libbibfs.so
	$(CXX) $(CXXFLAGS) -I$(PY_INC) -I$(PYBIND_INC) -shared $< -o $@ -L$(LIB) -lbibfs \
	  -Wl,-rpath,'$$ORIGIN/../$(LIB)' $(HIP_LD)

clean:
	rm -rf $(BUILD) build-asan $(PKG)/_native*.so

# Host code under AddressSanitizer + UndefinedBehaviorSanitizer (the GPU code
# is not instrumented: GPU ASan is not available on this pool).
asan:
	$(MAKE) BUILD=build-asan OPT="-O1 -g -fno-omit-frame-pointer" \
	  SANFLAGS="-fsanitize=address,undefined -fno-sanitize-recover=undefined" cpu mpi

$(BIN)/bibfs_selftest: tools/bibfs_selftest.cpp tools/cli_common.hpp $(LIB)/libbibfs.so
	@mkdir -p $(BIN)
	$(TOOL_CXX) $< -o $@ -L$(LIB) -lbibfs -Wl,-rpath,'$$ORIGIN/../lib' $(HIP_LD)
