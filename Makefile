# Build the native runtime in-tree for MI355X (gfx950).
#
#   make            -> distributed_llm_dissemination_amd/_core<ext>.so  (C++ core + HIP kernels + RCCL engine)
#   make tools      -> bin/diskspeed (NVMe -> pinned -> HBM calibration)
#   make sanitize   -> build/tests/*_{tsan,asan} (host-only core under Thread/Address sanitizer)
#
# The extension links the HIP runtime and RCCL that PyTorch-ROCm ships, so one
# process never holds two HIP runtimes (torch is imported before _core).

PY        ?= python3
ARCH      ?= gfx950
HIPCC     ?= /opt/rocm/bin/hipcc
CXX       := g++
JOBS      ?= 8

PYINC     := $(shell $(PY) -c "import sysconfig;print(sysconfig.get_paths()['include'])")
PYBIND    := $(shell $(PY) -c "import pybind11;print(pybind11.get_include())")
EXT       := $(shell $(PY) -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")
TORCHLIB  := $(shell $(PY) -c "import os,importlib.util as u;print(os.path.join(os.path.dirname(u.find_spec('torch').origin),'lib'))")
ROCM      := /opt/rocm

PKG       := distributed_llm_dissemination_amd
TARGET    := $(PKG)/_core$(EXT)
BUILD     := build

CXXFLAGS  := -O2 -g1 -std=c++17 -fPIC -Wall -Wno-sign-compare -Wno-unused-result -Icsrc -I$(PYINC) -I$(PYBIND) \
             -D__HIP_PLATFORM_AMD__ -I$(ROCM)/include -I$(ROCM)/include/rccl -fvisibility=hidden
HIPFLAGS  := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Icsrc -I$(ROCM)/include -Wno-unused-result \
             -fvisibility=hidden
LDFLAGS   := -shared -L$(TORCHLIB) -Wl,-rpath,$(TORCHLIB) -lamdhip64 -lrccl -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrocprofiler-sdk-roctx -lpthread

CORE_SRC  := csrc/core/vclock.cc csrc/core/json.cc csrc/core/log.cc csrc/core/wire.cc csrc/core/crc32c.cc csrc/core/fp8.cc csrc/core/trace.cc csrc/transport/inproc.cc \
             csrc/transport/tcp.cc csrc/store/store.cc csrc/sched/maxflow.cc csrc/sched/lp.cc csrc/roles/node.cc \
             csrc/roles/mode01.cc csrc/roles/mode2.cc csrc/roles/mode3.cc csrc/roles/multihost.cc \
             csrc/roles/recovery.cc csrc/roles/dispatch.cc \
             csrc/engine/host_engine.cc csrc/engine/planned_engine.cc csrc/engine/planned_stage.cc \
             csrc/engine/planned_recovery.cc csrc/engine/sim_backend.cc
BIND_SRC  := csrc/bindings.cc
GPU_SRC   := $(wildcard csrc/gpu/*.cc)
HIP_SRC   := $(wildcard csrc/kernels/*.hip)

CORE_OBJ  := $(patsubst csrc/%.cc,$(BUILD)/%.o,$(CORE_SRC))
BIND_OBJ  := $(patsubst csrc/%.cc,$(BUILD)/%.o,$(BIND_SRC))
GPU_OBJ   := $(patsubst csrc/%.cc,$(BUILD)/%.o,$(GPU_SRC))
HIP_OBJ   := $(patsubst csrc/%.hip,$(BUILD)/%.hip.o,$(HIP_SRC))

all: $(TARGET)

$(TARGET): $(CORE_OBJ) $(BIND_OBJ) $(GPU_OBJ) $(HIP_OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -o $@ $^ $(LDFLAGS)

$(BUILD)/%.hip.o: csrc/%.hip csrc/kernels/*.h
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/%.o: csrc/%.cc $(wildcard csrc/*/*.h) Makefile
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -c $< -o $@

tools: bin/diskspeed bin/h2dbench bin/contention bin/cvtprobe bin/walkprobe

bin/contention: $(BUILD)/tools/contention.hip.o $(BUILD)/kernels/crc32c.hip.o $(BUILD)/kernels/fill.hip.o $(BUILD)/core/crc32c.o
	@mkdir -p bin
	$(HIPCC) --offload-arch=$(ARCH) -o $@ $^ -L$(TORCHLIB) -Wl,-rpath,$(TORCHLIB) -lamdhip64 -lrccl \
	  -L$(ROCM)/lib -Wl,-rpath,$(ROCM)/lib

bin/cvtprobe: csrc/tools/cvtprobe.hip
	@mkdir -p bin
	$(HIPCC) -O2 -std=c++17 --offload-arch=$(ARCH) -Wno-unused-value -Wno-unused-result -o $@ $< -L$(TORCHLIB) -Wl,-rpath,$(TORCHLIB) -lamdhip64

bin/walkprobe: csrc/tools/walkprobe.hip
	@mkdir -p bin
	$(HIPCC) -O3 -std=c++17 --offload-arch=$(ARCH) -o $@ $< -L$(TORCHLIB) -Wl,-rpath,$(TORCHLIB) -lamdhip64

bin/h2dbench: csrc/tools/h2dbench.hip
	@mkdir -p bin
	$(HIPCC) -O3 -std=c++17 --offload-arch=$(ARCH) -o $@ $< -L$(TORCHLIB) -Wl,-rpath,$(TORCHLIB) -lamdhip64

bin/diskspeed: csrc/tools/diskspeed.cc
	@mkdir -p bin
	$(HIPCC) -O2 -std=c++17 --offload-arch=$(ARCH) -Icsrc -o $@ $< -L$(TORCHLIB) -Wl,-rpath,$(TORCHLIB) -lamdhip64 -lpthread

# ---- host-only sanitizer builds of the core
SAN_SRC := $(CORE_SRC) csrc/tests/core_selftest.cc
sanitize: $(BUILD)/tests/core_selftest_tsan $(BUILD)/tests/core_selftest_asan

$(BUILD)/tests/core_selftest_tsan: $(SAN_SRC)
	@mkdir -p $(dir $@)
	$(CXX) -O1 -g -std=c++17 -Icsrc -fsanitize=thread -I/opt/rocm/include -o $@ $(SAN_SRC) -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrocprofiler-sdk-roctx -lpthread

$(BUILD)/tests/core_selftest_asan: $(SAN_SRC)
	@mkdir -p $(dir $@)
	$(CXX) -O1 -g -std=c++17 -Icsrc -fsanitize=address,undefined -fno-omit-frame-pointer -I/opt/rocm/include -o $@ $(SAN_SRC) -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrocprofiler-sdk-roctx -lpthread

clean:
	rm -rf $(BUILD) $(PKG)/_core*.so bin/diskspeed bin/h2dbench bin/contention

.PHONY: all tools sanitize clean
