# LambdaGap-MI355X native build: host C++17 (g++/OpenMP) + HIP kernels for
# gfx950 (hipcc), linked into one shared library used by the Python package
# (ctypes) and by the CLI. Device code is cross-compiled; no GPU is needed to build.
ROCM ?= /opt/rocm
HIPCC ?= $(ROCM)/bin/hipcc
CXX ?= g++
ARCH ?= gfx950
BUILD ?= build
OUT ?= lambdagap_amd/lib
JOBS ?= 8

CXXFLAGS ?= -O3 -g0 -std=c++17 -fPIC -fopenmp -Wall -Wno-unused-function -Wno-sign-compare -Iinclude -Isrc \
            -D__HIP_PLATFORM_AMD__=1 -I$(ROCM)/include
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Iinclude -Isrc -munsafe-fp-atomics \
            -Wno-unused-result -ffp-contract=fast
LDFLAGS ?= -shared -fopenmp -L$(ROCM)/lib -lamdhip64 -lrccl -lrocprofiler-sdk-roctx -Wl,-rpath,$(ROCM)/lib

CPP_SRCS := $(shell find src -name '*.cpp' ! -path 'src/cli/*' | sort)
HIP_SRCS := $(shell find src -name '*.hip' | sort)
CPP_OBJS := $(patsubst src/%.cpp,$(BUILD)/%.o,$(CPP_SRCS))
HIP_OBJS := $(patsubst src/%.hip,$(BUILD)/%.hip.o,$(HIP_SRCS))
HEADERS := $(shell find include src -name '*.h' -o -name '*.def' -o -name '*.hpp')

LIB := $(OUT)/lib_lambdagap.so
CLI := $(OUT)/lambdagap

all: $(LIB) $(CLI)

$(BUILD)/%.o: src/%.cpp $(HEADERS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(BUILD)/%.hip.o: src/%.hip $(HEADERS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(CPP_OBJS) $(HIP_OBJS)
	@mkdir -p $(OUT)
	$(CXX) -o $@ $^ $(LDFLAGS)

$(CLI): src/cli/main.cpp $(LIB) $(HEADERS)
	@mkdir -p $(OUT)
	$(CXX) $(CXXFLAGS) -o $@ src/cli/main.cpp -L$(OUT) -l_lambdagap -Wl,-rpath,'$$ORIGIN' -fopenmp

# native unit tests (reference tests/cpp_tests analogue), linked against the library
CPPTEST := $(BUILD)/test_native
cpptest: $(CPPTEST)
$(CPPTEST): tests/cpp/test_native.cpp $(LIB) $(HEADERS)
	$(CXX) $(CXXFLAGS) -o $@ tests/cpp/test_native.cpp -L$(OUT) -l_lambdagap -Wl,-rpath,$(abspath $(OUT)) -fopenmp

# host code under AddressSanitizer + UBSan: every .cpp of the core and
# the test are rebuilt with the sanitizers; the HIP objects are linked as built (device
# code is never sanitized: GPU ASan / XNACK runs are unavailable on the target pool)
ASAN_DIR := $(BUILD)/asan
SANFLAGS := -fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=undefined
ASAN_OBJS := $(patsubst src/%.cpp,$(ASAN_DIR)/%.o,$(CPP_SRCS))
$(ASAN_DIR)/%.o: src/%.cpp $(HEADERS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -O1 $(SANFLAGS) -c $< -o $@
asan: $(ASAN_DIR)/test_native
$(ASAN_DIR)/test_native: tests/cpp/test_native.cpp $(ASAN_OBJS) $(HIP_OBJS) $(HEADERS)
	$(CXX) $(CXXFLAGS) -O1 $(SANFLAGS) -o $@ tests/cpp/test_native.cpp $(ASAN_OBJS) $(HIP_OBJS) \
	  -fopenmp -L$(ROCM)/lib -lamdhip64 -lrccl -lrocprofiler-sdk-roctx -Wl,-rpath,$(ROCM)/lib

clean:
	rm -rf $(BUILD) $(LIB) $(CLI)

.PHONY: all clean cpptest asan

# A/B variant of the library with extra compile-time flags on the device learner:
#   make variant NAME=k1 VFLAGS=-DLGAP_SCAN_K=1   ->  variants/lib_k1.so (LAMBDAGAP_LIB=...)
VARIANT_DIR := variants
variant: $(CPP_OBJS) $(HIP_OBJS)
	@mkdir -p $(BUILD)/variant_$(NAME) $(VARIANT_DIR)
	$(HIPCC) $(HIPFLAGS) $(VFLAGS) -c src/device/device_learner.hip -o $(BUILD)/variant_$(NAME)/device_learner.hip.o
	$(CXX) -o $(VARIANT_DIR)/lib_$(NAME).so $(CPP_OBJS) $(filter-out $(BUILD)/device/device_learner.hip.o,$(HIP_OBJS)) \
	  $(BUILD)/variant_$(NAME)/device_learner.hip.o $(LDFLAGS)
.PHONY: variant
