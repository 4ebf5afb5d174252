# Top-level build: the MI355X library, the host CLI binaries and the CPU oracle.
# hipcc cross-compiles gfx950 code objects without a GPU present.
ROCM ?= /opt/rocm
HIPCC ?= $(ROCM)/bin/hipcc
ARCH ?= gfx950
JOBS ?= 8

PKG := collaborative_filtering_amd
CSRC := $(PKG)/csrc
HOSTSRC := $(PKG)/host
BUILD := build

HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Iinclude -I$(CSRC) -Wall -Wno-unused-result
HOSTFLAGS := -O3 -std=c++17 -Iinclude -I$(HOSTSRC) -Wall

LIB := $(PKG)/libcf_mi355x.so
HIP_SRCS := $(wildcard $(CSRC)/*.hip)
HIP_OBJS := $(patsubst $(CSRC)/%.hip,$(BUILD)/%.o,$(HIP_SRCS))

HOST_BINS := $(patsubst $(HOSTSRC)/bin_%.cpp,bin/%,$(wildcard $(HOSTSRC)/bin_*.cpp))
HOST_COMMON := $(filter-out $(HOSTSRC)/bin_%.cpp,$(wildcard $(HOSTSRC)/*.cpp))
HOST_LIB := $(PKG)/libcf_host.so

all: $(LIB) $(HOST_LIB) $(HOST_BINS) oracle

$(BUILD)/%.o: $(CSRC)/%.hip $(wildcard $(CSRC)/*.h) $(wildcard $(CSRC)/*.hpp) include/cf_abi.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(HIP_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(HIP_OBJS)

$(HOST_LIB): $(HOST_COMMON) $(wildcard $(HOSTSRC)/*.hpp)
	g++ $(HOSTFLAGS) -fPIC -shared -o $@ $(HOST_COMMON) -lpthread

bin/%: $(HOSTSRC)/bin_%.cpp $(HOST_COMMON) $(wildcard $(HOSTSRC)/*.hpp) $(LIB)
	@mkdir -p bin
	$(HIPCC) $(HOSTFLAGS) -o $@ $< $(HOST_COMMON) -L$(PKG) -lcf_mi355x -Wl,-rpath,'$$ORIGIN/../$(PKG)' -lpthread

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf $(BUILD) $(LIB) $(HOST_LIB) bin/*
	$(MAKE) -C oracle clean

.PHONY: all oracle clean
