# Builds libsdgpu.so (gfx950 HIP kernels + C ABI) in-tree, and the CPU oracle.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CSRC := spacedrive_amd/csrc
BUILD := build/obj
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-function
HIPSRC := $(CSRC)/b3_batch.hip $(CSRC)/b3_tree.hip $(CSRC)/dedup.hip $(CSRC)/index.hip $(CSRC)/consumers.hip $(CSRC)/synth.hip $(CSRC)/link.hip
HOSTSRC := $(CSRC)/sdgpu.cpp $(CSRC)/shard.cpp
OBJS := $(patsubst $(CSRC)/%.hip,$(BUILD)/%.o,$(HIPSRC)) $(BUILD)/sdgpu.o $(BUILD)/shard.o
HDRS := $(wildcard $(CSRC)/*.hpp) include/sdgpu.h
LIB := spacedrive_amd/libsdgpu.so

all: $(LIB) oracle

$(BUILD)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -L/opt/rocm/lib -lrccl -lpthread

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -rf $(BUILD) $(LIB)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean
