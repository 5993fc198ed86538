# Build the gfx950 C-ABI library in-tree (travels to the GPU box with the snapshot).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
LIBDIR := preganplus_amd/_lib
LIB := $(LIBDIR)/libpreganplus.so
CSRC := preganplus_amd/csrc
SRCS := $(CSRC)/pgp_kernels.hip $(CSRC)/pgp_pack.cpp
HDRS := include/preganplus.h $(CSRC)/pgp_layout.hpp $(CSRC)/pgp_pack.hpp
CXXFLAGS := -O3 -std=c++17 -fPIC -Wall -Wno-unused-function

.PHONY: all clean resource-usage
all: $(LIB)

$(LIB): $(SRCS) $(HDRS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -shared -o $@ $(SRCS)

# per-kernel VGPR / spill / occupancy report
resource-usage:
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -c -o /tmp/pgp_k.o $(CSRC)/pgp_kernels.hip \
	  -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "Function Name|VGPRs:|AGPRs|Spill|Occupancy|LDS Size|SGPRs:" 

clean:
	rm -f $(LIB)
