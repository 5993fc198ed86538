# Build the gfx950 C-ABI library in-tree (travels to the GPU box with the snapshot).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
LIBDIR := preganplus_amd/_lib
LIB := $(LIBDIR)/libpreganplus.so
CSRC := preganplus_amd/csrc
KSRCS := $(CSRC)/pgp_tunef.hip $(CSRC)/pgp_dec.hip $(CSRC)/pgp_gat.hip $(CSRC)/pgp_encoder.hip $(CSRC)/pgp_decoder.hip $(CSRC)/pgp_gan.hip $(CSRC)/pgp_gansplit.hip $(CSRC)/pgp_train.hip $(CSRC)/pgp_tune.hip $(CSRC)/pgp_tune1.hip $(CSRC)/pgp_gan1.hip $(CSRC)/pgp_tunedp.hip $(CSRC)/pgp_gantrain.hip $(CSRC)/pgp_gobi.hip $(CSRC)/pgp_sim.hip $(CSRC)/pgp_fpe.hip $(CSRC)/pgp_fpetrain.hip $(CSRC)/pgp_decide.hip $(CSRC)/pgp_repack.hip $(CSRC)/pgp_online.hip $(CSRC)/pgp_capi.hip
SRCS := $(KSRCS) $(CSRC)/pgp_pack.cpp
OBJDIR := build/obj
OBJS := $(patsubst $(CSRC)/%,$(OBJDIR)/%.o,$(SRCS))
HDRS := include/preganplus.h $(CSRC)/pgp_tunef.hpp $(CSRC)/pgp_layout.hpp $(CSRC)/pgp_pack.hpp $(CSRC)/pgp_device.hpp $(CSRC)/pgp_train.hpp $(CSRC)/pgp_tune.hpp $(CSRC)/pgp_tunedp.hpp $(CSRC)/pgp_tunetargets.hpp $(CSRC)/pgp_gemm.hpp $(CSRC)/pgp_packcore.hpp $(CSRC)/pgp_repack.hpp
CXXFLAGS := -O3 -std=c++17 -fPIC -Wall -Wno-unused-function

.PHONY: all clean resource-usage variant asan
all: $(LIB)

$(OBJDIR)/%.o: $(CSRC)/% $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -c -o $@ $<

$(LIB): $(OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS)

# experiment builds: make variant NAME=w8 VFLAGS=-DPGP_GAN_WAVES=8
# -> preganplus_amd/_lib/var/libpreganplus_w8.so (select with PGP_LIB=...)
VOBJDIR := build/var_$(NAME)
variant:
	@mkdir -p $(VOBJDIR) $(LIBDIR)/var
	@for f in $(SRCS); do b=$$(basename $$f); \
	  $(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) $(VFLAGS) -c -o $(VOBJDIR)/$$b.o $$f & done; wait
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $(LIBDIR)/var/libpreganplus_$(NAME).so $(VOBJDIR)/*.o

# host-only sanitizer build of the weight packer (AddressSanitizer + UBSan):
# build/asan/pack_check packs every compiled host count and the FPE variant
asan: build/asan/pack_check
	./build/asan/pack_check
build/asan/pack_check: tools/pack_check.cpp $(CSRC)/pgp_pack.cpp $(CSRC)/pgp_packcore.hpp $(CSRC)/pgp_pack.hpp $(CSRC)/pgp_layout.hpp
	@mkdir -p build/asan
	g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all \
	  -o $@ tools/pack_check.cpp $(CSRC)/pgp_pack.cpp

# per-kernel VGPR / spill / occupancy report
resource-usage:
	python3 tools/resource_usage.py

clean:
	rm -f $(LIB) $(OBJS)
