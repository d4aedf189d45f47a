# Build of the MI355X volumetric path tracer (gfx950 only).
#   make            -> cudavolumerenderer_amd/libcvr.so + cudavolumerenderer_amd/cvr (CLI)
#   make oracle     -> oracle/liboracle.so (test infrastructure)
# -ffp-contract=off: the kernels must perform exactly the IEEE operations of
# the source (see include/cvr_detmath.h); the correctly-rounded fp32 divide /
# sqrt flag is the hipcc default, spelled out because parity depends on it.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
PKG := cudavolumerenderer_amd
CSRC := $(PKG)/csrc
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off \
            -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude -I$(CSRC) -Wall -Wno-unused-function
OBJDIR := build/obj
SRCS_HIP := $(CSRC)/cvr_kernels.hip $(CSRC)/cvr_persistent.hip $(CSRC)/cvr_pool.hip $(CSRC)/cvr_wpool.hip $(CSRC)/cvr_wavefront.hip
SRCS_CPP := $(CSRC)/cvr_api.cpp $(CSRC)/cvr_scene.cpp $(CSRC)/cvr_vdb.cpp $(CSRC)/cvr_mhd.cpp $(CSRC)/cvr_xml.cpp
OBJS := $(patsubst $(CSRC)/%.hip,$(OBJDIR)/%.o,$(SRCS_HIP)) $(patsubst $(CSRC)/%.cpp,$(OBJDIR)/%.o,$(SRCS_CPP))
HDRS := include/cvr.h include/cvr_detmath.h $(wildcard $(CSRC)/*.h)

all: $(PKG)/libcvr.so $(PKG)/cvr build/launcher_order oracle

$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(PKG)/libcvr.so: $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -Wl,-soname,libcvr.so -lz

$(PKG)/cvr: $(CSRC)/cvr_main.cpp $(PKG)/libcvr.so include/cvr.h
	g++ -O2 -std=c++17 -Iinclude -o $@ $< -L$(PKG) -lcvr -Wl,-rpath,'$$ORIGIN'

# Host-only C++ test: libcvr driven through include/cvr_launcher.hpp in
# CudaVolPath's call order (tests/test_launcher_adapter.py).
build/launcher_order: tests/cpp/launcher_order.cpp include/cvr_launcher.hpp include/cvr.h $(PKG)/libcvr.so
	@mkdir -p build
	g++ -O2 -std=c++17 -Wall -D__HIP_PLATFORM_AMD__ -Iinclude -I/opt/rocm/include -o $@ $< \
	    -L$(PKG) -lcvr -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,'$$ORIGIN/../$(PKG)' -Wl,-rpath,/opt/rocm/lib

oracle:
	$(MAKE) -C oracle

resource-usage:
	for f in $(SRCS_HIP); do $(HIPCC) $(HIPFLAGS) -Rpass-analysis=kernel-resource-usage -c $$f -o /dev/null; done

clean:
	rm -rf build $(PKG)/libcvr.so $(PKG)/cvr
	$(MAKE) -C oracle clean

.PHONY: all oracle clean resource-usage

# Diagnostic build with in-kernel phase stamps (never the shipped library).
stamps: build/stamps/libcvr.so
build/stamps/libcvr.so: $(SRCS_HIP) $(SRCS_CPP) $(HDRS)
	@mkdir -p build/stamps
	$(HIPCC) $(HIPFLAGS) -DCVR_STAMPS=1 -shared -o $@ $(SRCS_HIP) $(patsubst %,-x hip %,$(SRCS_CPP)) -lz
.PHONY: stamps

# Experiment builds: make variant NAME=u2 DEFS="-DCVR_WPOOL_UNROLL=2" -> build/variants/u2/libcvr.so
variant: $(SRCS_HIP) $(SRCS_CPP) $(HDRS)
	@mkdir -p build/variants/$(NAME)
	$(HIPCC) $(HIPFLAGS) $(DEFS) -shared -o build/variants/$(NAME)/libcvr.so $(SRCS_HIP) $(patsubst %,-x hip %,$(SRCS_CPP)) -lz
.PHONY: variant
# The workgroup-shared event-list experiment (k_wpair), kept out of libcvr.so:
#   make variant-pair; CVR_LIB=build/variants/pair/libcvr.so pytest tests/test_wave_pair.py -m gpu
variant-pair:
	$(MAKE) variant NAME=pair DEFS="-DCVR_WPOOL_PAIR=1"
.PHONY: variant-pair
# Cell fetches as track-ready work (round-6 experiment, measured slower: profiles/round6/ab/fetch_list/)
variant-fetchlist:
	$(MAKE) variant NAME=fetchlist DEFS="-DCVR_WPOOL_FETCH_LIST=1"
.PHONY: variant-fetchlist
