# Flags for building a world OUT OF TREE against this framework (reference:
# the user sources / flags of CompileConfig, include/madrona/mw_gpu.hpp:36-53,
# which the reference hands to NVRTC at run time).  Include this file from the
# world's Makefile and build a shared object:
#
#     MADRONA_MW := /path/to/gpu-ecs-madrona_amd
#     include $(MADRONA_MW)/world.mk
#     libmyworld.so: myworld.hip
#     	$(MW_HIPCC) $(MW_HIPFLAGS) -shared -o $@ $< $(MW_LDFLAGS)
#
# then mw_load_env("libmyworld.so") and mw_create("<WorldT>", ...).  The
# numerics flags are the framework's; the code object is v5
# like libmadrona_mw.so (one HIP runtime per process).
ROCM_PATH ?= /opt/rocm
MW_HIPCC ?= $(ROCM_PATH)/bin/hipcc
MW_ARCH ?= gfx950
MW_BUILD ?= build
MW_HIPFLAGS := -std=c++20 -O3 -fPIC --offload-arch=$(MW_ARCH) -mcode-object-version=5 \
               -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt \
               -I$(MADRONA_MW)/include
MW_LDFLAGS := -L$(MADRONA_MW)/$(MW_BUILD) -lmadrona_mw -Wl,-rpath,$(abspath $(MADRONA_MW)/$(MW_BUILD))

# The same world for the CPU back end (libmadrona_cpu.so): g++, no HIP.
#
#     libmyworld_cpu.so: myworld.hip
#     	$(MW_CPU_CXX) $(MW_CPU_CXXFLAGS) -shared -o $@ -x c++ $< $(MW_CPU_LDFLAGS)
MW_CPU_CXX ?= g++
MW_CPU_BUILD ?= build_cpu
MW_CPU_CXXFLAGS := -std=c++20 -O2 -fPIC -ffp-contract=off -fno-fast-math -pthread \
                   -DMW_CPU_BACKEND -I$(MADRONA_MW)/include
MW_CPU_LDFLAGS := -L$(MADRONA_MW)/$(MW_CPU_BUILD) -lmadrona_cpu \
                  -Wl,-rpath,$(abspath $(MADRONA_MW)/$(MW_CPU_BUILD))
