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

# The world walk's generated dispatch (MADRONA_MW_WORLD_WALK=1; the
# reference's generated megakernel dispatch, src/mw/cuda_exec.cpp:560-700):
# list the world's walk functions from its device IR, then compile the
# generated wrapper (it includes the source) instead of the source.  A world
# built directly from its source still walks, through device function
# pointers (slower: the indirect-call register budget).
#
#     build/myworld.ll: myworld.hip
#     	$(MW_HIPCC) $(MW_HIPFLAGS) $(MW_WALK_IR_FLAGS) $< -o $@
#     build/myworld_walk.hip: build/myworld.ll
#     	$(MW_WALK_GEN) myworld.hip $< $@
#     libmyworld.so: build/myworld_walk.hip
#     	$(MW_HIPCC) $(MW_HIPFLAGS) -shared -o $@ $< $(MW_LDFLAGS)
MW_WALK_IR_FLAGS := --cuda-device-only -S -emit-llvm -Xclang -disable-llvm-passes
MW_WALK_GEN := python3 $(MADRONA_MW)/tools/gen_walk_dispatch.py

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
