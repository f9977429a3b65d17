// Environment entry points (reference src/mw/device/include/madrona/
// mw_gpu_entry.hpp:12-101, CompileConfig::entryName / userSources in
// include/madrona/mw_gpu.hpp:36-53).
//
// The reference NVRTC-compiles a world's sources when the executor is built
// and finds its entry kernels by name.  Here a world is compiled AHEAD OF
// TIME by hipcc for gfx950 -- inside this library or as a separate shared
// object built against include/madrona and linked to libmadrona_mw.so --
// and registers a factory under a name when its object is loaded:
//
//     MADRONA_BUILD_MWGPU_ENTRY(MyEngine, MyWorld, MyConfig, MyInit)
//
// registers "MyWorld" (the world type as spelled at the call site);
// MADRONA_BUILD_MWGPU_ENTRY_NAMED("name", ...) picks the name.  C ABI:
// mw_load_env("libmyworld.so") loads an out-of-tree world, then
// mw_create("MyWorld", cfg, &config, sizeof(config), inits, sizeof(MyInit)).
// ConfigT and InitT cross the boundary as bytes, so both must be trivially
// copyable (the reference copies them to the device the same way,
// src/mw/cuda_exec.cpp:1149-1157).
#pragma once

#include <madrona/mw_gpu.hpp>

#include <cstddef>
#include <cstring>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

namespace madrona {

using EnvFactory = Executor *(*)(const ExecConfig &cfg, const void *user_cfg,
                                 size_t user_cfg_bytes, const void *inits,
                                 size_t init_stride);

struct EnvRegistration {
    EnvRegistration(const char *name, EnvFactory factory);
};

EnvFactory findEnv(const char *name);

namespace mwGPU {

template <typename ContextT, typename WorldT, typename ConfigT, typename InitT>
Executor *makeEntryExecutor(const ExecConfig &cfg, const void *user_cfg, size_t user_cfg_bytes,
                            const void *inits, size_t init_stride)
{
    static_assert(std::is_trivially_copyable_v<ConfigT>, "ConfigT crosses the C ABI as bytes");
    static_assert(std::is_trivially_copyable_v<InitT>, "InitT crosses the C ABI as bytes");
    if (user_cfg_bytes != sizeof(ConfigT)) {
        throw std::runtime_error("mw_create: user config is " + std::to_string(user_cfg_bytes) +
                                 " bytes, the world's ConfigT is " + std::to_string(sizeof(ConfigT)));
    }
    if (init_stride < sizeof(InitT) || (!inits && cfg.numWorlds > 0)) {
        throw std::runtime_error("mw_create: init records smaller than the world's InitT");
    }
    ConfigT c;
    memcpy((void *)&c, user_cfg, sizeof(ConfigT));
    std::vector<InitT> v(cfg.numWorlds);
    for (int32_t w = 0; w < cfg.numWorlds; w++) {
        memcpy((void *)&v[w], (const char *)inits + (size_t)w * init_stride, sizeof(InitT));
    }
    return new TaskGraphExecutor<ContextT, WorldT, ConfigT, InitT>(cfg, c, v.data());
}

}
}

#define MW_ENTRY_CAT2(a, b) a##b
#define MW_ENTRY_CAT(a, b) MW_ENTRY_CAT2(a, b)

#define MADRONA_BUILD_MWGPU_ENTRY_NAMED(name, ContextT, WorldT, ConfigT, InitT)            \
    static ::madrona::EnvRegistration MW_ENTRY_CAT(mw_env_entry_, __LINE__)(             \
        name, &::madrona::mwGPU::makeEntryExecutor<ContextT, WorldT, ConfigT, InitT>);

#define MADRONA_BUILD_MWGPU_ENTRY(ContextT, WorldT, ConfigT, InitT) \
    MADRONA_BUILD_MWGPU_ENTRY_NAMED(#WorldT, ContextT, WorldT, ConfigT, InitT)
