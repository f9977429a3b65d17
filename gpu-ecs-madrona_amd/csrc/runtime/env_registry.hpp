// Environments compiled into the library register a factory by name; the C
// ABI (capi.cpp) looks them up.  Replaces the reference's NVRTC compile of
// user sources named in CompileConfig (src/mw/cuda_exec.cpp:444-831).
#pragma once

#include <madrona/mw_gpu.hpp>

#include <cstddef>

namespace madrona {

using EnvFactory = Executor *(*)(const ExecConfig &cfg, const void *user_cfg,
                                 size_t user_cfg_bytes, const void *inits,
                                 size_t init_stride);

struct EnvRegistration {
    EnvRegistration(const char *name, EnvFactory factory);
};

EnvFactory findEnv(const char *name);

}
