// Environments register a factory by name (include/madrona/mw_gpu_entry.hpp);
// the C ABI (capi.cpp) looks them up.  Replaces the reference's NVRTC compile
// of user sources named in CompileConfig (src/mw/cuda_exec.cpp:444-831).
#pragma once

#include <madrona/mw_gpu_entry.hpp>
