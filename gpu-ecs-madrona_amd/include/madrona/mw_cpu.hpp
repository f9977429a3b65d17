// Reference include/madrona/mw_cpu.hpp:11-63 (ThreadPoolExecutor::Config,
// TaskGraphExecutor<ContextT, WorldT, ConfigT, InitT>(Config, ConfigT,
// InitT *)).  One TaskGraphExecutor template serves both back ends
// (mw_gpu.hpp): compiled by g++ against libmadrona_cpu.so it steps the worlds
// on pinned host threads, the reference's CPU executor.
#pragma once

#include <madrona/mw_gpu.hpp>
