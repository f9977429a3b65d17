// The ecs_ops world's user config and per-world init records (TEST
// WORKLOAD), shared by the world (ecs_ops.hip) and the host drivers that
// construct it through the reference-shaped executor classes
// (tests/drivers/), as a reference example's init.hpp is.
#pragma once

#include <cstdint>

namespace EcsOps {

struct Config {
    int32_t numAgents;
    int32_t growSpawns;     // 1: Spawn is a registerArchetype table (the executor grows it)
};
struct Init {
    int32_t worldIndex;
};

// exported singleton (slot 0); slot 1: the Spawn table's SpawnInfo column
struct Stats {
    int32_t tick;
    int32_t numPairs;
    int32_t numSpawns;
    int32_t sumHits;
    float sumD2;
    int32_t dynTicks;
};

}
