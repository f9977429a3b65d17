// "ecs_ops": a small user world that drives every structural ECS operation
// from row-parallel nodes (TEST WORKLOAD, not product code).  Shared by the
// two compilations of the same world:
//   * tests/ext_env/ecs_ops.hip    -- this framework's API, built OUT OF TREE
//     into tests/ext_env/build/libecs_ops.so and loaded with mw_load_env;
//   * oracle/ref_ecs.cpp           -- the reference's own API, compiled with
//     the reference sources into oracle/_ref/libmadrona_ref_ecs.so.
// Plain arithmetic only (no framework types), so both compile it unchanged.
//
// Per world: kNumAgents agents (Pos, Vel, Counter).  A step:
//   clear pairs -> move (ParallelFor) -> pairs (ParallelFor: makeTemporary
//   per overlapping agent pair, e.id < o.id, the shape of the reference's
//   findOverlappingEntry, src/physics/broadphase.cpp:897-932; tmpAlloc
//   scratch) -> pair distance (4 lanes x 2 rows per invocation) -> hits
//   (ParallelFor) -> spawn (ParallelFor: makeEntityNow<Spawn>) -> despawn
//   (ParallelFor over spawns: destroyEntityNow(self), and makeEntityNow of a
//   child in the same node) -> stats (one-off node per world) -> tick
//   (dynamic-count node) -> reset tmp alloc.
#pragma once

#include <cstdint>

#if defined(__HIPCC__)
#define ECS_OPS_HD __host__ __device__
#else
#define ECS_OPS_HD
#endif

namespace ecs_ops {

inline constexpr int32_t kNumAgents = 40;
inline constexpr int32_t kMaxSpawns = 512;
inline constexpr int32_t kMaxPairs = 1024;
inline constexpr int32_t kMaxLivePerAgent = 3;     // at most 40 x (3 + 1 child) spawns alive
inline constexpr float kDeltaT = 0.25f;
inline constexpr float kBound = 6.f;
inline constexpr float kPairRadius2 = 9.f;

// Deterministic per-(world, agent) initial state.
ECS_OPS_HD inline uint32_t mix(uint32_t x)
{
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

ECS_OPS_HD inline float unit(uint32_t h)      // [-1, 1)
{
    return (float)(h >> 8) * (1.f / 8388608.f) - 1.f;
}

ECS_OPS_HD inline void initAgent(uint32_t world, uint32_t i, float pos[3], float vel[3])
{
    for (uint32_t k = 0; k < 3; k++) {
        pos[k] = kBound * unit(mix(world * 7919u + i * 131u + k));
        vel[k] = unit(mix(world * 104729u + i * 977u + k + 17u));
    }
}

// move: p += v dt, reflect at the walls
ECS_OPS_HD inline void moveAxis(float &p, float &v)
{
    p = p + v * kDeltaT;
    if (p > kBound || p < -kBound) v = -v;
}

ECS_OPS_HD inline bool pairOverlaps(const float a[3], const float b[3])
{
    const float dx = a[0] - b[0], dy = a[1] - b[1], dz = a[2] - b[2];
    return (dx * dx + dy * dy) + dz * dz < kPairRadius2;
}

ECS_OPS_HD inline bool spawns(int32_t hits, int32_t tick, int32_t entity_id)
{
    return ((hits + tick + entity_id) % 5) == 0;
}

ECS_OPS_HD inline bool despawns(int32_t tick, int32_t born)
{
    return tick - born >= 3;
}

ECS_OPS_HD inline bool spawnsChild(int32_t born, int32_t hits)
{
    return ((born + hits) & 1) == 0;
}

}
