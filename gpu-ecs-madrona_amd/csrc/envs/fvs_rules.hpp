// Workload definition of the restated fantasy_vs:
// the reference example's constants (examples/fantasy_vs/fvs.cpp:42-214)
// and the counter-based draws that replace its racy thread_local mt19937.
// Shared by the HIP environment, the oracle restatement and the reference
// harness so all three run the same game; contains no simulation logic.
#pragma once

#include <cstdint>

#if defined(__HIPCC__)
#define FVS_HD __host__ __device__
#else
#define FVS_HD
#endif

namespace fvs_rules {

inline constexpr float kDeltaT = 1.f / 60.f;        // fvs.cpp:45
inline constexpr float kMoveSpeed = 0.1f;           // fvs.cpp:46
inline constexpr float kManaRegenRate = 1.f;        // fvs.cpp:47
inline constexpr float kCastTime = 2.f;             // fvs.cpp:48
inline constexpr float kShootTime = 0.5f;           // fvs.cpp:49
inline constexpr float kMoveCutoff = 0.5f;          // fvs.cpp:124
inline constexpr float kCastCost = 20.f;            // fvs.cpp:168
inline constexpr float kBlastRadius = 2.f;          // fvs.cpp:179
inline constexpr int32_t kBlastDamage = 20;         // fvs.cpp:180 (float 20 into atomic_int)
inline constexpr int32_t kArrowDamage = 15;         // fvs.cpp:207
inline constexpr int32_t kDragonHP = 1000;          // fvs.cpp:86
inline constexpr int32_t kKnightHP = 100;           // fvs.cpp:87

enum : uint32_t {
    kDrawMoveProb = 0, kDrawMoveX, kDrawMoveY, kDrawMoveZ,
    kDrawTargetX, kDrawTargetY, kDrawTargetZ, kDrawDragon,
};

FVS_HD inline uint64_t mix64(uint64_t z)
{                                                   // splitmix64 finaliser
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Draw k of entity `entity` in world `world` at tick `tick`.
struct Draw {
    uint32_t world, entity, tick;

    FVS_HD uint64_t bits(uint32_t k) const
    {
        return mix64(((uint64_t)world << 32 | entity) ^ mix64(((uint64_t)tick << 8) | k));
    }
    FVS_HD float uniform(uint32_t k) const          // [0, 1), 24 random bits, exact
    {
        return (float)(uint32_t)(bits(k) >> 40) * (1.0f / 16777216.0f);
    }
    FVS_HD float uniform(uint32_t k, float lo, float hi) const
    {
        return lo + (hi - lo) * uniform(k);
    }
    FVS_HD uint32_t index(uint32_t k, uint32_t n) const
    {
        return (uint32_t)(bits(k) % n);
    }
};

FVS_HD inline float clampRef(float v, float lo, float hi)
{                                                   // std::clamp
    return v < lo ? lo : (hi < v ? hi : v);
}

}
