// "cross_rows": a test world (TEST WORKLOAD, not product code) whose
// ParallelForNode bodies depend on the reference's serial row walk beyond
// structural ops (include/madrona/taskgraph.inl:63-71, state.inl:387-396):
//   * flow:  a row reads and writes ANOTHER row's plain (non-atomic) fields
//            through ctx.get<Cell>(other) -- rows after it see the result;
//   * scan:  state carried from row to row through a singleton (a running
//            hash each row reads, then overwrites);
//   * churn: makeEntityNow / destroyEntityNow of Sparks from the Cell walk
//            (the new entity's ID is stored in the cell), so entity IDs come
//            from the ID store's free list in walk order;
//   * split: from the Spark walk, makeEntityNow of Cells whose ID goes into
//            the source cell.  (Cells are not made from the Cell walk: growing
//            the walked table reallocates it under the reference's walk,
//            src/common/table.cpp:44-60, undefined behaviour.)
// Shared by the two compilations of the same world:
//   * tests/ext_env/cross_rows.hip -- this framework, built out of tree;
//   * oracle/ref_cross.cpp         -- the reference's own ECS.
// Plain arithmetic only (no framework types), so both compile it unchanged.
#pragma once

#include <cstdint>

#if defined(__HIPCC__)
#define CROSS_ROWS_HD __host__ __device__
#else
#define CROSS_ROWS_HD
#endif

namespace cross_rows {

inline constexpr int32_t kNumCells = 48;
inline constexpr int32_t kMaxCells = 192;
inline constexpr int32_t kMaxSparks = 160;
inline constexpr int32_t kSplitValue = 600;

CROSS_ROWS_HD inline uint32_t mix(uint32_t x)
{
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

CROSS_ROWS_HD inline void initCell(uint32_t world, uint32_t i, int32_t &value, float &heat)
{
    value = (int32_t)(mix(world * 7919u + i * 131u) % 400u);
    heat = (float)(mix(world * 104729u + i * 977u + 5u) >> 8) * (1.f / 16777216.f);
}

// initial link of cell i among the n initial cells (earlier and later rows)
CROSS_ROWS_HD inline int32_t linkTarget(int32_t i, int32_t n)
{
    return (i * 7 + 3) % n;
}

// a third of the cell's value moves to the cell it links to, heat blends
CROSS_ROWS_HD inline void flow(int32_t &v, float &h, int32_t &ov, float &oh)
{
    const int32_t moved = v / 3;
    ov += moved;
    v -= moved;
    oh = oh * 0.5f + h * 0.25f;
}

CROSS_ROWS_HD inline uint32_t scanStep(uint32_t running, int32_t value)
{
    return running * 31u + (uint32_t)value;
}

CROSS_ROWS_HD inline int32_t inject(uint32_t prefix)
{
    return (int32_t)(prefix % 13u);
}

CROSS_ROWS_HD inline bool dropsSpark(int32_t value, int32_t tick)
{
    return ((value + tick) % 3) == 0;
}

CROSS_ROWS_HD inline bool makesSpark(int32_t value)
{
    return (value % 5) == 0;
}

}
