// Host/device annotations for the MI355X-native framework.  Every header under
// include/madrona compiles with g++ (host-only users) and hipcc (gfx950).
#pragma once

#include <cstdint>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define MW_HD __host__ __device__
#define MW_DEV __device__
#define MW_INLINE __host__ __device__ inline __attribute__((always_inline))
#else
#define MW_HD
#define MW_DEV
#define MW_INLINE inline
#endif

#if defined(__HIP_DEVICE_COMPILE__)
#define MW_DEVICE_PASS 1
#else
#define MW_DEVICE_PASS 0
#endif

// 1 where node bodies execute: the device pass of hipcc and the CPU back
// end's g++ build (0 only in hipcc's host pass, where a device node's run()
// is compiled but never called).
#if defined(__HIP_DEVICE_COMPILE__) || !defined(__HIPCC__)
#define MW_EXEC_PASS 1
#else
#define MW_EXEC_PASS 0
#endif

namespace madrona {
using CountT = int64_t;

// State slabs are HBM allocations, but pointers read out of a StateView are
// generic to the compiler, which then emits flat loads that wait on both
// memory counters (every access serialised).  rowRef indexes a slab in the
// global address space and hands back an ordinary reference, so the backend
// emits global loads / stores with partial waits.
template <typename T>
MW_INLINE T &rowRef(T *base, int64_t r)
{
#if defined(__HIP_DEVICE_COMPILE__)
    using GT = __attribute__((address_space(1))) T;
    GT *g = (GT *)base;
    return *(T *)&g[r];
#else
    return base[r];
#endif
}
}
