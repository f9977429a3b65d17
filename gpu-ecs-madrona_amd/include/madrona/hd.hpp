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

namespace madrona {
using CountT = int64_t;
}
