// Kernel launch checks of the gfx950 back end.
//
// The reference aborts on every CUDA error (include/madrona/cuda_utils.hpp:
// 46-54, ERR_CUDA / REQ_CUDA).  Here every failure becomes a
// std::runtime_error that names the kernel; the C ABI turns it into a status
// code plus mw_last_error().  Two kinds of failure are caught:
//   * a launch shape the device cannot run: more LDS (static + dynamic) than
//     a workgroup may hold, more lanes than the kernel's launch bounds, or
//     zero resident blocks per CU.  A graph captured with such a launch
//     replays without running the kernel and without an error, so the shape
//     is checked on the host before every launch (cached per shape);
//   * an error the runtime reports for the launch (hipGetLastError right
//     after it).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstddef>
#include <cstdint>

namespace madrona::hipx {

[[noreturn]] void hipFail(hipError_t err, const char *expr, const char *file, int line);

// LDS one workgroup may hold on the current device (163840 B on gfx950).
size_t maxLDSPerBlock();

// Blocks of `threads` lanes with `dyn_lds` bytes of dynamic LDS that one CU
// holds at once (>= 1), or throws naming `name` and the byte counts.
int32_t residentBlocks(const void *fn, const char *name, int32_t threads, size_t dyn_lds);

// The same test without throwing: 0 when the shape cannot launch.
int32_t residentBlocksNoThrow(const void *fn, int32_t threads, size_t dyn_lds);

// hipGetLastError after a launch; throws naming the kernel.
void checkLaunched(const char *name);

// Live node timing (Executor::setTimedNode / timeNode).  While a
// TimedLaunch is installed on this thread, MW_LAUNCH / launchKernel bind an
// event pair to every kernel they launch (hipExtLaunchKernelGGL: the pair
// records that kernel's start and end): the first kernel takes (start,
// stop), each further kernel a fresh pair from next(ctx).  The timed time of
// a node (or walk run) is the SUM of its kernels' durations -- what a
// rocprofv3 kernel trace sums -- not the span from the first kernel's start
// to the last one's end, which for eagerly launched multi-kernel units
// includes the dispatch gaps between them (a walk run's walk and resume
// kernels: ~70 us of gap on the MI355X box against ~100 us of kernels).
struct TimedLaunch {
    hipEvent_t start = nullptr;
    hipEvent_t stop = nullptr;
    void (*next)(void *ctx, hipEvent_t *start, hipEvent_t *stop) = nullptr;
    void *ctx = nullptr;
    int32_t kernels = 0;          // kernels bound so far

    // the pair of the next kernel
    void bind(hipEvent_t *a, hipEvent_t *b)
    {
        if (kernels++ == 0 || !next) {
            *a = kernels == 1 ? start : nullptr;
            *b = stop;
        } else {
            next(ctx, a, b);
        }
    }
};
inline thread_local TimedLaunch *tlTimed = nullptr;

// hipLaunchKernel for the type-erased launchers (row / serial / node-function
// kernels), with the TimedLaunch binding of MW_LAUNCH.
inline hipError_t launchKernel(const void *fn, dim3 grid, dim3 block, void **args, size_t lds,
                               hipStream_t stream)
{
    if (TimedLaunch *t = tlTimed) {
        hipEvent_t a, b;
        t->bind(&a, &b);
        return hipExtLaunchKernel(fn, grid, block, args, lds, stream, a, b, 0);
    }
    return hipLaunchKernel(fn, grid, block, args, lds, stream);
}

}

#define MW_HIP_CHECK(expr)                                                          \
    do {                                                                            \
        const hipError_t err__ = (expr);                                            \
        if (err__ != hipSuccess) ::madrona::hipx::hipFail(err__, #expr, __FILE__, __LINE__); \
    } while (0)

// hipLaunchKernelGGL with the shape check before and the error check after.
#define MW_LAUNCH(kernel, grid, block, lds, stream, ...)                               \
    do {                                                                               \
        const dim3 blk__ = (block);                                                     \
        ::madrona::hipx::residentBlocks((const void *)&(kernel), #kernel,              \
                                        (int32_t)(blk__.x * blk__.y * blk__.z), (lds)); \
        if (::madrona::hipx::TimedLaunch *tl__ = ::madrona::hipx::tlTimed) {             \
            hipEvent_t start__, stop__;                                                 \
            tl__->bind(&start__, &stop__);                                              \
            hipExtLaunchKernelGGL(kernel, grid, blk__, lds, stream, start__, stop__,    \
                                  0u, __VA_ARGS__);                                     \
        } else {                                                                        \
            hipLaunchKernelGGL(kernel, grid, blk__, lds, stream, __VA_ARGS__);         \
        }                                                                               \
        ::madrona::hipx::checkLaunched(#kernel);                                       \
    } while (0)
