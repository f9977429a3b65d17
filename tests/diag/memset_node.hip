// Diagnosis harness (TEST INFRASTRUCTURE, not product code): does a
// hipMemsetAsync captured into a graph re-zero its target on every replay in
// the conditions the executor replays its step graph under (non-blocking
// stream, thread-local capture, host hipMemcpy calls between replays)?
//
// Round 2 saw two failures that both relied on a captured memset node to
// reset counters: the tmpAlloc offsets (executor.hip resetTmpAllocKernel
// note) and the reverted findOverlaps + first-substep fusion whose narrowphase
// work-list counters were reset by a memset node and which faulted with an
// illegal address.  This library replays the pattern in isolation:
//   graph = [reset counters] -> bump(+1) -> bump(+2 + (i & 3))
// and checks after every replay that counter i == 3 + (i & 3).
// reset: 0 = kernel (the executor's way), 1 = hipMemsetAsync node,
//        2 = hipMemsetD32Async node.
// Loaded with ctypes after torch, so it runs on the same HIP runtime as the
// framework's library.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <vector>

namespace {

__global__ void bumpKernel(uint32_t *c, int32_t n, uint32_t k, int32_t spread)
{
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) atomicAdd(&c[i], k + (spread ? (uint32_t)(i & 3) : 0u));
}

__global__ void resetKernel(uint32_t *c, int32_t n)
{
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) c[i] = 0;
}

#define DIAG_CHECK(x)                                                                          \
    do {                                                                                       \
        hipError_t e__ = (x);                                                                  \
        if (e__ != hipSuccess) {                                                               \
            std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e__));               \
            return -1;                                                                         \
        }                                                                                      \
    } while (0)

}

// The graph as the executor builds it: captured inside a helper whose
// stack frame is gone when the graph replays (the executor captures in
// captureSegments and replays from runAsync).
__attribute__((noinline)) static hipError_t captureInHelper(int32_t reset, uint32_t *c, int32_t n,
                                                            hipStream_t s, hipGraphExec_t *ge,
                                                            hipGraph_t *g)
{
    const dim3 grid((unsigned)((n + 255) / 256)), block(256);
    hipError_t e = hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    if (e != hipSuccess) return e;
    volatile uint32_t value = 0;               // a stack local, as a caller's would be
    if (reset == 0) {
        hipLaunchKernelGGL(resetKernel, grid, block, 0, s, c, n);
    } else if (reset == 1) {
        (void)hipMemsetAsync(c, (int)value, sizeof(uint32_t) * (size_t)n, s);
    } else {
        (void)hipMemsetD32Async((hipDeviceptr_t)c, (int)value, (size_t)n, s);
    }
    hipLaunchKernelGGL(bumpKernel, grid, block, 0, s, c, n, 1u, 0);
    hipLaunchKernelGGL(bumpKernel, grid, block, 0, s, c, n, 2u, 1);
    e = hipStreamEndCapture(s, g);
    if (e != hipSuccess) return e;
    return hipGraphInstantiate(ge, *g, nullptr, nullptr, 0);
}

// Overwrites a large stretch of the host stack with the pattern the fault
// log showed in every counter (0x7657500C), then returns.
__attribute__((noinline)) static uint32_t scribbleStack(uint32_t pattern)
{
    volatile uint32_t junk[16384];
    for (int32_t i = 0; i < 16384; i++) junk[i] = pattern;
    return junk[pattern & 1023];
}

// Allocates and fills many small host blocks with the pattern, then frees
// them: a runtime that kept a pointer to a freed parameter block of the
// captured node would read the pattern back at replay (the fault log's
// 0x7657500C looks like the low half of a host heap pointer).
__attribute__((noinline)) static void scribbleHeap(uint32_t pattern)
{
    std::vector<uint32_t *> blocks;
    for (int32_t k = 0; k < 4096; k++) {
        const size_t words = 4 + (size_t)(k % 128);
        uint32_t *b = (uint32_t *)malloc(words * 4);
        for (size_t i = 0; i < words; i++) b[i] = pattern;
        blocks.push_back(b);
    }
    for (uint32_t *b : blocks) free(b);
}

// Returns the number of replays after which at least one counter was wrong
// (out[0]), the first such replay (out[1], -1 if none) and the number of
// wrong counters summed over replays (out[2]); -1 on a HIP error.
extern "C" int memset_node_run(int32_t reset, int32_t n, int32_t replays, int32_t host_copies,
                               int64_t *out)
{
    uint32_t *c = nullptr;
    uint8_t *scratch = nullptr;
    const size_t scratch_bytes = 1 << 20;
    DIAG_CHECK(hipMalloc(&c, sizeof(uint32_t) * (size_t)n));
    DIAG_CHECK(hipMalloc(&scratch, scratch_bytes));
    DIAG_CHECK(hipMemset(c, 0xAB, sizeof(uint32_t) * (size_t)n));
    hipStream_t s;
    DIAG_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));

    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    DIAG_CHECK(captureInHelper(reset, c, n, s, &ge, &g));

    std::vector<uint32_t> host(n);
    std::vector<uint8_t> hs(scratch_bytes, 1);
    int64_t bad_replays = 0, first_bad = -1, bad_total = 0;
    for (int32_t r = 0; r < replays; r++) {
        DIAG_CHECK(hipGraphLaunch(ge, s));
        DIAG_CHECK(hipStreamSynchronize(s));
        if (host_copies >= 2) (void)scribbleStack(0x7657500Cu + (uint32_t)r);
        if (host_copies >= 4) scribbleHeap(0x7657500Cu);
        if (host_copies >= 3) {
            // the executor's sequence between replays: a D2H read-back of a
            // column (mw_read_column: hipMemcpy on the null stream) and a
            // fresh device allocation (hipMalloc, as a late export buffer)
            void *extra = nullptr;
            DIAG_CHECK(hipMalloc(&extra, 4096));
            DIAG_CHECK(hipMemcpy(hs.data(), c, sizeof(uint32_t) * (size_t)n, hipMemcpyDeviceToHost));
            DIAG_CHECK(hipFree(extra));
        }
        if (host_copies) {
            // what tests and exports do between steps: synchronous copies on
            // the null stream
            DIAG_CHECK(hipMemcpy(scratch, hs.data(), scratch_bytes, hipMemcpyHostToDevice));
            DIAG_CHECK(hipMemcpy(hs.data(), scratch, scratch_bytes, hipMemcpyDeviceToHost));
        }
        DIAG_CHECK(hipMemcpy(host.data(), c, sizeof(uint32_t) * (size_t)n, hipMemcpyDeviceToHost));
        int64_t bad = 0;
        for (int32_t i = 0; i < n; i++) bad += host[i] != 3u + (uint32_t)(i & 3);
        if (bad) {
            bad_replays++;
            bad_total += bad;
            if (first_bad < 0) first_bad = r;
        }
    }
    DIAG_CHECK(hipGraphExecDestroy(ge));
    DIAG_CHECK(hipGraphDestroy(g));
    DIAG_CHECK(hipStreamDestroy(s));
    DIAG_CHECK(hipFree(scratch));
    DIAG_CHECK(hipFree(c));
    out[0] = bad_replays;
    out[1] = first_bad;
    out[2] = bad_total;
    return 0;
}
