// Device tracing (reference src/mw/device/include/madrona/mw_gpu/tracing.hpp:
// 14-128): 40-byte DeviceLog records, the format
// scripts/parse_device_tracing.py reads.
//
// MI355X design.  The reference logs from inside its megakernel (node start /
// finish by the node's leader, block start / wait around each block's work).
// Here a step is a sequence of kernels, so:
//   * the executor brackets every node with two one-lane marker kernels
//     (nodeStart / nodeFinish) and the step with a calibration record (step
//     start, logIndex 0) and a blockExit record (step end) -- stream order
//     puts every block of the node between its markers;
//   * every kernel opens with MW_TRACE_BLOCK(disc): its first thread logs
//     blockStart on entry and blockWait on exit.  `numInvocations` of a block
//     record identifies the launch (source line of the kernel, plus `disc`
//     for kernels a node launches more than once), `nodeID` the node, so the
//     parser's per-SM key (numInvocations, nodeID, warp) is unique per step.
// Timestamps are the 100 MHz constant device clock (s_memrealtime) scaled to
// ns, the unit the reference's %globaltimer has.  The trace pointer is per
// process: one traced executor at a time.
#pragma once

#include <madrona/hd.hpp>

#include <cstdint>

namespace madrona::mwGPU {

enum class DeviceEvent : uint32_t {
    calibration = 0,
    nodeStart = 1,
    nodeFinish = 2,
    blockStart = 3,
    blockWait = 4,
    blockExit = 5,
};

struct DeviceLog {
    DeviceEvent event;
    uint32_t funcID;
    uint32_t numInvocations;
    uint32_t nodeID;
    uint32_t warpID;
    uint32_t blockID;
    uint32_t smID;
    uint32_t logIndex;        // index within the step (0 = its calibration record)
    uint64_t cycleCount;      // ns
};
static_assert(sizeof(DeviceLog) == 40);

// Device-resident trace state (one per traced executor).
struct TraceDev {
    uint32_t next;            // records written so far (all steps)
    uint32_t stepBase;        // index of the current step's calibration record
    uint32_t curNode;         // node being run (set by its nodeStart marker)
    uint32_t dropped;         // records lost to a full buffer
    uint32_t capacity;
    uint32_t nsPerTick;       // device clock period in ns
    DeviceLog *logs;
};

#if defined(__HIPCC__)

// One copy per translation unit: kernels are compiled without relocatable
// device code, so each TU's code object holds its own pointer; the executor
// sets all of them through the setters the TUs register at load time.
static __device__ TraceDev *g_mwTrace = nullptr;

using TraceSetter = void (*)(TraceDev *);
void registerTraceSetter(TraceSetter fn);       // csrc/runtime/executor.hip

namespace {
struct TraceTURegistrar {
    static void set(TraceDev *p)
    {
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_mwTrace), &p, sizeof(p));
    }
    TraceTURegistrar() { registerTraceSetter(&set); }
};
static TraceTURegistrar g_mwTraceRegistrar;
}

__device__ inline uint32_t traceSMID()
{
    // CU id (bits 3:0) and shader engine (bits 5:4) of HW_ID, XCC id on top:
    // a dense id space of 8 XCCs x 4 SEs x 16 CUs.
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t cu = __builtin_amdgcn_s_getreg(
        GETREG_IMMED(HW_ID_CU_ID_SIZE - 1, HW_ID_CU_ID_OFFSET, HW_ID)) & 0xf;
    const uint32_t se = __builtin_amdgcn_s_getreg(
        GETREG_IMMED(HW_ID_SE_ID_SIZE - 1, HW_ID_SE_ID_OFFSET, HW_ID)) & 0x3;
    const uint32_t xcc = __builtin_amdgcn_s_getreg(
        GETREG_IMMED(XCC_ID_XCC_ID_SIZE - 1, XCC_ID_XCC_ID_OFFSET, XCC_ID)) & 0x7;
    return (xcc * 4 + se) * 16 + cu;
#else
    return 0;
#endif
}

__device__ inline void traceLog(TraceDev *t, DeviceEvent ev, uint32_t func, uint32_t inv,
                                uint32_t node, uint32_t block)
{
    const uint32_t i = atomicAdd(&t->next, 1u);
    const uint64_t ts = (uint64_t)wall_clock64() * t->nsPerTick;
    if (i >= t->capacity) {
        atomicAdd(&t->dropped, 1u);
        return;
    }
    DeviceLog &l = t->logs[i];
    l.event = ev;
    l.funcID = func;
    l.numInvocations = inv;
    l.nodeID = node;
    l.warpID = 0;
    l.blockID = block;
    l.smID = traceSMID();
    l.logIndex = i - __hip_atomic_load(&t->stepBase, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    l.cycleCount = ts;
}

// Only the block's first wave touches the trace pointer, and it is re-read
// on exit instead of being kept live across the kernel (no register cost).
struct TraceBlockScope {
    uint32_t inv;
    __device__ inline explicit TraceBlockScope(uint32_t launch_id) : inv(launch_id)
    {
        if (threadIdx.x == 0 && threadIdx.y == 0) {
            TraceDev *t = g_mwTrace;
            if (__builtin_expect(t != nullptr, 0)) {
                traceLog(t, DeviceEvent::blockStart, 0, inv, t->curNode,
                         blockIdx.x + blockIdx.y * gridDim.x);
            }
        }
    }
    __device__ inline ~TraceBlockScope()
    {
        if (threadIdx.x == 0 && threadIdx.y == 0) {
            TraceDev *t = g_mwTrace;
            if (__builtin_expect(t != nullptr, 0)) {
                traceLog(t, DeviceEvent::blockWait, 0, inv, t->curNode,
                         blockIdx.x + blockIdx.y * gridDim.x);
            }
        }
    }
};

// Block records are compiled in only by the tracing build (-DMW_TRACING,
// build_trace/libmadrona_mw.so), as the reference compiles them only with
// MADRONA_TRACING: even unused, the per-block check costs the default build
// ~1.4 % of the collisions step (measured A/B).  Node / step records need no
// kernel code and work in every build.
#if defined(MW_TRACING)
#define MW_TRACE_BLOCK(disc) \
    ::madrona::mwGPU::TraceBlockScope mw_trace_scope__((uint32_t)(__LINE__ * 256 + (disc)))
constexpr bool kTraceBlockRecords = true;
#else
#define MW_TRACE_BLOCK(disc) ((void)0)
constexpr bool kTraceBlockRecords = false;
#endif

#endif

}
