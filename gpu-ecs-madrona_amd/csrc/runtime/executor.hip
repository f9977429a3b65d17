// Executor, TaskGraph build/launch and generic launch helpers (gfx950).
//
// Reference: src/core/taskgraph.cpp:18-122 (Builder/build/run),
// src/mw/cuda_exec.cpp:1519-1815 (run graph, getExported, export kernels).
#include <madrona/mw_gpu.hpp>
#include <madrona/tracing.hpp>
#include <madrona/commit.hpp>
#include <madrona/launch_config.hpp>

#include <hip/hip_runtime.h>

#include "hip_launch.hpp"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

namespace madrona {


// TaskGraph::Builder / build / launch: csrc/runtime/taskgraph.cpp (shared
// with the CPU back end).

// ---------------------------------------------------------------------------
// Generic launch helpers
// ---------------------------------------------------------------------------
namespace detail {

void launchWorldKernel(const void *kernel, LaunchCtx &lc)
{
    StateView *st = lc.devState;
    void *args[] = { &st };
    const uint32_t blocks = lc.capGrid((uint32_t)((lc.numWorlds + 63) / 64));
    if (blocks == 0) return;
    hipx::residentBlocks(kernel, "perWorldKernel", 64, 0);
    MW_HIP_CHECK(hipx::launchKernel(kernel, dim3(blocks), dim3(64), args, 0,
                                 (hipStream_t)lc.stream));
}

// Row-parallel kernels: numWorlds x ceil(capacity / items) invocations of
// `threads` lanes each, 256-lane blocks (grid-stride past capGrid).
void launchRowKernel(const void *kernel, LaunchCtx &lc, int32_t archetype, int32_t query_arch,
                     int32_t threads, int32_t items, const void *cols, size_t, bool world_waves)
{
    const int32_t cap = lc.view->arch[archetype].capacity;
    // world_waves: one wave per world (parallelForWorldKernel)
    const int64_t lanes = world_waves ? (cap > 0 ? (int64_t)lc.numWorlds * 64 : 0)
                                      : (int64_t)lc.numWorlds * ((cap + items - 1) / items) * threads;
    if (lanes == 0) return;
    dim3 block(256);
    const int64_t blocks = std::min<int64_t>((lanes + 255) / 256, 0x7fffffff);
    uint32_t g = lc.capGrid((uint32_t)blocks);
    const int32_t resident = hipx::residentBlocks(kernel, "parallelForKernel", 256, 0);
    // A capped grid strides over the rows in several passes; it is kept to
    // blocks that are all resident at once, so a row-parallel makeEntityNow
    // waiting for the earlier waves of its world (Context::lockedAcquire)
    // never waits on a block that cannot start.
    if ((int64_t)g < blocks && lc.numCUs > 0)
        g = (uint32_t)std::min<int64_t>(g, (int64_t)resident * lc.numCUs);
    dim3 grid(g);
    StateView *st = lc.devState;
    int32_t arch = archetype, qa = query_arch;
    void *kargs[] = { &st, &arch, &qa, const_cast<void *>(cols) };
    MW_HIP_CHECK(hipx::launchKernel(kernel, grid, block, kargs, 0, (hipStream_t)lc.stream));
}

// World-serial row nodes: numWorlds invocations of `threads` lanes.
void launchSerialKernel(const void *kernel, LaunchCtx &lc, int32_t threads, const void *query)
{
    const int64_t lanes = (int64_t)lc.numWorlds * threads;
    const uint32_t blocks = lc.capGrid((uint32_t)std::min<int64_t>((lanes + 255) / 256, 0x7fffffff));
    if (blocks == 0) return;
    StateView *st = lc.devState;
    void *kargs[] = { &st, const_cast<void *>(query) };
    hipx::residentBlocks(kernel, "serialForKernel", 256, 0);
    MW_HIP_CHECK(hipx::launchKernel(kernel, dim3(blocks), dim3(256), kargs, 0, (hipStream_t)lc.stream));
}

// addNodeFn nodes: a fixed count per world sizes the grid; a dynamic count
// is only known on the device, so its grid is persistent (grid-stride).
void launchNodeFnKernel(const void *kernel, LaunchCtx &lc, void *node_dev, uint32_t fixed_count,
                        uint32_t threads)
{
    uint32_t blocks;
    if (fixed_count == 0xFFFF'FFFFu) {
        blocks = 1;
    } else if (fixed_count > 0) {
        const int64_t lanes = (int64_t)lc.numWorlds * fixed_count * threads;
        blocks = lc.capGrid((uint32_t)std::min<int64_t>((lanes + 255) / 256, 0x7fffffff));
    } else {
        blocks = lc.persistentGrid((uint32_t)std::max(1, lc.numCUs) * 4);
    }
    if (blocks == 0) return;
    void *kargs[] = { &node_dev, &fixed_count, &threads };
    hipx::residentBlocks(kernel, "nodeFnKernel", 256, 0);
    MW_HIP_CHECK(hipx::launchKernel(kernel, dim3(blocks), dim3(256), kargs, 0,
                                 (hipStream_t)lc.stream));
}

}

// ---------------------------------------------------------------------------
// Ordered structural commit of a row-parallel node (madrona/commit.hpp) as
// its own kernel: one-wave blocks strided over the worlds, each world's
// working set in LDS.  Nodes whose every query table is walked one wave per
// world commit inside their row kernel instead (taskgraph.hpp).
// ---------------------------------------------------------------------------
struct CommitArgs {
    StateView *st;
    char *scratch;                 // [gridDim.x][scratchPerBlock]
    uint64_t scratchPerBlock;
    detail::CommitShape shape;
    int32_t grid;                  // blocks (all resident): worlds are strided over them
};

static size_t commitSharedBytes(const CommitArgs &A)
{
    return detail::commitWorkingBytes(A.shape);
}

// One wave per block: a world's commit is a chain of small steps (sorts of a
// few keys, a replay, a few row moves), each ending in a barrier, so a
// single-wave block's barriers cost nearly nothing and more worlds commit at
// once (256-lane blocks: 44 us per fantasy_vs destroy commit).
constexpr int32_t kCommitThreads = 64;

__global__ void __launch_bounds__(kCommitThreads) structuralCommitKernel(CommitArgs A)
{
    MW_TRACE_BLOCK(0);
    extern __shared__ __align__(16) char commit_lds[];
    StateView &st = *A.st;
    char *scratch = A.scratch + (size_t)blockIdx.x * A.scratchPerBlock;
    const int32_t tid = threadIdx.x;

    // the next node's waves mark themselves done with a new epoch
    // (row-ordered makeEntityNow); the next kernel sees the store
    if (st.makeEpoch && blockIdx.x == 0 && tid == 0) st.makeEpoch[0] = st.makeEpoch[0] + 1;
    // Most nodes mutate nothing: a block's lanes check 64 of its worlds
    // (strided over the resident grid) in one round of loads, then the block
    // walks the ones with work.  (A block per 256-world chunk walked its
    // chunk's worlds one after another: 64 busy blocks for 16384 worlds,
    // 0.2 ms per fantasy_vs destroy commit.)
    static_assert(kCommitThreads == 64, "one wave per block: the ballot covers the block");
    for (int64_t base = blockIdx.x; base < st.numWorlds; base += (int64_t)gridDim.x * 64) {
        const int64_t mine = base + (int64_t)tid * gridDim.x;
        const bool has_work = mine < st.numWorlds && (st.appendDirty[mine] != 0 || st.deferCount[mine] != 0);
        for (uint64_t todo = __ballot(has_work); todo != 0; todo &= todo - 1) {
            const int32_t w = (int32_t)(base + (int64_t)__builtin_ctzll(todo) * gridDim.x);
            detail::commitWorld(st, A.shape, commit_lds, scratch, w);
        }
    }
}

// A graph with no committable table still advances the epoch after every
// row node, so the next node's row-ordered makes wait on fresh marks.
__global__ void __launch_bounds__(64) bumpMakeEpochKernel(StateView *st)
{
    if (threadIdx.x == 0 && st->makeEpoch) st->makeEpoch[0] = st->makeEpoch[0] + 1;
}

namespace detail {

void readDeviceWord(const void *kernel, void *host_out)
{
    void *dev = nullptr;
    MW_HIP_CHECK(hipMalloc(&dev, 16));
    void *args[] = { &dev };
    const hipError_t e = hipLaunchKernel(kernel, dim3(1), dim3(1), args, 0, nullptr);
    if (e != hipSuccess) {
        (void)hipFree(dev);
        hipx::hipFail(e, "readDeviceWord launch", __FILE__, __LINE__);
    }
    MW_HIP_CHECK(hipMemcpy(host_out, dev, 8, hipMemcpyDeviceToHost));
    MW_HIP_CHECK(hipFree(dev));
}

void launchStructuralCommit(LaunchCtx &lc)
{
    const CommitArgs *A = lc.exec ? (const CommitArgs *)lc.exec->commitArgs() : nullptr;
    if (!A) return;
    if (A->shape.capMax <= 0) {
        MW_LAUNCH(bumpMakeEpochKernel, dim3(1), dim3(64), 0, (hipStream_t)lc.stream, A->st);
        return;
    }
    const size_t lds = commitSharedBytes(*A);
    MW_LAUNCH(structuralCommitKernel, dim3((uint32_t)A->grid), dim3(kCommitThreads), lds,
                       (hipStream_t)lc.stream, *A);
}

}

__global__ void clearRowsKernel(int32_t *num_rows, int32_t num_worlds)
{
    MW_TRACE_BLOCK(0);
    int32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w < num_worlds) num_rows[w] = 0;
}

void launchClearRows(LaunchCtx &lc, int32_t archetype)
{
    int32_t *rows = lc.view->arch[archetype].numRows;
    MW_LAUNCH(clearRowsKernel, dim3((lc.numWorlds + 255) / 256), dim3(256), 0,
                       (hipStream_t)lc.stream, rows, lc.numWorlds);
}

// A kernel rather than a memset node: measured on the MI355X box, a
// hipMemsetAsync captured into the step graph left every other world's
// offset unreset once host hipMemcpy calls ran between graph replays.
__global__ void resetTmpAllocKernel(uint32_t *offsets, int32_t num_worlds,
                                    unsigned long long *pool_offset)
{
    MW_TRACE_BLOCK(0);
    const int32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    if (offsets && w < num_worlds) offsets[w] = 0;
    if (pool_offset && w == 0) *pool_offset = 0;      // every world resets here
}

void launchResetTmpAlloc(LaunchCtx &lc)
{
    if (!lc.view->tmpOffset && !lc.view->tmpPoolOffset) return;
    MW_LAUNCH(resetTmpAllocKernel, dim3((lc.numWorlds + 255) / 256), dim3(256), 0,
              (hipStream_t)lc.stream, lc.view->tmpOffset, lc.numWorlds, lc.view->tmpPoolOffset);
}

// Packed export: world w's rows land at offset prefix(numRows)[w]
// (reference madronaMWGPUExportCopyOut, src/mw/device/consts.cpp:190-273,
// here one block-wide scan per exported archetype per step instead of
// O(blocks^2)).  Each thread owns a contiguous run of worlds; the run sums
// are scanned with wave shuffles and one LDS pass.
__global__ void __launch_bounds__(1024)
exportScanKernel(const int32_t *num_rows, int32_t num_worlds, int64_t *offsets)
{
    MW_TRACE_BLOCK(0);
    __shared__ int64_t wave_sums[1024 / 64];
    const int32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int32_t per = (num_worlds + 1023) / 1024;
    const int32_t beg = min(tid * per, num_worlds);
    const int32_t end = min(beg + per, num_worlds);
    // up to kScanPer counts per thread held in registers: their loads issue
    // together (the loop form waited on them one by one) and the write pass
    // reuses them
    constexpr int32_t kScanPer = 16;
    int32_t v[kScanPer];
    int64_t s = 0;
    if (per <= kScanPer) {
#pragma unroll
        for (int32_t j = 0; j < kScanPer; j++) v[j] = beg + j < end ? num_rows[beg + j] : 0;
#pragma unroll
        for (int32_t j = 0; j < kScanPer; j++) s += v[j];
    } else {
        for (int32_t w = beg; w < end; w++) s += num_rows[w];
    }
    int64_t x = s;
#pragma unroll
    for (int32_t off = 1; off < 64; off <<= 1) {
        const int64_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    if (lane == 63) wave_sums[wave] = x;
    __syncthreads();
    int64_t base = 0;
    for (int32_t i = 0; i < wave; i++) base += wave_sums[i];
    int64_t run = base + x - s;
    if (per <= kScanPer) {
#pragma unroll
        for (int32_t j = 0; j < kScanPer; j++) {
            if (beg + j < end) offsets[beg + j] = run;
            run += v[j];
        }
    } else {
        for (int32_t w = beg; w < end; w++) {
            offsets[w] = run;
            run += num_rows[w];
        }
    }
    if (tid == 1023) offsets[num_worlds] = base + x;
}

// A singleton's slab is already packed (capacity 1, one row per world): the
// export is a flat copy.
__global__ void __launch_bounds__(256)
exportFlatCopyKernel(const uint32_t *__restrict__ src, int64_t n, uint32_t *__restrict__ dst)
{
    MW_TRACE_BLOCK(0);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        dst[i] = src[i];
    }
}

// Small per-world tables (at most kExportWaveWords words of a world's
// column): one wave per world, four worlds per block, loads unrolled ahead
// of the stores.  The 2-D kernel below launched a 256-lane block per 256
// words of capacity and world -- for a 129-row Position column two blocks
// of mostly idle lanes per world -- and ran 13.5 us per collisions export.
constexpr int32_t kExportWaveWords = 4096;

__global__ void __launch_bounds__(256)
exportCopyWaveKernel(const uint32_t *__restrict__ col, int32_t capacity, uint32_t words_per_row,
                     int32_t num_worlds, const int32_t *__restrict__ num_rows,
                     const int64_t *__restrict__ offsets, uint32_t *__restrict__ out)
{
    MW_TRACE_BLOCK(0);
    const int32_t w = (int32_t)blockIdx.x * 4 + (int32_t)(threadIdx.x >> 6);
    if (w >= num_worlds) return;
    const int32_t lane = threadIdx.x & 63;
    const int32_t n = num_rows[w] * (int32_t)words_per_row;
    const uint32_t *__restrict__ src = col + (size_t)w * capacity * words_per_row;
    uint32_t *__restrict__ dst = out + (size_t)offsets[w] * words_per_row;
#pragma unroll 4
    for (int32_t i = lane; i < n; i += 64) dst[i] = src[i];
}

// Rows are whole 4-byte words for every exported component, so the gather
// moves dwords (one world per blockIdx.y).
__global__ void __launch_bounds__(256)
exportCopyKernel(const uint32_t *col, int32_t capacity, uint32_t words_per_row,
                 const int32_t *num_rows, const int64_t *offsets, uint32_t *out)
{
    MW_TRACE_BLOCK(0);
    const int32_t w = blockIdx.y;
    const int32_t n = num_rows[w] * (int32_t)words_per_row;
    const uint32_t *src = col + (size_t)w * capacity * words_per_row;
    uint32_t *dst = out + (size_t)offsets[w] * words_per_row;
    for (int32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        dst[i] = src[i];
    }
}

// ---------------------------------------------------------------------------
// Device tracing (include/madrona/tracing.hpp)
// ---------------------------------------------------------------------------
namespace mwGPU {

static std::vector<TraceSetter> &traceSetters()
{
    static std::vector<TraceSetter> v;
    return v;
}

void registerTraceSetter(TraceSetter fn) { traceSetters().push_back(fn); }

static void setTracePointer(TraceDev *p)
{
    for (TraceSetter fn : traceSetters()) fn(p);
}

// One lane: a step / node boundary record.  The calibration record opens a
// step (logIndex 0: funcID = loggers per block, numInvocations = blocks per
// CU accounted per record, nodeID = size of the SM id space -- the fields
// parse_device_tracing.py reads from it); nodeStart also publishes the node
// to the blocks of the kernels that follow it.
__global__ void traceMarkerKernel(TraceDev *t, uint32_t ev, uint32_t func, uint32_t inv,
                                  uint32_t node)
{
    if (ev == (uint32_t)DeviceEvent::calibration) {
        const uint32_t i = atomicAdd(&t->next, 1u);
        __hip_atomic_store(&t->stepBase, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t ts = (uint64_t)wall_clock64() * t->nsPerTick;
        if (i >= t->capacity) {
            atomicAdd(&t->dropped, 1u);
            return;
        }
        t->logs[i] = DeviceLog { DeviceEvent::calibration, func, inv, node, 0, 0, traceSMID(), 0,
                                 ts };
        return;
    }
    if (ev == (uint32_t)DeviceEvent::nodeStart) t->curNode = node;
    traceLog(t, (DeviceEvent)ev, func, inv, node, 0);
}

}

// ---------------------------------------------------------------------------
// Executor
// ---------------------------------------------------------------------------
struct GrowSet {
    int32_t n;
    int32_t arch[kMaxArchetypes];
};

// An export buffer of a growable archetype is a reserved device address
// range with physical memory mapped on demand (HIP virtual memory
// management): a table growth maps more of it behind the packed rows, so the
// buffer keeps its address and contents, as the reference's getExported
// pointer does (src/mw/cuda_exec.cpp:1777-1782, state.cpp exportColumn).
// Where the range cannot be reserved (or a growth outruns it) the buffer is
// reallocated with its packed rows copied over: then pointers handed out
// before the growth are stale (mw_get_exported again).
struct ExportMem {
    size_t reserved = 0;        // bytes of address space (0: a plain hipMalloc buffer)
    size_t mapped = 0;          // bytes backed by physical chunks from the start
    std::vector<std::pair<hipMemGenericAllocationHandle_t, size_t>> chunks;
};

struct ExportBuf {
    int32_t slot, archetype, column;
    uint32_t bytes;
    char *buf;
    int64_t *offsets;           // shared by the exports of one archetype
    bool scanOwner;             // this export launches the archetype's scan
    bool singleton;             // one row per world: offsets fixed (w), flat copy
    ExportMem mem;
    int64_t relocations = 0;    // growths that moved buf (0 with a reserved range)
};

static hipMemAllocationProp exportMemProp(int dev)
{
    hipMemAllocationProp prop {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = dev;
    return prop;
}

static size_t exportMemGranularity(int dev)
{
    const hipMemAllocationProp prop = exportMemProp(dev);
    size_t gran = 0;
    if (hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return gran;
}

static void releaseExportMem(ExportBuf &b)
{
    if (!b.buf) return;
    if (b.mem.reserved == 0) {
        (void)hipFree(b.buf);
    } else {
        size_t off = 0;
        for (auto &c : b.mem.chunks) {
            (void)hipMemUnmap(b.buf + off, c.second);
            (void)hipMemRelease(c.first);
            off += c.second;
        }
        (void)hipMemAddressFree(b.buf, b.mem.reserved);
    }
    b.buf = nullptr;
    b.mem = ExportMem {};
}

// Back [0, bytes) of the reserved range with physical memory (the new part
// only); false when the range or the device refuses it.
static bool mapExportMem(ExportBuf &b, size_t bytes, int dev)
{
    if (bytes <= b.mem.mapped) return true;
    const size_t gran = exportMemGranularity(dev);
    if (gran == 0) return false;
    const size_t need = (bytes - b.mem.mapped + gran - 1) / gran * gran;
    if (b.mem.mapped + need > b.mem.reserved) return false;
    const hipMemAllocationProp prop = exportMemProp(dev);
    auto refused = [&](const char *what, hipError_t e) {
        (void)hipGetLastError();
        if (getenv("MADRONA_MW_EXPORT_DEBUG"))
            fprintf(stderr, "export buffer: %s refused (%s): mapped %zu need %zu gran %zu reserved %zu\n",
                    what, hipGetErrorString(e), b.mem.mapped, need, gran, b.mem.reserved);
        return false;
    };
    hipMemGenericAllocationHandle_t h {};
    hipError_t e = hipMemCreate(&h, need, &prop, 0);
    if (e != hipSuccess) return refused("hipMemCreate", e);
    char *at = b.buf + b.mem.mapped;
    e = hipMemMap(at, need, 0, h, 0);
    if (e != hipSuccess) {
        (void)hipMemRelease(h);
        return refused("hipMemMap", e);
    }
    hipMemAccessDesc acc {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    // Access is set over the whole mapped prefix: ROCm refuses a range that
    // starts inside the reservation after an earlier chunk (measured: invalid
    // argument at offset 12 KiB), and accepts the prefix.
    e = hipMemSetAccess(b.buf, b.mem.mapped + need, &acc, 1);
    if (e != hipSuccess) {
        (void)hipMemUnmap(at, need);
        (void)hipMemRelease(h);
        return refused("hipMemSetAccess", e);
    }
    b.mem.chunks.push_back({ h, need });
    b.mem.mapped += need;
    return true;
}

// A new export buffer of `bytes`; a growable archetype's in a reserved range
// of 256x that (at least 4 GiB of address space, no memory behind it).
// MADRONA_MW_EXPORT_VMM=0: plain buffers (relocated on growth).
static void allocExportMem(ExportBuf &b, size_t bytes, bool growable, int dev)
{
    bytes = std::max<size_t>(bytes, 256);
    const char *env = getenv("MADRONA_MW_EXPORT_VMM");
    const size_t gran = growable && !(env && atoi(env) == 0) ? exportMemGranularity(dev) : 0;
    if (gran > 0) {
        size_t reserve = std::max<size_t>(bytes * 256, size_t(4) << 30);
        reserve = (reserve + gran - 1) / gran * gran;
        void *p = nullptr;
        if (hipMemAddressReserve(&p, reserve, 0, nullptr, 0) == hipSuccess && p) {
            b.buf = (char *)p;
            b.mem.reserved = reserve;
            if (mapExportMem(b, bytes, dev)) return;
            releaseExportMem(b);
        }
        (void)hipGetLastError();
    }
    MW_HIP_CHECK(hipMalloc(&b.buf, bytes));
}

// Growth probe ring: after every enqueued step the growable tables' largest
// per-world row counts go to pinned host memory, behind an event.
constexpr int32_t kGrowProbeSlots = 8;

struct Executor::Impl {
    ExecConfig cfg;
    std::unique_ptr<StateManager> mgr;
    hipStream_t stream = nullptr;
    hipStream_t sideStream = nullptr;   // LaunchCtx::sideStream
    hipEvent_t forkEvent = nullptr, joinEvent = nullptr;
    TaskGraph graph;
    // The step as replayable hipGraph segments.  Normally one segment holds
    // every node plus the export gathers; with live node timing enabled the
    // step is split at each timed node, which is launched directly on the
    // stream between its segments, its kernels bound to a HIP event pair.
    struct Segment {
        hipGraph_t graph = nullptr;
        hipGraphExec_t exec = nullptr;
        int32_t timedNode = -1;   // node launched (timed) after this segment
        int32_t timedEnd = -1;    // ... with the rest of the walk run it starts: [timedNode, timedEnd)
    };
    std::vector<Segment> segs;
    // Sampled live timing (timedEvery > 1): the unsplit step graph, replayed
    // on the steps that are not timed.
    std::vector<Segment> plainSegs;
    // Runs of untimed steps: K unsplit steps captured into one graph
    // (MADRONA_MW_STEPS_PER_GRAPH, default 16; 1 = off), launched when the
    // next K steps are all plain, so a run pays one graph launch instead of
    // K (fantasy_vs at 0.13 ms per tick: 125.7 -> 128.8 M env-steps/s with
    // K = 8; collisions unchanged).
    std::vector<Segment> multiSegs;
    int32_t stepsPerGraph = 16;
    int32_t multiK = 0;             // steps in multiSegs' graph (0: none)
    int32_t timedEvery = 1;
    int64_t stepIndex = 0;
    std::vector<ExportBuf> exports;
    int64_t *hostRowsTotal = nullptr;

    // Live per-node timing: a HIP event pair bound to the kernels of every
    // launch of one node kind inside each step (launchNodeTimed: first
    // kernel start to last kernel end), accumulated at each sync.
    std::string timedName;
    int32_t timedIndex = -1;        // setTimedNodeIndex: one node only
    // One event pair per timed launch per enqueued step: a burst of
    // runAsync steps keeps every step's pairs until the next sync.
    std::vector<std::pair<hipEvent_t, hipEvent_t>> timedPool;   // one pair per timed kernel
    size_t timedNext = 0;           // pairs used since the last sync
    int64_t timedUnits = 0;         // timed launches (nodes / walk runs) since the last sync
    int32_t timedPerStep = 0;       // timed launches in one step
    double timedMs = 0.0;
    int64_t timedLaunches = 0;

    // Device tracing: null unless enabled (Executor::enableTracing).
    mwGPU::TraceDev *trace = nullptr;
    mwGPU::DeviceLog *traceLogs = nullptr;
    std::vector<std::string> traceFuncs;      // funcID -> node kind
    std::vector<uint32_t> nodeFunc;           // node -> funcID

    // Launch configuration (reference MADRONA_MWGPU_EXEC_CONFIG_OVERRIDE /
    // _FILE, src/mw/cuda_exec.cpp:1534-1560): blocks per CU per node, -1 =
    // the default; numCUs = the CUs grids are sized for.
    int32_t defaultBlocksPerCU = 0;
    int32_t numCUs = 0;
    std::vector<int32_t> nodeBlocksPerCU;
    // ResetTmpAllocNodes with no possibly-allocating node since the previous
    // launched reset (the start of a step counts as one: the previous
    // step's tail) are no-ops: not launched.
    std::vector<uint8_t> nodeSkip;

    // Device copies of the graph's node data (TaskGraph::NodeData blocks).
    char *nodeDataDev = nullptr;
    // Ordered structural commit of row-parallel nodes.
    CommitArgs commit {};

    // World walk (TaskGraph::NodeFns::walk, planned when the graph is set):
    // per node 1 = walkable with walkKernel[i] / resumeKernel[i] and entries
    // [walkOff[i], walkOff[i + 1]) of walkEntriesDev, 2 = a no-op that may sit
    // inside a run (an elided reset), 0 = launched on its own.
    bool walkEnabled = true;
    std::vector<uint8_t> walkable;
    std::vector<uint8_t> walkCommits;        // the node's entries include a commit point
    std::vector<const void *> walkKernel;
    std::vector<const void *> resumeKernel;
    std::vector<int32_t> walkOff;
    detail::WalkEntry *walkEntriesDev = nullptr;
    int32_t *walkResume = nullptr;           // [W] commit point a world stopped at, -1
    // worldResumeKernel's per-block global scratch (commit working set +
    // move scratch) and grids
    char *walkScratch = nullptr;
    uint64_t walkPerBlock = 0;
    uint64_t walkWsBytes = 0;
    size_t walkLds = 0;             // resume kernel: dynamic LDS for the commit working set (0: in the slab)
    // table growth (growTables): the growable archetypes, their row maxima
    // per probe slot (device, pinned host), the slots in flight oldest first,
    // the latest maxima read back, and how many steps may run past the
    // newest maxima the host has seen (MADRONA_MW_GROW_LAG)
    GrowSet growable {};
    int32_t *growProbe = nullptr;             // [kGrowProbeSlots][kMaxArchetypes]
    int32_t *growProbeHost = nullptr;
    hipEvent_t growProbeEv[kGrowProbeSlots] = {};
    int32_t probeFifo[kGrowProbeSlots] = {};
    int32_t probeHead = 0, probeCount = 0, probeNext = 0;
    int64_t probeStepOf[kGrowProbeSlots] = {};
    int64_t stepsEnqueued = 0;                // probe k follows step k (0: the upload)
    int64_t lastProbeStep = -1;               // step of the maxima in lastMax (-1: none yet)
    int32_t growLag = 4;
    int32_t lastMax[kMaxArchetypes] = {};
    int32_t maxRise[kMaxArchetypes] = {};     // largest per-step rise seen, -1: none yet
    int64_t growths = 0;
    int64_t stepsRun = 0;                     // steps enqueued since creation (extension polls)
    std::vector<std::pair<const void *, int32_t>> walkGrid;   // kernel -> grid
};

static LaunchCtx makeLaunchCtx(Executor::Impl &I, Executor *exec)
{
    const StateView &dv = I.mgr->deviceViewHost();
    LaunchCtx lc { I.stream, I.mgr->deviceView(), &dv, I.cfg.numWorlds, exec };
    lc.nodeData = I.nodeDataDev;
    lc.serialNodes = I.cfg.serialNodes;
    if (const char *e = getenv("MADRONA_MW_WORLD_WAVE_LANES")) lc.worldWaveLanes = atoi(e);
    if (const char *e = getenv("MADRONA_MW_FUSE_ARCHETYPES")) lc.fuseArchetypes = atoi(e);
    // opt-in: in the replayed graph the join costs more than the overlap
    // saves (DESIGN.md round-3 dead ends)
    const char *side = getenv("MADRONA_MW_SIDE_STREAM");
    if (side && atoi(side) != 0) {
        lc.sideStream = I.sideStream;
        lc.forkEvent = I.forkEvent;
        lc.joinEvent = I.joinEvent;
    }
    return lc;
}

const void *Executor::commitArgs() const { return &impl_->commit; }

Executor::Executor(const ExecConfig &cfg) : impl_(new Impl)
{
    impl_->cfg = cfg;
    MW_HIP_CHECK(hipSetDevice(cfg.gpuID));
    MW_HIP_CHECK(hipStreamCreateWithFlags(&impl_->stream, hipStreamNonBlocking));
    MW_HIP_CHECK(hipStreamCreateWithFlags(&impl_->sideStream, hipStreamNonBlocking));
    MW_HIP_CHECK(hipEventCreateWithFlags(&impl_->forkEvent, hipEventDisableTiming));
    MW_HIP_CHECK(hipEventCreateWithFlags(&impl_->joinEvent, hipEventDisableTiming));
    impl_->mgr.reset(new StateManager(StateManager::Config {
        cfg.numWorlds, cfg.defaultCapacity,
        cfg.tmpAllocBytesPerWorld >= 0 ? cfg.tmpAllocBytesPerWorld : kDefaultTmpAllocBytes,
        cfg.maxDeferredPerWorld > 0 ? cfg.maxDeferredPerWorld : kDefaultDeferredPerWorld,
        cfg.tmpPoolBytes >= 0 ? cfg.tmpPoolBytes
                              : defaultTmpPoolBytes(cfg.numWorlds, cfg.tmpAllocBytesPerWorld >= 0
                                                                       ? cfg.tmpAllocBytesPerWorld
                                                                       : kDefaultTmpAllocBytes) }));
}

Executor::~Executor()
{
    for (auto &e : impl_->timedPool) {
        (void)hipEventDestroy(e.first);
        (void)hipEventDestroy(e.second);
    }
    for (auto *v : { &impl_->segs, &impl_->plainSegs, &impl_->multiSegs }) {
        for (auto &sg : *v) {
            if (sg.exec) (void)hipGraphExecDestroy(sg.exec);
            if (sg.graph) (void)hipGraphDestroy(sg.graph);
        }
    }
    if (impl_->trace) {
        (void)hipStreamSynchronize(impl_->stream);
        mwGPU::setTracePointer(nullptr);
        (void)hipFree(impl_->trace);
        (void)hipFree(impl_->traceLogs);
    }
    if (impl_->stream) (void)hipStreamSynchronize(impl_->stream);
    if (impl_->hostRowsTotal) (void)hipHostFree(impl_->hostRowsTotal);
    if (impl_->nodeDataDev) (void)hipFree(impl_->nodeDataDev);
    if (impl_->commit.scratch) (void)hipFree(impl_->commit.scratch);
    if (impl_->growProbe) (void)hipFree(impl_->growProbe);
    if (impl_->growProbeHost) (void)hipHostFree(impl_->growProbeHost);
    for (hipEvent_t e : impl_->growProbeEv) {
        if (e) (void)hipEventDestroy(e);
    }
    if (impl_->walkEntriesDev) (void)hipFree(impl_->walkEntriesDev);
    if (impl_->walkScratch) (void)hipFree(impl_->walkScratch);
    if (impl_->walkResume) (void)hipFree(impl_->walkResume);
    for (auto &e : impl_->exports) {
        releaseExportMem(e);
        if (e.scanOwner) (void)hipFree(e.offsets);
    }
    impl_->mgr.reset();
    if (impl_->stream) (void)hipStreamDestroy(impl_->stream);
    if (impl_->sideStream) (void)hipStreamDestroy(impl_->sideStream);
    if (impl_->forkEvent) (void)hipEventDestroy(impl_->forkEvent);
    if (impl_->joinEvent) (void)hipEventDestroy(impl_->joinEvent);
}

StateManager &Executor::stateManager() { return *impl_->mgr; }
ECSRegistry Executor::registry() { return ECSRegistry(impl_->mgr.get(), nullptr); }
int32_t Executor::numWorlds() const { return impl_->cfg.numWorlds; }
void *Executor::stream() const { return impl_->stream; }

void Executor::finalizeRegistration(uint32_t world_bytes, uint32_t world_align)
{
    impl_->mgr->finalizeLayout(world_bytes, world_align);
}

Context Executor::makeHostContext(int32_t world)
{
    return Context((WorldBase *)hostWorldData(world),
                   WorkerInit { &impl_->mgr->hostView(), world, impl_->mgr.get() });
}

char *Executor::hostWorldData(int32_t world)
{
    StateView &v = impl_->mgr->hostView();
    return v.worldData + (size_t)world * v.worldDataStride;
}

// Ordered-commit sizing (StateManager: the largest table that takes entity
// rows or row-parallel appends); one scratch slab per commit block holds a
// column of it.  Again after a table grows.
static void setupCommit(Executor::Impl &I)
{
    {
        Executor::Impl *impl_ = &I;
        const StateView &dv = impl_->mgr->deviceViewHost();
        CommitArgs &A = impl_->commit;
        if (A.scratch) {
            MW_HIP_CHECK(hipFree(A.scratch));
            A.scratch = nullptr;
        }
        A.st = impl_->mgr->deviceView();
        A.shape = detail::CommitShape { dv.commitCapMax, dv.commitSortA, dv.commitSortO };
        A.scratchPerBlock = ((uint64_t)dv.commitCapMax * dv.commitColMax + 255) / 256 * 256;
        A.grid = 1;
        if (A.shape.capMax > 0) {
            // refuse a configuration whose commit cannot launch (it would
            // silently drop every structural op of a row-parallel node)
            const size_t lds = commitSharedBytes(A);
            const int32_t per_cu =
                hipx::residentBlocksNoThrow((const void *)&structuralCommitKernel, kCommitThreads, lds);
            if (per_cu <= 0) {
                throw std::runtime_error(
                    "ordered commit needs " + std::to_string(lds) + " B of LDS per block (" +
                    std::to_string(A.shape.capMax) + " table rows, " + std::to_string(dv.deferCap) +
                    " deferred destroys per world) but a workgroup holds " +
                    std::to_string(hipx::maxLDSPerBlock()) +
                    " B: lower max_deferred_destroys or the table capacities");
            }
            // the resident grid, its scratch slabs bounded to 256 MiB
            int32_t cus = 0;
            MW_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, impl_->cfg.gpuID));
            int64_t blocks = std::min<int64_t>(dv.numWorlds, (int64_t)per_cu * std::max(cus, 1));
            blocks = std::min<int64_t>(blocks, std::max<int64_t>(1, (256ll << 20) / (int64_t)A.scratchPerBlock));
            A.grid = (int32_t)std::max<int64_t>(blocks, 1);
            MW_HIP_CHECK(hipMalloc(&A.scratch, std::max<size_t>(A.scratchPerBlock * A.grid, 256)));
        }
    }
}

// Growable tables (registerArchetype, StateManager::growable) and the
// per-archetype row-count maxima the growth check reads.
// One block: per growable archetype the maximum over worlds, plain stores
// (no reset needed between probes).
constexpr int32_t kMaxRowsThreads = 1024;
__global__ void __launch_bounds__(kMaxRowsThreads) maxRowsKernel(const StateView *__restrict__ st, GrowSet g,
                                                                 int32_t *out)
{
    __shared__ int32_t part[kMaxRowsThreads / 64];
    for (int32_t i = 0; i < g.n; i++) {
        const int32_t *rows = st->arch[g.arch[i]].numRows;
        int32_t m = 0;
        for (int32_t w = threadIdx.x; w < st->numWorlds; w += kMaxRowsThreads) m = max(m, rows[w]);
#pragma unroll
        for (int32_t o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o, 64));
        if ((threadIdx.x & 63) == 0) part[threadIdx.x / 64] = m;
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int32_t k = 1; k < kMaxRowsThreads / 64; k++) m = max(m, part[k]);
            out[i] = m;
        }
        __syncthreads();
    }
}

// Enqueue a growth probe behind the steps enqueued so far.
static void consumeOldestProbe(Executor::Impl &I, bool wait);
static void enqueueGrowProbe(Executor::Impl &I)
{
    if (I.growable.n == 0) return;
    if (I.probeCount == kGrowProbeSlots) consumeOldestProbe(I, true);
    const int32_t s = I.probeNext;
    I.probeNext = (I.probeNext + 1) % kGrowProbeSlots;
    int32_t *dev = I.growProbe + s * kMaxArchetypes;
    MW_LAUNCH(maxRowsKernel, dim3(1), dim3(kMaxRowsThreads), 0, I.stream, I.mgr->deviceView(), I.growable, dev);
    MW_HIP_CHECK(hipMemcpyAsync(I.growProbeHost + s * kMaxArchetypes, dev, sizeof(int32_t) * I.growable.n,
                                hipMemcpyDeviceToHost, I.stream));
    MW_HIP_CHECK(hipEventRecord(I.growProbeEv[s], I.stream));
    I.probeStepOf[s] = I.stepsEnqueued;
    I.probeFifo[(I.probeHead + I.probeCount) % kGrowProbeSlots] = s;
    I.probeCount++;
}

// Read the oldest probe in flight (waiting for it, or only if it is done);
// the maxima of later probes replace earlier ones, and the largest per-step
// rise between consecutive readings is kept.
static void consumeOldestProbe(Executor::Impl &I, bool wait)
{
    const int32_t s = I.probeFifo[I.probeHead];
    if (wait) {
        MW_HIP_CHECK(hipEventSynchronize(I.growProbeEv[s]));
    } else {
        const hipError_t q = hipEventQuery(I.growProbeEv[s]);
        if (q == hipErrorNotReady) {
            (void)hipGetLastError();
            return;
        }
        MW_HIP_CHECK(q);
    }
    const int64_t step = I.probeStepOf[s];
    for (int32_t i = 0; i < I.growable.n; i++) {
        const int32_t m = I.growProbeHost[s * kMaxArchetypes + i];
        if (I.lastProbeStep >= 0 && step > I.lastProbeStep) {
            const int64_t d = step - I.lastProbeStep;
            const int32_t rise = (int32_t)std::max<int64_t>(0, ((int64_t)m - I.lastMax[i] + d - 1) / d);
            I.maxRise[i] = std::max(I.maxRise[i], rise);
        }
        I.lastMax[i] = m;
    }
    I.lastProbeStep = step;
    I.probeHead = (I.probeHead + 1) % kGrowProbeSlots;
    I.probeCount--;
}

// Consume every finished probe; with wait, every probe.
static void drainGrowProbes(Executor::Impl &I, bool wait)
{
    while (I.probeCount > 0) {
        const int32_t before = I.probeCount;
        consumeOldestProbe(I, wait);
        if (I.probeCount == before) break;      // the oldest is still running
    }
}

// May the next step be enqueued before more probes are read?  The rows of
// the steps the host has not seen yet (those in flight and the next one)
// are projected with the largest per-step rise seen so far; before a rise
// is known only the step right after the newest reading is.
static bool enqueueSafe(const Executor::Impl &I)
{
    if (I.lastProbeStep < 0) return false;
    const StateView &dv = I.mgr->deviceViewHost();
    const int64_t ahead = I.stepsEnqueued + 1 - I.lastProbeStep;
    for (int32_t i = 0; i < I.growable.n; i++) {
        if (I.maxRise[i] < 0) {
            if (ahead > 1) return false;
            continue;
        }
        if ((int64_t)I.lastMax[i] + (int64_t)I.maxRise[i] * ahead > dv.arch[I.growable.arch[i]].capacity)
            return false;
    }
    return true;
}

// The capacity archetype i needs for the newest maxima: at most half full,
// and room for growLag + 1 steps at the largest rise seen.
static int64_t neededCapacity(const Executor::Impl &I, int32_t i, int64_t cap)
{
    const int64_t m = I.lastMax[i];
    const int64_t ahead = I.maxRise[i] > 0 ? m + (int64_t)I.maxRise[i] * (I.growLag + 1) : 0;
    int64_t nc = std::max<int64_t>(cap, 1);
    while (m * 2 > nc || ahead > nc) nc *= 2;
    return nc;
}

static bool growthDue(const Executor::Impl &I)
{
    const StateView &dv = I.mgr->deviceViewHost();
    for (int32_t i = 0; i < I.growable.n; i++) {
        const int32_t cap = dv.arch[I.growable.arch[i]].capacity;
        if (neededCapacity(I, i, cap) > cap) return true;
    }
    return false;
}

static void launchExports(Executor::Impl &I, const StateView &dv);

void Executor::uploadState()
{
    impl_->mgr->uploadToDevice(impl_->stream);
    setupCommit(*impl_);
    // growable tables: known once the modules have pinned theirs (upload)
    impl_->growable.n = 0;
    for (int32_t a = 0; a < impl_->mgr->numArchetypes(); a++) {
        if (impl_->mgr->growable(a) && impl_->growable.n < kMaxArchetypes) impl_->growable.arch[impl_->growable.n++] = a;
    }
    if (impl_->growable.n > 0) {
        const size_t pb = sizeof(int32_t) * kMaxArchetypes * kGrowProbeSlots;
        MW_HIP_CHECK(hipMalloc(&impl_->growProbe, pb));
        MW_HIP_CHECK(hipHostMalloc(&impl_->growProbeHost, pb));
        for (hipEvent_t &e : impl_->growProbeEv) MW_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        if (const char *e = std::getenv("MADRONA_MW_GROW_LAG")) impl_->growLag = std::max(0, atoi(e));
        impl_->growLag = std::min(impl_->growLag, kGrowProbeSlots - 1);
        for (int32_t &r : impl_->maxRise) r = -1;
    }

    int32_t num_exports = 0;
    const StateManager::ExportDesc *ex = impl_->mgr->exports(&num_exports);
    const StateView &dv = impl_->mgr->deviceViewHost();
    for (int32_t i = 0; i < num_exports; i++) {
        ExportBuf b {};
        b.slot = ex[i].slot;
        b.archetype = ex[i].archetype;
        b.column = ex[i].column;
        b.bytes = ex[i].bytes;
        size_t bytes = (size_t)dv.numWorlds * dv.arch[b.archetype].capacity * b.bytes;
        if (b.bytes % 4 != 0) {
            throw std::runtime_error("exportColumn: component size must be a multiple of 4 bytes");
        }
        allocExportMem(b, bytes, impl_->mgr->growable(b.archetype), impl_->cfg.gpuID);
        // offsets are per archetype: exports of one archetype share them
        for (const ExportBuf &o : impl_->exports) {
            if (o.archetype == b.archetype) { b.offsets = o.offsets; b.scanOwner = false; }
        }
        b.singleton = (dv.arch[b.archetype].flags & kArchSingleton) != 0;
        if (!b.offsets) {
            MW_HIP_CHECK(hipMalloc(&b.offsets, sizeof(int64_t) * (dv.numWorlds + 1)));
            // a singleton's packed rows never move: world w at row w, no scan
            b.scanOwner = !b.singleton;
            if (b.singleton) {
                std::vector<int64_t> off(dv.numWorlds + 1);
                for (int32_t w = 0; w <= dv.numWorlds; w++) off[w] = w;
                MW_HIP_CHECK(hipMemcpy(b.offsets, off.data(), sizeof(int64_t) * off.size(),
                                       hipMemcpyHostToDevice));
            }
        }
        impl_->exports.push_back(b);
    }
    // the packed exports of the initial state (a getExported before the
    // first step reads the worlds as created, not uninitialised offsets)
    launchExports(*impl_, dv);
    enqueueGrowProbe(*impl_);            // the initial rows
}

static void traceMarker(Executor::Impl &I, mwGPU::DeviceEvent ev, uint32_t func, uint32_t inv,
                        uint32_t node);

// With tracing on, each export gather is its own trace node (IDs after the
// graph's nodes, funcID of the "ExportNode" kind).
static void launchExports(Executor::Impl &I, const StateView &dv)
{
    for (size_t e = 0; e < I.exports.size(); e++) {
        ExportBuf &b = I.exports[e];
        const uint32_t trace_node = (uint32_t)(I.graph.numNodes() + e);
        const uint32_t trace_func = (uint32_t)I.traceFuncs.size() - 1;
        if (I.trace) {
            traceMarker(I, mwGPU::DeviceEvent::nodeStart, trace_func, (uint32_t)dv.numWorlds,
                        trace_node);
        }
        const ArchetypeView &av = dv.arch[b.archetype];
        const uint32_t words = b.bytes / 4;
        if (b.singleton) {
            const int64_t n = (int64_t)dv.numWorlds * words;
            MW_LAUNCH(exportFlatCopyKernel, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 4096)),
                      dim3(256), 0, I.stream, (const uint32_t *)av.cols[b.column], n, (uint32_t *)b.buf);
        } else {
            if (b.scanOwner) {
                MW_LAUNCH(exportScanKernel, dim3(1), dim3(1024), 0, I.stream, av.numRows, dv.numWorlds,
                          b.offsets);
            }
            if ((int64_t)av.capacity * words <= kExportWaveWords) {
                MW_LAUNCH(exportCopyWaveKernel, dim3((unsigned)((dv.numWorlds + 3) / 4)), dim3(256), 0,
                          I.stream, (const uint32_t *)av.cols[b.column], av.capacity, words,
                          dv.numWorlds, av.numRows, b.offsets, (uint32_t *)b.buf);
            } else {
                const unsigned bx = (unsigned)std::max<int64_t>(1, ((int64_t)av.capacity * words + 255) / 256);
                MW_LAUNCH(exportCopyKernel, dim3(bx, dv.numWorlds), dim3(256), 0, I.stream,
                          (const uint32_t *)av.cols[b.column], av.capacity, words, av.numRows, b.offsets,
                          (uint32_t *)b.buf);
            }
        }
        if (I.trace) {
            traceMarker(I, mwGPU::DeviceEvent::nodeFinish, trace_func, (uint32_t)dv.numWorlds,
                        trace_node);
        }
    }
}

static bool isTimed(const Executor::Impl &I, int32_t node)
{
    if (I.timedIndex >= 0) return node == I.timedIndex;
    return !I.timedName.empty() && I.timedName == I.graph.nodeName(node);
}

static void traceMarker(Executor::Impl &I, mwGPU::DeviceEvent ev, uint32_t func, uint32_t inv,
                        uint32_t node)
{
    MW_LAUNCH(mwGPU::traceMarkerKernel, dim3(1), dim3(1), 0, I.stream, I.trace,
                       (uint32_t)ev, func, inv, node);
}

// A node's launches; with tracing on, bracketed by nodeStart / nodeFinish.
static void launchNode(Executor::Impl &I, int32_t i, LaunchCtx &lc)
{
    if (i < (int32_t)I.nodeSkip.size() && I.nodeSkip[i]) {
        if (I.trace) {              // an elided node still appears in the trace, empty
            const uint32_t f = I.nodeFunc[i], n = (uint32_t)I.cfg.numWorlds;
            traceMarker(I, mwGPU::DeviceEvent::nodeStart, f, n, (uint32_t)i);
            traceMarker(I, mwGPU::DeviceEvent::nodeFinish, f, n, (uint32_t)i);
        }
        return;
    }
    const int32_t bpc = i < (int32_t)I.nodeBlocksPerCU.size() ? I.nodeBlocksPerCU[i] : -1;
    lc.blocksPerCU = bpc >= 0 ? bpc : I.defaultBlocksPerCU;
    lc.numCUs = I.numCUs;
    if (!I.trace) {
        I.graph.launchNode(i, lc);
        return;
    }
    const uint32_t f = I.nodeFunc[i], n = (uint32_t)I.cfg.numWorlds;
    traceMarker(I, mwGPU::DeviceEvent::nodeStart, f, n, (uint32_t)i);
    I.graph.launchNode(i, lc);
    traceMarker(I, mwGPU::DeviceEvent::nodeFinish, f, n, (uint32_t)i);
}

// Step boundaries of the trace (calibration record / blockExit record).
static constexpr uint32_t kTraceSMIDs = 8 * 4 * 16;

static void traceStepBegin(Executor::Impl &I)
{
    if (I.trace) traceMarker(I, mwGPU::DeviceEvent::calibration, 1, 1, kTraceSMIDs);
}

static void traceStepEnd(Executor::Impl &I)
{
    if (I.trace) {
        traceMarker(I, mwGPU::DeviceEvent::blockExit, 0, 0, (uint32_t)I.graph.numNodes());
    }
}

// The next free event pair of the timing pool (created on first use); the
// pool is read back and recycled at the next sync.
static std::pair<hipEvent_t, hipEvent_t> &timedPair(Executor::Impl &I)
{
    while (I.timedPool.size() <= I.timedNext) {
        hipEvent_t a, b;
        MW_HIP_CHECK(hipEventCreate(&a));
        MW_HIP_CHECK(hipEventCreate(&b));
        I.timedPool.push_back({ a, b });
    }
    return I.timedPool[I.timedNext++];
}

static void nextTimedPair(void *ctx, hipEvent_t *a, hipEvent_t *b)
{
    const auto &pr = timedPair(*(Executor::Impl *)ctx);
    *a = pr.first;
    *b = pr.second;
}

// Sum of the elapsed times of the pool's used pairs (after a stream sync);
// recycles them.
static double drainTimedPairs(Executor::Impl &I)
{
    double total = 0.0;
    for (size_t i = 0; i < I.timedNext; i++) {
        float ms = 0;
        MW_HIP_CHECK(hipEventElapsedTime(&ms, I.timedPool[i].first, I.timedPool[i].second));
        total += ms;
    }
    I.timedNext = 0;
    return total;
}

static void launchUnit(Executor::Impl &I, int32_t k, int32_t j, LaunchCtx &lc);

// Node i (or the walk run [i, j) it starts: timed as one unit, its walk and
// resume kernels) with each of its kernels bound to an event pair of the
// pool (hipx::TimedLaunch: the unit's time is the sum of its kernels').  A
// unit none of whose kernels took a binding (a world library launching
// through its own calls) is timed by a stream-order pair around it.
static void launchNodeTimed(Executor::Impl &I, int32_t i, int32_t j, LaunchCtx &lc)
{
    const auto &pr = timedPair(I);
    MW_HIP_CHECK(hipEventRecord(pr.first, I.stream));
    hipx::TimedLaunch t { pr.first, pr.second, &nextTimedPair, &I };
    hipx::tlTimed = &t;
    try {
        launchUnit(I, i, j, lc);
    } catch (...) {
        hipx::tlTimed = nullptr;
        throw;
    }
    hipx::tlTimed = nullptr;
    if (t.kernels == 0) MW_HIP_CHECK(hipEventRecord(pr.second, I.stream));
    I.timedUnits++;
}

// World walk planning (before any capture: a node's walk plan may read a
// device address back with a synchronous launch).  Opt-in,
// MADRONA_MW_WORLD_WALK=1: on fantasy_vs the walk is 0.25 ms per tick against
// 0.14 for the per-node launches -- the world functions are
// called through pointers and compiled with the function ABI, the heaviest
// (the caster's row code) at ~100 VGPRs, so the walk holds 4-5 waves per
// SIMD where the per-node world-wave kernels hold 8.
static void planWorldWalk(Executor::Impl &I, LaunchCtx &lc)
{
    const int32_t n = I.graph.numNodes();
    I.walkable.assign(n, 0);
    I.walkCommits.assign(n, 0);
    I.walkKernel.assign(n, nullptr);
    I.resumeKernel.assign(n, nullptr);
    I.walkOff.assign(n + 1, 0);
    if (const char *e = getenv("MADRONA_MW_WORLD_WALK")) I.walkEnabled = atoi(e) != 0;
    std::vector<detail::WalkEntry> all;
    for (int32_t i = 0; i < n; i++) {
        I.walkOff[i] = (int32_t)all.size();
        if (!I.walkEnabled) continue;
        if (i < (int32_t)I.nodeSkip.size() && I.nodeSkip[i]) {
            I.walkable[i] = 2;
            continue;
        }
        const TaskGraph::NodeFns &f = I.graph.nodeFns(i);
        if (!f.walk) continue;
        detail::WalkEntry tmp[detail::kMaxWalkEntriesPerNode];
        const void *kernels[2] = { nullptr, nullptr };
        const int32_t ne = f.walk(I.graph.nodeState(i), lc, tmp, kernels);
        if (ne <= 0 || ne > detail::kMaxWalkEntriesPerNode || !kernels[0] || !kernels[1]) continue;
        I.walkable[i] = 1;
        I.walkKernel[i] = kernels[0];
        I.resumeKernel[i] = kernels[1];
        for (int32_t k = 0; k < ne; k++) I.walkCommits[i] |= tmp[k].kind == detail::kWalkCommit;
        all.insert(all.end(), tmp, tmp + ne);
    }
    I.walkOff[n] = (int32_t)all.size();
    if (I.walkEntriesDev) {
        MW_HIP_CHECK(hipFree(I.walkEntriesDev));
        I.walkEntriesDev = nullptr;
    }
    if (all.empty()) return;
    MW_HIP_CHECK(hipMalloc(&I.walkEntriesDev, sizeof(detail::WalkEntry) * all.size()));
    MW_HIP_CHECK(hipMemcpy(I.walkEntriesDev, all.data(), sizeof(detail::WalkEntry) * all.size(),
                           hipMemcpyHostToDevice));
    if (!I.walkResume) {
        MW_HIP_CHECK(hipMalloc(&I.walkResume, sizeof(int32_t) * std::max(I.cfg.numWorlds, 1)));
        MW_HIP_CHECK(hipMemset(I.walkResume, 0xFF, sizeof(int32_t) * std::max(I.cfg.numWorlds, 1)));
    }
    // resident grids (one wave per block); the resume kernel's blocks each
    // own a global scratch slab for the commit's row moves and keep its
    // working set in LDS, as the ordered-commit kernel does (in the slab
    // too when it does not fit: measured 43 vs ~20 us per fantasy_vs tick)
    const CommitArgs &A = I.commit;
    const size_t ws = detail::commitWorkingBytes(A.shape);
    bool ws_in_lds = A.shape.capMax > 0;
    for (int32_t i = 0; i < n && ws_in_lds; i++) {
        if (I.walkable[i] == 1)
            ws_in_lds = hipx::residentBlocksNoThrow(I.resumeKernel[i], 64, ws) > 0;
    }
    I.walkLds = ws_in_lds ? ws : 0;
    I.walkWsBytes = ws_in_lds ? 0 : (ws + 255) / 256 * 256;
    I.walkPerBlock = I.walkWsBytes + (A.scratchPerBlock + 255) / 256 * 256;
    int64_t max_resume = 1;
    I.walkGrid.clear();
    auto add_grid = [&](const void *k, bool resume) {
        for (auto &g : I.walkGrid) {
            if (g.first == k) return;
        }
        const int32_t per_cu = hipx::residentBlocks(k, resume ? "worldResumeKernel" : "worldWalkKernel", 64,
                                                    resume ? I.walkLds : 0);
        int64_t grid = std::min<int64_t>(I.cfg.numWorlds, (int64_t)per_cu * std::max(I.numCUs, 1));
        // the walk: one block per world -- the hardware dispatcher balances
        // the worlds (fantasy_vs: 120 vs 118 M env-steps/s for the resident
        // grid striding over them); MADRONA_MW_WALK_FULL_GRID=0: resident grid
        const char *fg = getenv("MADRONA_MW_WALK_FULL_GRID");
        if (!resume && !(fg && atoi(fg) == 0)) grid = I.cfg.numWorlds;
        if (resume) {
            // enough blocks for the usual handful of stopped worlds; slabs
            // bounded to 256 MiB
            grid = std::min<int64_t>(grid, std::max<int64_t>(1, (256ll << 20) / (int64_t)I.walkPerBlock));
            max_resume = std::max(max_resume, grid);
        }
        I.walkGrid.push_back({ k, (int32_t)std::max<int64_t>(grid, 1) });
    };
    for (int32_t i = 0; i < n; i++) {
        if (I.walkable[i] != 1) continue;
        add_grid(I.walkKernel[i], false);
        add_grid(I.resumeKernel[i], true);
    }
    if (I.walkScratch) {
        MW_HIP_CHECK(hipFree(I.walkScratch));
        I.walkScratch = nullptr;
    }
    MW_HIP_CHECK(hipMalloc(&I.walkScratch, std::max<size_t>(I.walkPerBlock * max_resume, 256)));
}

static int32_t walkGridOf(const Executor::Impl &I, const void *kernel)
{
    for (auto &g : I.walkGrid) {
        if (g.first == kernel) return g.second;
    }
    return 1;
}

// One walk run: the walk over every world, then (if the run has commit
// points) the resume pass over the worlds that stopped at one.
static void launchWorldWalk(Executor::Impl &I, LaunchCtx &lc, int32_t b, int32_t e, bool commits)
{
    const void *walk = I.walkKernel[b], *resume = I.resumeKernel[b];
    const detail::WalkEntry *entries = I.walkEntriesDev + I.walkOff[b];
    int32_t n = I.walkOff[e] - I.walkOff[b];
    StateView *st = lc.devState;
    int32_t *res = I.walkResume;
    {
        void *args[] = { &entries, &n, &st, &res };
        hipx::residentBlocks(walk, "worldWalkKernel", 64, 0);
        MW_HIP_CHECK(hipx::launchKernel(walk, dim3((uint32_t)walkGridOf(I, walk)), dim3(64), args, 0, I.stream));
        hipx::checkLaunched("worldWalkKernel");
    }
    if (!commits) return;
    char *scratch = I.walkScratch;
    uint64_t per_block = I.walkPerBlock, ws_bytes = I.walkWsBytes;
    detail::CommitShape shape = I.commit.shape;
    void *args[] = { &entries, &n, &st, &res, &scratch, &per_block, &shape, &ws_bytes };
    hipx::residentBlocks(resume, "worldResumeKernel", 64, I.walkLds);
    MW_HIP_CHECK(hipx::launchKernel(resume, dim3((uint32_t)walkGridOf(I, resume)), dim3(64), args,
                                    I.walkLds, I.stream));
    hipx::checkLaunched("worldResumeKernel");
}

// The end of the walk run starting at node k within [k, e): a maximal run of
// walkable nodes of one walk kernel with at least two real nodes; k + 1 when
// node k starts none (tracing keeps per-node launches, for its markers).
static int32_t walkRunEnd(const Executor::Impl &I, int32_t k, int32_t e)
{
    if (I.trace || k >= (int32_t)I.walkable.size() || I.walkable[k] != 1) return k + 1;
    const void *kern = I.walkKernel[k];
    int32_t j = k, real = 0;
    while (j < e && (I.walkable[j] == 2 || (I.walkable[j] == 1 && I.walkKernel[j] == kern))) {
        real += I.walkable[j] == 1;
        j++;
    }
    return real >= 2 ? j : k + 1;
}

// Nodes [k, j) as one unit: a walk run (walkRunEnd) or the single node k.
static void launchUnit(Executor::Impl &I, int32_t k, int32_t j, LaunchCtx &lc)
{
    if (j > k + 1) {
        bool commits = false;
        for (int32_t q = k; q < j; q++) commits |= I.walkCommits[q] != 0;
        launchWorldWalk(I, lc, k, j, commits);
    } else {
        launchNode(I, k, lc);
    }
}

// Nodes [b, e) in order, walk runs as one walk launch each, the rest node by
// node.
static void launchRange(Executor::Impl &I, int32_t b, int32_t e, LaunchCtx &lc)
{
    for (int32_t k = b; k < e;) {
        const int32_t j = walkRunEnd(I, k, e);
        launchUnit(I, k, j, lc);
        k = j;
    }
}

// One step's launch sequence: every node in sorted order, then the export
// gathers.  Nodes of the timed kind are bracketed by their own event pair.
static void launchStep(Executor::Impl &I, LaunchCtx &lc, const StateView &dv)
{
    traceStepBegin(I);
    int32_t start = 0;
    for (int32_t i = 0; i < I.graph.numNodes(); i++) {
        if (i >= start && isTimed(I, i)) {
            launchRange(I, start, i, lc);
            const int32_t j = walkRunEnd(I, i, I.graph.numNodes());
            launchNodeTimed(I, i, j, lc);
            start = j;
        }
    }
    launchRange(I, start, I.graph.numNodes(), lc);
    launchExports(I, dv);
    traceStepEnd(I);
}

static void destroySegments(std::vector<Executor::Impl::Segment> &segs)
{
    for (auto &sg : segs) {
        if (sg.exec) MW_HIP_CHECK(hipGraphExecDestroy(sg.exec));
        if (sg.graph) MW_HIP_CHECK(hipGraphDestroy(sg.graph));
    }
    segs.clear();
}

static void captureSegments(Executor::Impl &I, LaunchCtx &lc, const StateView &dv, bool split);

// K plain steps back to back in one graph (the unsplit step's launches and
// exports, K times); none while tracing (each step brackets its records).
static void captureMultiStep(Executor::Impl &I, LaunchCtx &lc, const StateView &dv)
{
    destroySegments(I.multiSegs);
    I.multiK = 0;
    // with sampled live timing the plain runs are timedEvery - 1 steps long
    int32_t K = I.stepsPerGraph;
    if (I.timedPerStep > 0) K = I.timedEvery > 1 ? std::min(K, I.timedEvery - 1) : 0;
    if (K <= 1 || I.trace) return;
    Executor::Impl::Segment sg;
    MW_HIP_CHECK(hipStreamBeginCapture(I.stream, hipStreamCaptureModeThreadLocal));
    try {
        for (int32_t k = 0; k < K; k++) {
            launchRange(I, 0, I.graph.numNodes(), lc);
            launchExports(I, dv);
        }
    } catch (...) {
        hipGraph_t partial = nullptr;
        (void)hipStreamEndCapture(I.stream, &partial);
        if (partial) (void)hipGraphDestroy(partial);
        (void)hipGetLastError();
        throw;
    }
    MW_HIP_CHECK(hipStreamEndCapture(I.stream, &sg.graph));
    if (!sg.graph) throw std::runtime_error("multi-step graph capture returned no graph");
    MW_HIP_CHECK(hipGraphInstantiate(&sg.exec, sg.graph, nullptr, nullptr, 0));
    I.multiSegs.push_back(sg);
    I.multiK = K;
}

static void captureGraph(Executor::Impl &I, LaunchCtx &lc, const StateView &dv)
{
    destroySegments(I.segs);
    destroySegments(I.plainSegs);
    captureSegments(I, lc, dv, true);
    if (I.timedPerStep > 0 && I.timedEvery > 1) {
        std::swap(I.segs, I.plainSegs);
        captureSegments(I, lc, dv, false);
        std::swap(I.segs, I.plainSegs);
    }
    captureMultiStep(I, lc, dv);
}

// The step graph into I.segs; split: at every launch of the timed kind.
static void captureSegments(Executor::Impl &I, LaunchCtx &lc, const StateView &dv, bool split)
{
    const int32_t n = I.graph.numNodes();
    // Live node timing splits the step graph at each launch of the timed
    // kind, which runs on the stream between segments bracketed by events:
    // HIP here refuses event records captured into a graph for timing
    // (hipEventRecordWithFlags(..., hipEventRecordExternal) during capture:
    // "invalid argument" on the MI355X box).  Cost measured there: +2 % per
    // step with SolverNode timed (4 splits).
    int32_t start = 0;
    for (int32_t i = 0; i <= n; i++) {
        const bool last = i == n;
        if (!last && !(split && i >= start && isTimed(I, i))) continue;
        Executor::Impl::Segment sg;
        sg.timedNode = last ? -1 : i;
        sg.timedEnd = last ? -1 : walkRunEnd(I, i, n);
        if (i > start || last || (start == 0 && I.trace)) {
            MW_HIP_CHECK(hipStreamBeginCapture(I.stream, hipStreamCaptureModeThreadLocal));
            try {
                if (start == 0) traceStepBegin(I);
                launchRange(I, start, i, lc);
                if (last) {
                    launchExports(I, dv);
                    traceStepEnd(I);
                }
            } catch (...) {
                // a launch refused its shape: leave the stream usable
                hipGraph_t partial = nullptr;
                (void)hipStreamEndCapture(I.stream, &partial);
                if (partial) (void)hipGraphDestroy(partial);
                (void)hipGetLastError();
                throw;
            }
            MW_HIP_CHECK(hipStreamEndCapture(I.stream, &sg.graph));
            if (!sg.graph) throw std::runtime_error("step graph capture returned no graph");
            MW_HIP_CHECK(hipGraphInstantiate(&sg.exec, sg.graph, nullptr, nullptr, 0));
        }
        I.segs.push_back(sg);
        start = last ? n + 1 : sg.timedEnd;
    }
}

// The reference's launch-configuration environment (src/mw/cuda_exec.cpp:
// 1534-1560): the override sets the default blocks per CU (and the CU
// count), the file one value per node index; both are read when the step
// graph is captured.  Node indices past the graph are an error here (the
// reference silently grows its table).
static void applyLaunchConfigEnv(Executor::Impl &I)
{
    int dev = 0, cus = 0;
    MW_HIP_CHECK(hipGetDevice(&dev));
    MW_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    I.numCUs = cus;
    I.nodeBlocksPerCU.assign(I.graph.numNodes(), -1);
    if (const char *ov = std::getenv("MADRONA_MWGPU_EXEC_CONFIG_OVERRIDE")) {
        const ExecConfigOverride o = parseExecConfigOverride(ov);
        I.defaultBlocksPerCU = (int32_t)o.blocksPerCU;
        if (o.numCUs > 0) I.numCUs = (int32_t)o.numCUs;
        std::fprintf(stderr, "Using %u %u %u as the default launch configuration\n",
                     o.numThreads, o.blocksPerCU, (unsigned)I.numCUs);
    }
    if (const char *path = std::getenv("MADRONA_MWGPU_EXEC_CONFIG_FILE")) {
        std::ifstream f(path);
        if (!f) throw std::runtime_error(std::string("MADRONA_MWGPU_EXEC_CONFIG_FILE: cannot open ") + path);
        std::stringstream ss;
        ss << f.rdbuf();
        for (const NodeBlocks &nb : parseExecConfigFile(ss.str())) {
            if (nb.node < 0 || nb.node >= I.graph.numNodes()) {
                throw std::runtime_error("MADRONA_MWGPU_EXEC_CONFIG_FILE: node index past the graph");
            }
            I.nodeBlocksPerCU[nb.node] = nb.blocksPerCU;
            std::fprintf(stderr, "Taskgraph node %d (%s): using %d blocks per CU\n", nb.node,
                         I.graph.nodeName(nb.node), nb.blocksPerCU);
        }
    }
}

int32_t Executor::numNodes() const { return impl_->graph.numNodes(); }

int32_t Executor::worldWalkRuns() const
{
    const Impl &I = *impl_;
    const int32_t n = (int32_t)I.walkable.size();
    int32_t runs = 0;
    for (int32_t k = 0; k < n;) {
        const int32_t j = ::madrona::walkRunEnd(I, k, n);
        runs += j > k + 1;
        k = j;
    }
    return runs;
}

int32_t Executor::walkRunEnd(int32_t node) const
{
    const int32_t n = impl_->graph.numNodes();
    if (node < 0 || node >= n) throw std::runtime_error("walkRunEnd: node index past the graph");
    return ::madrona::walkRunEnd(*impl_, node, n);
}
const char *Executor::nodeName(int32_t node) const
{
    if (node < 0 || node >= impl_->graph.numNodes()) return nullptr;
    return impl_->graph.nodeName(node);
}

int32_t Executor::nodeBlocksPerCU(int32_t node) const
{
    if (node < 0) return impl_->defaultBlocksPerCU;
    if (node >= impl_->graph.numNodes()) return -1;
    const int32_t v = impl_->nodeBlocksPerCU[node];
    return v >= 0 ? v : impl_->defaultBlocksPerCU;
}

void Executor::setNodeBlocksPerCU(int32_t node, int32_t blocks_per_cu)
{
    Impl &I = *impl_;
    if (node >= I.graph.numNodes() || node < -1 || blocks_per_cu < -1 ||
        blocks_per_cu > kMaxBlocksPerCU || (node < 0 && blocks_per_cu < 0)) {
        throw std::runtime_error("setNodeBlocksPerCU: bad node index or block count");
    }
    sync();
    if (node < 0) {
        I.defaultBlocksPerCU = blocks_per_cu;
    } else {
        I.nodeBlocksPerCU[node] = blocks_per_cu;
    }
    const StateView &dv = I.mgr->deviceViewHost();
    LaunchCtx lc = makeLaunchCtx(I, this);
    if (I.cfg.useGraph) captureGraph(I, lc, dv);
}

void Executor::setGraph(TaskGraph &&graph)
{
    impl_->graph = std::move(graph);
    {
        const TaskGraph &g = impl_->graph;
        impl_->nodeSkip.assign(g.numNodes(), 0);
        bool alloc_since = true;
        for (int32_t i = 0; i < g.numNodes(); i++) {
            const uint32_t f = g.nodeFlags(i);
            if (f & TaskGraph::kNodeTmpAllocReset) {
                impl_->nodeSkip[i] = alloc_since ? 0 : 1;
                alloc_since = false;
            } else if (!(f & TaskGraph::kNodeNoTmpAlloc)) {
                alloc_since = true;
            }
        }
    }
    // Node data blocks to the device; NodeBase-derived blocks learn the
    // device state first (NodeBase::makeContext).
    {
        const TaskGraph &g = impl_->graph;
        const int32_t nd = g.numNodeDatas();
        if (nd > 0) {
            std::vector<TaskGraph::NodeData> blocks(g.nodeDatas(), g.nodeDatas() + nd);
            for (int32_t i = 0; i < nd; i++) {
                if (!g.nodeDataIsNodeBase(i)) continue;
                NodeBase *nb = (NodeBase *)blocks[i].userData;
                nb->mwState = impl_->mgr->deviceView();
                nb->mwNumWorlds = impl_->cfg.numWorlds;
            }
            const size_t bytes = sizeof(TaskGraph::NodeData) * nd;
            MW_HIP_CHECK(hipMalloc(&impl_->nodeDataDev, bytes));
            MW_HIP_CHECK(hipMemcpy(impl_->nodeDataDev, blocks.data(), bytes, hipMemcpyHostToDevice));
        }
    }
    applyLaunchConfigEnv(*impl_);
    if (const char *e = std::getenv("MADRONA_MW_STEPS_PER_GRAPH")) impl_->stepsPerGraph = std::max(1, atoi(e));
    const StateView &dv = impl_->mgr->deviceViewHost();
    LaunchCtx lc = makeLaunchCtx(*impl_, this);
    planWorldWalk(*impl_, lc);
    if (impl_->cfg.useGraph) captureGraph(*impl_, lc, dv);
}

static bool growTables(Executor &E, Executor::Impl &I);

void Executor::runAsync()
{
    Impl &I = *impl_;
    growTables(*this, I);
    const StateView &dv = I.mgr->deviceViewHost();
    LaunchCtx lc = makeLaunchCtx(I, this);
    // sampled timing: the first step of every run of timedEvery is the
    // split, timed one
    const bool sampled = I.plainSegs.empty() || I.stepIndex % I.timedEvery == 0;
    I.stepIndex++;
    if (!I.segs.empty()) {
        for (auto &sg : sampled ? I.segs : I.plainSegs) {
            if (sg.exec) MW_HIP_CHECK(hipGraphLaunch(sg.exec, I.stream));
            if (sg.timedNode >= 0) launchNodeTimed(I, sg.timedNode, sg.timedEnd, lc);
        }
    } else {
        launchStep(I, lc, dv);
    }
    I.stepsEnqueued++;
    I.stepsRun++;
    enqueueGrowProbe(I);
}

// Is step `idx` an unsplit step?  With live timing every step is split
// (timedEvery 1) or the first of every run of timedEvery is.
static bool plainStep(const Executor::Impl &I, int64_t idx)
{
    if (I.timedPerStep == 0) return true;
    return !I.plainSegs.empty() && idx % I.timedEvery != 0;
}

void Executor::runSteps(int32_t n)
{
    Impl &I = *impl_;
    const int32_t K = I.multiK;
    for (int32_t i = 0; i < n;) {
        // growable tables: one step per launch, so the growth check runs
        // between any two steps
        bool multi = !I.multiSegs.empty() && n - i >= K && I.growable.n == 0;
        for (int32_t k = 0; multi && k < K; k++) multi = plainStep(I, I.stepIndex + k);
        if (multi) {
            MW_HIP_CHECK(hipGraphLaunch(I.multiSegs[0].exec, I.stream));
            I.stepIndex += K;
            I.stepsRun += K;
            i += K;
        } else {
            runAsync();
            i++;
        }
    }
}

// Table growth between steps (reference Table::addRow, src/common/table.cpp:
// 44-61, x2 when full; the reference's device runtime grows by device
// malloc).  Behind every enqueued step a probe copies the growable tables'
// largest per-world row counts to pinned host memory (enqueueGrowProbe).
// Before the next step is enqueued the host reads the probes that have
// finished and waits for older ones only while the rows of the steps it has
// not seen, projected at the largest per-step rise seen so far, could pass a
// table's capacity (enqueueSafe), or more than growLag steps are unseen.  A
// table past half full, or without room for growLag + 1 steps at that rise,
// then doubles (neededCapacity) before the step is enqueued.  So the tables
// grow between any two steps -- inside mw_step(n), async bursts and at every
// sync -- without a host synchronisation per step; a step whose rows rise
// past any rise seen before (or that fills a table inside itself) still
// overflows and raises the table-full flag.  The growth itself is a
// synchronisation point: it re-strides the slabs
// (StateManager::growArchetype), extends the export buffers of that
// archetype in place (mapping more of their reserved range), resizes the
// commit scratch and re-plans / re-captures the step.
static bool growTables(Executor &E, Executor::Impl &I)
{
    if (I.growable.n == 0) return false;
    drainGrowProbes(I, false);
    while (I.probeCount > 0 && (I.probeCount > I.growLag || !enqueueSafe(I))) consumeOldestProbe(I, true);
    if (!growthDue(I)) return false;
    MW_HIP_CHECK(hipStreamSynchronize(I.stream));
    drainGrowProbes(I, true);                   // every step so far
    const StateView &dv = I.mgr->deviceViewHost();
    bool grown = false;
    for (int32_t i = 0; i < I.growable.n; i++) {
        const int32_t a = I.growable.arch[i];
        const int32_t cap = dv.arch[a].capacity;
        const int64_t nc = neededCapacity(I, i, cap);
        if (nc <= cap) continue;
        if (nc > (1 << 28)) throw std::runtime_error("table growth past 2^28 rows per world");
        I.mgr->growArchetype(a, (int32_t)nc, I.stream);
        for (ExportBuf &b : I.exports) {
            if (b.archetype != a) continue;
            const size_t old_bytes = std::max<size_t>((size_t)dv.numWorlds * cap * b.bytes, 256);
            const size_t new_bytes = std::max<size_t>((size_t)dv.numWorlds * nc * b.bytes, 256);
            if (b.mem.reserved > 0 && mapExportMem(b, new_bytes, I.cfg.gpuID)) continue;
            // no reserved range (or past it): a new buffer with the packed
            // rows of the last step copied over
            char *nb = nullptr;
            MW_HIP_CHECK(hipMalloc(&nb, new_bytes));
            MW_HIP_CHECK(hipMemcpyAsync(nb, b.buf, old_bytes, hipMemcpyDeviceToDevice, I.stream));
            MW_HIP_CHECK(hipStreamSynchronize(I.stream));
            releaseExportMem(b);
            b.buf = nb;
            b.relocations++;
        }
        grown = true;
    }
    if (!grown) return false;
    I.growths++;
    setupCommit(I);
    LaunchCtx lc = makeLaunchCtx(I, &E);
    planWorldWalk(I, lc);
    if (I.cfg.useGraph) captureGraph(I, lc, I.mgr->deviceViewHost());
    return true;
}

void Executor::sync()
{
    Impl &I = *impl_;
    MW_HIP_CHECK(hipStreamSynchronize(I.stream));
    // every enqueued step's timed launches since the last sync
    I.timedMs += drainTimedPairs(I);
    I.timedLaunches += I.timedUnits;
    I.timedUnits = 0;
    // the probes behind the last step are complete: no launch, no second sync
    drainGrowProbes(I, true);
    if (growthDue(I)) growTables(*this, I);
    // extensions that change their launches from what the steps measured
    // (the physics module's solver lanes) ask for a re-capture here
    if (I.mgr->pollExtensions(I.stream, I.stepsRun)) {
        LaunchCtx lc = makeLaunchCtx(I, this);
        if (I.cfg.useGraph) captureGraph(I, lc, I.mgr->deviceViewHost());
    }
}

void Executor::run()
{
    runAsync();
    sync();
}

static void setTimed(Executor &E, Executor::Impl &I, const char *name, int32_t index, int32_t every)
{
    E.sync();
    I.timedName = name ? name : "";
    I.timedIndex = index;
    I.timedEvery = std::max(1, every);
    I.stepIndex = 0;
    I.timedMs = 0.0;
    I.timedLaunches = 0;
    I.timedPerStep = 0;
    for (int32_t i = 0; i < I.graph.numNodes(); i++) I.timedPerStep += isTimed(I, i);
    const StateView &dv = I.mgr->deviceViewHost();
    LaunchCtx lc = makeLaunchCtx(I, &E);
    if (I.cfg.useGraph) captureGraph(I, lc, dv);
}

void Executor::setTimedNode(const char *name, int32_t every)
{
    setTimed(*this, *impl_, name, -1, every);
}

void Executor::setTimedNodeIndex(int32_t node, int32_t every)
{
    if (node < 0 || node >= impl_->graph.numNodes()) {
        throw std::runtime_error("setTimedNodeIndex: node index past the graph");
    }
    setTimed(*this, *impl_, impl_->graph.nodeName(node), node, every);
}

void Executor::enableTracing(int64_t max_records)
{
    Impl &I = *impl_;
    sync();
    if (I.trace) {
        mwGPU::setTracePointer(nullptr);
        MW_HIP_CHECK(hipFree(I.trace));
        MW_HIP_CHECK(hipFree(I.traceLogs));
        I.trace = nullptr;
        I.traceLogs = nullptr;
    }
    if (max_records > 0) {
        if (max_records > 0xffffffffll) throw std::runtime_error("tracing: too many records");
        int rate_khz = 0;
        MW_HIP_CHECK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate,
                                           I.cfg.gpuID));
        if (rate_khz <= 0) rate_khz = 100000;
        MW_HIP_CHECK(hipMalloc(&I.traceLogs, sizeof(mwGPU::DeviceLog) * (size_t)max_records));
        MW_HIP_CHECK(hipMalloc(&I.trace, sizeof(mwGPU::TraceDev)));
        mwGPU::TraceDev t {};
        t.capacity = (uint32_t)max_records;
        t.nsPerTick = (uint32_t)std::max(1, 1000000 / rate_khz);
        t.logs = I.traceLogs;
        MW_HIP_CHECK(hipMemcpy(I.trace, &t, sizeof(t), hipMemcpyHostToDevice));
        mwGPU::setTracePointer(I.trace);
        // funcID: node kind, numbered in first-appearance order
        I.traceFuncs.clear();
        I.nodeFunc.clear();
        for (int32_t i = 0; i < I.graph.numNodes(); i++) {
            const std::string name = I.graph.nodeName(i);
            auto it = std::find(I.traceFuncs.begin(), I.traceFuncs.end(), name);
            I.nodeFunc.push_back((uint32_t)(it - I.traceFuncs.begin()));
            if (it == I.traceFuncs.end()) I.traceFuncs.push_back(name);
        }
        I.traceFuncs.push_back("ExportNode");
    }
    MW_HIP_CHECK(hipDeviceSynchronize());
    const StateView &dv = I.mgr->deviceViewHost();
    LaunchCtx lc = makeLaunchCtx(I, this);
    if (I.cfg.useGraph) captureGraph(I, lc, dv);
}

int64_t Executor::readTrace(void *dst, int64_t max_bytes, int64_t *dropped)
{
    Impl &I = *impl_;
    sync();
    if (!I.trace) return -1;
    mwGPU::TraceDev t {};
    MW_HIP_CHECK(hipMemcpy(&t, I.trace, sizeof(t), hipMemcpyDeviceToHost));
    const int64_t n = std::min<int64_t>(t.next, t.capacity);
    if (dropped) *dropped = t.dropped;
    const int64_t bytes = n * (int64_t)sizeof(mwGPU::DeviceLog);
    if (dst) {
        MW_HIP_CHECK(hipMemcpy(dst, I.traceLogs, (size_t)std::min(bytes, std::max<int64_t>(0, max_bytes)),
                               hipMemcpyDeviceToHost));
    }
    return bytes;
}

const char *Executor::traceFuncName(int32_t func_id)
{
    if (func_id < 0 || func_id >= (int32_t)impl_->traceFuncs.size()) return nullptr;
    return impl_->traceFuncs[func_id].c_str();
}

double Executor::timedNodeMs(int64_t *launches)
{
    sync();
    if (launches) *launches = impl_->timedLaunches;
    return impl_->timedMs;
}

// The packed row total is read on the executor stream (into pinned host
// memory), so it is the total of the last enqueued step even after
// runAsync(); a null-stream hipMemcpy would not wait for the non-blocking
// executor stream.
static int64_t *pinnedRowsTotal(Executor::Impl &I)
{
    if (!I.hostRowsTotal) MW_HIP_CHECK(hipHostMalloc(&I.hostRowsTotal, sizeof(int64_t)));
    return I.hostRowsTotal;
}

void *Executor::getExported(int32_t slot, int64_t *num_rows)
{
    for (ExportBuf &b : impl_->exports) {
        if (b.slot == slot) {
            if (num_rows) {
                int64_t *total = pinnedRowsTotal(*impl_);
                MW_HIP_CHECK(hipMemcpyAsync(total, b.offsets + impl_->cfg.numWorlds, sizeof(int64_t),
                                            hipMemcpyDeviceToHost, impl_->stream));
                sync();
                *num_rows = *total;
            }
            return b.buf;
        }
    }
    return nullptr;
}

// Stream-ordered copy of the packed rows into dst with one host sync: the
// copy spans min(max_bytes, the export buffer) -- bytes of dst past the
// returned count are unspecified -- and the row total travels with it.
int64_t Executor::copyExported(int32_t slot, void *dst, int64_t max_bytes)
{
    for (ExportBuf &b : impl_->exports) {
        if (b.slot != slot) continue;
        const StateView &dv = impl_->mgr->deviceViewHost();
        const int64_t buf_bytes = (int64_t)dv.numWorlds * dv.arch[b.archetype].capacity * b.bytes;
        const int64_t span = std::min(std::max<int64_t>(max_bytes, 0), buf_bytes);
        int64_t *total = pinnedRowsTotal(*impl_);
        MW_HIP_CHECK(hipMemcpyAsync(total, b.offsets + impl_->cfg.numWorlds, sizeof(int64_t),
                                    hipMemcpyDeviceToHost, impl_->stream));
        if (span > 0) {
            MW_HIP_CHECK(hipMemcpyAsync(dst, b.buf, (size_t)span, hipMemcpyDefault, impl_->stream));
        }
        sync();
        return std::min(*total * (int64_t)b.bytes, span);
    }
    return -1;
}

// Device-side hand-off: the copy is enqueued on the executor stream behind
// the steps enqueued so far and the host does not wait (the learner orders
// its stream after it with mw_stream_wait).  dst receives min(max_bytes, the
// export buffer) bytes; bytes past the packed rows are unspecified.
int64_t Executor::copyExportedAsync(int32_t slot, void *dst, int64_t max_bytes)
{
    for (ExportBuf &b : impl_->exports) {
        if (b.slot != slot) continue;
        const StateView &dv = impl_->mgr->deviceViewHost();
        const int64_t buf_bytes = (int64_t)dv.numWorlds * dv.arch[b.archetype].capacity * b.bytes;
        const int64_t span = std::min(std::max<int64_t>(max_bytes, 0), buf_bytes);
        if (span > 0) {
            MW_HIP_CHECK(hipMemcpyAsync(dst, b.buf, (size_t)span, hipMemcpyDeviceToDevice,
                                        impl_->stream));
        }
        return span;
    }
    return -1;
}

int32_t Executor::exportRowBytes(int32_t slot)
{
    for (ExportBuf &b : impl_->exports) {
        if (b.slot == slot) return (int32_t)b.bytes;
    }
    return 0;
}

int64_t Executor::exportBufferBytes(int32_t slot)
{
    const StateView &dv = impl_->mgr->deviceViewHost();
    for (ExportBuf &b : impl_->exports) {
        if (b.slot == slot) return (int64_t)dv.numWorlds * dv.arch[b.archetype].capacity * b.bytes;
    }
    return -1;
}

void Executor::copyOutExports() { launchExports(*impl_, impl_->mgr->deviceViewHost()); }

void *Executor::columnBase(int32_t archetype, int32_t column, int32_t *capacity, uint32_t *bytes)
{
    const StateView &dv = impl_->mgr->deviceViewHost();
    if (archetype < 0 || archetype >= dv.numArchetypes) return nullptr;
    const ArchetypeView &av = dv.arch[archetype];
    if (column < 0 || column >= av.numColumns) return nullptr;
    if (capacity) *capacity = av.capacity;
    if (bytes) *bytes = av.colBytes[column];
    return av.cols[column];
}

int32_t Executor::numRows(int32_t archetype, int32_t world)
{
    const StateView &dv = impl_->mgr->deviceViewHost();
    int32_t n = 0;
    MW_HIP_CHECK(hipMemcpy(&n, dv.arch[archetype].numRows + world, sizeof(int32_t),
                           hipMemcpyDeviceToHost));
    return n;
}

double Executor::timeNode(const char *name, int32_t num_steps)
{
    Impl &I = *impl_;
    sync();        // live timing so far is accounted before the pool is reused
    const StateView &dv = I.mgr->deviceViewHost();
    LaunchCtx lc = makeLaunchCtx(I, this);
    for (int32_t s = 0; s < num_steps; s++) {
        for (int32_t i = 0; i < I.graph.numNodes(); i++) {
            if (strcmp(I.graph.nodeName(i), name) == 0) {
                launchNodeTimed(I, i, i + 1, lc);
            } else {
                launchNode(I, i, lc);
            }
        }
        launchExports(I, dv);
        I.stepsEnqueued++;
        enqueueGrowProbe(I);
    }
    MW_HIP_CHECK(hipStreamSynchronize(I.stream));
    const int64_t units = I.timedUnits;
    const double total = drainTimedPairs(I);
    I.timedUnits = 0;
    return units == 0 ? -1.0 : total / (double)units;
}

bool Executor::entityLoc(int32_t world, Entity e, Loc *out)
{
    sync();
    const StateView &dv = impl_->mgr->deviceViewHost();
    if (world < 0 || world >= dv.numWorlds) return false;
    IDMapState st {};
    MW_HIP_CHECK(hipMemcpy(&st, dv.idState + world, sizeof(st), hipMemcpyDeviceToHost));
    if (e.id < 0 || e.id >= st.numIDs) return false;
    IDNode n {};
    MW_HIP_CHECK(hipMemcpy(&n, dv.idNodes + (size_t)world * dv.idsPerWorld + e.id, sizeof(n),
                           hipMemcpyDeviceToHost));
    if (n.gen != e.gen) return false;
    *out = n.val;
    return true;
}

void Executor::downloadState() { impl_->mgr->downloadFromDevice(impl_->stream); }
const StateView &Executor::hostView() { return impl_->mgr->hostView(); }

// Ordered on the executor stream behind every enqueued step (the stream is
// non-blocking, so a null-stream copy could read flags from before them).
int32_t Executor::errorFlags()
{
    const StateView &dv = impl_->mgr->deviceViewHost();
    std::vector<int32_t> f(dv.numWorlds);
    MW_HIP_CHECK(hipMemcpyAsync(f.data(), dv.errorFlags, sizeof(int32_t) * dv.numWorlds,
                                hipMemcpyDeviceToHost, impl_->stream));
    sync();
    int32_t r = 0;
    for (int32_t v : f) r |= v;
    return r;
}

}
