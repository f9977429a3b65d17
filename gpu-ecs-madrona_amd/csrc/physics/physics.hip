// MI355X rigid-body physics: the gfx950 back end of the physics module --
// device slabs, launch sizing and the graph nodes that launch the kernels of
// broadphase.hip / narrowphase.hip / solver.hip (the host side shared with
// the CPU back end is physics_host.cpp).
//
// Reference: src/physics/{physics,broadphase,narrowphase,geometry}.cpp and
// include/madrona/physics.{hpp,inl}.  Every kernel processes ALL worlds in one
// launch.  Float evaluation order follows the reference CPU path exactly
// (see include/madrona/math.hpp); DESIGN.md §3 lists kernel <-> reference
// function correspondences and the parallel-but-order-preserving schemes:
//   * candidates: per-world block scan keeps the reference's
//     (row order, BVH DFS order) candidate sequence;
//   * narrowphase: one lane per candidate, results stored per candidate slot
//     and compacted in candidate order;
//   * XPBD solver: contacts are level-scheduled per world: a contact's level
//     is 1 + the max level of earlier contacts sharing a non-static body, so
//     all contacts of one level touch disjoint bodies and commute exactly;
//     the result equals the reference's serial Gauss-Seidel sweep bit for bit.
#include "physics_module.hpp"
#include "physics_device.hpp"

#include <hip/hip_runtime.h>

#include "../runtime/hip_launch.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace madrona::phys {

using namespace math;
using namespace base;

#if defined(MW_SAT_CUTS)
static const PhysArgs *g_cutArgs = nullptr;     // mw_debug_time_sat
#endif


PhysicsModule::~PhysicsModule()
{
    for (void *p : allocs) (void)hipFree(p);
}

void *PhysicsModule::rawAlloc(size_t bytes, void *stream)
{
    void *p = nullptr;
    MW_HIP_CHECK(hipMalloc(&p, bytes));
    MW_HIP_CHECK(hipMemsetAsync(p, 0, bytes, (hipStream_t)stream));
    allocs.push_back(p);
    return p;
}

void PhysicsModule::rawCopy(void *dst, const void *src, size_t bytes, void *stream)
{
    MW_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
}

// Launch sizing and the LDS-image decision of every LDS-staging kernel.  A
// kernel whose image (a world's leaves, BVH nodes or bodies; a block's hull
// staging or clip polygons) does not fit a workgroup's LDS runs its
// global-image variant (the same code on a global slab: same bits); a shape
// that cannot launch either way throws here, at mw_create, naming the kernel
// and the bytes (hip_launch.hpp).  MADRONA_MW_FORCE_GLOBAL_IMAGES=1 selects
// the global variants everywhere (the parity tests of the fallback).
// The solver's lane variant, once, from the level widths of the worlds' last
// solve (the stream is idle at a poll).
bool PhysicsModule::poll(void *stream_ptr, int64_t steps)
{
    if (!uploaded || solverLanesMode != 0 || steps < solverLanesNextCheck) return false;
    const int32_t W = args.numWorlds;
    std::vector<uint32_t> st(W);
    MW_HIP_CHECK(hipMemcpyAsync(st.data(), args.solverLevelStats, sizeof(uint32_t) * W, hipMemcpyDeviceToHost,
                                (hipStream_t)stream_ptr));
    MW_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream_ptr));
    double items = 0, levels = 0;
    for (uint32_t v : st) {
        items += v & 0xffffu;
        levels += v >> 16;
    }
    if (levels == 0) return false;                   // no contacts yet: ask again at the next sync
    solverLanesNextCheck = steps + kSolverLanesEvery;
    solverItemsPerLevel = items / levels;
    int32_t lanes = solverLanes;
    if (solverItemsPerLevel <= kSolverNarrowLevel) lanes = 32;
    if (solverItemsPerLevel >= kSolverWideLevel) lanes = 64;
    if (lanes == solverLanes) return false;
    solverLanes = lanes;
    args.solverImage = solverImages[lanes == 32];
    return true;
}

void PhysicsModule::upload(void *stream_ptr)
{
    if (!initialized) return;          // physics types registered but never used
    buildArgs(stream_ptr);
    PhysArgs &P = args;
    int dev = 0, cus = 0;
    MW_HIP_CHECK(hipGetDevice(&dev));
    MW_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const char *force_env = std::getenv("MADRONA_MW_FORCE_GLOBAL_IMAGES");
    const bool force = force_env && force_env[0] && force_env[0] != '0';
    auto fitsLDS = [&](const void *fn, int32_t threads, size_t lds) {
        return !force && hipx::residentBlocksNoThrow(fn, threads, lds) > 0;
    };
    const int32_t W = P.numWorlds;

    // broadphase: the BVH rebuild picks its variant per launch (<= 64 KB)
    // refit: LDS for about two thirds of the node capacity -- a rebuild uses
    // ≈0.7 nodes per leaf of the capacity's 1.33 (collisions: 81-97 of
    // 172), so the full capacity would cost blocks per CU for nodes no world
    // uses; a world past it refits in place in HBM inside the same kernel.
    // MADRONA_MW_REFIT_LDS_NODES overrides (the mixed-path parity tests).
    P.refitLDSNodes = std::min(P.maxNodes, (P.maxNodes * 2 + 2) / 3);
    if (const char *e = std::getenv("MADRONA_MW_REFIT_LDS_NODES"))
        P.refitLDSNodes = std::max(1, std::min(P.maxNodes, atoi(e)));
    P.refitGlobal = fitsLDS((const void *)&refitKernel, kRefitBlock, refitSharedBytes(P)) ? 0 : 1;
    if (P.refitGlobal) hipx::residentBlocks((const void *)&refitGlobalKernel, "refitGlobalKernel", kRefitBlock, 0);
    // findOverlaps: BVH traversal for worlds past 512 leaves (the sweep is
    // O(leaves) per body); MADRONA_MW_OVERLAP_DFS_LEAVES overrides (0: every
    // world, -1: never) -- both forms give the same candidates in the same order
    // findOverlaps keeps leaf ranks as 16-bit values (per-lane hit buffers,
    // the candidate stage): refuse a world it cannot index
    if (P.maxLeaves > 65535)
        throw std::runtime_error("physics: more than 65535 objects per world (findOverlaps leaf ranks)");
    P.overlapDFSLeaves = 512;
    if (const char *e = std::getenv("MADRONA_MW_OVERLAP_DFS_LEAVES")) P.overlapDFSLeaves = atoi(e);
    if (P.maxNodes > 32767) P.overlapDFSLeaves = -1;      // int16 traversal stack
    if (P.overlapDFSLeaves >= P.maxLeaves) P.overlapDFSLeaves = -1;   // no world traverses
    P.overlapImage = nullptr;
    if (!fitsLDS((const void *)&findOverlapsKernel, kOverlapBlock, findOverlapsSharedBytes(P))) {
        hipx::residentBlocks((const void *)&findOverlapsGlobalKernel, "findOverlapsGlobalKernel",
                             kOverlapBlock, findOverlapsGlobalSharedBytes(P));
        P.overlapImage = alloc<char>((size_t)W * findOverlapsImageBytes(P), stream_ptr);
    }
    P.dfsChunks = 0;
    P.dfsRowCap = 0;
    if (P.overlapDFSLeaves >= 0) {
        P.dfsChunks = (P.maxLeaves + kDfsBlock - 1) / kDfsBlock;
        P.dfsRowCap = P.dfsChunks * kDfsBlock;
        const size_t WL = (size_t)W * P.maxLeaves, WR = (size_t)W * P.dfsRowCap;
        P.dfsImage = alloc<char>(WL * kOrderedLeafBytes, stream_ptr);
        P.dfsKeys = alloc<int32_t>(WL * 2, stream_ptr);
        P.dfsHits = alloc<uint16_t>(WR * kOverlapBufRanks, stream_ptr);
        P.dfsRows = alloc<int32_t>(WR * 2, stream_ptr);
        P.dfsChunkTotals = alloc<int32_t>((size_t)W * P.dfsChunks, stream_ptr);
    }

    // SAT: persistent grid of exactly the blocks that can be resident (hull
    // tables in LDS up to 16 KB, else read from HBM; from HBM under
    // MADRONA_MW_FORCE_GLOBAL_IMAGES, so the fallback tests cover both)
    P.satGeoBytes = force ? 0 : (int32_t)satGeoSharedBytes(P);
#if defined(MW_SAT_CUTS)
    g_cutArgs = &args;
#endif
    // MADRONA_MW_SAT_TABLES=0: the SAT edge query without its Minkowski-test
    // tables (the per-pair form; parity tests of both)
    if (const char *t = std::getenv("MADRONA_MW_SAT_TABLES"); t && t[0] == '0') P.objs.minkStride = 0;
    P.satImage = nullptr;
    P.satImageBlocks = 0;
    const bool sat_geo = P.satGeoBytes > 0;
    const void *sat_lds = sat_geo ? (const void *)&narrowSATKernel : (const void *)&narrowSATNoGeoKernel;
    if (fitsLDS(sat_lds, kNarrowBlock, narrowphaseSharedBytes(P))) {
        P.satGrid = cus * hipx::residentBlocks(sat_lds, sat_geo ? "narrowSATKernel" : "narrowSATNoGeoKernel",
                                               kNarrowBlock, narrowphaseSharedBytes(P));
    } else {
        const int32_t per_cu = hipx::residentBlocks((const void *)&narrowSATGlobalKernel,
                                                    "narrowSATGlobalKernel", kNarrowBlock,
                                                    narrowphaseGlobalSharedBytes(P));
        P.satGrid = cus * std::min(per_cu, 2);
        P.satImageBlocks = P.satGrid;
        P.satImage = alloc<char>((size_t)P.satGrid * narrowphaseImageBytes(P), stream_ptr);
    }

    int32_t max_face_verts = 1;
    for (const HullDev &h : hulls) {
        for (int32_t f = 0; f < h.numFaces; f++) {
            int32_t n = 0;
            uint32_t e = polygons[h.faceOffset + f], start = e;
            do {
                e = hedges[h.hedgeOffset + e].next;
                n++;
            } while (e != start && n <= h.numHedges);
            max_face_verts = std::max(max_face_verts, n);
        }
    }
    // clipping an incident face against a reference face's side planes
    // yields at most |incident| + |reference| vertices
    P.clipCap = 2 * max_face_verts;
    P.clipImage = nullptr;
    P.clipImageBlocks = 0;
    if (fitsLDS((const void *)&narrowContactKernel, kContactBlock, contactSharedBytes(P))) {
        P.contactGrid = cus * hipx::residentBlocks((const void *)&narrowContactKernel,
                                                   "narrowContactKernel", kContactBlock,
                                                   contactSharedBytes(P));
    } else {
        const int32_t per_cu = hipx::residentBlocks((const void *)&narrowContactGlobalKernel,
                                                    "narrowContactGlobalKernel", kContactBlock, 0);
        P.contactGrid = cus * std::min(per_cu, 2);
        P.clipImageBlocks = P.contactGrid;
        P.clipImage = alloc<char>((size_t)P.contactGrid * contactImageBytes(P), stream_ptr);
    }
    // plane kernel: hull tables in LDS up to 16 KB, else read from HBM
    P.planeGeoBytes = force ? 0 : (int32_t)planeSharedBytes(P);
    P.planeGrid = cus * (P.planeGeoBytes > 0
                             ? hipx::residentBlocks((const void *)&narrowPlaneKernel, "narrowPlaneKernel",
                                                    kContactBlock, P.planeGeoBytes)
                             : hipx::residentBlocks((const void *)&narrowPlaneNoGeoKernel,
                                                    "narrowPlaneNoGeoKernel", kContactBlock, 0));

    // solver: both lane variants, each with its global-image slab when its
    // block image does not fit (SolverNode picks one per launch)
    for (int32_t v = 0; v < 2; v++) {
        const SolverVariant sv = v ? lanes32::solverVariant() : lanes64::solverVariant();
        const int32_t blocks = (W + sv.worldsPerBlock - 1) / sv.worldsPerBlock;
        solverImages[v] = nullptr;
        if (!fitsLDS(sv.kernel, sv.threads, sv.sharedBytes(P))) {
            hipx::residentBlocks(sv.globalKernel, v ? "solverGlobalKernel (32 lanes)" : "solverGlobalKernel",
                                 sv.threads, sv.globalSharedBytes(P));
            solverImages[v] = alloc<char>((size_t)blocks * sv.imageBytes(P), stream_ptr);
        }
    }
    P.solverLevelStats = alloc<uint32_t>(W, stream_ptr);
    solverLanesMode = 0;
    if (const char *e = std::getenv("MADRONA_MW_SOLVER_LANES")) {
        const int32_t v = atoi(e);
        if (v == 32 || v == 64) solverLanesMode = v;
        else if (strcmp(e, "auto") != 0) throw std::runtime_error("MADRONA_MW_SOLVER_LANES: 32, 64 or auto");
    }
    solverLanes = solverLanesMode ? solverLanesMode : 64;
    solverLanesNextCheck = kSolverLanesAfterSteps;
    P.solverImage = solverImages[solverLanes == 32];
    // the remaining kernels stage nothing of variable size
    hipx::residentBlocks((const void *)&narrowFilterKernel, "narrowFilterKernel", kNarrowBlock, 0);
    hipx::residentBlocks((const void *)&narrowFilterWaveKernel, "narrowFilterWaveKernel", kNarrowBlock, 0);
    uploaded = true;
}


// ===========================================================================
// Graph nodes
// ===========================================================================
static dim3 rowGrid(const PhysArgs &P)
{
    int64_t maxcap = 0;
    for (int i = 0; i < P.numBodyArchs; i++) maxcap = std::max<int64_t>(maxcap, P.body[i].capacity);
    int64_t total = (int64_t)P.numWorlds * maxcap;
    return dim3((unsigned)((total + 255) / 256), (unsigned)P.numBodyArchs);
}

struct PhysNodeBase : NodeBase {
    PhysicsModule *mod;
    explicit PhysNodeBase(Context &ctx) : mod(&physicsModule(ctxManager(ctx))) {}
};

#define MW_PHYS_NODE(NAME, BODY)                                                     \
    struct NAME : PhysNodeBase {                                                     \
        using PhysNodeBase::PhysNodeBase;                                            \
        static TaskGraph::NodeID addToGraph(Context &ctx, TaskGraph::Builder &b,     \
                                            Span<const TaskGraph::NodeID> deps)      \
        {                                                                            \
            return b.addDefaultNode<NAME>(deps, ctx);                                \
        }                                                                            \
        static const char *nodeName() { return #NAME; }                             \
        static constexpr bool kNoTmpAlloc = true;                                    \
        static void launch(NAME *self, LaunchCtx &lc)                                \
        {                                                                            \
            const PhysArgs &P = self->mod->args;                                     \
            hipStream_t stream = (hipStream_t)lc.stream;                             \
            (void)stream;                                                            \
            BODY                                                                     \
        }                                                                            \
    };

MW_PHYS_NODE(UpdateLeafPositionsNode,
    if (P.numBodyArchs > 0)
        MW_LAUNCH(leafUpdateKernel, rowGrid(P), dim3(256), 0, stream, P);)

// One wave per world while the world's leaves fit the LDS image (129 leaves:
// ≈11 KB); the lane-per-world kernel otherwise.
MW_PHYS_NODE(UpdateBVHNode,
    if (rebuildSharedBytes(P) <= 64 * 1024)
        MW_LAUNCH(bvhRebuildWaveKernel, dim3(P.numWorlds), dim3(64),
                           rebuildSharedBytes(P), stream, P);
    else
        MW_LAUNCH(bvhRebuildKernel, dim3((P.numWorlds + 63) / 64), dim3(64), 0, stream, P);)

MW_PHYS_NODE(RefitNode,
    if (P.numBodyArchs == 0) return;
    if (P.refitGlobal)
        MW_LAUNCH(refitGlobalKernel, dim3(P.numWorlds), dim3(kRefitBlock), 0, stream, P);
    else
        MW_LAUNCH(refitKernel, dim3(P.numWorlds), dim3(kRefitBlock), refitSharedBytes(P), stream, P);)

// Sweep worlds in the one-block kernels, then the traversal worlds (the
// sweep kernels skip them, the dfs kernels skip the others).
MW_PHYS_NODE(FindOverlappingNode,
    if (P.overlapImage)
        MW_LAUNCH(findOverlapsGlobalKernel, dim3(P.numWorlds), dim3(kOverlapBlock),
                  findOverlapsGlobalSharedBytes(P), stream, P);
    else if (P.maxLeaves <= kOverlapSmallLeaves && P.overlapDFSLeaves < 0)
        MW_LAUNCH(findOverlapsSmallKernel, dim3(P.numWorlds), dim3(kOverlapBlock),
                  findOverlapsSharedBytes(P), stream, P);
    else
        MW_LAUNCH(findOverlapsKernel, dim3(P.numWorlds), dim3(kOverlapBlock),
                  findOverlapsSharedBytes(P), stream, P);
    if (P.dfsChunks > 0) {
        const dim3 grid(P.numWorlds, P.dfsChunks);
        MW_LAUNCH(dfsStageKernel, grid, dim3(kDfsBlock), 0, stream, P);
        MW_LAUNCH(dfsCountKernel, grid, dim3(kDfsBlock), 0, stream, P);
        MW_LAUNCH(dfsWriteKernel, grid, dim3(kDfsBlock), 0, stream, P);
    })

// Work units of a live-timed launch (PhysArgs::unitAccum): the probe sums
// the worlds' candidates and this substep's contact manifolds -- after a
// solver launch the solver's own count (lastNumContacts), after a
// narrowphase launch the survivor slots that got a manifold -- and adds
// them to the accumulators.  Launched only behind a node whose kernels are
// bound to a timing event pair (hipx::tlTimed), outside that pair, so the
// replayed (untimed) steps never run it.
constexpr int32_t kProbeThreads = 256;
constexpr int32_t kProbeBlocks = 256;

__global__ void __launch_bounds__(kProbeThreads) unitProbeKernel(PhysArgs P, int32_t from_solver,
                                                       int32_t fused_extra)
{
    // one wave per world (grid-stride), one set of atomics per block
    const int32_t lane = threadIdx.x & 63;
    const int32_t waves = (int32_t)(gridDim.x * blockDim.x) >> 6;
    unsigned long long cands = 0, contacts = 0, survivors = 0;
    for (int32_t w = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < P.numWorlds;
         w += waves) {
        if (lane == 0) {
            cands += (unsigned long long)P.lastNumCands[w];
            if (from_solver) contacts += (unsigned long long)P.lastNumContacts[w];
        }
        if (!from_solver) {
            const int32_t n = min(P.survCount[w], P.candCapacity);
            if (lane == 0) survivors += (unsigned long long)n;
            const uint32_t *info = P.survInfo + (size_t)w * P.candCapacity;
            for (int32_t i = lane; i < n; i += 64) contacts += info[i] != kNoManifold;
        }
    }
#pragma unroll
    for (int32_t o = 32; o > 0; o >>= 1) {
        cands += __shfl_down(cands, o, 64);
        contacts += __shfl_down(contacts, o, 64);
        survivors += __shfl_down(survivors, o, 64);
    }
    // the block's waves summed in LDS, one set of atomics per block (one
    // per wave, all on three addresses, serialised into ~0.2 ms)
    __shared__ unsigned long long s_sum[3][kProbeThreads / 64];
    const int32_t wave = threadIdx.x >> 6;
    if (lane == 0) {
        s_sum[0][wave] = cands;
        s_sum[1][wave] = contacts;
        s_sum[2][wave] = survivors;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        unsigned long long x = 0;
        for (int32_t i = 0; i < kProbeThreads / 64; i++) x += s_sum[threadIdx.x][i];
        if (x) atomicAdd(P.unitAccum + (threadIdx.x == 0 ? 1 : threadIdx.x == 1 ? 2 : 4), x);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        atomicAdd(P.unitAccum + 0, 1ull);
        if (fused_extra) atomicAdd(P.unitAccum + 3, 1ull);
    }
}

static void probeUnits(const PhysArgs &P, LaunchCtx &lc, bool from_solver, bool fused_extra)
{
    if (!hipx::tlTimed || !P.unitAccum) return;
    hipx::TimedLaunch *t = hipx::tlTimed;
    hipx::tlTimed = nullptr;        // not part of the node's timed span
    try {
        MW_LAUNCH(unitProbeKernel, dim3((uint32_t)std::min((P.numWorlds + 3) / 4, kProbeBlocks)),
                  dim3(kProbeThreads), 0,
                  (hipStream_t)lc.stream, P,
                  from_solver ? 1 : 0, fused_extra ? 1 : 0);
    } catch (...) {
        hipx::tlTimed = t;
        throw;
    }
    hipx::tlTimed = t;
}

// The narrowphase work lists come in two sets (PhysArgs::satWorkSet):
// substep i's narrowphase reads set i % 2, and its filter for substep i + 1
// (fused into substep i's solver) appends to set (i + 1) % 2.  The launch
// copies of PhysArgs point satWork / satWorkCount at the set a kernel reads
// and nextSatWork / nextSatWorkCount at the set it fills or resets.
static PhysArgs substepArgs(const PhysArgs &P, int32_t i, bool reset_next)
{
    PhysArgs Q = P;
    Q.satWork = P.satWorkSet[i & 1];
    Q.satWorkCount = P.satWorkCountSet[i & 1];
    Q.nextSatWork = P.satWorkSet[(i + 1) & 1];
    Q.nextSatWorkCount = reset_next || i > 0 ? P.satWorkCountSet[(i + 1) & 1] : nullptr;
    return Q;
}

#if defined(MW_SAT_CUTS)
// Timing build only (narrowphase.hip MW_SAT_CUTS): the SAT kernel relaunched
// `reps` times on the list substep `substep` of the last step read, cut after
// phase `cut` (0: whole SAT); the mean ms per launch.  The relaunches rewrite
// solverOrder only (rewritten again before its next read), write no
// verdict and reset no list.
extern "C" int mw_debug_set_sat_exp(int32_t cut);
extern "C" double mw_debug_time_sat(int32_t cut, int32_t reps, int32_t substep)
{
    if (!g_cutArgs || g_cutArgs->satImage) return -1.0;
    PhysArgs Q = substepArgs(*g_cutArgs, substep, false);
    Q.nextSatWorkCount = nullptr;
    Q.hhJobs = nullptr;                // no verdicts written
    if (hipDeviceSynchronize() != hipSuccess || mw_debug_set_sat_exp(cut) != 0) return -1.0;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a, nullptr);
    for (int32_t r = 0; r < reps; r++)
        if (Q.satGeoBytes > 0)
            hipLaunchKernelGGL(narrowSATKernel, dim3(Q.satGrid), dim3(kNarrowBlock),
                               narrowphaseSharedBytes(Q), nullptr, Q);
        else
            hipLaunchKernelGGL(narrowSATNoGeoKernel, dim3(Q.satGrid), dim3(kNarrowBlock),
                               narrowphaseSharedBytes(Q), nullptr, Q);
    (void)hipEventRecord(b, nullptr);
    float ms = -1.f;
    if (hipEventSynchronize(b) != hipSuccess || hipEventElapsedTime(&ms, a, b) != hipSuccess) ms = -1.f;
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    mw_debug_set_sat_exp(0);
    return ms / reps;
}

// The solver kernel relaunched `reps` times on substep `substep`'s inputs,
// cut after phase `cut` (solver.hip MW_SOLVER_CUT; 0: whole), without the
// fused integration of the next substep; the mean ms per launch.
extern "C" int mw_debug_set_solver_cut(int32_t cut);
extern "C" double mw_debug_time_solver(int32_t cut, int32_t reps, int32_t substep)
{
    if (!g_cutArgs || g_cutArgs->solverImage) return -1.0;
    const PhysArgs Q = substepArgs(*g_cutArgs, substep, true);
    if (hipDeviceSynchronize() != hipSuccess || mw_debug_set_solver_cut(cut) != 0) return -1.0;
    const dim3 grid((Q.numWorlds + kSolverWorlds - 1) / kSolverWorlds);   // the lanes64 variant
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a, nullptr);
    for (int32_t r = 0; r < reps; r++)
        hipLaunchKernelGGL(lanes64::solverKernel, grid, dim3(kSolverThreads), lanes64::solverSharedBytes(Q),
                           nullptr, Q, 0);
    (void)hipEventRecord(b, nullptr);
    float ms = -1.f;
    if (hipEventSynchronize(b) != hipSuccess || hipEventElapsedTime(&ms, a, b) != hipSuccess) ms = -1.f;
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    mw_debug_set_solver_cut(0);
    return ms / reps;
}
#endif

// substepRigidBodies.  Substeps after the first are integrated by the
// previous substep's solver kernel as it writes its bodies back (fused: the
// bodies are already in its LDS); their nodes keep the graph shape.
struct SubstepRigidBodiesNode : PhysNodeBase {
    bool fused;
    SubstepRigidBodiesNode(Context &ctx, bool fused_into_solver)
        : PhysNodeBase(ctx), fused(fused_into_solver) {}
    static TaskGraph::NodeID addToGraph(Context &ctx, TaskGraph::Builder &b,
                                        Span<const TaskGraph::NodeID> deps)
    {
        return b.addDefaultNode<SubstepRigidBodiesNode>(deps, ctx, false);
    }
    static const char *nodeName() { return "SubstepRigidBodiesNode"; }
    static constexpr bool kNoTmpAlloc = true;
    static void launch(SubstepRigidBodiesNode *self, LaunchCtx &lc)
    {
        const PhysArgs &P = self->mod->args;
        if (self->fused || P.numBodyArchs == 0) return;
        // resets both list sets
        MW_LAUNCH(integrateKernel, rowGrid(P), dim3(256), 0, (hipStream_t)lc.stream,
                           substepArgs(P, 0, true));
    }
};

// Narrowphase = AABB recheck + survivor numbering (the first substep's
// filter kernel, block per world; later substeps' filters run in the
// previous solver's tail), a persistent SAT kernel (8-lane group per
// hull-hull pair; its block 0 also sorts the worlds for the solver grid), a
// plane kernel and a persistent contact kernel (lane per manifold); see
// narrowphase.hip.  The node's launch configuration (blocks
// per CU) sizes the persistent grids; by default they are exactly the
// resident blocks.  The solver turns the per-survivor manifolds into the
// ordered contact list.
struct NarrowphaseNode : PhysNodeBase {
    int32_t substep;
    NarrowphaseNode(Context &ctx, int32_t i) : PhysNodeBase(ctx), substep(i) {}
    static TaskGraph::NodeID addToGraph(Context &ctx, TaskGraph::Builder &b,
                                        Span<const TaskGraph::NodeID> deps)
    {
        return b.addDefaultNode<NarrowphaseNode>(deps, ctx, 0);
    }
    static const char *nodeName() { return "NarrowphaseNode"; }
    static constexpr bool kNoTmpAlloc = true;
    static void launch(NarrowphaseNode *self, LaunchCtx &lc)
    {
        const PhysArgs Q = substepArgs(self->mod->args, self->substep, false);
        hipStream_t stream = (hipStream_t)lc.stream;
        if (self->substep == 0) {
#ifndef MW_FILTER_WAVE
#define MW_FILTER_WAVE 1
#endif
            if (MW_FILTER_WAVE)
                MW_LAUNCH(narrowFilterWaveKernel, dim3((Q.numWorlds + kNarrowBlock / 64 - 1) / (kNarrowBlock / 64)),
                          dim3(kNarrowBlock), 0, stream, Q);
            else
                MW_LAUNCH(narrowFilterKernel, dim3(Q.numWorlds), dim3(kNarrowBlock), 0, stream, Q);
        }
        // The hull-plane pairs share nothing with the hull-hull ones (own
        // list, own contact slots): their kernel runs on the side stream,
        // beside SAT + contact clipping (a parallel branch of the graph).
        hipStream_t side = (hipStream_t)lc.sideStream;
        if (side) {
            MW_HIP_CHECK(hipEventRecord((hipEvent_t)lc.forkEvent, stream));
            MW_HIP_CHECK(hipStreamWaitEvent(side, (hipEvent_t)lc.forkEvent, 0));
        }
        if (Q.planeGeoBytes > 0)
            MW_LAUNCH(narrowPlaneKernel, dim3(lc.persistentGrid(Q.planeGrid)),
                      dim3(kContactBlock), Q.planeGeoBytes, side ? side : stream, Q);
        else
            MW_LAUNCH(narrowPlaneNoGeoKernel, dim3(lc.persistentGrid(Q.planeGrid)),
                      dim3(kContactBlock), 0, side ? side : stream, Q);
        if (side) MW_HIP_CHECK(hipEventRecord((hipEvent_t)lc.joinEvent, side));
        if (Q.satImage) {       // the grid never exceeds the slabs of the image
            const uint32_t g = std::min<uint32_t>(lc.persistentGrid(Q.satGrid), Q.satImageBlocks);
            MW_LAUNCH(narrowSATGlobalKernel, dim3(g), dim3(kNarrowBlock),
                      narrowphaseGlobalSharedBytes(Q), stream, Q);
        } else {
            if (Q.satGeoBytes > 0)
                MW_LAUNCH(narrowSATKernel, dim3(lc.persistentGrid(Q.satGrid)), dim3(kNarrowBlock),
                          narrowphaseSharedBytes(Q), stream, Q);
            else
                MW_LAUNCH(narrowSATNoGeoKernel, dim3(lc.persistentGrid(Q.satGrid)), dim3(kNarrowBlock),
                          narrowphaseSharedBytes(Q), stream, Q);
        }
        if (Q.clipImage) {
            const uint32_t g = std::min<uint32_t>(lc.persistentGrid(Q.contactGrid), Q.clipImageBlocks);
            MW_LAUNCH(narrowContactGlobalKernel, dim3(g), dim3(kContactBlock), 0, stream, Q);
        } else {
            MW_LAUNCH(narrowContactKernel, dim3(lc.persistentGrid(Q.contactGrid)),
                      dim3(kContactBlock), contactSharedBytes(Q), stream, Q);
        }
        if (side) MW_HIP_CHECK(hipStreamWaitEvent(stream, (hipEvent_t)lc.joinEvent, 0));
        probeUnits(Q, lc, false, self->substep == 0);
    }
};

// solvePositions + setVelocities + solveVelocities (one per-world kernel);
// integrate_next: also substepRigidBodies and the narrowphase filter of the
// next substep.
struct SolverNode : PhysNodeBase {
    int32_t substep;
    int32_t integrateNext;
    SolverNode(Context &ctx, int32_t i, bool integrate_next)
        : PhysNodeBase(ctx), substep(i), integrateNext(integrate_next ? 1 : 0) {}
    static TaskGraph::NodeID addToGraph(Context &ctx, TaskGraph::Builder &b,
                                        Span<const TaskGraph::NodeID> deps)
    {
        return b.addDefaultNode<SolverNode>(deps, ctx, 0, false);
    }
    static const char *nodeName() { return "SolverNode"; }
    static constexpr bool kNoTmpAlloc = true;
    static void launch(SolverNode *self, LaunchCtx &lc)
    {
        PhysArgs Q = substepArgs(self->mod->args, self->substep, true);
        const bool l32 = self->mod->solverLanes == 32;
        const SolverVariant sv = l32 ? lanes32::solverVariant() : lanes64::solverVariant();
        Q.solverImage = self->mod->solverImages[l32];
        const dim3 grid((Q.numWorlds + sv.worldsPerBlock - 1) / sv.worldsPerBlock);
        const hipStream_t st = (hipStream_t)lc.stream;
        if (l32) {
            if (Q.solverImage)
                MW_LAUNCH(lanes32::solverGlobalKernel, grid, dim3(sv.threads), sv.globalSharedBytes(Q), st, Q,
                          self->integrateNext);
            else
                MW_LAUNCH(lanes32::solverKernel, grid, dim3(sv.threads), sv.sharedBytes(Q), st, Q,
                          self->integrateNext);
        } else {
            if (Q.solverImage)
                MW_LAUNCH(lanes64::solverGlobalKernel, grid, dim3(sv.threads), sv.globalSharedBytes(Q), st, Q,
                          self->integrateNext);
            else
                MW_LAUNCH(lanes64::solverKernel, grid, dim3(sv.threads), sv.sharedBytes(Q), st, Q,
                          self->integrateNext);
        }
        probeUnits(Q, lc, true, self->integrateNext != 0);
    }
};

// Joint constraints are collected per substep in the reference
// (collectConstraintsSystem, physics.cpp:34-40: ConstraintData rows copied
// in row order into SolverData).  Nothing mutates those rows during a step,
// so the solver kernel reads them in place, in the same order; the node only
// keeps the graph shape.
MW_PHYS_NODE(CollectConstraintsNode, (void)P;)

TaskGraph::NodeID RigidBodyPhysicsSystem::setupBroadphaseTasks(TaskGraph::Builder &builder,
                                                               Span<const TaskGraph::NodeID> deps)
{                                                          // broadphase.cpp:934-956
    auto update_leaves = builder.addToGraph<UpdateLeafPositionsNode>(deps);
    auto bvh_update = builder.addToGraph<UpdateBVHNode>({ update_leaves });
    return builder.addToGraph<RefitNode>({ bvh_update });
}

TaskGraph::NodeID RigidBodyPhysicsSystem::setupSubstepTasks(TaskGraph::Builder &builder,
                                                            Span<const TaskGraph::NodeID> deps,
                                                            CountT num_substeps)
{                                                          // physics.cpp:1149-1199
    auto cur = builder.addToGraph<FindOverlappingNode>(deps);
    for (CountT i = 0; i < num_substeps; i++) {
        auto collect = builder.addToGraph<CollectConstraintsNode>({ cur });
        auto integrate = builder.addDefaultNode<SubstepRigidBodiesNode>({ cur }, builder.context(),
                                                                        i > 0);
        auto narrow = builder.addDefaultNode<NarrowphaseNode>({ integrate }, builder.context(),
                                                              (int32_t)i);
        auto reset1 = builder.addToGraph<ResetTmpAllocNode>({ narrow });
        // solvePositions + setVelocities + solveVelocities: one per-world
        // kernel (the three reference nodes are consecutive per world).
        auto solve = builder.addDefaultNode<SolverNode>({ reset1, collect }, builder.context(),
                                                        (int32_t)i, i + 1 < num_substeps);
        cur = builder.addToGraph<ResetTmpAllocNode>({ solve });
    }
    auto clear = builder.addToGraph<ClearTmpNode<CandidateTemporary>>({ cur });
    auto post_leaves = builder.addToGraph<UpdateLeafPositionsNode>({ clear });
    return builder.addToGraph<RefitNode>({ post_leaves });
}

TaskGraph::NodeID RigidBodyPhysicsSystem::setupCleanupTasks(TaskGraph::Builder &builder,
                                                            Span<const TaskGraph::NodeID> deps)
{
    return builder.addToGraph<ClearTmpNode<CollisionEventTemporary>>(deps);
}

}
