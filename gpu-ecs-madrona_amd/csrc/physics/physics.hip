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

#include <cstdio>

namespace madrona::phys {

using namespace math;
using namespace base;

#define MW_HIP_CHECK(expr)                                                          \
    do {                                                                            \
        hipError_t err__ = (expr);                                                  \
        if (err__ != hipSuccess) {                                                  \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(err__),    \
                    __FILE__, __LINE__);                                            \
            throw std::runtime_error(hipGetErrorString(err__));                     \
        }                                                                           \
    } while (0)

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

void PhysicsModule::upload(void *stream_ptr)
{
    if (!initialized) return;          // physics types registered but never used
    buildArgs(stream_ptr);
    PhysArgs &P = args;
    // Persistent SAT grid: exactly the blocks that can be resident at once.
    int dev = 0, cus = 0, per_cu = 0;
    MW_HIP_CHECK(hipGetDevice(&dev));
    MW_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    MW_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per_cu, narrowSATKernel, kNarrowBlock, narrowphaseSharedBytes(P)));
    P.satGrid = std::max(1, cus * std::max(per_cu, 1));
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
    MW_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per_cu, narrowContactKernel, kContactBlock, contactSharedBytes(P)));
    P.contactGrid = std::max(1, cus * std::max(per_cu, 1));
    P.planeGeoBytes = (int32_t)planeSharedBytes(P);
    MW_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, narrowPlaneKernel,
                                                              kContactBlock, P.planeGeoBytes));
    P.planeGrid = std::max(1, cus * std::max(per_cu, 1));
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
        hipLaunchKernelGGL(leafUpdateKernel, rowGrid(P), dim3(256), 0, stream, P);)

// One wave per world while the world's leaves fit the LDS image (129 leaves:
// ≈11 KB); the lane-per-world kernel otherwise.
MW_PHYS_NODE(UpdateBVHNode,
    if (rebuildSharedBytes(P) <= 64 * 1024)
        hipLaunchKernelGGL(bvhRebuildWaveKernel, dim3(P.numWorlds), dim3(64),
                           rebuildSharedBytes(P), stream, P);
    else
        hipLaunchKernelGGL(bvhRebuildKernel, dim3((P.numWorlds + 63) / 64), dim3(64), 0, stream, P);)

MW_PHYS_NODE(RefitNode,
    if (P.numBodyArchs > 0)
        hipLaunchKernelGGL(refitKernel, dim3(P.numWorlds), dim3(kRefitBlock),
                           refitSharedBytes(P), stream, P);)

MW_PHYS_NODE(FindOverlappingNode,
    hipLaunchKernelGGL(findOverlapsKernel, dim3(P.numWorlds), dim3(kOverlapBlock),
                       findOverlapsSharedBytes(P), stream, P);)

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
        hipLaunchKernelGGL(integrateKernel, rowGrid(P), dim3(256), 0, (hipStream_t)lc.stream,
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
        if (self->substep == 0)
            hipLaunchKernelGGL(narrowFilterKernel, dim3(Q.numWorlds), dim3(kNarrowBlock), 0, stream, Q);
        hipLaunchKernelGGL(narrowSATKernel, dim3(lc.persistentGrid(Q.satGrid)), dim3(kNarrowBlock),
                           narrowphaseSharedBytes(Q), stream, Q);
        hipLaunchKernelGGL(narrowPlaneKernel, dim3(lc.persistentGrid(Q.planeGrid)),
                           dim3(kContactBlock), Q.planeGeoBytes, stream, Q);
        hipLaunchKernelGGL(narrowContactKernel, dim3(lc.persistentGrid(Q.contactGrid)),
                           dim3(kContactBlock), contactSharedBytes(Q), stream, Q);
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
        const PhysArgs Q = substepArgs(self->mod->args, self->substep, true);
        hipLaunchKernelGGL(solverKernel, dim3((Q.numWorlds + kSolverWorlds - 1) / kSolverWorlds),
                           dim3(kSolverThreads), solverSharedBytes(Q), (hipStream_t)lc.stream, Q,
                           self->integrateNext);
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
