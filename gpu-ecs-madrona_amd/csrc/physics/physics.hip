// MI355X rigid-body physics: host setup + gfx950 kernels.
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
#include <madrona/mw_gpu.hpp>
#include <madrona/physics.hpp>

#include "physics_impl.hpp"
#include "physics_device.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <map>
#include <stdexcept>
#include <vector>

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

// ===========================================================================
// Host geometry (restates src/physics/geometry.cpp:14-194)
// ===========================================================================
namespace geometry {

void FastPolygonList::allocate(uint32_t maxIdx)
{
    maxIndices = maxIdx;
    buffer = (uint32_t *)malloc(sizeof(uint32_t) * maxIndices);
    size = 0;
    edgeCount = 0;
    polygonCount = 0;
}

void FastPolygonList::free() { ::free(buffer); }

void FastPolygonList::addPolygon(Span<const uint32_t> indices)
{
    uint32_t index_count = (uint32_t)indices.size();
    buffer[size] = index_count;
    memcpy(buffer + size + 1, indices.data(), sizeof(uint32_t) * index_count);
    size += index_count + 1;
    polygonCount += 1;
    edgeCount += index_count;
}

void HalfEdgeMesh::construct(FastPolygonList &polygons, uint32_t vertexCount,
                             const Vector3 *vertices)
{
    std::vector<PolygonData> polys;
    std::vector<Plane> planes;
    std::vector<HalfEdge> hedges(polygons.edgeCount);
    std::vector<EdgeData> edges;
    std::map<std::pair<VertexID, VertexID>, HalfEdgeID> pair_to_hedge;
    uint32_t he_count = 0;

    uint32_t poly_idx = 0;
    for (uint32_t *polygon = polygons.begin(); polygon != polygons.end();
         polygon = polygons.next(polygon), ++poly_idx) {
        uint32_t vtx_count = polygons.getPolygonVertexCount(polygon);
        HalfEdge dummy {};
        HalfEdge *prev = &dummy;
        uint32_t first = he_count;
        PolygonData new_polygon = 0;
        for (uint32_t v = 0; v < vtx_count; v++) {
            VertexID a = polygon[v];
            VertexID b = polygon[(v + 1) % vtx_count];
            if (pair_to_hedge.count({ a, b })) {
                throw std::runtime_error("Invalid input mesh to halfedge construction");
            }
            uint32_t hidx = he_count++;
            HalfEdge *ne = &hedges[hidx];
            ne->rootVertex = a;
            ne->polygon = poly_idx;
            auto twin = pair_to_hedge.find({ b, a });
            if (twin != pair_to_hedge.end()) {
                ne->twin = twin->second;
                hedges[twin->second].twin = hidx;
                edges.push_back(twin->second);
            }
            prev->next = hidx;
            prev = ne;
            pair_to_hedge[{ a, b }] = hidx;
            new_polygon = hidx;
        }
        prev->next = first;
        polys.push_back(new_polygon);

        Vector3 fp[3];
        const HalfEdge *he = &hedges[new_polygon];
        for (int i = 0; i < 3; i++) {
            fp[i] = vertices[he->rootVertex];
            he = &hedges[he->next];
        }
        Vector3 a = fp[1] - fp[0];
        Vector3 b = fp[2] - fp[0];
        Vector3 n = cross(a, b).normalize();
        planes.push_back(Plane { n, dot(n, fp[0]) });
    }

    auto dup = [](const auto &vec) {
        using T = typename std::decay_t<decltype(vec)>::value_type;
        T *p = (T *)malloc(sizeof(T) * std::max<size_t>(vec.size(), 1));
        memcpy(p, vec.data(), sizeof(T) * vec.size());
        return p;
    };
    mPolygons = dup(polys);
    mPolygonCount = (uint32_t)polys.size();
    mFacePlanes = dup(planes);
    mEdges = dup(edges);
    mEdgeCount = (uint32_t)edges.size();
    mHalfEdges = dup(hedges);
    mHalfEdgeCount = he_count;
    mVertices = (Vector3 *)malloc(sizeof(Vector3) * vertexCount);
    memcpy(mVertices, vertices, sizeof(Vector3) * vertexCount);
    mVertexCount = vertexCount;
}

}

// ===========================================================================
// Module state (host side)
// ===========================================================================
struct PhysicsModule : StateExtension {
    StateManager *mgr = nullptr;
    int32_t numWorlds = 0;
    bool initialized = false;
    int32_t maxLeaves = 0;
    int32_t maxNodes = 0;
    int32_t maxContacts = 0;
    int32_t maxJoints = 0;
    int32_t candCapacity = 0;

    std::vector<Entity> leafEntitiesHost;        // [W][maxLeaves]

    // flattened object table (host staging)
    ObjDev objHost {};
    std::vector<RigidBodyMetadata> metadata;
    std::vector<AABB> aabbs;
    std::vector<uint32_t> types;
    std::vector<HullDev> hulls;
    std::vector<Vector3> vertices;
    std::vector<geometry::Plane> planes;
    std::vector<geometry::HalfEdge> hedges;
    std::vector<uint32_t> edges;
    std::vector<uint32_t> polygons;
    std::vector<EdgeQuad> edgeQuads;

    PhysArgs args {};
    std::vector<void *> devAllocs;
    bool uploaded = false;

    ~PhysicsModule() override
    {
        for (void *p : devAllocs) (void)hipFree(p);
    }

    template <typename T>
    T *devAlloc(size_t count, hipStream_t stream)
    {
        void *p = nullptr;
        size_t bytes = std::max<size_t>(count * sizeof(T), 256);
        MW_HIP_CHECK(hipMalloc(&p, bytes));
        MW_HIP_CHECK(hipMemsetAsync(p, 0, bytes, stream));
        devAllocs.push_back(p);
        return (T *)p;
    }

    template <typename T>
    T *devUpload(const std::vector<T> &v, hipStream_t stream)
    {
        T *p = devAlloc<T>(v.size(), stream);
        if (!v.empty()) {
            MW_HIP_CHECK(hipMemcpyAsync(p, v.data(), sizeof(T) * v.size(),
                                        hipMemcpyHostToDevice, stream));
        }
        return p;
    }

    void upload(void *stream_ptr) override;
};

static PhysicsModule &module(StateManager &mgr)
{
    auto *m = (PhysicsModule *)mgr.getExtension("physics");
    if (!m) throw std::runtime_error("physics module not registered");
    return *m;
}

struct HostCtxPeek : Context {
    StateManager *mgr() { return mgr_; }
    int32_t world() { return world_; }
};

static StateManager &ctxManager(Context &ctx) { return *static_cast<HostCtxPeek &>(ctx).mgr(); }


void PhysicsModule::upload(void *stream_ptr)
{
    hipStream_t stream = (hipStream_t)stream_ptr;
    if (!initialized) return;          // physics types registered but never used
    const StateView &dv = mgr->deviceViewHost();
    const int32_t W = numWorlds;

    PhysArgs &P = args;
    P.numWorlds = W;

    // Body archetypes: every archetype with the physics column set, in
    // archetype order (the reference query iteration order).
    uint64_t keys[13] = {
        typeKey<Entity>(), typeKey<Position>(), typeKey<Rotation>(), typeKey<Scale>(),
        typeKey<Velocity>(), typeKey<ObjectID>(), typeKey<ResponseType>(),
        typeKey<solver::SubstepPrevState>(), typeKey<solver::PreSolvePositional>(),
        typeKey<solver::PreSolveVelocity>(), typeKey<ExternalForce>(),
        typeKey<ExternalTorque>(), typeKey<broadphase::LeafID>(),
    };
    int32_t archs[kMaxQueryArchetypes];
    int32_t cols[kMaxQueryArchetypes * kMaxQueryComponents];
    int32_t n = mgr->resolveQuery(keys + 1, 12, archs, cols, kMaxQueryArchetypes);
    if (n > kMaxBodyArchetypes) throw std::runtime_error("too many physics body archetypes");
    P.numBodyArchs = n;
    int32_t slot = 0;
    for (int32_t i = 0; i < n; i++) {
        BodyArch &B = P.body[i];
        B.archetype = archs[i];
        const ArchetypeView &av = dv.arch[archs[i]];
        B.capacity = av.capacity;
        B.numRows = av.numRows;
        B.slotBase = slot;
        slot += av.capacity;
        B.cols[0] = av.cols[0];
        for (int32_t c = 0; c < 12; c++) {
            int32_t col = cols[i * kMaxQueryComponents + c];
            // Reference physics ABI: Cols::Position..LeafID are columns 1..12.
            if (col != c + 1) {
                throw std::runtime_error("physics body archetype must list Position, Rotation, "
                                         "Scale, Velocity, ObjectID, ResponseType, SubstepPrevState, "
                                         "PreSolvePositional, PreSolveVelocity, ExternalForce, "
                                         "ExternalTorque, LeafID first, in that order");
            }
            B.cols[c + 1] = av.cols[col];
        }
    }
    P.maxBodiesPerWorld = slot;

    int32_t bvh_arch = mgr->archetypeIndex(typeKey<SingletonArchetype<broadphase::BVH>>());
    int32_t solver_arch = mgr->archetypeIndex(typeKey<SingletonArchetype<SolverData>>());
    P.bvh = (broadphase::BVH *)dv.arch[bvh_arch].cols[1];
    P.solver = (SolverData *)dv.arch[solver_arch].cols[1];
    P.candArchetype = mgr->archetypeIndex(typeKey<CandidateTemporary>());
    P.candCapacity = dv.arch[P.candArchetype].capacity;
    if (P.candCapacity > 32767 || P.maxBodiesPerWorld > 32767) {
        // solver contact records hold survivor slots and body slots as int16
        throw std::runtime_error("physics: max candidates / bodies per world must be <= 32767");
    }
    P.numCands = dv.arch[P.candArchetype].numRows;
    P.cands = (CandidateCollision *)dv.arch[P.candArchetype].cols[1];
    P.idNodes = dv.idNodes;
    P.idsPerWorld = dv.idsPerWorld;
    P.errorFlags = dv.errorFlags;

    P.maxLeaves = maxLeaves;
    P.maxNodes = maxNodes;
    P.nodes = devAlloc<BVHNode>((size_t)W * maxNodes, stream);
    P.leafEntities = devUpload(leafEntitiesHost, stream);
    P.leafAABBs = devAlloc<AABB>((size_t)W * maxLeaves, stream);
    P.leafParents = devAlloc<uint32_t>((size_t)W * maxLeaves, stream);
    P.sortedLeaves = devAlloc<int32_t>((size_t)W * maxLeaves, stream);
    P.leafOrder = devAlloc<int32_t>((size_t)W * maxLeaves, stream);

    ObjDev &O = P.objs;
    O.numObjects = (int32_t)metadata.size();
    O.maxVerts = 0;
    O.maxFaces = 0;
    O.maxEdges = 0;
    for (const HullDev &h : hulls) {
        O.maxVerts = std::max(O.maxVerts, h.numVerts);
        O.maxFaces = std::max(O.maxFaces, h.numFaces);
        O.maxEdges = std::max(O.maxEdges, h.numEdges);
    }
    O.metadata = devUpload(metadata, stream);
    O.aabbs = devUpload(aabbs, stream);
    O.types = devUpload(types, stream);
    O.hulls = devUpload(hulls, stream);
    O.vertices = devUpload(vertices, stream);
    O.planes = devUpload(planes, stream);
    O.hedges = devUpload(hedges, stream);
    O.edges = devUpload(edges, stream);
    O.edgeQuads = devUpload(edgeQuads, stream);
    O.polygons = devUpload(polygons, stream);

    P.bodyAABBs = devAlloc<AABB>((size_t)W * std::max(P.maxBodiesPerWorld, 1), stream);
    P.survInfo = devAlloc<uint32_t>((size_t)W * P.candCapacity, stream);
    P.survCount = devAlloc<int32_t>(W, stream);
    P.binCap = (W + kNarrowBins - 1) / kNarrowBins * P.candCapacity;
    P.satWork = devAlloc<SatWork>((size_t)kNarrowBins * P.binCap, stream);
    P.satWorkCount = devAlloc<int32_t>(kNarrowBins * kBinStride, stream);
    P.hhJobs = devAlloc<ContactJob>((size_t)W * P.candCapacity, stream);
    P.candContacts = devAlloc<Contact>((size_t)W * P.candCapacity, stream);
    P.maxContacts = maxContacts;
    P.contactOrder = devAlloc<int32_t>((size_t)W * P.candCapacity, stream);
    const int32_t joint_arch = mgr->archetypeIndex(typeKey<ConstraintData>());
    P.jointCapacity = dv.arch[joint_arch].capacity;
    P.numJointRows = dv.arch[joint_arch].numRows;
    P.joints = (JointConstraint *)dv.arch[joint_arch].cols[1];
    P.maxJoints = maxJoints;
    P.recStride = P.candCapacity + std::min(maxJoints, P.jointCapacity);
    if (P.recStride > 32767) {
        throw std::runtime_error("physics: max candidates + joints per world must be <= 32767");
    }
    P.solverRecs = devAlloc<uint64_t>((size_t)W * P.recStride, stream);
    P.solverPrevs = devAlloc<int32_t>((size_t)W * P.recStride, stream);
    P.lastNumContacts = devAlloc<int32_t>(W, stream);
    P.lastNumCands = devAlloc<int32_t>(W, stream);

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
    MW_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, narrowPlaneKernel,
                                                              kContactBlock, 0));
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
    explicit PhysNodeBase(Context &ctx) : mod(&module(ctxManager(ctx))) {}
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
        hipLaunchKernelGGL(integrateKernel, rowGrid(P), dim3(256), 0, (hipStream_t)lc.stream, P);
    }
};

// Narrowphase = AABB recheck + survivor numbering (block per world), a
// per-world compaction into flat lists, a persistent SAT kernel (16-lane
// group per hull-hull pair) and a persistent contact kernel (lane per
// manifold); see narrowphase.hip.  The node's launch configuration (blocks
// per CU) sizes the two persistent grids; by default they are exactly the
// resident blocks.  The solver turns
// the per-survivor manifolds into the ordered contact list.
MW_PHYS_NODE(NarrowphaseNode,
    hipLaunchKernelGGL(narrowFilterKernel, dim3(P.numWorlds), dim3(kNarrowBlock), 0, stream, P);
    hipLaunchKernelGGL(narrowSATKernel, dim3(lc.persistentGrid(P.satGrid)), dim3(kNarrowBlock),
                       narrowphaseSharedBytes(P), stream, P);
    hipLaunchKernelGGL(narrowPlaneKernel, dim3(lc.persistentGrid(P.planeGrid)),
                       dim3(kContactBlock), 0, stream, P);
    hipLaunchKernelGGL(narrowContactKernel, dim3(lc.persistentGrid(P.contactGrid)),
                       dim3(kContactBlock), contactSharedBytes(P), stream, P);)

// solvePositions + setVelocities + solveVelocities (one per-world kernel);
// integrate_next: also substepRigidBodies of the next substep.
struct SolverNode : PhysNodeBase {
    int32_t integrateNext;
    SolverNode(Context &ctx, bool integrate_next)
        : PhysNodeBase(ctx), integrateNext(integrate_next ? 1 : 0) {}
    static TaskGraph::NodeID addToGraph(Context &ctx, TaskGraph::Builder &b,
                                        Span<const TaskGraph::NodeID> deps)
    {
        return b.addDefaultNode<SolverNode>(deps, ctx, false);
    }
    static const char *nodeName() { return "SolverNode"; }
    static constexpr bool kNoTmpAlloc = true;
    static void launch(SolverNode *self, LaunchCtx &lc)
    {
        const PhysArgs &P = self->mod->args;
        hipLaunchKernelGGL(solverKernel, dim3((P.numWorlds + kSolverWorlds - 1) / kSolverWorlds),
                           dim3(kSolverThreads), solverSharedBytes(P), (hipStream_t)lc.stream, P,
                           self->integrateNext);
    }
};

// Joint constraints are collected per substep in the reference
// (collectConstraintsSystem, physics.cpp:34-40: ConstraintData rows copied
// in row order into SolverData).  Nothing mutates those rows during a step,
// so the solver kernel reads them in place, in the same order; the node only
// keeps the graph shape.
MW_PHYS_NODE(CollectConstraintsNode, (void)P;)

// ===========================================================================
// RigidBodyPhysicsSystem
// ===========================================================================
void RigidBodyPhysicsSystem::registerTypes(ECSRegistry &registry)
{                                                          // physics.cpp:1055-1081
    StateManager &mgr = registry.stateManager();
    registry.registerComponent<broadphase::LeafID>();
    registry.registerSingleton<broadphase::BVH>();
    registry.registerComponent<ExternalForce>();
    registry.registerComponent<ExternalTorque>();
    registry.registerComponent<ResponseType>();
    registry.registerComponent<Velocity>();
    registry.registerComponent<solver::SubstepPrevState>();
    registry.registerComponent<solver::PreSolvePositional>();
    registry.registerComponent<solver::PreSolveVelocity>();
    registry.registerComponent<CollisionEvent>();
    registry.registerArchetype<CollisionEventTemporary>();
    mgr.setTemporary(typeKey<CollisionEventTemporary>());
    mgr.setModuleRows(typeKey<CollisionEventTemporary>());
    registry.registerComponent<CandidateCollision>();
    registry.registerArchetype<CandidateTemporary>();
    mgr.setTemporary(typeKey<CandidateTemporary>());
    mgr.setModuleRows(typeKey<CandidateTemporary>());
    registry.registerComponent<JointConstraint>();
    registry.registerArchetype<ConstraintData>();
    registry.registerSingleton<SolverData>();
    registry.registerSingleton<ObjectData>();

    if (!mgr.getExtension("physics")) {
        auto *m = new PhysicsModule();
        m->mgr = &mgr;
        m->numWorlds = mgr.numWorlds();
        mgr.setExtension("physics", m);
    }
}

void RigidBodyPhysicsSystem::setMaxCandidatesPerWorld(ECSRegistry &registry, int32_t max_candidates)
{
    registry.stateManager().setCapacityHint(typeKey<CandidateTemporary>(), max_candidates);
}

void RigidBodyPhysicsSystem::init(Context &ctx, ObjectManager *obj_mgr, float delta_t,
                                  CountT num_substeps, Vector3 gravity,
                                  CountT max_dynamic_objects, CountT max_contacts_per_world,
                                  CountT max_joint_constraints_per_world)
{                                                          // physics.cpp:1012-1036
    StateManager &mgr = ctxManager(ctx);
    PhysicsModule &m = module(mgr);
    const int32_t W = m.numWorlds;
    const int32_t world = static_cast<HostCtxPeek &>(ctx).world();

    if (!m.initialized) {
        m.initialized = true;
        m.maxLeaves = (int32_t)max_dynamic_objects;
        m.maxNodes = numInternalNodes((int32_t)max_dynamic_objects);
        m.maxContacts = (int32_t)max_contacts_per_world;
        m.maxJoints = (int32_t)max_joint_constraints_per_world;
        m.leafEntitiesHost.assign((size_t)W * m.maxLeaves, Entity::none());

        // Flatten the host object table.
        for (int32_t o = 0; o < obj_mgr->numObjects; o++) {
            m.metadata.push_back(obj_mgr->metadata[o]);
            m.aabbs.push_back(obj_mgr->aabbs[o]);
            const CollisionPrimitive &prim = obj_mgr->primitives[o];
            m.types.push_back((uint32_t)prim.type);
            HullDev hd {};
            if (prim.type == CollisionPrimitive::Type::Hull) {
                const geometry::HalfEdgeMesh &he = prim.hull.halfEdgeMesh;
                hd.vertOffset = (int32_t)m.vertices.size();
                hd.numVerts = (int32_t)he.mVertexCount;
                hd.faceOffset = (int32_t)m.planes.size();
                hd.numFaces = (int32_t)he.mPolygonCount;
                hd.hedgeOffset = (int32_t)m.hedges.size();
                hd.numHedges = (int32_t)he.mHalfEdgeCount;
                hd.edgeOffset = (int32_t)m.edges.size();
                hd.numEdges = (int32_t)he.mEdgeCount;
                m.vertices.insert(m.vertices.end(), he.mVertices, he.mVertices + he.mVertexCount);
                m.planes.insert(m.planes.end(), he.mFacePlanes, he.mFacePlanes + he.mPolygonCount);
                m.polygons.insert(m.polygons.end(), he.mPolygons, he.mPolygons + he.mPolygonCount);
                m.hedges.insert(m.hedges.end(), he.mHalfEdges, he.mHalfEdges + he.mHalfEdgeCount);
                m.edges.insert(m.edges.end(), he.mEdges, he.mEdges + he.mEdgeCount);
                if (he.mVertexCount > 65535 || he.mPolygonCount > 65535) {
                    throw std::runtime_error("hull too large (edge topology is 16-bit)");
                }
                for (uint32_t e = 0; e < he.mEdgeCount; e++) {
                    const geometry::HalfEdge &h = he.mHalfEdges[he.mEdges[e]];
                    m.edgeQuads.push_back(EdgeQuad {
                        (uint16_t)h.polygon, (uint16_t)he.mHalfEdges[h.twin].polygon,
                        (uint16_t)h.rootVertex, (uint16_t)he.mHalfEdges[h.next].rootVertex });
                }
            } else if (prim.type == CollisionPrimitive::Type::Sphere) {
                throw std::runtime_error("sphere primitives are unsupported (the reference asserts, "
                                         "narrowphase.cpp:1197-1313)");
            }
            m.hulls.push_back(hd);
        }
    } else if (m.maxLeaves != (int32_t)max_dynamic_objects ||
               m.maxContacts != (int32_t)max_contacts_per_world ||
               m.maxJoints != (int32_t)max_joint_constraints_per_world) {
        throw std::runtime_error("RigidBodyPhysicsSystem::init: per-world sizes must match");
    }

    broadphase::BVH &bvh = ctx.getSingleton<broadphase::BVH>();
    bvh.numLeaves = 0;
    bvh.maxLeaves = m.maxLeaves;
    bvh.numNodes = 0;
    bvh.usedNodes = 0;
    bvh.forceRebuild = 0;
    bvh.leafVelocityExpansion = 2.f * delta_t;
    bvh.leafAccelExpansion = 100.f * delta_t * delta_t;
    bvh.worldIdx = world;

    SolverData &solver = ctx.getSingleton<SolverData>();
    solver.numContacts = 0;
    solver.maxContacts = (int32_t)max_contacts_per_world;
    solver.numJointConstraints = 0;
    solver.maxJointConstraints = (int32_t)max_joint_constraints_per_world;
    solver.deltaT = delta_t;
    solver.h = delta_t / (float)num_substeps;
    solver.g = gravity;
    solver.gMagnitude = gravity.length();
    solver.restitutionThreshold = 2.f * solver.gMagnitude * solver.h;

    ctx.getSingleton<ObjectData>().mgr = nullptr;
}

void RigidBodyPhysicsSystem::reset(Context &ctx)
{
    broadphase::BVH &bvh = ctx.getSingleton<broadphase::BVH>();
    bvh.rebuildOnUpdate();
    bvh.clearLeaves();
}

broadphase::LeafID RigidBodyPhysicsSystem::registerEntity(Context &ctx, Entity e, ObjectID obj_id)
{                                                          // physics.cpp:1045-1053
    (void)obj_id;
    PhysicsModule &m = module(ctxManager(ctx));
    broadphase::BVH &bvh = ctx.getSingleton<broadphase::BVH>();
    int32_t leaf = bvh.numLeaves++;
    if (leaf >= m.maxLeaves) throw std::runtime_error("BVH leaf capacity exceeded");
    m.leafEntitiesHost[(size_t)bvh.worldIdx * m.maxLeaves + leaf] = e;
    return broadphase::LeafID { leaf };
}

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
        auto narrow = builder.addToGraph<NarrowphaseNode>({ integrate });
        auto reset1 = builder.addToGraph<ResetTmpAllocNode>({ narrow });
        // solvePositions + setVelocities + solveVelocities: one per-world
        // kernel (the three reference nodes are consecutive per world).
        auto solve = builder.addDefaultNode<SolverNode>({ reset1, collect }, builder.context(),
                                                        i + 1 < num_substeps);
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

// Debug / test access to module slabs (used by the C ABI).
PhysArgs *physicsArgs(StateManager &mgr)
{
    auto *m = (PhysicsModule *)mgr.getExtension("physics");
    return m && m->uploaded ? &m->args : nullptr;
}

}
