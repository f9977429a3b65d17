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

__host__ __device__ inline int32_t numInternalNodes(int32_t num_leaves)   // broadphase.cpp:33-40
{
    int32_t a = (num_leaves - 1 + 2) / 3;
    return (a > 1 ? a : 1) + num_leaves;
}

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

    ObjDev &O = P.objs;
    O.numObjects = (int32_t)metadata.size();
    O.maxVerts = 0;
    O.maxFaces = 0;
    for (const HullDev &h : hulls) {
        O.maxVerts = std::max(O.maxVerts, h.numVerts);
        O.maxFaces = std::max(O.maxFaces, h.numFaces);
    }
    O.metadata = devUpload(metadata, stream);
    O.aabbs = devUpload(aabbs, stream);
    O.types = devUpload(types, stream);
    O.hulls = devUpload(hulls, stream);
    O.vertices = devUpload(vertices, stream);
    O.planes = devUpload(planes, stream);
    O.hedges = devUpload(hedges, stream);
    O.edges = devUpload(edges, stream);
    O.polygons = devUpload(polygons, stream);

    P.hullVerts = devAlloc<Vector3>((size_t)W * maxLeaves * std::max(O.maxVerts, 1), stream);
    P.hullPlanes = devAlloc<geometry::Plane>((size_t)W * maxLeaves * std::max(O.maxFaces, 1), stream);
    P.candContacts = devAlloc<Contact>((size_t)W * P.candCapacity, stream);
    P.maxContacts = maxContacts;
    P.contactOrder = devAlloc<int32_t>((size_t)W * P.candCapacity, stream);
    P.lastNumContacts = devAlloc<int32_t>(W, stream);
    P.lastNumCands = devAlloc<int32_t>(W, stream);
    uploaded = true;
}

// ===========================================================================
// Device helpers
// ===========================================================================
template <typename T>
__device__ __forceinline__ T &bcol(const BodyArch &B, int col, int32_t w, int32_t r)
{
    return ((T *)B.cols[col])[(size_t)w * B.capacity + r];
}

__device__ __forceinline__ int bodyArchIndex(const PhysArgs &P, uint32_t archetype)
{
    for (int i = 0; i < P.numBodyArchs; i++) {
        if ((uint32_t)P.body[i].archetype == archetype) return i;
    }
    return 0;
}

__device__ __forceinline__ Loc entityLoc(const PhysArgs &P, int32_t w, Entity e)
{
    const IDNode &n = P.idNodes[(size_t)w * P.idsPerWorld + e.id];
    if (n.gen != e.gen) return Loc::none();
    return n.val;
}

// Float min/max updates with the reference's "v < old" rule; CAS loop so
// concurrent leaves of one world compose like the reference's atomicMinF
// (broadphase.cpp:494-543).  Values only shrink (min) / grow (max), so a
// stale first read is safe.
__device__ __forceinline__ float atomicMinRef(float *addr, float v)
{
    uint32_t *p = (uint32_t *)addr;
    uint32_t old = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (true) {
        float of = __uint_as_float(old);
        if (!(v < of)) return of;
        uint32_t prev = atomicCAS(p, old, __float_as_uint(v));
        if (prev == old) return of;
        old = prev;
    }
}

__device__ __forceinline__ float atomicMaxRef(float *addr, float v)
{
    uint32_t *p = (uint32_t *)addr;
    uint32_t old = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (true) {
        float of = __uint_as_float(old);
        if (!(v > of)) return of;
        uint32_t prev = atomicCAS(p, old, __float_as_uint(v));
        if (prev == old) return of;
        old = prev;
    }
}

// Grid helper: lanes over (world, row) of body archetype blockIdx.y.
struct RowIdx {
    int32_t w, r;
    bool valid;
};

__device__ __forceinline__ RowIdx rowIndex(const PhysArgs &P, const BodyArch &B)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    RowIdx ri;
    ri.w = (int32_t)(t / B.capacity);
    ri.r = (int32_t)(t - (int64_t)ri.w * B.capacity);
    ri.valid = ri.w < P.numWorlds && ri.r < B.numRows[ri.w];
    return ri;
}

// ===========================================================================
// Broadphase kernels (src/physics/broadphase.cpp)
// ===========================================================================
__device__ __forceinline__ AABB expandAABBWithMotion(AABB aabb, const Vector3 &v,
                                                     float vel_exp, float acc_exp)
{                                                          // broadphase.cpp:435-459
#pragma unroll
    for (int32_t i = 0; i < 3; i++) {
        float pos_delta = vel_exp * v[i];
        float min_delta = pos_delta - acc_exp;
        float max_delta = pos_delta + acc_exp;
        if (min_delta < 0.f) aabb.pMin[i] += min_delta;
        if (max_delta > 0.f) aabb.pMax[i] += max_delta;
    }
    return aabb;
}

// updateLeafPositionsEntry (broadphase.cpp:858-873, 461-480)
__global__ void __launch_bounds__(256) leafUpdateKernel(PhysArgs P)
{
    const BodyArch &B = P.body[blockIdx.y];
    RowIdx ri = rowIndex(P, B);
    if (!ri.valid) return;
    const int32_t w = ri.w, r = ri.r;
    const int32_t leaf = bcol<broadphase::LeafID>(B, Cols::LeafID, w, r).id;
    const Vector3 pos = bcol<Vector3>(B, Cols::Position, w, r);
    const Quat rot = bcol<Quat>(B, Cols::Rotation, w, r);
    const Diag3x3 scale = bcol<Diag3x3>(B, Cols::Scale, w, r);
    const int32_t obj = bcol<ObjectID>(B, Cols::ObjectID, w, r).idx;
    const Vector3 lin = bcol<Velocity>(B, Cols::Velocity, w, r).linear;
    const broadphase::BVH &bvh = P.bvh[w];
    AABB world_aabb = P.objs.aabbs[obj].applyTRS(pos, rot, scale);
    const size_t li = (size_t)w * P.maxLeaves + leaf;
    P.leafAABBs[li] = expandAABBWithMotion(world_aabb, lin, bvh.leafVelocityExpansion,
                                           bvh.leafAccelExpansion);
    P.sortedLeaves[li] = leaf;
}

// BVH::rebuild (broadphase.cpp:42-280): top-down midpoint 4-way split, one
// lane per world, only for worlds with force_rebuild_ set (first step).
__device__ __forceinline__ Vector3 leafCenter(const AABB *aabbs, const int32_t *sorted, int32_t i)
{
    AABB a = aabbs[sorted[i]];
    return (a.pMin + a.pMax) / 2.f;
}

__device__ int32_t midpointSplit(const AABB *aabbs, int32_t *sorted, int32_t base, int32_t n)
{
    Vector3 cmin { FLT_MAX, FLT_MAX, FLT_MAX };
    Vector3 cmax { -FLT_MAX, -FLT_MAX, -FLT_MAX };
    for (int32_t i = 0; i < n; i++) {
        Vector3 c = leafCenter(aabbs, sorted, base + i);
        cmin = Vector3::min(cmin, c);
        cmax = Vector3::max(cmax, c);
    }
    Vector3 d = cmax - cmin;
    int axis;
    if (d.x > d.y && d.x > d.z) axis = 0;
    else if (d.y > d.x && d.y > d.z) axis = 1;
    else axis = 2;
    float split_val = 0.5f * (cmin[axis] + cmax[axis]);
    int32_t start = 0, end = n;
    while (start < end) {
        while (start < end && leafCenter(aabbs, sorted, base + start)[axis] < split_val) ++start;
        while (start < end && leafCenter(aabbs, sorted, base + end - 1)[axis] >= split_val) --end;
        if (start < end) {
            int32_t tmp = sorted[base + start];
            sorted[base + start] = sorted[base + end - 1];
            sorted[base + end - 1] = tmp;
            ++start;
            --end;
        }
    }
    if (start > 0 && start < n) return start;
    return n / 2;
}

__global__ void __launch_bounds__(64) bvhRebuildKernel(PhysArgs P)
{
    const int32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= P.numWorlds) return;
    broadphase::BVH &bvh = P.bvh[w];
    if (!bvh.forceRebuild) return;                       // BVH::updateTree
    bvh.forceRebuild = 0;

    BVHNode *nodes = P.nodes + (size_t)w * P.maxNodes;
    const AABB *aabbs = P.leafAABBs + (size_t)w * P.maxLeaves;
    int32_t *sorted = P.sortedLeaves + (size_t)w * P.maxLeaves;
    uint32_t *parents = P.leafParents + (size_t)w * P.maxLeaves;

    bvh.numNodes = numInternalNodes(bvh.numLeaves);
    struct StackEntry { int32_t nodeID, parentID, offset, numObjs; };
    StackEntry stack[128];
    stack[0] = { -1, -1, 0, bvh.numLeaves };
    int32_t cur_node_offset = 0;
    int32_t stack_size = 1;
    while (stack_size > 0) {
        StackEntry &entry = stack[stack_size - 1];
        int32_t node_id;
        if (entry.numObjs <= 4) {
            node_id = cur_node_offset++;
            BVHNode &node = nodes[node_id];
            node.parentID = entry.parentID;
            for (int i = 0; i < 4; i++) {
                if (i < entry.numObjs) {
                    int32_t leaf_id = sorted[entry.offset + i];
                    const AABB a = aabbs[leaf_id];
                    parents[leaf_id] = ((uint32_t)node_id << 2) | (uint32_t)i;
                    node.children[i] = (int32_t)(0x80000000u | (uint32_t)leaf_id);
                    node.minX[i] = a.pMin.x; node.minY[i] = a.pMin.y; node.minZ[i] = a.pMin.z;
                    node.maxX[i] = a.pMax.x; node.maxY[i] = a.pMax.y; node.maxZ[i] = a.pMax.z;
                } else {
                    node.children[i] = -1;
                    node.minX[i] = FLT_MAX; node.minY[i] = FLT_MAX; node.minZ[i] = FLT_MAX;
                    node.maxX[i] = -FLT_MAX; node.maxY[i] = -FLT_MAX; node.maxZ[i] = -FLT_MAX;
                }
            }
        } else if (entry.nodeID == -1) {
            node_id = cur_node_offset++;
            entry.nodeID = node_id;
            BVHNode &node = nodes[node_id];
            for (int i = 0; i < 4; i++) node.children[i] = -1;
            node.parentID = entry.parentID;
            int32_t second = midpointSplit(aabbs, sorted, entry.offset, entry.numObjs);
            int32_t nh1 = second;
            int32_t nh2 = entry.numObjs - second;
            int32_t first = midpointSplit(aabbs, sorted, entry.offset, nh1);
            int32_t third = midpointSplit(aabbs, sorted, entry.offset + second, nh2);
            int32_t eid = entry.nodeID, eoff = entry.offset;
            if (stack_size + 4 > 128) { atomicOr(P.errorFlags + w, kErrBVHStack); return; }
            stack[stack_size++] = { -1, eid, eoff + nh1 + third, nh2 - third };
            stack[stack_size++] = { -1, eid, eoff + nh1, third };
            stack[stack_size++] = { -1, eid, eoff + first, nh1 - first };
            stack[stack_size++] = { -1, eid, eoff, first };
            continue;
        } else {
            node_id = entry.nodeID;
        }
        stack_size -= 1;
        BVHNode &node = nodes[node_id];
        if (node.parentID == -1) continue;
        AABB combined = AABB::invalid();
        for (int i = 0; i < 4; i++) {
            if (node.children[i] == -1) break;
            combined = AABB::merge(combined, AABB {
                { node.minX[i], node.minY[i], node.minZ[i] },
                { node.maxX[i], node.maxY[i], node.maxZ[i] } });
        }
        BVHNode &parent = nodes[node.parentID];
        int c;
        for (c = 0; c < 4; c++) if (parent.children[c] == -1) break;
        parent.children[c] = node_id;
        parent.minX[c] = combined.pMin.x; parent.minY[c] = combined.pMin.y;
        parent.minZ[c] = combined.pMin.z; parent.maxX[c] = combined.pMax.x;
        parent.maxY[c] = combined.pMax.y; parent.maxZ[c] = combined.pMax.z;
    }
    bvh.usedNodes = cur_node_offset;
}

// refitEntry -> BVH::refitLeaf (broadphase.cpp:545-642, 891-895)
__global__ void __launch_bounds__(256) refitKernel(PhysArgs P)
{
    const BodyArch &B = P.body[blockIdx.y];
    RowIdx ri = rowIndex(P, B);
    if (!ri.valid) return;
    const int32_t w = ri.w;
    const int32_t leaf = bcol<broadphase::LeafID>(B, Cols::LeafID, w, ri.r).id;
    const size_t li = (size_t)w * P.maxLeaves + leaf;
    const AABB a = P.leafAABBs[li];
    const uint32_t lp = P.leafParents[li];
    BVHNode *nodes = P.nodes + (size_t)w * P.maxNodes;
    int32_t node_idx = (int32_t)(lp >> 2);
    const int sub = (int)(lp & 3);

    {   // leaf slot: owned by this leaf alone -> plain read-modify-write
        BVHNode &n = nodes[node_idx];
        float xm = n.minX[sub], ym = n.minY[sub], zm = n.minZ[sub];
        float xM = n.maxX[sub], yM = n.maxY[sub], zM = n.maxZ[sub];
        if (a.pMin.x < xm) n.minX[sub] = a.pMin.x;
        if (a.pMin.y < ym) n.minY[sub] = a.pMin.y;
        if (a.pMin.z < zm) n.minZ[sub] = a.pMin.z;
        if (a.pMax.x > xM) n.maxX[sub] = a.pMax.x;
        if (a.pMax.y > yM) n.maxY[sub] = a.pMax.y;
        if (a.pMax.z > zM) n.maxZ[sub] = a.pMax.z;
        bool expanded = a.pMin.x < xm || a.pMin.y < ym || a.pMin.z < zm ||
                        a.pMax.x > xM || a.pMax.y > yM || a.pMax.z > zM;
        if (!expanded) return;
    }
    int32_t child_idx = node_idx;
    node_idx = nodes[node_idx].parentID;
    while (node_idx != -1) {
        BVHNode &n = nodes[node_idx];
        int c = -1;
        for (int j = 0; j < 4; j++) {
            if (n.children[j] == child_idx) { c = j; break; }
        }
        if (c < 0) return;
        float xm = atomicMinRef(&n.minX[c], a.pMin.x);
        float ym = atomicMinRef(&n.minY[c], a.pMin.y);
        float zm = atomicMinRef(&n.minZ[c], a.pMin.z);
        float xM = atomicMaxRef(&n.maxX[c], a.pMax.x);
        float yM = atomicMaxRef(&n.maxY[c], a.pMax.y);
        float zM = atomicMaxRef(&n.maxZ[c], a.pMax.z);
        bool expanded = a.pMin.x < xm || a.pMin.y < ym || a.pMin.z < zm ||
                        a.pMax.x > xM || a.pMax.y > yM || a.pMax.z > zM;
        if (!expanded) break;
        child_idx = node_idx;
        node_idx = n.parentID;
    }
}

// findOverlappingEntry + BVH::findOverlaps (broadphase.cpp:897-932,
// physics.inl:61-100).  One block per world; lanes own rows.  Pass 1 counts
// each row's candidates, a block scan gives the reference's append order,
// pass 2 writes them.
constexpr int32_t kOverlapBlock = 128;
constexpr int32_t kOverlapStack = 48;

template <bool kWrite>
__device__ __forceinline__ int32_t traverseOverlaps(const PhysArgs &P, int32_t w,
                                                    const BodyArch &B, int32_t row,
                                                    int32_t *stack, int32_t out_base)
{
    const Entity e = bcol<Entity>(B, 0, w, row);
    const Loc a_loc = entityLoc(P, w, e);
    const bool a_static = bcol<ResponseType>(B, Cols::ResponseType, w, row) == ResponseType::Static;
    const int32_t leaf = bcol<broadphase::LeafID>(B, Cols::LeafID, w, row).id;
    const AABB q = P.leafAABBs[(size_t)w * P.maxLeaves + leaf];
    const BVHNode *nodes = P.nodes + (size_t)w * P.maxNodes;
    const Entity *leaf_entities = P.leafEntities + (size_t)w * P.maxLeaves;

    int32_t count = 0;
    stack[0] = 0;
    int32_t ss = 1;
    while (ss > 0) {
        const BVHNode &n = nodes[stack[--ss]];
        for (int i = 0; i < 4; i++) {
            const int32_t child = n.children[i];
            if (child == -1) continue;
            AABB c { { n.minX[i], n.minY[i], n.minZ[i] }, { n.maxX[i], n.maxY[i], n.maxZ[i] } };
            if (!q.overlaps(c)) continue;
            if (child & 0x80000000) {
                const Entity o = leaf_entities[child & ~0x80000000];
                if (e.id < o.id) {
                    const Loc b_loc = entityLoc(P, w, o);
                    if (a_static) {
                        const BodyArch &OB = P.body[bodyArchIndex(P, b_loc.archetype)];
                        if (bcol<ResponseType>(OB, Cols::ResponseType, w, b_loc.row) ==
                            ResponseType::Static) {
                            continue;
                        }
                    }
                    if (kWrite) {
                        int32_t slot = out_base + count;
                        if (slot < P.candCapacity) {
                            P.cands[(size_t)w * P.candCapacity + slot] = CandidateCollision { a_loc, b_loc };
                        }
                    }
                    count++;
                }
            } else {
                if (ss < kOverlapStack) {
                    stack[ss++] = child;
                } else {
                    atomicOr(P.errorFlags + w, kErrBVHStack);
                }
            }
        }
    }
    return count;
}

__device__ __forceinline__ int32_t blockExclusiveScan(int32_t v, int32_t *scratch, int32_t *total)
{
    // Wave-level inclusive scan with DPP-friendly shuffles, then across waves.
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    int32_t x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        int32_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    if (lane == 63) scratch[wave] = x;
    __syncthreads();
    const int nwaves = blockDim.x >> 6;
    int32_t wave_base = 0, sum = 0;
    for (int i = 0; i < nwaves; i++) {
        int32_t s = scratch[i];
        if (i < wave) wave_base += s;
        sum += s;
    }
    __syncthreads();
    *total = sum;
    return wave_base + x - v;
}

__global__ void __launch_bounds__(kOverlapBlock) findOverlapsKernel(PhysArgs P)
{
    __shared__ int32_t stacks[kOverlapBlock * kOverlapStack];
    __shared__ int32_t scan_scratch[kOverlapBlock / 64];
    const int32_t w = blockIdx.x;
    int32_t *stack = stacks + threadIdx.x * kOverlapStack;
    int32_t base = 0;
    for (int32_t ba = 0; ba < P.numBodyArchs; ba++) {
        const BodyArch &B = P.body[ba];
        const int32_t rows = B.numRows[w];
        for (int32_t chunk = 0; chunk < rows; chunk += kOverlapBlock) {
            const int32_t row = chunk + threadIdx.x;
            int32_t cnt = 0;
            if (row < rows) cnt = traverseOverlaps<false>(P, w, B, row, stack, 0);
            int32_t total;
            int32_t off = blockExclusiveScan(cnt, scan_scratch, &total);
            if (row < rows && cnt > 0) traverseOverlaps<true>(P, w, B, row, stack, base + off);
            base += total;
        }
    }
    if (threadIdx.x == 0) {
        if (base > P.candCapacity) {
            atomicOr(P.errorFlags + w, kErrCandidateOverflow);
            base = P.candCapacity;
        }
        P.numCands[w] = base;
        P.lastNumCands[w] = base;
    }
}

// ===========================================================================
// Substep integration (physics.cpp:79-164) fused with the world-space hull
// transform the narrowphase needs (narrowphase.cpp:139-212, CPU branch).
// ===========================================================================
__device__ __forceinline__ Vector3 multDiag(Vector3 d, Vector3 v)
{
    return Vector3 { d.x * v.x, d.y * v.y, d.z * v.z };
}

__global__ void __launch_bounds__(256) integrateKernel(PhysArgs P)
{
    const BodyArch &B = P.body[blockIdx.y];
    RowIdx ri = rowIndex(P, B);
    if (!ri.valid) return;
    const int32_t w = ri.w, r = ri.r;

    Vector3 &pos = bcol<Vector3>(B, Cols::Position, w, r);
    Quat &rot = bcol<Quat>(B, Cols::Rotation, w, r);
    const Velocity vel = bcol<Velocity>(B, Cols::Velocity, w, r);
    const int32_t obj = bcol<ObjectID>(B, Cols::ObjectID, w, r).idx;
    const ResponseType rt = bcol<ResponseType>(B, Cols::ResponseType, w, r);
    auto &prev = bcol<solver::SubstepPrevState>(B, Cols::SubstepPrevState, w, r);
    auto &ps_pos = bcol<solver::PreSolvePositional>(B, Cols::PreSolvePositional, w, r);
    auto &ps_vel = bcol<solver::PreSolveVelocity>(B, Cols::PreSolveVelocity, w, r);

    Vector3 x = pos;
    Quat q = rot;
    if (rt == ResponseType::Static) {
        prev.prevPosition = x;
        prev.prevRotation = q;
        ps_pos.x = x;
        ps_pos.q = q;
        ps_vel.v = Vector3::zero();
        ps_vel.omega = Vector3::zero();
    } else {
        Vector3 v = vel.linear;
        Vector3 omega = vel.angular;
        prev.prevPosition = x;
        prev.prevRotation = q;
        const SolverData &solver = P.solver[w];
        const RigidBodyMetadata md = P.objs.metadata[obj];
        const float inv_m = md.invMass;
        const Vector3 inv_I = md.invInertiaTensor;
        const float h = solver.h;
        const Vector3 ext_force = bcol<Vector3>(B, Cols::ExternalForce, w, r);
        const Vector3 ext_torque = bcol<Vector3>(B, Cols::ExternalTorque, w, r);
        if (rt == ResponseType::Dynamic) v += h * solver.g;
        v += h * inv_m * ext_force;
        x += h * v;
        Vector3 I {
            (inv_I.x == 0) ? 0.0f : 1.0f / inv_I.x,
            (inv_I.y == 0) ? 0.0f : 1.0f / inv_I.y,
            (inv_I.z == 0) ? 0.0f : 1.0f / inv_I.z,
        };
        Quat to_local = q.inv();
        Vector3 tau_ext_local = to_local.rotateVec(ext_torque);
        Vector3 omega_local = to_local.rotateVec(omega);
        Vector3 I_omega_local = multDiag(I, omega_local);
        omega_local += h * multDiag(inv_I, tau_ext_local - cross(omega_local, I_omega_local));
        omega = q.rotateVec(omega_local);
        Quat apply_omega = Quat::fromAngularVec(0.5f * h * omega);
        q += apply_omega * q;
        q = q.normalize();
        pos = x;
        rot = q;
        ps_pos.x = x;
        ps_pos.q = q;
        ps_vel.v = v;
        ps_vel.omega = omega;
    }

    // World-space hull for this body (makeHullState with dst buffers).
    if (P.objs.types[obj] == (uint32_t)CollisionPrimitive::Type::Hull) {
        const HullDev hd = P.objs.hulls[obj];
        const Diag3x3 scale = bcol<Diag3x3>(B, Cols::Scale, w, r);
        const int32_t leaf = bcol<broadphase::LeafID>(B, Cols::LeafID, w, r).id;
        Mat3x3 unscaled_rot = Mat3x3::fromQuat(q);
        Mat3x3 vertex_txfm = unscaled_rot * scale;
        Mat3x3 normal_txfm = unscaled_rot * scale.inv();
        Vector3 *dv = P.hullVerts + ((size_t)w * P.maxLeaves + leaf) * P.objs.maxVerts;
        geometry::Plane *dp = P.hullPlanes + ((size_t)w * P.maxLeaves + leaf) * P.objs.maxFaces;
        for (int32_t i = 0; i < hd.numVerts; i++) {
            dv[i] = vertex_txfm * P.objs.vertices[hd.vertOffset + i] + x;
        }
        for (int32_t i = 0; i < hd.numFaces; i++) {
            geometry::Plane op = P.objs.planes[hd.faceOffset + i];
            Vector3 origin = vertex_txfm * (op.normal * op.d) + x;
            Vector3 n = (normal_txfm * op.normal).normalize();
            dp[i] = geometry::Plane { n, dot(n, origin) };
        }
    }
}

// ===========================================================================
// Narrowphase (narrowphase.cpp, CPU branch), one lane per candidate
// ===========================================================================
struct HullRef {
    const Vector3 *verts;          // world space
    const geometry::Plane *planes; // world space
    HullDev hd;
    Vector3 center;
};

__device__ __forceinline__ float distFromPlane(const geometry::Plane &p, const Vector3 &a)
{
    float adotn = a.dot(p.normal);
    return adotn - p.d;
}

__device__ __forceinline__ Vector3 planeIntersection(const geometry::Plane &p, const Vector3 &p1,
                                                     const Vector3 &p2)
{
    float distance = distFromPlane(p, p1);
    return p1 + (p2 - p1) * (-distance / p.normal.dot(p2 - p1));
}

__device__ __forceinline__ float hullDistFromPlane(const geometry::Plane &p, const HullRef &h)
{
    float min_dot = FLT_MAX;
    for (int32_t i = 0; i < h.hd.numVerts; i++) {
        float d = p.normal.dot(h.verts[i]);
        if (d < min_dot) min_dot = d;
    }
    return min_dot - p.d;
}

struct FaceQuery {
    float separation;
    int32_t faceIdx;
    geometry::Plane plane;
};

__device__ FaceQuery queryFaceDirections(const HullRef &a, const HullRef &b)
{
    geometry::Plane max_plane { { 0, 0, 0 }, 0 };
    int32_t max_face = -1;
    float max_dist = -FLT_MAX;
    for (int32_t f = 0; f < a.hd.numFaces; f++) {
        geometry::Plane p = a.planes[f];
        float d = hullDistFromPlane(p, b);
        if (d > max_dist) {
            max_dist = d;
            max_face = f;
            max_plane = p;
            if (max_dist > 0) break;
        }
    }
    return { max_dist, max_face, max_plane };
}

__device__ __forceinline__ bool isMinkowskiFace(const Vector3 &a, const Vector3 &b,
                                                const Vector3 &c, const Vector3 &d)
{
    Vector3 bxa = b.cross(a);
    Vector3 dxc = d.cross(c);
    float cba = c.dot(bxa);
    float dba = d.dot(bxa);
    float adc = a.dot(dxc);
    float bdc = b.dot(dxc);
    return cba * dba < 0.0f && adc * bdc < 0.0f && cba * bdc > 0.0f;
}

struct EdgeQuery {
    float separation;
    Vector3 normal;
    int32_t edgeA;
    int32_t edgeB;
};

__device__ EdgeQuery queryEdgeDirections(const ObjDev &O, const HullRef &a, const HullRef &b)
{
    Vector3 normal { 0, 0, 0 };
    int32_t ea_max = 0, eb_max = 0;
    float max_d = -FLT_MAX;
    const geometry::HalfEdge *ha = O.hedges + a.hd.hedgeOffset;
    const geometry::HalfEdge *hb = O.hedges + b.hd.hedgeOffset;
    for (int32_t i = 0; i < a.hd.numEdges; i++) {
        const int32_t he_a = (int32_t)O.edges[a.hd.edgeOffset + i];
        const geometry::HalfEdge ea = ha[he_a];
        const Vector3 an1 = a.planes[ea.polygon].normal;
        const Vector3 an2 = a.planes[ha[ea.twin].polygon].normal;
        const Vector3 pa1 = a.verts[ea.rootVertex];
        const Vector3 pa2 = a.verts[ha[ea.next].rootVertex];
        for (int32_t j = 0; j < b.hd.numEdges; j++) {
            const int32_t he_b = (int32_t)O.edges[b.hd.edgeOffset + j];
            const geometry::HalfEdge eb = hb[he_b];
            const Vector3 bn1 = b.planes[eb.polygon].normal;
            const Vector3 bn2 = b.planes[hb[eb.twin].polygon].normal;
            float sep = -FLT_MAX;
            Vector3 n { 0, 0, 0 };
            if (isMinkowskiFace(an1, an2, -bn1, -bn2)) {      // edgeDistance :433-472
                const Vector3 pb1 = b.verts[eb.rootVertex];
                const Vector3 pb2 = b.verts[hb[eb.next].rootVertex];
                Vector3 da = pa2 - pa1, db = pb2 - pb1;
                Vector3 uc = da.cross(db);
                float l2 = uc.length2();
                if (l2 != 0) {
                    float inv = 1.f / sqrtf(l2);
                    n = uc * inv;
                    if (n.dot(pa1 - a.center) < 0.0f) n = -n;
                    sep = n.dot(pb1 - pa1);
                }
            }
            if (sep > max_d) {
                max_d = sep;
                normal = n;
                ea_max = he_a;
                eb_max = he_b;
                if (max_d > 0) return { max_d, normal, ea_max, eb_max };
            }
        }
    }
    return { max_d, normal, ea_max, eb_max };
}

__device__ __forceinline__ int32_t findIncidentFace(const HullRef &h, Vector3 ref_normal)
{
    float min_dot = FLT_MAX;
    int32_t face = -1;
    for (int32_t f = 0; f < h.hd.numFaces; f++) {
        float d = dot(h.planes[f].normal, ref_normal);
        if (d < min_dot) { min_dot = d; face = f; }
    }
    return face;
}

constexpr int32_t kMaxClip = 32;

__device__ __forceinline__ int32_t clipPolygon(Vector3 *dst, geometry::Plane cp,
                                               const Vector3 *in, int32_t n)
{                                                          // narrowphase.cpp:626-661
    if (n == 0) return 0;
    int32_t out = 0;
    Vector3 v1 = in[n - 1];
    float d1 = distFromPlane(cp, v1);
    for (int32_t i = 0; i < n; i++) {
        Vector3 v2 = in[i];
        float d2 = distFromPlane(cp, v2);
        if (d1 <= 0.0f && d2 <= 0.0f) {
            if (out < kMaxClip) dst[out++] = v2;
        } else if (d1 <= 0.0f && d2 > 0.0f) {
            if (out < kMaxClip) dst[out++] = planeIntersection(cp, v1, v2);
        } else if (d2 <= 0.0f && d1 > 0.0f) {
            if (out < kMaxClip) dst[out++] = planeIntersection(cp, v1, v2);
            if (out < kMaxClip) dst[out++] = v2;
        }
        v1 = v2;
        d1 = d2;
    }
    return out;
}

struct Manifold {
    Vector3 cp[4];
    float depth[4];
    int32_t num;
    Vector3 normal;
};

__device__ Manifold buildFaceContactManifold(Vector3 n, Vector3 *contacts, float *depths,
                                             int32_t num)
{                                                          // narrowphase.cpp:790-864
    Manifold m;
    for (int i = 0; i < 4; i++) { m.cp[i] = Vector3::zero(); m.depth[i] = 0.f; }
    if (num <= 4) {
        m.num = num;
        for (int32_t i = 0; i < num; i++) { m.cp[i] = contacts[i]; m.depth[i] = depths[i]; }
    } else {
        m.num = 4;
        m.cp[0] = contacts[0];
        m.depth[0] = depths[0];
        Vector3 p0 = m.cp[0];
        float largest_d2 = 0.0f;
        int32_t largest_d2_idx = 0;
        for (int32_t i = 1; i < num; i++) {
            Vector3 c = contacts[i];
            float d2 = p0.distance2(c);
            if (d2 > largest_d2) {
                largest_d2 = d2;
                m.cp[1] = c;
                m.depth[1] = depths[i];
                largest_d2_idx = i;
            }
        }
        contacts[largest_d2_idx] = m.cp[0];
        Vector3 diff0 = m.cp[1] - p0;
        const float largest_area = 0.0f;        // never updated in the reference
        int32_t largest_area_idx = 0;
        for (int32_t i = 1; i < num; i++) {
            Vector3 c = contacts[i];
            Vector3 diff1 = c - p0;
            float area = n.dot(diff0.cross(diff1));
            if (area > largest_area) {
                m.cp[2] = c;
                m.depth[2] = depths[i];
                largest_area_idx = i;
            }
        }
        contacts[largest_area_idx] = m.cp[0];
        for (int32_t i = 1; i < num; i++) {
            Vector3 c = contacts[i];
            Vector3 diff1 = c - p0;
            float area = n.dot(diff0.cross(diff1));
            if (area < largest_area) {
                m.cp[3] = c;
                m.depth[3] = depths[i];
            }
        }
    }
    const Quat ident { 1, 0, 0, 0 };
    for (int32_t i = 0; i < m.num; i++) m.cp[i] = ident.rotateVec(m.cp[i]) + Vector3::zero();
    m.normal = ident.rotateVec(n);
    return m;
}

__device__ __forceinline__ geometry::Segment shortestSegmentBetween(const geometry::Segment &s1,
                                                                    const geometry::Segment &s2)
{                                                          // narrowphase.cpp:1020-1051
    Vector3 v1 = s1.p2 - s1.p1;
    Vector3 v2 = s2.p2 - s2.p1;
    Vector3 v21 = s2.p1 - s1.p1;
    float dotv22 = v2.dot(v2);
    float dotv11 = v1.dot(v1);
    float dotv21 = v2.dot(v1);
    float dotv211 = v21.dot(v1);
    float dotv212 = v21.dot(v2);
    float denom = dotv21 * dotv21 - dotv22 * dotv11;
    float s, t;
    if (fabsf(denom) < 0.00001f) {
        s = 0.0f;
        t = (dotv11 * s - dotv211) / dotv21;
    } else {
        s = (dotv212 * dotv21 - dotv22 * dotv211) / denom;
        t = (-dotv211 * dotv21 + dotv11 * dotv212) / denom;
    }
    s = fmaxRef(fminRef(s, 1.0f), 0.0f);
    t = fmaxRef(fminRef(t, 1.0f), 0.0f);
    return { s1.p1 + s * v1, s2.p1 + t * v2 };
}

__device__ __forceinline__ void storeManifold(Contact &c, const Manifold &m, Loc ref, Loc alt)
{
    c.ref = ref;
    c.alt = alt;
    for (int i = 0; i < 4; i++) c.points[i] = Vector4::fromVector3(m.cp[i], m.depth[i]);
    c.numPoints = m.num;
    c.normal = m.normal;
    for (int i = 0; i < 4; i++) c.lambdaN[i] = 0.f;
}

constexpr int32_t kNarrowBlock = 128;

__global__ void __launch_bounds__(kNarrowBlock) narrowphaseKernel(PhysArgs P)
{
    const int32_t w = blockIdx.x;
    const int32_t num = min(P.numCands[w], P.candCapacity);
    const ObjDev &O = P.objs;
    for (int32_t ci = threadIdx.x; ci < num; ci += kNarrowBlock) {
        Contact &out = P.candContacts[(size_t)w * P.candCapacity + ci];
        out.numPoints = 0;
        const CandidateCollision cand = P.cands[(size_t)w * P.candCapacity + ci];
        Loc a_loc = cand.a, b_loc = cand.b;
        const BodyArch *BA = &P.body[bodyArchIndex(P, a_loc.archetype)];
        const BodyArch *BB = &P.body[bodyArchIndex(P, b_loc.archetype)];
        int32_t a_obj = bcol<ObjectID>(*BA, Cols::ObjectID, w, a_loc.row).idx;
        int32_t b_obj = bcol<ObjectID>(*BB, Cols::ObjectID, w, b_loc.row).idx;
        uint32_t ta = O.types[a_obj], tb = O.types[b_obj];
        if (ta > tb) {
            Loc tl = a_loc; a_loc = b_loc; b_loc = tl;
            const BodyArch *tB = BA; BA = BB; BB = tB;
            int32_t to = a_obj; a_obj = b_obj; b_obj = to;
            uint32_t tt = ta; ta = tb; tb = tt;
        }
        const Vector3 a_pos = bcol<Vector3>(*BA, Cols::Position, w, a_loc.row);
        const Vector3 b_pos = bcol<Vector3>(*BB, Cols::Position, w, b_loc.row);
        const Quat a_rot = bcol<Quat>(*BA, Cols::Rotation, w, a_loc.row);
        const Quat b_rot = bcol<Quat>(*BB, Cols::Rotation, w, b_loc.row);
        const Diag3x3 a_scale = bcol<Diag3x3>(*BA, Cols::Scale, w, a_loc.row);
        const Diag3x3 b_scale = bcol<Diag3x3>(*BB, Cols::Scale, w, b_loc.row);
        {
            AABB aw = O.aabbs[a_obj].applyTRS(a_pos, a_rot, a_scale);
            AABB bw = O.aabbs[b_obj].applyTRS(b_pos, b_rot, b_scale);
            if (!aw.overlaps(bw)) continue;
        }
        const uint32_t test = ta | tb;
        const int32_t a_leaf = bcol<broadphase::LeafID>(*BA, Cols::LeafID, w, a_loc.row).id;
        HullRef ha;
        ha.hd = O.hulls[a_obj];
        ha.verts = P.hullVerts + ((size_t)w * P.maxLeaves + a_leaf) * O.maxVerts;
        ha.planes = P.hullPlanes + ((size_t)w * P.maxLeaves + a_leaf) * O.maxFaces;
        ha.center = a_pos;
        Vector3 tmp1[kMaxClip], tmp2[kMaxClip];
        float depths[kMaxClip];

        if (test == (uint32_t)CollisionPrimitive::Type::Hull) {
            const int32_t b_leaf = bcol<broadphase::LeafID>(*BB, Cols::LeafID, w, b_loc.row).id;
            HullRef hb;
            hb.hd = O.hulls[b_obj];
            hb.verts = P.hullVerts + ((size_t)w * P.maxLeaves + b_leaf) * O.maxVerts;
            hb.planes = P.hullPlanes + ((size_t)w * P.maxLeaves + b_leaf) * O.maxFaces;
            hb.center = b_pos;

            // doSAT (narrowphase.cpp:678-758)
            FaceQuery fa = queryFaceDirections(ha, hb);
            if (fa.separation > 0.0f) continue;
            FaceQuery fb = queryFaceDirections(hb, ha);
            if (fb.separation > 0.0f) continue;
            EdgeQuery eq = queryEdgeDirections(O, ha, hb);
            if (eq.separation > 0.0f) continue;

            Manifold m;
            Loc ref_loc, other_loc;
            if (fa.separation > eq.separation || fb.separation > eq.separation) {
                const bool a_is_ref = fa.separation >= fb.separation;
                const geometry::Plane ref_plane = a_is_ref ? fa.plane : fb.plane;
                const int32_t ref_face = a_is_ref ? fa.faceIdx : fb.faceIdx;
                const HullRef &ref = a_is_ref ? ha : hb;
                const HullRef &inc = a_is_ref ? hb : ha;
                const int32_t inc_face = findIncidentFace(inc, ref_plane.normal);
                ref_loc = a_is_ref ? a_loc : b_loc;
                other_loc = a_is_ref ? b_loc : a_loc;

                // createFaceContact (narrowphase.cpp:866-972)
                const geometry::HalfEdge *rh = O.hedges + ref.hd.hedgeOffset;
                const geometry::HalfEdge *oh = O.hedges + inc.hd.hedgeOffset;
                int32_t n_in = 0;
                {
                    uint32_t hidx = O.polygons[inc.hd.faceOffset + inc_face], start = hidx;
                    do {
                        const geometry::HalfEdge he = oh[hidx];
                        hidx = he.next;
                        if (n_in < kMaxClip) tmp1[n_in++] = inc.verts[he.rootVertex];
                    } while (hidx != start);
                }
                Vector3 *cin = tmp1, *cdst = tmp2;
                int32_t n_clip = n_in;
                {
                    uint32_t hidx = O.polygons[ref.hd.faceOffset + ref_face], start = hidx;
                    geometry::HalfEdge che = rh[hidx];
                    Vector3 cur = ref.verts[che.rootVertex];
                    do {
                        hidx = che.next;
                        che = rh[hidx];
                        Vector3 next = ref.verts[che.rootVertex];
                        Vector3 edge = next - cur;
                        Vector3 pn = cross(edge, ref_plane.normal);
                        float d = dot(pn, cur);
                        cur = next;
                        n_clip = clipPolygon(cdst, geometry::Plane { pn, d }, cin, n_clip);
                        Vector3 *t = cdst; cdst = cin; cin = t;
                    } while (hidx != start);
                }
                int32_t n_below = 0;
                for (int32_t i = 0; i < n_clip; i++) {
                    Vector3 v = cin[i];
                    float d = distFromPlane(ref_plane, v);
                    if (d < 0.0f) {
                        cin[n_below] = v - d * ref_plane.normal;
                        depths[n_below] = -d;
                        n_below++;
                    }
                }
                m = buildFaceContactManifold(ref_plane.normal, cin, depths, n_below);
            } else {
                // createEdgeContact (narrowphase.cpp:1053-1121)
                ref_loc = a_loc;
                other_loc = b_loc;
                const geometry::HalfEdge *ha_e = O.hedges + ha.hd.hedgeOffset;
                const geometry::HalfEdge *hb_e = O.hedges + hb.hd.hedgeOffset;
                const geometry::HalfEdge ea = ha_e[eq.edgeA];
                const geometry::HalfEdge eb = hb_e[eq.edgeB];
                geometry::Segment sa { ha.verts[ea.rootVertex], ha.verts[ha_e[ea.next].rootVertex] };
                geometry::Segment sb { hb.verts[eb.rootVertex], hb.verts[hb_e[eb.next].rootVertex] };
                geometry::Segment s = shortestSegmentBetween(sa, sb);
                const Quat ident { 1, 0, 0, 0 };
                for (int i = 0; i < 4; i++) { m.cp[i] = Vector3::zero(); m.depth[i] = 0.f; }
                m.cp[0] = ident.rotateVec(s.p1) + Vector3::zero();
                m.depth[0] = -eq.separation;
                m.num = 1;
                m.normal = ident.rotateVec(eq.normal);
            }
            if (m.num > 0) storeManifold(out, m, ref_loc, other_loc);
        } else if (test == ((uint32_t)CollisionPrimitive::Type::Hull |
                            (uint32_t)CollisionPrimitive::Type::Plane)) {
            Vector3 pn = b_rot.rotateVec(Vector3 { 0, 0, 1 });
            geometry::Plane plane { pn, dot(pn, b_pos) };
            // doSATPlane (narrowphase.cpp:760-788)
            float sep = hullDistFromPlane(plane, ha);
            if (sep > 0.0f) continue;
            int32_t inc_face = findIncidentFace(ha, plane.normal);
            // createFacePlaneContact (narrowphase.cpp:974-1017)
            const geometry::HalfEdge *hh = O.hedges + ha.hd.hedgeOffset;
            int32_t n = 0;
            uint32_t hidx = O.polygons[ha.hd.faceOffset + inc_face], start = hidx;
            do {
                const geometry::HalfEdge he = hh[hidx];
                hidx = he.next;
                Vector3 v = ha.verts[he.rootVertex];
                float d = distFromPlane(plane, v);
                if (d < 0.0f && n < kMaxClip) {
                    tmp1[n] = v - d * plane.normal;
                    depths[n] = -d;
                    n++;
                }
            } while (hidx != start);
            Manifold m = buildFaceContactManifold(plane.normal, tmp1, depths, n);
            if (m.num > 0) storeManifold(out, m, b_loc, a_loc);
        }
        // sphere / plane-plane: the reference asserts (narrowphase.cpp:1197-1313)
    }
}

// ===========================================================================
// XPBD solver: solvePositions + setVelocities + solveVelocities
// (physics.cpp:166-1008), one wave per world, body state in LDS,
// level-scheduled contacts.
// ===========================================================================
struct SBody {
    Vector3 x;
    Quat q;
    Vector3 v;
    Vector3 omega;
    Vector3 prevX;
    Quat prevQ;
    Vector3 psX;
    Quat psQ;
    Vector3 psV;
    Vector3 psOmega;
    Vector3 invI;
    float invMass;
    float muS;
    float muD;
    uint32_t resp;
};

constexpr int32_t kSolverBlock = 64;

__device__ __forceinline__ int32_t bodySlot(const PhysArgs &P, Loc l)
{
    return P.body[bodyArchIndex(P, l.archetype)].slotBase + l.row;
}

__device__ __forceinline__ float computePositionalLambda(Vector3 ta1, Vector3 ta2, Vector3 ra1,
                                                         Vector3 ra2, float im1, float im2,
                                                         float c, float alpha)
{                                                          // physics.cpp:166-183
    float w1 = im1 + dot(ta1, ra1);
    float w2 = im2 + dot(ta2, ra2);
    return -c / (w1 + w2 + alpha);
}

__device__ __forceinline__ void applyPositionalUpdate(Vector3 &x1, Vector3 &x2, Quat &q1, Quat &q2,
                                                      Vector3 ral1, Vector3 ral2, float im1,
                                                      float im2, Vector3 n, float dl)
{                                                          // physics.cpp:185-211
    x1 += dl * im1 * n;
    x2 -= dl * im2 * n;
    float half = 0.5f * dl;
    Vector3 q1u = q1.rotateVec(half * ral1);
    Vector3 q2u = q2.rotateVec(half * ral2);
    q1 += Quat::fromAngularVec(q1u) * q1;
    q2 -= Quat::fromAngularVec(q2u) * q2;
    q1 = q1.normalize();
    q2 = q2.normalize();
}

__device__ void solveContactPositions(SBody &b1, SBody &b2, Contact &c)
{                                                          // physics.cpp:281-476
    Vector3 x1 = b1.x, x2 = b2.x;
    Quat q1 = b1.q, q2 = b2.q;
    float im1 = b1.invMass, im2 = b2.invMass;
    Vector3 iI1 = b1.invI, iI2 = b2.invI;
    if (b1.resp == (uint32_t)ResponseType::Static) { im1 = 0.f; iI1 = Vector3::zero(); }
    if (b2.resp == (uint32_t)ResponseType::Static) { im2 = 0.f; iI2 = Vector3::zero(); }
    const float avg_mu_s = 0.5f * (b1.muS + b2.muS);
    const Vector3 n = c.normal;
    for (int i = 0; i < 4; i++) {
        if (i >= c.numPoints) continue;
        Vector3 c1 = c.points[i].xyz();
        float depth = c.points[i].w;
        Vector3 c2 = c1 - n * depth;
        Vector3 r1 = b1.psQ.inv().rotateVec(c1 - b1.psX);
        Vector3 r2 = b2.psQ.inv().rotateVec(c2 - b2.psX);
        float lambda_n = 0.f;
        Vector3 p1 = q1.rotateVec(r1) + x1;
        Vector3 p2 = q2.rotateVec(r2) + x2;
        float d = dot(p1 - p2, n);
        if (d > 0) {
            Vector3 nl1 = q1.inv().rotateVec(n);
            Vector3 nl2 = q2.inv().rotateVec(n);
            Vector3 ta1 = cross(r1, nl1);
            Vector3 ta2 = cross(r2, nl2);
            Vector3 ra1 = multDiag(iI1, ta1);
            Vector3 ra2 = multDiag(iI2, ta2);
            lambda_n = computePositionalLambda(ta1, ta2, ra1, ra2, im1, im2, d, 0);
            applyPositionalUpdate(x1, x2, q1, q2, ra1, ra2, im1, im2, n, lambda_n);

            Vector3 p1_hat = b1.prevQ.rotateVec(r1) + b1.prevX;
            Vector3 p2_hat = b2.prevQ.rotateVec(r2) + b2.prevX;
            p1 = q1.rotateVec(r1) + x1;
            p2 = q2.rotateVec(r2) + x2;
            Vector3 dp = (p1 - p1_hat) - (p2 - p2_hat);
            Vector3 dpt = dp - dot(dp, n) * n;
            float tmag = dpt.length();
            if (tmag > 0.f) {
                Vector3 tw = dpt / tmag;
                Vector3 tl1 = q1.inv().rotateVec(tw);
                Vector3 tl2 = q2.inv().rotateVec(tw);
                Vector3 fta1 = cross(r1, tl1);
                Vector3 fta2 = cross(r2, tl2);
                Vector3 fra1 = multDiag(iI1, fta1);
                Vector3 fra2 = multDiag(iI2, fta2);
                float lambda_t = computePositionalLambda(fta1, fta2, fra1, fra2, im1, im2, tmag, 0);
                float thresh = lambda_n * avg_mu_s;
                if (lambda_t > thresh) {
                    applyPositionalUpdate(x1, x2, q1, q2, fra1, fra2, im1, im2, tw, lambda_t);
                }
            }
        }
        c.lambdaN[i] = lambda_n;
    }
    b1.x = x1; b2.x = x2;
    b1.q = q1; b2.q = q2;
}

__device__ __forceinline__ Vector3 relVel(Vector3 v1, Vector3 v2, Vector3 o1, Vector3 o2,
                                          Vector3 d1, Vector3 d2)
{
    return (v1 + cross(o1, d1)) - (v2 + cross(o2, d2));
}

__device__ __forceinline__ void applyVelocityUpdate(Vector3 &v1, Vector3 &v2, Vector3 &o1,
                                                    Vector3 &o2, Quat q1, Quat q2, Vector3 ta1,
                                                    Vector3 ta2, float im1, float im2,
                                                    Vector3 iI1, Vector3 iI2, Vector3 dv,
                                                    float mag)
{                                                          // physics.cpp:724-750
    Vector3 ra1 = multDiag(iI1, ta1);
    Vector3 ra2 = multDiag(iI2, ta2);
    float w1 = im1 + dot(ta1, ra1);
    float w2 = im2 + dot(ta2, ra2);
    mag *= 1.f / (w1 + w2);
    v1 += mag * im1 * dv;
    v2 -= mag * im2 * dv;
    Vector3 o1u = mag * ra1;
    Vector3 o2u = mag * ra2;
    o1 += q1.rotateVec(o1u);
    o2 -= q2.rotateVec(o2u);
}

__device__ void solveContactVelocities(SBody &b1, SBody &b2, const Contact &c, float h,
                                       float rest_thresh)
{                                                          // physics.cpp:865-993
    const Quat q1 = b1.q, q2 = b2.q;
    Vector3 v1 = b1.v, o1 = b1.omega, v2 = b2.v, o2 = b2.omega;
    float im1 = b1.invMass, im2 = b2.invMass;
    Vector3 iI1 = b1.invI, iI2 = b2.invI;
    if (b1.resp == (uint32_t)ResponseType::Static) { im1 = 0.f; iI1 = Vector3::zero(); }
    if (b2.resp == (uint32_t)ResponseType::Static) { im2 = 0.f; iI2 = Vector3::zero(); }
    const float mu_d = 0.5f * (b1.muD + b2.muD);
    const Vector3 n = c.normal;

    Vector3 r1l[4], r2l[4], r1w[4], r2w[4], rt1[4], rt2[4];
    float vn_bars[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        if (i >= c.numPoints) continue;
        Vector3 c1 = c.points[i].xyz();
        float depth = c.points[i].w;
        Vector3 c2 = c1 - n * depth;
        Vector3 r1 = b1.psQ.inv().rotateVec(c1 - b1.psX);
        Vector3 r2 = b2.psQ.inv().rotateVec(c2 - b2.psX);
        Vector3 r1p = b1.psQ.rotateVec(r1);
        Vector3 r2p = b2.psQ.rotateVec(r2);
        Vector3 vbar = relVel(b1.psV, b2.psV, b1.psOmega, b2.psOmega, r1p, r2p);
        vn_bars[i] = dot(n, vbar);
        r1l[i] = r1;
        r2l[i] = r2;
        r1w[i] = q1.rotateVec(r1);
        r2w[i] = q2.rotateVec(r2);
        rt1[i] = cross(r1, q1.inv().rotateVec(n));
        rt2[i] = cross(r2, q2.inv().rotateVec(n));
    }
    for (int it = 0; it < 2; it++) {                       // :813-863
#pragma unroll
        for (int i = 0; i < 4; i++) {
            if (i >= c.numPoints) continue;
            Vector3 v = relVel(v1, v2, o1, o2, r1w[i], r2w[i]);
            float vn = dot(n, v);
            float vn_bar = vn_bars[i];
            float e = 0.3f;
            if (fabsf(vn_bar) <= rest_thresh) e = 0.f;
            float mag = fminRef(-e * vn_bar, 0) - vn;
            applyVelocityUpdate(v1, v2, o1, o2, q1, q2, rt1[i], rt2[i], im1, im2, iI1, iI2, n, mag);
        }
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {                          // :752-811
        if (i >= c.numPoints) continue;
        Vector3 v = relVel(v1, v2, o1, o2, r1w[i], r2w[i]);
        float dfm = mu_d * fabsf(c.lambdaN[i]) / h;
        float vn = dot(n, v);
        Vector3 vt = v - n * vn;
        float vt_len = vt.length();
        if (vt_len != 0 && dfm != 0.f) {
            float corrected = -fminRef(dfm, vt_len);
            Vector3 dw = vt / vt_len;
            Vector3 d1l = q1.inv().rotateVec(dw);
            Vector3 d2l = q2.inv().rotateVec(dw);
            Vector3 fta1 = cross(r1l[i], d1l);
            Vector3 fta2 = cross(r2l[i], d2l);
            applyVelocityUpdate(v1, v2, o1, o2, q1, q2, fta1, fta2, im1, im2, iI1, iI2, dw,
                                corrected);
        }
    }
    b1.v = v1; b1.omega = o1;
    b2.v = v2; b2.omega = o2;
}

__device__ __forceinline__ bool isNegZero(float f) { return __float_as_uint(f) == 0x80000000u; }

// A static body is never written through if every solver write to it is an
// exact no-op: x +- (+-0) and q +- (+-0) keep bits when no component is -0,
// and normalize() must be idempotent on its rotation (static velocities are
// always +0 after setVelocities).  Such bodies add no ordering edge.
__device__ __forceinline__ bool staticInvariant(const SBody &b)
{
    if (b.resp != (uint32_t)ResponseType::Static) return false;
    if (isNegZero(b.x.x) || isNegZero(b.x.y) || isNegZero(b.x.z)) return false;
    if (isNegZero(b.q.w) || isNegZero(b.q.x) || isNegZero(b.q.y) || isNegZero(b.q.z)) return false;
    Quat nq = b.q.normalize();
    return __float_as_uint(nq.w) == __float_as_uint(b.q.w) &&
           __float_as_uint(nq.x) == __float_as_uint(b.q.x) &&
           __float_as_uint(nq.y) == __float_as_uint(b.q.y) &&
           __float_as_uint(nq.z) == __float_as_uint(b.q.z);
}

struct SolverLDS {
    SBody *bodies;        // [nb]
    int16_t *lastLevel;   // [nb]
    int16_t *lvl;         // [maxContacts]
    int16_t *slot1;       // [maxContacts]
    int16_t *slot2;       // [maxContacts]
};

__host__ __device__ inline size_t solverLDSBytes(int32_t nb, int32_t max_contacts)
{
    auto a16 = [](size_t b) { return (b + 15) & ~size_t(15); };
    return a16(sizeof(SBody) * nb) + a16(sizeof(int16_t) * nb) + 3 * a16(sizeof(int16_t) * max_contacts);
}

__device__ __forceinline__ SolverLDS solverLDS(char *smem, int32_t nb, int32_t max_contacts)
{
    auto a16 = [](size_t b) { return (b + 15) & ~size_t(15); };
    SolverLDS L;
    L.bodies = (SBody *)smem;
    char *p = smem + a16(sizeof(SBody) * nb);
    L.lastLevel = (int16_t *)p;
    p += a16(sizeof(int16_t) * nb);
    L.lvl = (int16_t *)p;
    p += a16(sizeof(int16_t) * max_contacts);
    L.slot1 = (int16_t *)p;
    p += a16(sizeof(int16_t) * max_contacts);
    L.slot2 = (int16_t *)p;
    return L;
}

__global__ void __launch_bounds__(kSolverBlock) solverKernel(PhysArgs P)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int32_t w = blockIdx.x;
    const int32_t nb = P.maxBodiesPerWorld;
    SolverLDS L = solverLDS(smem, nb, P.maxContacts);
    SBody *bodies = L.bodies;
    __shared__ int32_t s_num_contacts, s_max_level, s_scan[kSolverBlock / 64];

    // 1. load bodies into LDS
    for (int32_t ba = 0; ba < P.numBodyArchs; ba++) {
        const BodyArch &B = P.body[ba];
        const int32_t rows = B.numRows[w];
        for (int32_t r = threadIdx.x; r < rows; r += kSolverBlock) {
            SBody &s = bodies[B.slotBase + r];
            s.x = bcol<Vector3>(B, Cols::Position, w, r);
            s.q = bcol<Quat>(B, Cols::Rotation, w, r);
            const Velocity vel = bcol<Velocity>(B, Cols::Velocity, w, r);
            s.v = vel.linear;
            s.omega = vel.angular;
            const auto prev = bcol<solver::SubstepPrevState>(B, Cols::SubstepPrevState, w, r);
            s.prevX = prev.prevPosition;
            s.prevQ = prev.prevRotation;
            const auto psp = bcol<solver::PreSolvePositional>(B, Cols::PreSolvePositional, w, r);
            s.psX = psp.x;
            s.psQ = psp.q;
            const auto psv = bcol<solver::PreSolveVelocity>(B, Cols::PreSolveVelocity, w, r);
            s.psV = psv.v;
            s.psOmega = psv.omega;
            const int32_t obj = bcol<ObjectID>(B, Cols::ObjectID, w, r).idx;
            const RigidBodyMetadata md = P.objs.metadata[obj];
            s.invI = md.invInertiaTensor;
            s.invMass = md.invMass;
            s.muS = md.muS;
            s.muD = md.muD;
            s.resp = (uint32_t)bcol<ResponseType>(B, Cols::ResponseType, w, r);
            L.lastLevel[B.slotBase + r] = staticInvariant(s) ? (int16_t)-1 : (int16_t)0;
        }
    }

    // 2. ordered contact list: candidates with a manifold, in candidate order
    const int32_t ncand = min(P.numCands[w], P.candCapacity);
    const Contact *cslots = P.candContacts + (size_t)w * P.candCapacity;
    int32_t *order = P.contactOrder + (size_t)w * P.candCapacity;
    int32_t base = 0;
    for (int32_t chunk = 0; chunk < ncand; chunk += kSolverBlock) {
        const int32_t ci = chunk + threadIdx.x;
        const int32_t has = (ci < ncand && cslots[ci].numPoints > 0) ? 1 : 0;
        int32_t total;
        int32_t off = blockExclusiveScan(has, s_scan, &total);
        if (has) order[base + off] = ci;
        base += total;
    }
    if (base > P.maxContacts) {
        // The reference asserts here (narrowphase.cpp:1130); flag and truncate.
        if (threadIdx.x == 0) atomicOr(P.errorFlags + w, kErrContactOverflow);
        base = P.maxContacts;
    }
    const int32_t K = base;
    __syncthreads();
    for (int32_t k = threadIdx.x; k < K; k += kSolverBlock) {
        const Contact &c = cslots[order[k]];
        L.slot1[k] = (int16_t)bodySlot(P, c.ref);
        L.slot2[k] = (int16_t)bodySlot(P, c.alt);
    }
    __syncthreads();

    // 3. levels (serial, one lane, LDS only)
    if (threadIdx.x == 0) {
        int32_t max_level = 0;
        for (int32_t k = 0; k < K; k++) {
            const int32_t s1 = L.slot1[k], s2 = L.slot2[k];
            const int32_t l1 = L.lastLevel[s1], l2 = L.lastLevel[s2];
            const int32_t l = max(max(l1, l2), 0) + 1;
            L.lvl[k] = (int16_t)l;
            if (l1 >= 0) L.lastLevel[s1] = (int16_t)l;
            if (l2 >= 0) L.lastLevel[s2] = (int16_t)l;
            max_level = max(max_level, l);
        }
        s_num_contacts = K;
        s_max_level = max_level;
        P.lastNumContacts[w] = K;
    }
    __syncthreads();
    const int32_t max_level = s_max_level;
    const SolverData &sd = P.solver[w];
    int16_t *lvl = L.lvl;
    (void)s_num_contacts;

    // 4. solvePositions, level by level
    for (int32_t l = 1; l <= max_level; l++) {
        for (int32_t k = threadIdx.x; k < K; k += kSolverBlock) {
            if (lvl[k] != l) continue;
            Contact &c = P.candContacts[(size_t)w * P.candCapacity + order[k]];
            solveContactPositions(bodies[L.slot1[k]], bodies[L.slot2[k]], c);
        }
        __syncthreads();
    }

    // 5. setVelocities (physics.cpp:673-714)
    const float h = sd.h;
    for (int32_t ba = 0; ba < P.numBodyArchs; ba++) {
        const BodyArch &B = P.body[ba];
        const int32_t rows = B.numRows[w];
        for (int32_t r = threadIdx.x; r < rows; r += kSolverBlock) {
            SBody &s = bodies[B.slotBase + r];
            const Quat q = s.q, qp = s.prevQ;
            Quat dq;
            if (q.w != qp.w || q.x != qp.x || q.y != qp.y || q.z != qp.z) {
                dq = q * qp.inv();
            } else {
                dq = Quat { 1, 0, 0, 0 };
            }
            Vector3 new_omega = 2.f / h * Vector3 { dq.x, dq.y, dq.z };
            s.v = (s.x - s.prevX) / h;
            s.omega = dq.w > 0.f ? new_omega : -new_omega;
        }
    }
    __syncthreads();

    // 6. solveVelocities, same levels
    for (int32_t l = 1; l <= max_level; l++) {
        for (int32_t k = threadIdx.x; k < K; k += kSolverBlock) {
            if (lvl[k] != l) continue;
            const Contact &c = P.candContacts[(size_t)w * P.candCapacity + order[k]];
            solveContactVelocities(bodies[L.slot1[k]], bodies[L.slot2[k]], c, h,
                                   sd.restitutionThreshold);
        }
        __syncthreads();
    }

    // 7. write back
    for (int32_t ba = 0; ba < P.numBodyArchs; ba++) {
        const BodyArch &B = P.body[ba];
        const int32_t rows = B.numRows[w];
        for (int32_t r = threadIdx.x; r < rows; r += kSolverBlock) {
            const SBody &s = bodies[B.slotBase + r];
            bcol<Vector3>(B, Cols::Position, w, r) = s.x;
            bcol<Quat>(B, Cols::Rotation, w, r) = s.q;
            bcol<Velocity>(B, Cols::Velocity, w, r) = Velocity { s.v, s.omega };
        }
    }
}

static size_t solverSharedBytes(const PhysArgs &P)
{
    return solverLDSBytes(P.maxBodiesPerWorld, P.maxContacts);
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

MW_PHYS_NODE(UpdateBVHNode,
    hipLaunchKernelGGL(bvhRebuildKernel, dim3((P.numWorlds + 63) / 64), dim3(64), 0, stream, P);)

MW_PHYS_NODE(RefitNode,
    if (P.numBodyArchs > 0)
        hipLaunchKernelGGL(refitKernel, rowGrid(P), dim3(256), 0, stream, P);)

MW_PHYS_NODE(FindOverlappingNode,
    hipLaunchKernelGGL(findOverlapsKernel, dim3(P.numWorlds), dim3(kOverlapBlock), 0, stream, P);)

MW_PHYS_NODE(SubstepRigidBodiesNode,
    if (P.numBodyArchs > 0)
        hipLaunchKernelGGL(integrateKernel, rowGrid(P), dim3(256), 0, stream, P);)

MW_PHYS_NODE(NarrowphaseNode,
    hipLaunchKernelGGL(narrowphaseKernel, dim3(P.numWorlds), dim3(kNarrowBlock), 0, stream, P);)

MW_PHYS_NODE(SolverNode,
    hipLaunchKernelGGL(solverKernel, dim3(P.numWorlds), dim3(kSolverBlock),
                       solverSharedBytes(P), stream, P);)

// Joint constraints are collected per substep in the reference
// (collectConstraintsSystem, physics.cpp:34-40).  Joint solving is not on
// the scoped path; the node keeps the graph shape.
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
    registry.registerComponent<CandidateCollision>();
    registry.registerArchetype<CandidateTemporary>();
    mgr.setTemporary(typeKey<CandidateTemporary>());
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
            } else if (prim.type == CollisionPrimitive::Type::Sphere) {
                throw std::runtime_error("sphere primitives are unsupported (the reference asserts, "
                                         "narrowphase.cpp:1197-1313)");
            }
            m.hulls.push_back(hd);
        }
    } else if (m.maxLeaves != (int32_t)max_dynamic_objects ||
               m.maxContacts != (int32_t)max_contacts_per_world) {
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
        auto integrate = builder.addToGraph<SubstepRigidBodiesNode>({ cur });
        auto narrow = builder.addToGraph<NarrowphaseNode>({ integrate });
        auto reset1 = builder.addToGraph<ResetTmpAllocNode>({ narrow });
        // solvePositions + setVelocities + solveVelocities: one per-world
        // kernel (the three reference nodes are consecutive per world).
        auto solve = builder.addToGraph<SolverNode>({ reset1, collect });
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
