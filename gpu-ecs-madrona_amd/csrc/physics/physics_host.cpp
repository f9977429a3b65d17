// Host side of the rigid-body physics module, shared by the gfx950 library
// and the CPU back end: half-edge geometry (restates src/physics/
// geometry.cpp:14-194), RigidBodyPhysicsSystem registration / init /
// registerEntity (src/physics/physics.cpp:1012-1081) and the PhysArgs
// layout of the module's per-world slabs.
#include "physics_module.hpp"

#include <cstdio>
#include <cstring>
#include <map>

namespace madrona::phys {

using namespace math;
using namespace base;

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
        if (!vec.empty()) memcpy(p, vec.data(), sizeof(T) * vec.size());
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
// Module state
// ===========================================================================
PhysicsModule &physicsModule(StateManager &mgr)
{
    auto *m = (PhysicsModule *)mgr.getExtension("physics");
    if (!m) throw std::runtime_error("physics module not registered");
    return *m;
}

namespace {
struct HostCtxPeek : Context {
    StateManager *mgr() { return mgr_; }
    int32_t world() { return world_; }
};
}

StateManager &ctxManager(Context &ctx) { return *static_cast<HostCtxPeek &>(ctx).mgr(); }

void PhysicsModule::buildArgs(void *stream)
{
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
        mgr->pinCapacity(archs[i]);       // PhysArgs keeps its slab pointers and capacity
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
    P.nodes = alloc<BVHNode>((size_t)W * maxNodes, stream);
    P.leafEntities = upload(leafEntitiesHost, stream);
    P.leafAABBs = alloc<AABB>((size_t)W * maxLeaves, stream);
    P.leafParents = alloc<uint32_t>((size_t)W * maxLeaves, stream);
    P.sortedLeaves = alloc<int32_t>((size_t)W * maxLeaves, stream);
    P.leafOrder = alloc<int32_t>((size_t)W * maxLeaves, stream);

    ObjDev &O = P.objs;
    O.numObjects = (int32_t)metadata.size();
    if (O.numObjects > 65535) {
        // narrowphase work entries hold object ids in 16 bits (PackedSatWork)
        throw std::runtime_error("physics: more than 65535 collision objects");
    }
    O.maxVerts = 0;
    O.maxFaces = 0;
    O.maxEdges = 0;
    for (const HullDev &h : hulls) {
        O.maxVerts = std::max(O.maxVerts, h.numVerts);
        O.maxFaces = std::max(O.maxFaces, h.numFaces);
        O.maxEdges = std::max(O.maxEdges, h.numEdges);
    }
    O.minkStride = O.maxEdges * O.maxFaces <= 128 ? O.maxFaces : 0;
    O.metadata = upload(metadata, stream);
    O.aabbs = upload(aabbs, stream);
    O.types = upload(types, stream);
    O.hulls = upload(hulls, stream);
    O.vertices = upload(vertices, stream);
    O.planes = upload(planes, stream);
    O.hedges = upload(hedges, stream);
    O.edges = upload(edges, stream);
    O.edgeQuads = upload(edgeQuads, stream);
    O.polygons = upload(polygons, stream);
    O.numVertsTotal = (int32_t)vertices.size();
    O.numPlanesTotal = (int32_t)planes.size();
    O.numHedgesTotal = (int32_t)hedges.size();
    O.numPolygonsTotal = (int32_t)polygons.size();
    O.numEdgesTotal = (int32_t)edgeQuads.size();

    P.bodyBoxes = alloc<BodyBox>((size_t)W * std::max(P.maxBodiesPerWorld, 1), stream);
    P.survInfo = alloc<uint32_t>((size_t)W * P.candCapacity, stream);
    P.candSlots = alloc<uint64_t>((size_t)W * P.candCapacity, stream);
    P.survCount = alloc<int32_t>(W, stream);
    P.solverOrder = alloc<int32_t>(W, stream);
    P.binCap = (W + kNarrowBins - 1) / kNarrowBins * P.candCapacity;
    for (int32_t set = 0; set < 2; set++) {
        P.satWorkSet[set] = alloc<PackedSatWork>((size_t)kNarrowBins * P.binCap, stream);
        P.satWorkCountSet[set] = alloc<int32_t>(kNarrowBins * kBinStride, stream);
    }
    P.satWork = P.satWorkSet[0];
    P.satWorkCount = P.satWorkCountSet[0];
    P.nextSatWork = P.satWorkSet[1];
    P.nextSatWorkCount = P.satWorkCountSet[1];
    P.hhJobs = alloc<ContactJob>((size_t)W * P.candCapacity, stream);
    P.hhKinds = alloc<int8_t>((size_t)W * P.candCapacity, stream);
    P.candContacts = alloc<Contact>((size_t)W * P.candCapacity, stream);
    P.maxContacts = maxContacts;
    P.contactOrder = alloc<int32_t>((size_t)W * P.candCapacity, stream);
    const int32_t joint_arch = mgr->archetypeIndex(typeKey<ConstraintData>());
    mgr->pinCapacity(joint_arch);         // PhysArgs keeps its slab pointer and capacity
    P.jointCapacity = dv.arch[joint_arch].capacity;
    P.numJointRows = dv.arch[joint_arch].numRows;
    P.joints = (JointConstraint *)dv.arch[joint_arch].cols[1];
    P.maxJoints = maxJoints;
    P.recStride = P.candCapacity + std::min(maxJoints, P.jointCapacity);
    if (P.recStride > 32767) {
        throw std::runtime_error("physics: max candidates + joints per world must be <= 32767");
    }
    P.solverRecs = alloc<uint64_t>((size_t)W * P.recStride, stream);
    P.solverPrevs = alloc<int32_t>((size_t)W * P.recStride, stream);
    P.lastNumContacts = alloc<int32_t>(W, stream);
    P.lastNumCands = alloc<int32_t>(W, stream);
    P.unitAccum = alloc<unsigned long long>(kUnitSlots, stream);

}

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
    PhysicsModule &m = physicsModule(mgr);
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
    PhysicsModule &m = physicsModule(ctxManager(ctx));
    broadphase::BVH &bvh = ctx.getSingleton<broadphase::BVH>();
    int32_t leaf = bvh.numLeaves++;
    if (leaf >= m.maxLeaves) throw std::runtime_error("BVH leaf capacity exceeded");
    m.leafEntitiesHost[(size_t)bvh.worldIdx * m.maxLeaves + leaf] = e;
    return broadphase::LeafID { leaf };
}

// Debug / test access to module slabs (used by the C ABI).
PhysArgs *physicsArgs(StateManager &mgr)
{
    auto *m = (PhysicsModule *)mgr.getExtension("physics");
    return m && m->uploaded ? &m->args : nullptr;
}

}
