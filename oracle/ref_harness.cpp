// Reference harness (TEST INFRASTRUCTURE ONLY).
//
// Drives the *reference* CPU executor path of shacklettbp/gpu-ecs-madrona
// (compiled from the untouched sources under /root/reference by
// oracle/Makefile.ref) in single-world mode, which is the only mode in which
// the reference physics reads the right columns.  Every
// world owns a StateManager + StateCache + TaskGraph, exactly the recipe of
// SURVEY.md Appendix B.  The world definition below is the "collisions"
// physics workload of SURVEY.md §8(d) written against the reference's own
// registration API (registerTypes / setupTasks / world ctor).
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
// the resulting oracle/_ref/libmadrona_ref.so.  Nothing here is product code.

#include <madrona/taskgraph.hpp>
#include <madrona/custom_context.hpp>
#include <madrona/components.hpp>
#include <madrona/physics.hpp>
#include <madrona/state.hpp>

#include "core/worker_init.hpp"
#include "physics/physics_impl.hpp"

#include <cfloat>
#include <cstdio>
#include <cstring>
#include <new>
#include <thread>

#include <pthread.h>
#include <sched.h>
#include <vector>

using namespace madrona;
using namespace madrona::math;
using namespace madrona::base;
using namespace madrona::phys;

namespace refh {

// Body archetype: column order is the reference physics ABI (Cols 1..12,
// include/madrona/physics.hpp:449-464).
struct PhysicsBody : Archetype<
    Position, Rotation, Scale, Velocity, ObjectID, ResponseType,
    solver::SubstepPrevState, solver::PreSolvePositional,
    solver::PreSolveVelocity, ExternalForce, ExternalTorque,
    broadphase::LeafID> {};

// simple_taskgraph bodies (examples/simple_taskgraph/simple.hpp), same
// physics column layout, two archetypes.
struct SphereBody : Archetype<
    Position, Rotation, Scale, Velocity, ObjectID, ResponseType,
    solver::SubstepPrevState, solver::PreSolvePositional,
    solver::PreSolveVelocity, ExternalForce, ExternalTorque,
    broadphase::LeafID> {};
struct AgentBody : Archetype<
    Position, Rotation, Scale, Velocity, ObjectID, ResponseType,
    solver::SubstepPrevState, solver::PreSolvePositional,
    solver::PreSolveVelocity, ExternalForce, ExternalTorque,
    broadphase::LeafID> {};

struct RefPhysConfig {
    int32_t numCubes;
    int32_t numSubsteps;
    float deltaT;
    float gravityZ;
    int32_t maxContacts;
    float cubeInvMass;
    float cubeInvInertia;
    float muS;
    float muD;
    int32_t numJoints;      // joint pairs per world, 0 = none
    int32_t numHingeJoints; // the last numHingeJoints of them are hinges
};

struct WorldInit {
    const float *pos;   // numCubes * 3
    const float *rot;   // numCubes * 4 (w, x, y, z)
};

class Engine;

struct PhysWorld : public WorldBase {
    PhysWorld(Engine &ctx, ObjectManager *mgr, const RefPhysConfig &cfg,
              const WorldInit &init, bool simple = false, int32_t num_hulls = 1);

    AABB worldBounds;
};

class Engine : public CustomContext<Engine, PhysWorld> {
public:
    using CustomContext::CustomContext;
};

static void registerWorldTypes(ECSRegistry &reg)
{
    base::registerTypes(reg);
    RigidBodyPhysicsSystem::registerTypes(reg);
    reg.registerArchetype<PhysicsBody>();
}

// simple_taskgraph (examples/simple_taskgraph/simple.cpp:22-66), restated
// with cube hulls: clamp Position to the world bounds, then physics.
static void registerSimpleTypes(ECSRegistry &reg)
{
    base::registerTypes(reg);
    RigidBodyPhysicsSystem::registerTypes(reg);
    reg.registerArchetype<SphereBody>();
    reg.registerArchetype<AgentBody>();
}

static inline float clampRef(float v, float lo, float hi)
{
    return v < lo ? lo : (hi < v ? hi : v);
}

static void clampSystem(Engine &ctx, Position &position);

static void setupSimpleTasks(TaskGraph::Builder &builder, int32_t num_substeps)
{
    auto clamp = builder.addToGraph<ParallelForNode<Engine, clampSystem, Position>>({});
    auto bp = RigidBodyPhysicsSystem::setupBroadphaseTasks(builder, { clamp });
    auto sub = RigidBodyPhysicsSystem::setupSubstepTasks(builder, {bp},
                                                         num_substeps);
    RigidBodyPhysicsSystem::setupCleanupTasks(builder, {sub});
}

static void setupTasks(TaskGraph::Builder &builder, int32_t num_substeps)
{
    auto bp = RigidBodyPhysicsSystem::setupBroadphaseTasks(builder, {});
    auto sub = RigidBodyPhysicsSystem::setupSubstepTasks(builder, {bp},
                                                         num_substeps);
    RigidBodyPhysicsSystem::setupCleanupTasks(builder, {sub});
}

static void clampSystem(Engine &ctx, Position &position)
{
    const AABB &b = ctx.data().worldBounds;
    position.x = clampRef(position.x, b.pMin.x, b.pMax.x);
    position.y = clampRef(position.y, b.pMin.y, b.pMax.y);
    position.z = clampRef(position.z, b.pMin.z, b.pMax.z);
}

PhysWorld::PhysWorld(Engine &ctx, ObjectManager *mgr,
                     const RefPhysConfig &cfg, const WorldInit &init, bool simple,
                     int32_t num_hulls)
    : WorldBase(ctx),
      worldBounds { { -10, -10, 0 }, { 10, 10, 10 } }
{
    RigidBodyPhysicsSystem::init(ctx, mgr, cfg.deltaT, cfg.numSubsteps,
        Vector3 { 0.f, 0.f, cfg.gravityZ }, cfg.numCubes + (simple ? 2 : 1),
        cfg.maxContacts, cfg.numJoints > 16 ? cfg.numJoints : 16);

    auto setup = [&](Entity e, Vector3 p, Quat q, int32_t obj,
                     ResponseType rt) {
        ctx.getUnsafe<Position>(e) = Position { p };
        ctx.getUnsafe<Rotation>(e) = Rotation { q };
        ctx.getUnsafe<Scale>(e) = Scale { Diag3x3 { 1.f, 1.f, 1.f } };
        ctx.getUnsafe<Velocity>(e) = Velocity { Vector3::zero(),
                                                Vector3::zero() };
        ctx.getUnsafe<ObjectID>(e) = ObjectID { obj };
        ctx.getUnsafe<ResponseType>(e) = rt;
        ctx.getUnsafe<solver::SubstepPrevState>(e) = { p, q };
        ctx.getUnsafe<solver::PreSolvePositional>(e) = { p, q };
        ctx.getUnsafe<solver::PreSolveVelocity>(e) = {
            Vector3::zero(), Vector3::zero() };
        ctx.getUnsafe<ExternalForce>(e) = ExternalForce { Vector3::zero() };
        ctx.getUnsafe<ExternalTorque>(e) = ExternalTorque { Vector3::zero() };
        ctx.getUnsafe<broadphase::LeafID>(e) =
            RigidBodyPhysicsSystem::registerEntity(ctx, e, ObjectID { obj });
    };

    if (simple) {                          // simple.cpp:94-117
        for (int32_t i = 0; i < cfg.numCubes; i++) {
            Entity e = ctx.makeEntityNow<SphereBody>();
            Vector3 p { init.pos[3 * i], init.pos[3 * i + 1], init.pos[3 * i + 2] };
            Quat q { init.rot[4 * i], init.rot[4 * i + 1], init.rot[4 * i + 2],
                     init.rot[4 * i + 3] };
            setup(e, p, q, 0, ResponseType::Dynamic);
        }
        Entity agent = ctx.makeEntityNow<AgentBody>();
        setup(agent, Vector3 { 0, 0, 0 }, Quat::angleAxis(0.f, { 0, 1, 0 }), 0,
              ResponseType::Dynamic);
        Entity test = ctx.makeEntityNow<SphereBody>();
        setup(test, Vector3 { -10, 0, 0 }, Quat::angleAxis(0.f, { 0, 1, 0 }), 0,
              ResponseType::Dynamic);
        ctx.getSingleton<broadphase::BVH>().rebuildOnUpdate();
        return;
    }

    std::vector<Entity> cubes;
    for (int32_t i = 0; i < cfg.numCubes; i++) {
        Entity e = ctx.makeEntityNow<PhysicsBody>();
        Vector3 p { init.pos[3 * i], init.pos[3 * i + 1], init.pos[3 * i + 2] };
        Quat q { init.rot[4 * i], init.rot[4 * i + 1], init.rot[4 * i + 2],
                 init.rot[4 * i + 3] };
        setup(e, p, q, i % num_hulls, ResponseType::Dynamic);
        cubes.push_back(e);
    }

    Entity plane = ctx.makeEntityNow<PhysicsBody>();
    setup(plane, Vector3::zero(), Quat { 1.f, 0.f, 0.f, 0.f }, num_hulls,
          ResponseType::Static);

    // Joint workload (shared with the oracle and the collisions
    // environment): joint j ties cube 2j to cube 2j + 1, fixed,
    // or hinge for the last numHingeJoints, through the reference's own
    // setup helpers.
    for (int32_t j = 0; j < cfg.numJoints; j++) {
        Entity e1 = cubes[2 * j], e2 = cubes[2 * j + 1];
        Entity je = ctx.makeEntityNow<ConstraintData>();
        if (j < cfg.numJoints - cfg.numHingeJoints) {
            ctx.getUnsafe<JointConstraint>(je) = JointConstraint::setupFixed(
                e1, e2, Quat { 1.f, 0.f, 0.f, 0.f },
                Quat { 0.70710678f, 0.f, 0.f, 0.70710678f },
                Vector3 { 0.f, 1.5f, 0.f }, Vector3 { 0.f, -1.5f, 0.f }, 0.5f);
        } else {
            ctx.getUnsafe<JointConstraint>(je) = JointConstraint::setupHinge(
                e1, e2, Vector3 { 1, 0, 0 }, Vector3 { 1, 0, 0 },
                Vector3 { 0, 1, 0 }, Vector3 { 0, 1, 0 },
                Vector3 { 0.f, 0.f, 1.5f }, Vector3 { 0.f, 0.f, -1.5f });
        }
    }

    ctx.getSingleton<broadphase::BVH>().rebuildOnUpdate();
}

// Object table: object 0 = cube hull (half extent 1), object 1 = plane.
static ObjectManager * makeObjectManager(const RefPhysConfig &cfg)
{
    auto *mgr = new ObjectManager {};
    mgr->metadata = new RigidBodyMetadata[2];
    mgr->aabbs = new AABB[2];
    mgr->primitives = new CollisionPrimitive[2];

    const Vector3 verts[8] = {
        { -1, -1, -1 }, {  1, -1, -1 }, {  1,  1, -1 }, { -1,  1, -1 },
        { -1, -1,  1 }, {  1, -1,  1 }, {  1,  1,  1 }, { -1,  1,  1 },
    };
    const uint32_t faces[6][4] = {
        { 0, 3, 2, 1 }, { 4, 5, 6, 7 }, { 0, 1, 5, 4 },
        { 3, 7, 6, 2 }, { 0, 4, 7, 3 }, { 1, 2, 6, 5 },
    };

    geometry::FastPolygonList pl {};
    pl.allocate(6 * 5);
    pl.polygonCount = 0;
    pl.edgeCount = 0;
    for (int f = 0; f < 6; f++) {
        pl.addPolygon(Span<const uint32_t>(faces[f], 4));
    }

    mgr->primitives[0].type = CollisionPrimitive::Type::Hull;
    mgr->primitives[0].hull.halfEdgeMesh.construct(pl, 8, verts);

    mgr->metadata[0] = RigidBodyMetadata {
        { cfg.cubeInvInertia, cfg.cubeInvInertia, cfg.cubeInvInertia },
        cfg.cubeInvMass, cfg.muS, cfg.muD,
    };
    mgr->aabbs[0] = AABB { { -1, -1, -1 }, { 1, 1, 1 } };

    mgr->primitives[1].type = CollisionPrimitive::Type::Plane;
    mgr->metadata[1] = RigidBodyMetadata {
        { 0.f, 0.f, 0.f }, 0.f, cfg.muS, cfg.muD,
    };
    mgr->aabbs[1] = AABB {
        { -FLT_MAX, -FLT_MAX, -FLT_MAX },
        { FLT_MAX, FLT_MAX, 0.f },
    };

    return mgr;
}

// Object table of OBJ hulls, built the way PhysicsLoader::loadHullFromDisk
// does after import (physics_assets.cpp:205-254): FastPolygonList of the
// faces, HalfEdgeMesh::construct, AABB::point + AABB::expand; then the plane.
static ObjectManager * makeHullObjectManager(const RefPhysConfig &cfg,
    int32_t num_hulls, const int32_t *num_verts, const float *verts,
    const int32_t *num_faces, const int32_t *face_counts,
    const uint32_t *indices)
{
    auto *mgr = new ObjectManager {};
    mgr->metadata = new RigidBodyMetadata[num_hulls + 1];
    mgr->aabbs = new AABB[num_hulls + 1];
    mgr->primitives = new CollisionPrimitive[num_hulls + 1];
    for (int32_t h = 0; h < num_hulls; h++) {
        auto *vs = new Vector3[num_verts[h]];
        for (int32_t v = 0; v < num_verts[h]; v++) {
            vs[v] = Vector3 { verts[0], verts[1], verts[2] };
            verts += 3;
        }
        uint32_t space = 0;
        for (int32_t f = 0; f < num_faces[h]; f++) space += face_counts[f] + 1;
        geometry::FastPolygonList pl {};
        pl.allocate(space);
        pl.polygonCount = 0;
        pl.edgeCount = 0;
        for (int32_t f = 0; f < num_faces[h]; f++) {
            pl.addPolygon(Span<const uint32_t>(indices, face_counts[f]));
            indices += face_counts[f];
        }
        face_counts += num_faces[h];
        mgr->primitives[h].type = CollisionPrimitive::Type::Hull;
        mgr->primitives[h].hull.halfEdgeMesh.construct(pl, num_verts[h], vs);
        AABB box = AABB::point(vs[0]);
        for (int32_t v = 1; v < num_verts[h]; v++) box.expand(vs[v]);
        mgr->aabbs[h] = box;
        mgr->metadata[h] = RigidBodyMetadata {
            { cfg.cubeInvInertia, cfg.cubeInvInertia, cfg.cubeInvInertia },
            cfg.cubeInvMass, cfg.muS, cfg.muD,
        };
    }
    mgr->primitives[num_hulls].type = CollisionPrimitive::Type::Plane;
    mgr->metadata[num_hulls] = RigidBodyMetadata {
        { 0.f, 0.f, 0.f }, 0.f, cfg.muS, cfg.muD,
    };
    mgr->aabbs[num_hulls] = AABB {
        { -FLT_MAX, -FLT_MAX, -FLT_MAX },
        { FLT_MAX, FLT_MAX, 0.f },
    };
    return mgr;
}

struct RefWorld {
    StateManager sm;
    StateCache sc;
    PhysWorld *world;
    Engine *ctx;
    TaskGraph *graph;
    bool logCandidates = false;
    std::vector<CandidateCollision> candidates;   // logCandidates mode only
    int32_t numSubsteps = 0;
    // logCandidates mode: SolverData::numContacts right after the last
    // substep's narrowphase node (-1 when the node layout check fails)
    int32_t lastContactCount = -1;
};

// Mirror of TaskGraph's private layout (include/madrona/taskgraph.hpp:15-27,
// 89-94: HeapArray<Node> sorted_nodes_, HeapArray<NodeData> node_datas_) so
// a logged step can walk the built graph node by node, exactly as
// TaskGraph::run does (src/core/taskgraph.cpp:117-122), without editing the
// reference headers.
struct TaskGraphMirror {
    struct Node {
        void (*fn)(NodeBase *, Context *);
        uint32_t dataIDX;
        uint32_t numChildren;
    };
    struct alignas(128) NodeData {
        char userData[128];
    };
    Node *nodes;
    CountT numNodes;
    NodeData *datas;
    CountT numDatas;
};
static_assert(sizeof(TaskGraphMirror) == sizeof(TaskGraph));

// One step of a logged world: TaskGraph::run's loop, plus a read-only copy
// of the CandidateTemporary rows at the first node boundary where the table
// is non-empty.  Only findOverlapping appends to it and only the
// ClearTmpNode<CandidateTemporary> of setupSubstepTasks
// (src/physics/physics.cpp:1184-1185) empties it (Table::clear,
// src/common/table.cpp:83-86), so that copy is the step's full candidate
// list in emission order.  Nothing is written to world state.
//
// The step's contact count: the nodes are sorted in registration order
// (src/core/taskgraph.cpp:18-108), so after findOverlapping (node F, the one
// after which the candidate table is first non-empty) each substep adds 8
// nodes -- collectConstraints, substepRigidBodies, narrowphase and its
// ResetTmpAllocNode (narrowphase.cpp:1766-1785), solvePositions,
// setVelocities, solveVelocities, ResetTmpAlloc (src/physics/physics.cpp:
// 1157-1183) -- and SolverData::numContacts, which only narrowphase raises
// (narrowphase.cpp:1127) and solveVelocities resets (physics.cpp:1007), is
// read right after the last substep's narrowphase node (F + 3 + 8 (S - 1)).
// Layout checks: the count is 0 just before that node and again after its
// substep's solveVelocities (4 nodes later); otherwise -1.
static void runLogged(RefWorld *rw)
{
    auto *g = (TaskGraphMirror *)rw->graph;
    Engine &ctx = *rw->ctx;
    SolverData &solver = ctx.getSingleton<SolverData>();
    auto q = ctx.query<CandidateCollision>();
    bool done = false;
    CountT last_np = -1;
    rw->candidates.clear();
    rw->lastContactCount = 0;      // no candidates: no contacts
    bool layout_ok = true;
    for (CountT i = 0; i < g->numNodes; i++) {
        if (!done) {
            ctx.forEach(q, [&](CandidateCollision &c) {
                rw->candidates.push_back(c);
            });
            done = !rw->candidates.empty();
            if (done) last_np = i + 2 + 8 * (CountT)(rw->numSubsteps - 1);
        }
        if (i == last_np) layout_ok = layout_ok && solver.numContacts.load_relaxed() == 0;
        const auto &n = g->nodes[i];
        n.fn((NodeBase *)&g->datas[n.dataIDX].userData[0], rw->ctx);
        if (i == last_np) rw->lastContactCount = (int32_t)solver.numContacts.load_relaxed();
        if (last_np >= 0 && i == last_np + 4) {
            layout_ok = layout_ok && solver.numContacts.load_relaxed() == 0;
        }
    }
    if (!layout_ok || (done && last_np + 4 >= g->numNodes)) rw->lastContactCount = -1;
}

// Set before ref_phys_create: worlds created afterwards log their candidate
// pairs (ref_phys_set_candidate_log).  Off for the CPU baseline.
static bool g_logCandidates = false;

struct RefPhys {
    RefPhysConfig cfg;
    ObjectManager *mgr;
    std::vector<RefWorld *> worlds;
};

// Mirror of broadphase::BVH's private layout (include/madrona/physics.hpp:
// 303-396) so the harness can read node / leaf arrays without editing the
// reference headers.
struct BVHMirror {
    void *nodes;
    CountT numNodes;
    CountT numAllocatedNodes;
    Entity *leafEntities;
    CollisionPrimitive **leafPrimitives;
    AABB *leafAABBs;
    void *leafTransforms;
    uint32_t *leafParents;
    int32_t *sortedLeaves;
    AtomicI32 numLeaves;
    int32_t numAllocatedLeaves;
    float leafVelocityExpansion;
    float leafAccelExpansion;
    bool forceRebuild;
};
static_assert(sizeof(BVHMirror) == sizeof(broadphase::BVH));

}

using namespace refh;

extern "C" {

struct RefBodyState {
    uint32_t gen;
    int32_t id;
    float pos[3];
    float rot[4];
    float vel[6];
    float prevPos[3];
    float prevRot[4];
    float presolvePos[3];
    float presolveRot[4];
    float presolveVel[6];
    int32_t leafID;
    int32_t objID;
    uint32_t responseType;
};

static void * createWorlds(bool simple, int32_t num_worlds,
                                      const RefPhysConfig *cfg,
                                      const float *init_pos,
                                      const float *init_rot,
                                      ObjectManager *mgr = nullptr,
                                      int32_t num_hulls = 1)
{
    auto *h = new RefPhys {};
    h->cfg = *cfg;
    h->mgr = mgr ? mgr : makeObjectManager(*cfg);

    for (int32_t w = 0; w < num_worlds; w++) {
        auto *rw = new RefWorld {};
        ECSRegistry reg(&rw->sm, nullptr);
        if (simple) registerSimpleTypes(reg); else registerWorldTypes(reg);

        rw->world = (PhysWorld *)::operator new(sizeof(PhysWorld));
        rw->ctx = new Engine(rw->world, WorkerInit { &rw->sm, &rw->sc });

        WorldInit init {
            init_pos + (size_t)w * cfg->numCubes * 3,
            init_rot + (size_t)w * cfg->numCubes * 4,
        };
        new (rw->world) PhysWorld(*rw->ctx, h->mgr, *cfg, init, simple, num_hulls);
        rw->logCandidates = g_logCandidates && !simple;
        rw->numSubsteps = cfg->numSubsteps;

        TaskGraph::Builder builder(*rw->ctx);
        if (simple) setupSimpleTasks(builder, cfg->numSubsteps);
        else setupTasks(builder, cfg->numSubsteps);
        rw->graph = new TaskGraph(builder.build());
        h->worlds.push_back(rw);
    }

    return h;
}

MADRONA_EXPORT void * ref_phys_create(int32_t num_worlds,
                                      const RefPhysConfig *cfg,
                                      const float *init_pos,
                                      const float *init_rot)
{
    return createWorlds(false, num_worlds, cfg, init_pos, init_rot);
}

// One hull through the reference's HalfEdgeMesh::construct + AABB (same
// arguments as the oracle's orc_build_hull).
MADRONA_EXPORT void ref_build_hull(int32_t num_verts, const float *verts,
    int32_t num_faces, const int32_t *face_counts, const uint32_t *indices,
    int32_t *counts_out, float *verts_out, float *planes_out,
    uint32_t *half_edges_out, uint32_t *polys_out, uint32_t *edges_out,
    float *aabb_out)
{
    RefPhysConfig cfg {};
    ObjectManager *mgr = makeHullObjectManager(cfg, 1, &num_verts, verts,
        &num_faces, face_counts, indices);
    const geometry::HalfEdgeMesh &m = mgr->primitives[0].hull.halfEdgeMesh;
    counts_out[0] = (int32_t)m.mVertexCount;
    counts_out[1] = (int32_t)m.mPolygonCount;
    counts_out[2] = (int32_t)m.mEdgeCount;
    counts_out[3] = (int32_t)m.mHalfEdgeCount;
    memcpy(verts_out, m.mVertices, 12 * (size_t)m.mVertexCount);
    memcpy(planes_out, m.mFacePlanes, 16 * (size_t)m.mPolygonCount);
    memcpy(half_edges_out, m.mHalfEdges, 16 * (size_t)m.mHalfEdgeCount);
    memcpy(polys_out, m.mPolygons, 4 * (size_t)m.mPolygonCount);
    memcpy(edges_out, m.mEdges, 4 * (size_t)m.mEdgeCount);
    memcpy(aabb_out, &mgr->aabbs[0], 24);
}

// Collisions worlds over OBJ hulls (body i uses hull i % num_hulls); same
// geometry arguments as the oracle's orc_phys_create_hulls.
MADRONA_EXPORT void * ref_phys_create_hulls(int32_t num_worlds,
    const RefPhysConfig *cfg, const float *init_pos, const float *init_rot,
    int32_t num_hulls, const int32_t *num_verts, const float *verts,
    const int32_t *num_faces, const int32_t *face_counts,
    const uint32_t *indices)
{
    ObjectManager *mgr = makeHullObjectManager(*cfg, num_hulls, num_verts,
        verts, num_faces, face_counts, indices);
    return createWorlds(false, num_worlds, cfg, init_pos, init_rot, mgr,
                        num_hulls);
}

// simple_taskgraph worlds: cfg->numCubes objects + agent + test object.
MADRONA_EXPORT void * ref_simple_create(int32_t num_worlds,
                                        const RefPhysConfig *cfg,
                                        const float *init_pos,
                                        const float *init_rot)
{
    return createWorlds(true, num_worlds, cfg, init_pos, init_rot);
}

MADRONA_EXPORT void ref_phys_step(void *handle, int32_t num_steps)
{
    auto *h = (RefPhys *)handle;
    for (int32_t s = 0; s < num_steps; s++) {
        for (RefWorld *rw : h->worlds) {
            SolverData &solver = rw->ctx->getSingleton<SolverData>();
            // Poison the contact array so a reader can tell which prefix
            // the last substep wrote.
            memset((void *)solver.contacts, 0xFF,
                   sizeof(Contact) * solver.maxContacts);
            if (rw->logCandidates) runLogged(rw);
            else rw->graph->run(rw->ctx);
        }
    }
}

// Worlds are independent (one StateManager each), so a world-parallel loop
// over host threads is the reference ThreadPoolExecutor's job model
// (src/mw/cpu_exec.cpp:244-284) without its (unbuildable) render plumbing.
MADRONA_EXPORT void ref_phys_step_mt(void *handle, int32_t num_steps,
                                     int32_t num_threads)
{
    auto *h = (RefPhys *)handle;
    int32_t W = (int32_t)h->worlds.size();
    // One worker pinned per usable core, as ThreadPoolExecutor pins its
    // workers (src/mw/cpu_exec.cpp:56-93): the t-th CPU of this process's
    // affinity mask.
    cpu_set_t allowed;
    CPU_ZERO(&allowed);
    sched_getaffinity(0, sizeof(allowed), &allowed);
    std::vector<int> cpus;
    for (int c = 0; c < CPU_SETSIZE; c++) {
        if (CPU_ISSET(c, &allowed)) cpus.push_back(c);
    }
    std::vector<std::thread> pool;
    for (int32_t t = 0; t < num_threads; t++) {
        pool.emplace_back([=, &cpus]() {
            if (!cpus.empty()) {
                cpu_set_t one;
                CPU_ZERO(&one);
                CPU_SET(cpus[t % cpus.size()], &one);
                pthread_setaffinity_np(pthread_self(), sizeof(one), &one);
            }
            for (int32_t w = t; w < W; w += num_threads) {
                RefWorld *rw = h->worlds[w];
                for (int32_t s = 0; s < num_steps; s++) {
                    rw->graph->run(rw->ctx);
                }
            }
        });
    }
    for (auto &th : pool) th.join();
}

MADRONA_EXPORT int32_t ref_phys_num_bodies(void *handle)
{
    auto *h = (RefPhys *)handle;
    return h->cfg.numCubes + 1;
}

MADRONA_EXPORT void ref_phys_read_bodies(void *handle, int32_t world,
                                         RefBodyState *out)
{
    auto *h = (RefPhys *)handle;
    RefWorld *rw = h->worlds[world];
    Engine &ctx = *rw->ctx;

    Query<Entity, Position, Rotation, Velocity, solver::SubstepPrevState,
          solver::PreSolvePositional, solver::PreSolveVelocity,
          broadphase::LeafID, ObjectID, ResponseType> q =
        ctx.query<Entity, Position, Rotation, Velocity,
                  solver::SubstepPrevState, solver::PreSolvePositional,
                  solver::PreSolveVelocity, broadphase::LeafID, ObjectID,
                  ResponseType>();

    int32_t idx = 0;
    ctx.forEach(q, [&](Entity e, Position &p, Rotation &r, Velocity &v,
                       solver::SubstepPrevState &prev,
                       solver::PreSolvePositional &psp,
                       solver::PreSolveVelocity &psv,
                       broadphase::LeafID &leaf, ObjectID &obj,
                       ResponseType &rt) {
        RefBodyState &o = out[idx++];
        o.gen = e.gen;
        o.id = e.id;
        memcpy(o.pos, &p, 12);
        memcpy(o.rot, &r, 16);
        memcpy(o.vel, &v, 24);
        memcpy(o.prevPos, &prev.prevPosition, 12);
        memcpy(o.prevRot, &prev.prevRotation, 16);
        memcpy(o.presolvePos, &psp.x, 12);
        memcpy(o.presolveRot, &psp.q, 16);
        memcpy(o.presolveVel, &psv, 24);
        o.leafID = leaf.id;
        o.objID = obj.idx;
        o.responseType = (uint32_t)rt;
    });
}

// BVH snapshot: node array (116 B / node), leaf AABBs (24 B / leaf),
// leaf parents, sorted leaves.  Returns the number of nodes.
MADRONA_EXPORT int32_t ref_phys_read_bvh(void *handle, int32_t world,
                                         void *nodes_out,
                                         float *leaf_aabbs_out,
                                         uint32_t *leaf_parents_out,
                                         int32_t *sorted_leaves_out)
{
    auto *h = (RefPhys *)handle;
    RefWorld *rw = h->worlds[world];
    auto &bvh = rw->ctx->getSingleton<broadphase::BVH>();
    auto *m = (BVHMirror *)&bvh;
    int32_t num_leaves = m->numLeaves.load_relaxed();
    if (nodes_out) {
        memcpy(nodes_out, m->nodes, 116 * m->numNodes);
    }
    if (leaf_aabbs_out) {
        memcpy(leaf_aabbs_out, m->leafAABBs, sizeof(AABB) * num_leaves);
    }
    if (leaf_parents_out) {
        memcpy(leaf_parents_out, m->leafParents, 4 * num_leaves);
    }
    if (sorted_leaves_out) {
        memcpy(sorted_leaves_out, m->sortedLeaves, 4 * num_leaves);
    }
    return (int32_t)m->numNodes;
}

// Raw contact array (maxContacts * 112 B).  Entries written by the last
// substep form a prefix; untouched entries are 0xFF-poisoned.
MADRONA_EXPORT int32_t ref_phys_read_contacts(void *handle, int32_t world,
                                              void *out)
{
    auto *h = (RefPhys *)handle;
    RefWorld *rw = h->worlds[world];
    SolverData &solver = rw->ctx->getSingleton<SolverData>();
    memcpy(out, (void *)solver.contacts, sizeof(Contact) * solver.maxContacts);
    return (int32_t)solver.maxContacts;
}

MADRONA_EXPORT void ref_phys_set_candidate_log(int32_t on)
{
    g_logCandidates = on != 0;
}

// The last step's candidate pairs (Loc a, Loc b) in the reference's
// findOverlapping emission order; -1 when the worlds were created without
// the candidate log.  Returns the total count (copies at most cap).
MADRONA_EXPORT int32_t ref_phys_read_candidates(void *handle, int32_t world,
                                                void *out, int32_t cap)
{
    auto *h = (RefPhys *)handle;
    RefWorld *rw = h->worlds[world];
    if (!rw->logCandidates) return -1;
    int32_t n = (int32_t)rw->candidates.size();
    memcpy(out, rw->candidates.data(),
           sizeof(CandidateCollision) * (size_t)(n < cap ? n : cap));
    return n;
}

// The last step's last-substep contact count (logCandidates worlds; -1
// otherwise, or when runLogged's node layout check failed).
MADRONA_EXPORT int32_t ref_phys_last_contact_count(void *handle, int32_t world)
{
    auto *h = (RefPhys *)handle;
    RefWorld *rw = h->worlds[world];
    return rw->logCandidates ? rw->lastContactCount : -1;
}

MADRONA_EXPORT int32_t ref_sizeof(int32_t what)
{
    switch (what) {
    case 0: return sizeof(Contact);
    case 1: return sizeof(RefBodyState);
    case 2: return sizeof(JointConstraint);
    case 3: return sizeof(CandidateCollision);
    default: return -1;
    }
}

MADRONA_EXPORT void ref_phys_destroy(void *handle)
{
    // The reference has no teardown path for worlds that is safe to call
    // piecemeal (TaskGraph / StateManager own raw allocations); the harness
    // is process-scoped, so leak deliberately.
    (void)handle;
}

}
