// "phys_grow" test world (TEST WORKLOAD): simple_taskgraph's physics world
// (csrc/envs/simple.hip: Sphere bodies + one Agent, clamp -> rigid-body
// physics) plus a growable "Mark" table that the agent fills with kMarksPerStep
// entities every step.  Built out of tree like ecs_ops.hip.
//
// Every growth of Mark re-allocates the entity ID store, whose pointer and
// size the physics module caches in its kernel arguments (the
// module read the freed store after a growth).  The marks never touch a
// body, so the bodies must stay bit-identical to the built-in
// simple_taskgraph world stepping the same inits
// (tests/test_phys_grow.py).
#include <madrona/mw_gpu.hpp>
#include <madrona/mw_gpu_entry.hpp>
#include <madrona/physics.hpp>

#include "../../gpu-ecs-madrona_amd/csrc/envs/cube_assets.hpp"

#include <cstring>
#include <stdexcept>
#include <vector>

using namespace madrona;
using namespace madrona::math;
using namespace madrona::base;
using namespace madrona::phys;

namespace PhysGrow {

constexpr int32_t kMarksPerStep = 8;

#define PG_BODY_COLS                                                       \
    Position, Rotation, Scale, Velocity, ObjectID, ResponseType,           \
        solver::SubstepPrevState, solver::PreSolvePositional,              \
        solver::PreSolveVelocity, ExternalForce, ExternalTorque, broadphase::LeafID

// the same archetypes in the same order as simple_taskgraph, then Mark
struct Sphere : Archetype<PG_BODY_COLS> {};
struct Agent : Archetype<PG_BODY_COLS> {};

struct MarkInfo {
    Entity agent;
    int32_t tick;
    int32_t serial;
};
struct Mark : Archetype<MarkInfo> {};

struct Config {
    mw_collisions_config c;
    ObjectManager *objMgr;
};

class Engine;

struct World : public WorldBase {
    static void registerTypes(ECSRegistry &reg, const Config &cfg)
    {
        base::registerTypes(reg);
        RigidBodyPhysicsSystem::setMaxCandidatesPerWorld(reg, cfg.c.max_candidates);
        RigidBodyPhysicsSystem::registerTypes(reg);
        reg.registerFixedSizeArchetype<Sphere>(cfg.c.num_cubes + 1);
        reg.registerFixedSizeArchetype<Agent>(1);
        reg.registerComponent<MarkInfo>();
        reg.registerArchetype<Mark>();        // grows past mw_config.default_capacity
    }

    static void setupTasks(TaskGraph::Builder &builder, const Config &cfg)
    {
        auto clamp = builder.addToGraph<ParallelForNode<Engine, clampSystem, Position>>({});
        auto mark = builder.addToGraph<ParallelForNode<Engine, markSystem, Entity, ObjectID,
                                                       broadphase::LeafID>>({ clamp });
        auto bp = RigidBodyPhysicsSystem::setupBroadphaseTasks(builder, { mark });
        auto sub = RigidBodyPhysicsSystem::setupSubstepTasks(builder, { bp }, cfg.c.num_substeps);
        RigidBodyPhysicsSystem::setupCleanupTasks(builder, { sub });
    }

    World(Engine &ctx, const Config &cfg, const mw_collisions_init &init);

    static MW_HD void clampSystem(Engine &ctx, Position &position);
    static MW_HD void markSystem(Engine &ctx, Entity e, ObjectID &, broadphase::LeafID &);

    AABB worldBounds;
    int32_t tick;
    int32_t marks;
    Entity agent;
};

class Engine : public CustomContext<Engine, World> {
public:
    using CustomContext::CustomContext;
};

MW_HD static inline float clampRef(float v, float lo, float hi)
{
    return v < lo ? lo : (hi < v ? hi : v);
}

MW_HD void World::clampSystem(Engine &ctx, Position &position)
{
    const AABB &b = ctx.data().worldBounds;
    position.x = clampRef(position.x, b.pMin.x, b.pMax.x);
    position.y = clampRef(position.y, b.pMin.y, b.pMax.y);
    position.z = clampRef(position.z, b.pMin.z, b.pMax.z);
}

// Runs for every body row; only the agent's row makes marks.
MW_HD void World::markSystem(Engine &ctx, Entity e, ObjectID &, broadphase::LeafID &)
{
    World &d = ctx.data();
    if (e != d.agent) return;
    for (int32_t i = 0; i < kMarksPerStep; i++) {
        ctx.makeEntityNow<Mark>(MarkInfo { e, d.tick, d.marks });
        d.marks++;
    }
    d.tick++;
}

World::World(Engine &ctx, const Config &cfg, const mw_collisions_init &init)
    : WorldBase(ctx)
{
    const mw_collisions_config &c = cfg.c;
    worldBounds = AABB { { -10, -10, 0 }, { 10, 10, 10 } };
    tick = 0;
    marks = 0;
    RigidBodyPhysicsSystem::init(ctx, cfg.objMgr, c.delta_t, c.num_substeps,
                                 Vector3 { 0.f, 0.f, c.gravity_z }, c.num_cubes + 2,
                                 c.max_contacts, 16);
    auto setup = [&](Entity e, Vector3 p, Quat q) {
        ctx.getUnsafe<Position>(e) = Position { p };
        ctx.getUnsafe<Rotation>(e) = Rotation { q };
        ctx.getUnsafe<Scale>(e) = Scale { Diag3x3 { 1.f, 1.f, 1.f } };
        ctx.getUnsafe<Velocity>(e) = Velocity { Vector3::zero(), Vector3::zero() };
        ctx.getUnsafe<ObjectID>(e) = ObjectID { 0 };
        ctx.getUnsafe<ResponseType>(e) = ResponseType::Dynamic;
        ctx.getUnsafe<solver::SubstepPrevState>(e) = { p, q };
        ctx.getUnsafe<solver::PreSolvePositional>(e) = { p, q };
        ctx.getUnsafe<solver::PreSolveVelocity>(e) = { Vector3::zero(), Vector3::zero() };
        ctx.getUnsafe<ExternalForce>(e) = ExternalForce { Vector3::zero() };
        ctx.getUnsafe<ExternalTorque>(e) = ExternalTorque { Vector3::zero() };
        ctx.getUnsafe<broadphase::LeafID>(e) =
            RigidBodyPhysicsSystem::registerEntity(ctx, e, ObjectID { 0 });
    };
    for (int32_t i = 0; i < c.num_cubes; i++) {
        Entity e = ctx.makeEntityNow<Sphere>();
        setup(e, Vector3 { init.pos[3 * i], init.pos[3 * i + 1], init.pos[3 * i + 2] },
              Quat { init.rot[4 * i], init.rot[4 * i + 1], init.rot[4 * i + 2], init.rot[4 * i + 3] });
    }
    agent = ctx.makeEntityNow<Agent>();
    setup(agent, Vector3 { 0, 0, 0 }, Quat::angleAxis(0.f, Vector3 { 0, 1, 0 }));
    Entity test = ctx.makeEntityNow<Sphere>();
    setup(test, Vector3 { -10, 0, 0 }, Quat::angleAxis(0.f, Vector3 { 0, 1, 0 }));
    ctx.getSingleton<broadphase::BVH>().rebuildOnUpdate();
}

using Exec = TaskGraphExecutor<Engine, World, Config, mw_collisions_init>;

static Executor *create(const ExecConfig &ecfg, const void *user_cfg, size_t cfg_bytes,
                        const void *inits, size_t init_stride)
{
    if (cfg_bytes != sizeof(mw_collisions_config)) throw std::runtime_error("phys_grow: config size");
    if (init_stride < sizeof(mw_collisions_init)) throw std::runtime_error("phys_grow: init stride");
    Config cfg;
    memcpy(&cfg.c, user_cfg, sizeof(cfg.c));
    cfg.objMgr = envs::makeCubeObjectManager(cfg.c);
    std::vector<mw_collisions_init> v(ecfg.numWorlds);
    for (int32_t w = 0; w < ecfg.numWorlds; w++)
        memcpy(&v[w], (const char *)inits + (size_t)w * init_stride, sizeof(mw_collisions_init));
    return new Exec(ecfg, cfg, v.data());
}

static EnvRegistration reg("phys_grow", &create);

}
