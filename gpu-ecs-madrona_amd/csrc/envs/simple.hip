// "simple_taskgraph" environment (BASELINE.json configs[0] / [1], SURVEY.md
// §8(d) C1 / C2): examples/simple_taskgraph/simple.cpp:22-122 restated onto
// the current physics API (the example targets an older one and does not
// build): per world num_objects "Sphere" bodies at the
// reference init positions, one "Agent" body at the origin and one test
// Sphere at (-10, 0, 0) (simple.cpp:94-117); sphere narrowphase asserts in
// the reference (narrowphase.cpp:1197-1225), so every body is the unit-cube
// hull.  Nodes: clampSystem (ParallelForNode<Position>, simple.cpp:22-35) ->
// rigid-body physics -> physics cleanup (simple.cpp:51-66).  Two body
// archetypes exercise the multi-archetype physics path.
#include <madrona/mw_gpu.hpp>
#include <madrona/physics.hpp>

#include "../runtime/env_registry.hpp"
#include "cube_assets.hpp"

#include <cstring>

using namespace madrona;
using namespace madrona::math;
using namespace madrona::base;
using namespace madrona::phys;

namespace SimpleTaskgraph {

#define SIMPLE_BODY_COLS                                                   \
    Position, Rotation, Scale, Velocity, ObjectID, ResponseType,           \
        solver::SubstepPrevState, solver::PreSolvePositional,              \
        solver::PreSolveVelocity, ExternalForce, ExternalTorque, broadphase::LeafID

struct Sphere : Archetype<SIMPLE_BODY_COLS> {};
struct Agent : Archetype<SIMPLE_BODY_COLS> {};

struct Config {
    mw_collisions_config c;        // num_cubes = objects per world
    ObjectManager *objMgr;
};

class Engine;

struct SimpleSim : public WorldBase {
    static void registerTypes(ECSRegistry &reg, const Config &cfg)
    {                                                      // simple.cpp:37-49
        base::registerTypes(reg);
        RigidBodyPhysicsSystem::setMaxCandidatesPerWorld(reg, cfg.c.max_candidates);
        RigidBodyPhysicsSystem::registerTypes(reg);
        reg.registerFixedSizeArchetype<Sphere>(cfg.c.num_cubes + 1);
        reg.registerFixedSizeArchetype<Agent>(1);
        reg.exportColumn<Agent, Position>(0);
        reg.exportColumn<Agent, Rotation>(1);
    }

    static void setupTasks(TaskGraph::Builder &builder, const Config &cfg)
    {                                                      // simple.cpp:51-66
        auto clamp = builder.addToGraph<ParallelForNode<Engine, clampSystem, Position>>({});
        auto bp = RigidBodyPhysicsSystem::setupBroadphaseTasks(builder, { clamp });
        auto sub = RigidBodyPhysicsSystem::setupSubstepTasks(builder, { bp },
                                                             cfg.c.num_substeps);
        RigidBodyPhysicsSystem::setupCleanupTasks(builder, { sub });
    }

    SimpleSim(Engine &ctx, const Config &cfg, const mw_collisions_init &init);

    static MW_HD void clampSystem(Engine &ctx, Position &position);

    AABB worldBounds;
};

class Engine : public CustomContext<Engine, SimpleSim> {
public:
    using CustomContext::CustomContext;
};

MW_HD static inline float clampRef(float v, float lo, float hi)
{                                                          // std::clamp
    return v < lo ? lo : (hi < v ? hi : v);
}

MW_HD void SimpleSim::clampSystem(Engine &ctx, Position &position)
{                                                          // simple.cpp:22-35
    const AABB &b = ctx.data().worldBounds;
    position.x = clampRef(position.x, b.pMin.x, b.pMax.x);
    position.y = clampRef(position.y, b.pMin.y, b.pMax.y);
    position.z = clampRef(position.z, b.pMin.z, b.pMax.z);
}

SimpleSim::SimpleSim(Engine &ctx, const Config &cfg, const mw_collisions_init &init)
    : WorldBase(ctx)
{                                                          // simple.cpp:68-117
    const mw_collisions_config &c = cfg.c;
    worldBounds = AABB { { -10, -10, 0 }, { 10, 10, 10 } };   // init.cpp:38-41
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
    Entity agent = ctx.makeEntityNow<Agent>();
    setup(agent, Vector3 { 0, 0, 0 }, Quat::angleAxis(0.f, Vector3 { 0, 1, 0 }));
    Entity test = ctx.makeEntityNow<Sphere>();
    setup(test, Vector3 { -10, 0, 0 }, Quat::angleAxis(0.f, Vector3 { 0, 1, 0 }));

    ctx.getSingleton<broadphase::BVH>().rebuildOnUpdate();
}

using Exec = TaskGraphExecutor<Engine, SimpleSim, Config, mw_collisions_init>;

static Executor *create(const ExecConfig &ecfg, const void *user_cfg, size_t cfg_bytes,
                        const void *inits, size_t init_stride)
{
    if (cfg_bytes != sizeof(mw_collisions_config)) {
        throw std::runtime_error("simple_taskgraph: user config size mismatch");
    }
    Config cfg;
    memcpy(&cfg.c, user_cfg, sizeof(cfg.c));
    cfg.objMgr = envs::makeCubeObjectManager(cfg.c);
    std::vector<mw_collisions_init> init_vec(ecfg.numWorlds);
    for (int32_t w = 0; w < ecfg.numWorlds; w++) {
        memcpy(&init_vec[w], (const char *)inits + (size_t)w * init_stride,
               sizeof(mw_collisions_init));
    }
    return new Exec(ecfg, cfg, init_vec.data());
}

static EnvRegistration reg("simple_taskgraph", &create);

}
