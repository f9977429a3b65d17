// "collisions" environment: the rigid-body workload of SURVEY.md §8(d)
// (C3/C4): per world num_cubes unit-cube hulls + one static ground plane,
// stepped by RigidBodyPhysicsSystem.  Written against the reference's
// registration API (registerTypes / setupTasks / world ctor, reference
// include/madrona/mw_cpu.inl:15-69) exactly like oracle/ref_harness.cpp's
// world, which is the same world compiled against the reference itself.
#include <madrona/mw_gpu.hpp>
#include <madrona/physics.hpp>

#include "../runtime/env_registry.hpp"
#include "cube_assets.hpp"
#include "../../../include/madrona_mw.h"

#include <cfloat>
#include <cstring>
#include <random>

using namespace madrona;
using namespace madrona::math;
using namespace madrona::base;
using namespace madrona::phys;

namespace CollisionsEnv {

struct PhysicsBody : Archetype<
    Position, Rotation, Scale, Velocity, ObjectID, ResponseType,
    solver::SubstepPrevState, solver::PreSolvePositional,
    solver::PreSolveVelocity, ExternalForce, ExternalTorque,
    broadphase::LeafID> {};

struct Config {
    mw_collisions_config c;
    ObjectManager *objMgr;
    int32_t numHulls;             // body i uses object i % numHulls
};

// Per-world episode return handed to a learner: the running
// sum over steps of the mean height of the dynamic bodies.  Exported as a
// singleton column, all-gathered across GPUs by bench.py / the trainer.
struct EpisodeReturn {
    float value;
};

class Engine;

struct PhysWorld : public WorldBase {
    static void registerTypes(ECSRegistry &reg, const Config &cfg)
    {
        base::registerTypes(reg);
        RigidBodyPhysicsSystem::setMaxCandidatesPerWorld(reg, cfg.c.max_candidates);
        RigidBodyPhysicsSystem::registerTypes(reg);
        reg.registerFixedSizeArchetype<PhysicsBody>(cfg.c.num_cubes + 1);
        reg.registerSingleton<EpisodeReturn>();
        reg.exportColumn<PhysicsBody, Position>(0);
        reg.exportColumn<PhysicsBody, Rotation>(1);
        reg.exportSingleton<EpisodeReturn>(2);
    }

    static void setupTasks(TaskGraph::Builder &builder, const Config &cfg)
    {
        auto bp = RigidBodyPhysicsSystem::setupBroadphaseTasks(builder, {});
        auto sub = RigidBodyPhysicsSystem::setupSubstepTasks(builder, { bp },
                                                             cfg.c.num_substeps);
        auto cleanup = RigidBodyPhysicsSystem::setupCleanupTasks(builder, { sub });
        // one wave per world (the world's one EpisodeReturn row)
        builder.addToGraph<CustomParallelForNode<Engine, accumulateReturn, 64, 1, EpisodeReturn>>(
            { cleanup });
    }

    PhysWorld(Engine &ctx, const Config &cfg, const mw_collisions_init &init);

    static MW_HD void accumulateReturn(Engine &ctx, EpisodeReturn &ret);

    Query<Position, ResponseType> bodyQuery;
};

class Engine : public CustomContext<Engine, PhysWorld> {
public:
    using CustomContext::CustomContext;
};

// The mean height of the world's dynamic bodies, summed in row order (a
// deterministic serial sum).  On the device the world's wave loads its rows
// cooperatively (coalesced, 64 per round) and every lane replays the serial
// sum over them through shuffles -- the same additions in the same order as
// the host's walk, without one lane's chain of strided loads.
MW_HD void PhysWorld::accumulateReturn(Engine &ctx, EpisodeReturn &ret)
{
    float sum = 0.f;
    int32_t n = 0;
#if defined(__HIP_DEVICE_COMPILE__)
    const int32_t lane = mwGPU::invocationLane<64>();
    const Query<Position, ResponseType> &q = ctx.data().bodyQuery;
    StateView &st = ctx.state();
    const int32_t w = ctx.worldID().idx;
    for (int32_t a = 0; a < q.numArchetypes; a++) {
        const int32_t arch = q.archetypes[a];
        const int32_t rows = st.arch[arch].numRows[w];
        const Position *pos = st.column<Position>(arch, q.cols[a][0], w);
        const ResponseType *rts = st.column<ResponseType>(arch, q.cols[a][1], w);
        for (int32_t r0 = 0; r0 < rows; r0 += 64) {
            const int32_t r = r0 + lane;
            const float z = r < rows ? pos[r].z : 0.f;
            const int32_t dyn = r < rows && rts[r] == ResponseType::Dynamic ? 1 : 0;
            const int32_t cnt = min(64, rows - r0);
            const uint64_t dmask = __ballot(dyn != 0);
            // lane k's value to a scalar register (v_readlane, independent of
            // the running sum, so the reads run ahead of the add chain)
#pragma unroll
            for (int32_t k = 0; k < 64; k++) {
                if (k >= cnt) break;
                const float zk = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(z), k));
                const bool dk = (dmask >> k) & 1ull;
                sum = dk ? sum + zk : sum;
            }
            n += __popcll(dmask);
        }
    }
    if (lane != 0) return;
#else
#if !defined(__HIPCC__)
    // CPU back end: the invocation's lanes run one after another; one sums
    if (mwGPU::invocationLane<64>() != 0) return;
#endif
    ctx.forEach(ctx.data().bodyQuery, [&](const Position &p, const ResponseType &rt) {
        const bool dyn = rt == ResponseType::Dynamic;
        const float z = p.z;
        sum = dyn ? sum + z : sum;
        n += dyn ? 1 : 0;
    });
#endif
    ret.value += n > 0 ? sum / (float)n : 0.f;
}

PhysWorld::PhysWorld(Engine &ctx, const Config &cfg, const mw_collisions_init &init)
    : WorldBase(ctx)
{
    const mw_collisions_config &c = cfg.c;
    RigidBodyPhysicsSystem::init(ctx, cfg.objMgr, c.delta_t, c.num_substeps,
                                 Vector3 { 0.f, 0.f, c.gravity_z }, c.num_cubes + 1,
                                 c.max_contacts, c.num_joints > 16 ? c.num_joints : 16);

    auto setup = [&](Entity e, Vector3 p, Quat q, int32_t obj, ResponseType rt) {
        ctx.getUnsafe<Position>(e) = Position { p };
        ctx.getUnsafe<Rotation>(e) = Rotation { q };
        ctx.getUnsafe<Scale>(e) = Scale { Diag3x3 { 1.f, 1.f, 1.f } };
        ctx.getUnsafe<Velocity>(e) = Velocity { Vector3::zero(), Vector3::zero() };
        ctx.getUnsafe<ObjectID>(e) = ObjectID { obj };
        ctx.getUnsafe<ResponseType>(e) = rt;
        ctx.getUnsafe<solver::SubstepPrevState>(e) = { p, q };
        ctx.getUnsafe<solver::PreSolvePositional>(e) = { p, q };
        ctx.getUnsafe<solver::PreSolveVelocity>(e) = { Vector3::zero(), Vector3::zero() };
        ctx.getUnsafe<ExternalForce>(e) = ExternalForce { Vector3::zero() };
        ctx.getUnsafe<ExternalTorque>(e) = ExternalTorque { Vector3::zero() };
        ctx.getUnsafe<broadphase::LeafID>(e) =
            RigidBodyPhysicsSystem::registerEntity(ctx, e, ObjectID { obj });
    };

    std::vector<Entity> cubes;
    for (int32_t i = 0; i < c.num_cubes; i++) {
        Entity e = ctx.makeEntityNow<PhysicsBody>();
        Vector3 p { init.pos[3 * i], init.pos[3 * i + 1], init.pos[3 * i + 2] };
        Quat q { init.rot[4 * i], init.rot[4 * i + 1], init.rot[4 * i + 2], init.rot[4 * i + 3] };
        setup(e, p, q, i % cfg.numHulls, ResponseType::Dynamic);
        cubes.push_back(e);
    }
    Entity plane = ctx.makeEntityNow<PhysicsBody>();
    setup(plane, Vector3::zero(), Quat { 1.f, 0.f, 0.f, 0.f }, cfg.numHulls, ResponseType::Static);

    // Joint workload (mw_collisions_config::num_joints): joint j ties cube
    // 2j to cube 2j + 1, fixed, or hinge for the last num_hinge_joints --
    // the same ConstraintData rows oracle/ref_harness.cpp builds on the
    // reference.
    for (int32_t j = 0; j < c.num_joints; j++) {
        Entity e1 = cubes[2 * j], e2 = cubes[2 * j + 1];
        Entity je = ctx.makeEntityNow<ConstraintData>();
        if (j < c.num_joints - c.num_hinge_joints) {
            ctx.getUnsafe<JointConstraint>(je) = JointConstraint::setupFixed(
                e1, e2, Quat { 1.f, 0.f, 0.f, 0.f }, Quat { 0.70710678f, 0.f, 0.f, 0.70710678f },
                Vector3 { 0.f, 1.5f, 0.f }, Vector3 { 0.f, -1.5f, 0.f }, 0.5f);
        } else {
            ctx.getUnsafe<JointConstraint>(je) = JointConstraint::setupHinge(
                e1, e2, Vector3 { 1, 0, 0 }, Vector3 { 1, 0, 0 }, Vector3 { 0, 1, 0 },
                Vector3 { 0, 1, 0 }, Vector3 { 0.f, 0.f, 1.5f }, Vector3 { 0.f, 0.f, -1.5f });
        }
    }

    ctx.getSingleton<broadphase::BVH>().rebuildOnUpdate();
    ctx.getSingleton<EpisodeReturn>().value = 0.f;
    bodyQuery = ctx.query<Position, ResponseType>();
}

using Exec = TaskGraphExecutor<Engine, PhysWorld, Config, mw_collisions_init>;

static Executor *create(const ExecConfig &ecfg, const void *user_cfg, size_t cfg_bytes,
                        const void *inits, size_t init_stride)
{
    if (cfg_bytes != sizeof(mw_collisions_config)) {
        throw std::runtime_error("collisions: user config size mismatch");
    }
    Config cfg;
    memcpy(&cfg.c, user_cfg, sizeof(cfg.c));
    if (cfg.c.num_joints < 0 || 2 * cfg.c.num_joints > cfg.c.num_cubes ||
        cfg.c.num_hinge_joints < 0 || cfg.c.num_hinge_joints > cfg.c.num_joints) {
        throw std::runtime_error("collisions: need 0 <= 2 * num_joints <= num_cubes and "
                                 "0 <= num_hinge_joints <= num_joints");
    }
    const std::vector<std::string> hulls = envs::splitHullPaths(cfg.c.hull_paths);
    if (hulls.empty()) {
        cfg.objMgr = envs::makeCubeObjectManager(cfg.c);
        cfg.numHulls = 1;
    } else {
        cfg.objMgr = envs::makeHullObjectManager(cfg.c, hulls);
        cfg.numHulls = (int32_t)hulls.size();
    }
    std::vector<mw_collisions_init> init_vec(ecfg.numWorlds);
    for (int32_t w = 0; w < ecfg.numWorlds; w++) {
        memcpy(&init_vec[w], (const char *)inits + (size_t)w * init_stride, sizeof(mw_collisions_init));
    }
    return new Exec(ecfg, cfg, init_vec.data());
}

static EnvRegistration reg("collisions", &create);

}

// Deterministic synthetic inputs (examples/collisions/collisions.cpp:20-39,
// 48-51, 76-80): one mt19937 drawn serially over worlds; per body x, y, z
// then the rotation angle about +Y.  first_world lets a rank draw only its
// shard while staying identical to the serial sequence.
extern "C" void mw_gen_collisions_inits(int32_t first_world, int32_t num_worlds,
                                        int32_t num_cubes, uint32_t seed,
                                        float *pos_out, float *rot_out)
{
    std::mt19937 gen(seed);
    std::uniform_real_distribution<float> xd(-10.f, 10.f), yd(-10.f, 10.f), zd(0.f, 10.f);
    std::uniform_real_distribution<float> ad(0.f, madrona::math::pi);
    for (int64_t w = 0; w < (int64_t)first_world + num_worlds; w++) {
        for (int64_t i = 0; i < num_cubes; i++) {
            float x = xd(gen), y = yd(gen), z = zd(gen);
            float angle = ad(gen);
            if (w < first_world) continue;
            int64_t k = (w - first_world) * num_cubes + i;
            pos_out[3 * k] = x;
            pos_out[3 * k + 1] = y;
            pos_out[3 * k + 2] = z;
            Quat q = Quat::angleAxis(angle, Vector3 { 0, 1, 0 });
            rot_out[4 * k] = q.w;
            rot_out[4 * k + 1] = q.x;
            rot_out[4 * k + 2] = q.y;
            rot_out[4 * k + 3] = q.z;
        }
    }
}
