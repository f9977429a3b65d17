// "collisions_jobs": examples/collisions as the reference wrote it, against
// the job API (collisions.cpp:88-227): a brute-force broadphase (a nested
// parallelFor over every ordered pair), a pass-through narrowphase (contact
// normal = direction between the two translations) and a serial solver that
// pushes each pair apart, with CollisionCandidate / Contact entities made by
// makeEntityNow and released by clearArchetype every tick.  Run through the
// Context job API (include/madrona/context.hpp): the loop is a PerWorldNode
// and each world's jobs run on the lane that owns the world, in submission
// order.  Edits from the reference source: the SpinLocks
// around makeEntityNow are gone (one lane owns the world), the tick printf is
// dropped, and the constructor takes its initial state from the init struct
// (the reference draws it inside the constructor from a thread_local
// mt19937; mw_gen_collisions_inits makes the same serial draws).  The
// physics workload (configs[2]) is csrc/envs/collisions.hip; this is the
// example's own toy system, kept for API compatibility.
#include <madrona/math.hpp>
#include <madrona/mw_gpu.hpp>

#include "../runtime/env_registry.hpp"
#include "../../../include/madrona_mw.h"

#include <cstring>

using namespace madrona;
using namespace madrona::math;

namespace CollisionExample {

// Components (collisions.hpp:15-43)
struct Translation : Vector3 {
    MW_INLINE Translation(Vector3 v) : Vector3(v) {}
};

struct Rotation : Quat {
    MW_INLINE Rotation(Quat q) : Quat(q) {}
};

struct PhysicsAABB : AABB {
    MW_INLINE PhysicsAABB(AABB b) : AABB(b) {}
};

struct CandidatePair {
    Entity a;
    Entity b;
};

struct ContactData {
    Vector3 normal;
    Entity a;
    Entity b;
};

// Archetypes (collisions.hpp:45-48)
struct CubeObject : Archetype<Translation, Rotation, PhysicsAABB> {};
struct CollisionCandidate : Archetype<CandidatePair> {};
struct Contact : Archetype<ContactData> {};

struct Config {
    mw_jobs_collisions_config c;
};

class Engine;

struct CollisionSim : public WorldBase {
    static void registerTypes(ECSRegistry &reg, const Config &cfg)
    {                                                      // collisions.cpp:53-63
        reg.registerComponent<Translation>();
        reg.registerComponent<Rotation>();
        reg.registerComponent<PhysicsAABB>();
        reg.registerComponent<CandidatePair>();
        reg.registerComponent<ContactData>();
        reg.registerFixedSizeArchetype<CubeObject>(cfg.c.num_objects);
        reg.registerFixedSizeArchetype<CollisionCandidate>(cfg.c.max_candidates);
        reg.registerFixedSizeArchetype<Contact>(cfg.c.max_candidates);
    }

    // CollisionSim::entry (collisions.cpp:220-227) starts simLoop once; the
    // loop's body is the job the step graph replays.
    static void setupTasks(TaskGraph::Builder &builder, const Config &)
    {
        builder.addToGraph<PerWorldNode<Engine, entry>>({});
    }

    CollisionSim(Engine &ctx, const Config &cfg, const mw_collisions_init &init);

    static MW_HD void entry(Engine &ctx);

    uint64_t tickCount;
    float deltaT;

    AABB worldBounds;

    Query<const Translation, const Rotation, PhysicsAABB> physicsPreprocessQuery;
    Query<const Entity, const PhysicsAABB> broadphaseQuery;
    Query<const CandidatePair> candidateQuery;
};

class Engine : public CustomContext<Engine, CollisionSim> {
public:
    using CustomContext::CustomContext;
    MW_INLINE CollisionSim &sim() { return data(); }
};

MW_HD static JobID broadphaseSystem(Engine &ctx)
{                                                          // collisions.cpp:88-137
    // Update all entity bounding boxes:
    JobID preprocess = ctx.parallelFor(ctx.sim().physicsPreprocessQuery,
            [](Engine &, const Translation &translation,
               const Rotation &rotation, PhysicsAABB &aabb) {
        // No actual mesh, just a 2-unit cube centered around translation
        Mat3x4 model_mat = Mat3x4::fromTRS(translation, rotation);

        Vector3 cube[8] = {
            model_mat.txfmPoint(Vector3 {-1.f, -1.f, -1.f}),
            model_mat.txfmPoint(Vector3 { 1.f, -1.f, -1.f}),
            model_mat.txfmPoint(Vector3 { 1.f,  1.f, -1.f}),
            model_mat.txfmPoint(Vector3 {-1.f,  1.f, -1.f}),
            model_mat.txfmPoint(Vector3 {-1.f, -1.f,  1.f}),
            model_mat.txfmPoint(Vector3 { 1.f, -1.f,  1.f}),
            model_mat.txfmPoint(Vector3 { 1.f,  1.f,  1.f}),
            model_mat.txfmPoint(Vector3 {-1.f,  1.f,  1.f}),
        };

        aabb = AABB::point(cube[0]);
        for (int i = 1; i < 8; i++) {
            aabb.expand(cube[i]);
        }
    });

    // Generate list of CollisionCandidates for narrowphase
    return ctx.parallelFor(ctx.sim().broadphaseQuery,
            [](Engine &ctx, Entity a, const PhysicsAABB &a_bbox) {
        ctx.parallelFor(ctx.sim().broadphaseQuery,
                [a, &a_bbox](Engine &ctx, Entity b,
                             const PhysicsAABB &b_bbox) {
            if (a == b) {
                return;
            }

            if (a_bbox.overlaps(b_bbox)) {
                ctx.makeEntityNow<CollisionCandidate>(CandidatePair { a, b });
            }
        });
    }, true, preprocess);
}

MW_HD static JobID narrowphaseSystem(Engine &ctx, JobID broadphase_job)
{                                                          // collisions.cpp:139-167
    JobID contact_job = ctx.parallelFor(ctx.sim().candidateQuery,
            [](Engine &ctx, const CandidatePair &pair) {
        // Narrow phase is a pass-through in the example
        Translation a_pos = ctx.get<Translation>(pair.a).value();
        Translation b_pos = ctx.get<Translation>(pair.b).value();

        Vector3 to_b = (b_pos - a_pos).normalize();
        ctx.makeEntityNow<Contact>(ContactData {
            to_b,
            pair.a,
            pair.b,
        });
    }, true, broadphase_job);

    // Once narrowphase is done, wipe CollisionCandidate table for next frame
    return ctx.submit([](Engine &ctx) {
        ctx.clearArchetype<CollisionCandidate>();
    }, true, contact_job);
}

MW_HD static JobID solverSystem(Engine &ctx, JobID narrowphase_job)
{                                                          // collisions.cpp:170-193
    return ctx.submit([](Engine &ctx) {
        // Push objects in serial based on the contact normal
        auto contacts = ctx.archetype<Contact>();
        int num_contacts = (int)contacts.size();
        ContactData *contacts_data = contacts.component<ContactData>().data();

        for (int i = 0; i < num_contacts; i++) {
            ContactData &contact = contacts_data[i];

            Translation &a_pos = ctx.get<Translation>(contact.a).value();
            Translation &b_pos = ctx.get<Translation>(contact.b).value();

            a_pos -= contact.normal;
            b_pos += contact.normal;
        }

        ctx.clearArchetype<Contact>();
    }, true, narrowphase_job);
}

MW_HD static void tick(Engine &ctx)
{                                                          // collisions.cpp:195-201
    JobID broadphase_job = broadphaseSystem(ctx);
    JobID narrowphase_job = narrowphaseSystem(ctx, broadphase_job);

    solverSystem(ctx, narrowphase_job);
}

MW_HD static void simLoop(Engine &ctx)
{                                                          // collisions.cpp:203-218
    ctx.submit([](Engine &ctx) {
        tick(ctx);

        ctx.sim().tickCount += 1;

        // Queues the loop again behind the current job: the next step.
        simLoop(ctx);
    }, /* not a child of the current job */ false, ctx.currentJobID());
}

MW_HD void CollisionSim::entry(Engine &ctx)
{
    simLoop(ctx);
}

CollisionSim::CollisionSim(Engine &ctx, const Config &cfg, const mw_collisions_init &init)
    : WorldBase(ctx)
{                                                          // collisions.cpp:41-86
    tickCount = 0;
    deltaT = 1.f / 60.f;

    worldBounds = AABB { { -10, -10, 0 }, { 10, 10, 10 } };

    physicsPreprocessQuery = ctx.query<const Translation, const Rotation, PhysicsAABB>();
    broadphaseQuery = ctx.query<const Entity, const PhysicsAABB>();
    candidateQuery = ctx.query<const CandidatePair>();

    for (int32_t i = 0; i < cfg.c.num_objects; i++) {
        Translation rand_pos = Vector3 { init.pos[3 * i], init.pos[3 * i + 1], init.pos[3 * i + 2] };
        Rotation rand_rot = Quat { init.rot[4 * i], init.rot[4 * i + 1], init.rot[4 * i + 2],
                                   init.rot[4 * i + 3] };
        PhysicsAABB aabb = AABB::invalid();

        ctx.makeEntityNow<CubeObject>(rand_pos, rand_rot, aabb);
    }
}

using Exec = TaskGraphExecutor<Engine, CollisionSim, Config, mw_collisions_init>;

static Executor *create(const ExecConfig &ecfg, const void *user_cfg, size_t cfg_bytes,
                        const void *inits, size_t init_stride)
{
    if (cfg_bytes != sizeof(mw_jobs_collisions_config)) {
        throw std::runtime_error("collisions_jobs: user config size mismatch");
    }
    Config cfg;
    memcpy(&cfg.c, user_cfg, sizeof(cfg.c));
    if (cfg.c.num_objects < 0 || cfg.c.max_candidates < 0) {
        throw std::runtime_error("collisions_jobs: negative sizes");
    }
    std::vector<mw_collisions_init> init_vec(ecfg.numWorlds);
    for (int32_t w = 0; w < ecfg.numWorlds; w++) {
        memcpy(&init_vec[w], (const char *)inits + (size_t)w * init_stride, sizeof(mw_collisions_init));
    }
    return new Exec(ecfg, cfg, init_vec.data());
}

static EnvRegistration reg("collisions_jobs", &create);

}
