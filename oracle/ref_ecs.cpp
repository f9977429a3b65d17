// Reference harness, "ecs_ops" world (TEST INFRASTRUCTURE ONLY).
//
// The world of tests/ext_env/ecs_ops.hip written against the REFERENCE's own
// API and compiled with the untouched reference sources (src/core,
// src/common) by oracle/Makefile.ref into oracle/_ref/libmadrona_ref_ecs.so,
// single-world mode (one StateManager + StateCache + TaskGraph per world,
// SURVEY.md Appendix B).  Here every structural operation runs the way the
// reference runs it: ParallelForNode walks a world's rows serially
// (include/madrona/taskgraph.inl:63-71) and makeTemporary / makeEntityNow /
// destroyEntityNow act immediately (state.inl:398-472, src/core/state.cpp:
// 181-202); custom nodes use the reference's addDefaultNode / NodeT::run.
// tests/test_ecs_ops_gpu.py compares the HIP build of the same world (rows
// made and removed by parallel lanes, ordered by the commit) against this.

#include <madrona/taskgraph.hpp>
#include <madrona/custom_context.hpp>
#include <madrona/state.hpp>

#include "core/worker_init.hpp"
#include "../tests/ext_env/ecs_ops_rules.hpp"

#include <cstring>
#include <new>
#include <vector>

using namespace madrona;
using namespace ecs_ops;

namespace refecs {

struct Pos { float v[3]; };
struct Vel { float v[3]; };
struct Counter {
    int32_t hits;
    int32_t spawned;
    int32_t pairsMade;
    int32_t destroyed;
};
struct PairInfo {
    Entity a;
    Entity b;
    float d2;
    int32_t pad;
};
struct SpawnInfo {
    Entity parent;
    int32_t born;
    int32_t hits;
    int32_t serial;
    int32_t pad;
};
struct Stats {
    int32_t tick;
    int32_t numPairs;
    int32_t numSpawns;
    int32_t sumHits;
    float sumD2;
    int32_t dynTicks;
};

struct Agent : Archetype<Pos, Vel, Counter> {};
struct PairTemp : Archetype<PairInfo> {};
struct Spawn : Archetype<SpawnInfo> {};

class Engine;

struct World : public WorldBase {
    World(Engine &ctx, int32_t num_agents, int32_t world_index);

    int32_t tick;
    Query<Entity, Pos> agentQuery;
    Query<PairInfo> pairQuery;
    Query<Entity, SpawnInfo> spawnEntityQuery;
    Query<Counter> counterQuery;
};

class Engine : public CustomContext<Engine, World> {
public:
    using CustomContext::CustomContext;
};

static void moveSystem(Engine &, Pos &p, Vel &v)
{
    for (int32_t k = 0; k < 3; k++) moveAxis(p.v[k], v.v[k]);
}

static void pairSystem(Engine &ctx, Entity e, Pos &p, Counter &c)
{
    int32_t *scratch = (int32_t *)ctx.tmpAlloc(64);
    int32_t n = 0;
    ctx.forEach(ctx.data().agentQuery, [&](Entity o, Pos &q) {
        if (e.id < o.id && pairOverlaps(p.v, q.v)) {
            Loc l = ctx.makeTemporary<PairTemp>();
            ctx.getDirect<PairInfo>(1, l) = PairInfo { e, o, 0.f, 0 };
            n++;
        }
    });
    if (scratch) scratch[0] = n;
    c.pairsMade = scratch ? scratch[0] : -1;
}

static void pairDistSystem(Engine &ctx, PairInfo &pi)
{
    const Pos &a = ctx.getUnsafe<Pos>(pi.a);
    const Pos &b = ctx.getUnsafe<Pos>(pi.b);
    const float dx = a.v[0] - b.v[0], dy = a.v[1] - b.v[1], dz = a.v[2] - b.v[2];
    pi.d2 = (dx * dx + dy * dy) + dz * dz;
}

static void hitSystem(Engine &ctx, Entity e, Counter &c)
{
    ctx.forEach(ctx.data().pairQuery, [&](PairInfo &pi) {
        if (pi.a == e || pi.b == e) c.hits++;
    });
}

static void spawnSystem(Engine &ctx, Entity e, Counter &c)
{
    const int32_t tick = ctx.data().tick;
    struct Item {
        Entity self;
        SpawnInfo info;
    };
    Item *items = (Item *)ctx.tmpAlloc(sizeof(Item) * 32);
    int32_t n = 0;
    ctx.forEach(ctx.data().spawnEntityQuery, [&](Entity s, SpawnInfo &si) {
        if (si.parent == e && despawns(tick, si.born) && items && n < 32) {
            items[n++] = Item { s, si };
        }
    });
    for (int32_t i = 1; i < n; i++) {
        Item x = items[i];
        int32_t j = i - 1;
        while (j >= 0 && items[j].info.serial > x.info.serial) {
            items[j + 1] = items[j];
            j--;
        }
        items[j + 1] = x;
    }
    for (int32_t i = 0; i < n; i++) {
        const SpawnInfo si = items[i].info;
        if (spawnsChild(si.born, si.hits)) {
            ctx.makeEntityNow<Spawn>(SpawnInfo { e, tick, si.hits + 1, c.spawned, 0 });
            c.spawned++;
        }
        ctx.destroyEntityNow(items[i].self);
        if (si.serial % 7 == 0) ctx.destroyEntityNow(items[i].self);
        c.destroyed++;
    }
    if (spawns(c.hits, tick, e.id) && c.spawned - c.destroyed < kMaxLivePerAgent) {
        ctx.makeEntityNow<Spawn>(SpawnInfo { e, tick, c.hits, c.spawned, 0 });
        c.spawned++;
    }
}

struct StatsNode : NodeBase {
    static TaskGraph::NodeID addToGraph(Context &, TaskGraph::Builder &builder,
                                        Span<const TaskGraph::NodeID> deps)
    {
        return builder.addDefaultNode<StatsNode>(deps);
    }
    void run(Context *ctx_base)
    {
        Engine &ctx = *static_cast<Engine *>(ctx_base);
        Stats &st = ctx.getSingleton<Stats>();
        st.numPairs = (int32_t)ctx.numMatches(ctx.data().pairQuery);
        Query<SpawnInfo> sq = ctx.query<SpawnInfo>();
        st.numSpawns = (int32_t)ctx.numMatches(sq);
        int32_t hits = 0;
        ctx.forEach(ctx.data().counterQuery, [&](Counter &c) { hits += c.hits; });
        st.sumHits = hits;
        float d2 = 0.f;
        ctx.forEach(ctx.data().pairQuery, [&](PairInfo &pi) { d2 += pi.d2; });
        st.sumD2 = d2;
    }
};

struct TickNode : NodeBase {
    static TaskGraph::NodeID addToGraph(Context &, TaskGraph::Builder &builder,
                                        Span<const TaskGraph::NodeID> deps)
    {
        return builder.addDefaultNode<TickNode>(deps);
    }
    void run(Context *ctx_base)
    {
        Engine &ctx = *static_cast<Engine *>(ctx_base);
        ctx.data().tick += 1;
        ctx.getSingleton<Stats>().tick = ctx.data().tick;
        ctx.getSingleton<Stats>().dynTicks += 1;
    }
};

static void registerTypes(ECSRegistry &reg)
{
    reg.registerComponent<Pos>();
    reg.registerComponent<Vel>();
    reg.registerComponent<Counter>();
    reg.registerComponent<PairInfo>();
    reg.registerComponent<SpawnInfo>();
    reg.registerArchetype<Agent>();
    reg.registerArchetype<PairTemp>();
    reg.registerArchetype<Spawn>();
    reg.registerSingleton<Stats>();
}

static void setupTasks(TaskGraph::Builder &b)
{
    auto clear = b.addToGraph<ClearTmpNode<PairTemp>>({});
    auto move = b.addToGraph<ParallelForNode<Engine, moveSystem, Pos, Vel>>({ clear });
    auto pairs = b.addToGraph<ParallelForNode<Engine, pairSystem, Entity, Pos, Counter>>({ move });
    auto dist = b.addToGraph<ParallelForNode<Engine, pairDistSystem, PairInfo>>({ pairs });
    auto hits = b.addToGraph<ParallelForNode<Engine, hitSystem, Entity, Counter>>({ dist });
    auto spawn = b.addToGraph<ParallelForNode<Engine, spawnSystem, Entity, Counter>>({ hits });
    auto stats = b.addToGraph<StatsNode>({ spawn });
    auto tick = b.addToGraph<TickNode>({ stats });
    b.addToGraph<ResetTmpAllocNode>({ tick });
}

World::World(Engine &ctx, int32_t num_agents, int32_t world_index)
    : WorldBase(ctx), tick(0)
{
    for (int32_t i = 0; i < num_agents; i++) {
        Pos p;
        Vel v;
        initAgent((uint32_t)world_index, (uint32_t)i, p.v, v.v);
        ctx.makeEntityNow<Agent>(p, v, Counter { 0, 0, 0, 0 });
    }
    ctx.getSingleton<Stats>() = Stats { 0, 0, 0, 0, 0.f, 0 };
    agentQuery = ctx.query<Entity, Pos>();
    pairQuery = ctx.query<PairInfo>();
    spawnEntityQuery = ctx.query<Entity, SpawnInfo>();
    counterQuery = ctx.query<Counter>();
}

struct RefWorld {
    StateManager sm;
    StateCache sc;
    World *world;
    Engine *ctx;
    TaskGraph *graph;
};

}

using namespace refecs;

extern "C" {

struct RefEcsAgent {
    uint32_t gen;
    int32_t id;
    Pos pos;
    Vel vel;
    Counter counter;
};

struct RefEcsSpawn {
    uint32_t gen;
    int32_t id;
    SpawnInfo info;
};

MADRONA_EXPORT void *ref_ecs_create(int32_t num_worlds, int32_t num_agents, int32_t first_world_index)
{
    auto *v = new std::vector<RefWorld *>();
    for (int32_t w = 0; w < num_worlds; w++) {
        auto *rw = new RefWorld {};
        ECSRegistry reg(&rw->sm, nullptr);
        registerTypes(reg);
        rw->world = (World *)::operator new(sizeof(World));
        rw->ctx = new Engine(rw->world, WorkerInit { &rw->sm, &rw->sc });
        new (rw->world) World(*rw->ctx, num_agents, first_world_index + w);
        TaskGraph::Builder builder(*rw->ctx);
        setupTasks(builder);
        rw->graph = new TaskGraph(builder.build());
        v->push_back(rw);
    }
    return v;
}

MADRONA_EXPORT void ref_ecs_step(void *handle, int32_t num_steps)
{
    auto *v = (std::vector<RefWorld *> *)handle;
    for (int32_t s = 0; s < num_steps; s++) {
        for (RefWorld *rw : *v) rw->graph->run(rw->ctx);
    }
}

MADRONA_EXPORT int32_t ref_ecs_read_agents(void *handle, int32_t world, RefEcsAgent *out, int32_t cap)
{
    RefWorld *rw = (*(std::vector<RefWorld *> *)handle)[world];
    int32_t n = 0;
    auto q = rw->ctx->query<Entity, Pos, Vel, Counter>();
    rw->ctx->forEach(q, [&](Entity e, Pos &p, Vel &vel, Counter &c) {
        if (n < cap) out[n] = RefEcsAgent { e.gen, e.id, p, vel, c };
        n++;
    });
    return n;
}

MADRONA_EXPORT int32_t ref_ecs_read_pairs(void *handle, int32_t world, PairInfo *out, int32_t cap)
{
    RefWorld *rw = (*(std::vector<RefWorld *> *)handle)[world];
    int32_t n = 0;
    rw->ctx->forEach(rw->world->pairQuery, [&](PairInfo &pi) {
        if (n < cap) out[n] = pi;
        n++;
    });
    return n;
}

MADRONA_EXPORT int32_t ref_ecs_read_spawns(void *handle, int32_t world, RefEcsSpawn *out, int32_t cap)
{
    RefWorld *rw = (*(std::vector<RefWorld *> *)handle)[world];
    int32_t n = 0;
    rw->ctx->forEach(rw->world->spawnEntityQuery, [&](Entity e, SpawnInfo &si) {
        if (n < cap) out[n] = RefEcsSpawn { e.gen, e.id, si };
        n++;
    });
    return n;
}

MADRONA_EXPORT void ref_ecs_read_stats(void *handle, int32_t world, Stats *out)
{
    RefWorld *rw = (*(std::vector<RefWorld *> *)handle)[world];
    *out = rw->ctx->getSingleton<Stats>();
}

// Entity lookup in the world's ID store (getLoc): 0 + row when alive.
MADRONA_EXPORT int32_t ref_ecs_entity_row(void *handle, int32_t world, int32_t id, uint32_t gen,
                                          int32_t *row)
{
    RefWorld *rw = (*(std::vector<RefWorld *> *)handle)[world];
    Loc l = rw->ctx->getLoc(Entity { gen, id });
    if (!l.valid()) return 1;
    *row = (int32_t)l.row;
    return 0;
}

}
