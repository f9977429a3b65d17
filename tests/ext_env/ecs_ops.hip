// "ecs_ops" test world (TEST WORKLOAD; see ecs_ops_rules.hpp), written
// against this framework's include/madrona API and built OUT OF TREE
// (tests/ext_env/Makefile -> build/libecs_ops.so, linked to
// libmadrona_mw.so, loaded at run time with mw_load_env).  It registers
// itself with MADRONA_BUILD_MWGPU_ENTRY under the name "EcsOps::World".
//
// Every structural operation runs from row-parallel lanes, where the
// reference walks rows serially: makeTemporary per overlapping pair (the
// shape of findOverlappingEntry, src/physics/broadphase.cpp:897-932),
// makeEntityNow / destroyEntityNow of Spawn entities interleaved in one
// node, tmpAlloc scratch; plus CustomParallelForNode (4 lanes x 2 rows per
// invocation), addOneOffNode and addDynamicCountNode.  oracle/ref_ecs.cpp is
// the same world on the reference's own ECS.
#include <madrona/mw_gpu_entry.hpp>
#include <madrona/taskgraph.hpp>

#include "ecs_ops_init.hpp"
#include "ecs_ops_rules.hpp"

using namespace madrona;

namespace EcsOps {

using namespace ecs_ops;

struct Pos {
    float v[3];
};
struct Vel {
    float v[3];
};
struct Counter {
    int32_t hits;
    int32_t spawned;       // spawns made so far (the next spawn's serial)
    int32_t pairsMade;     // read back through the tmpAlloc scratch
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

struct Agent : Archetype<Pos, Vel, Counter> {};
struct PairTemp : Archetype<PairInfo> {};
struct Spawn : Archetype<SpawnInfo> {};


class Engine;

struct World : public WorldBase {
    static void registerTypes(ECSRegistry &reg, const Config &cfg);
    static void setupTasks(TaskGraph::Builder &builder, const Config &cfg);
    World(Engine &ctx, const Config &cfg, const Init &init);

    static MW_HD void moveSystem(Engine &ctx, Pos &p, Vel &v);
    static MW_HD void pairSystem(Engine &ctx, Entity e, Pos &p, Counter &c);
    static MW_HD void pairDistSystem(Engine &ctx, PairInfo &pi);
    static MW_HD void hitSystem(Engine &ctx, Entity e, Counter &c);
    static MW_HD void spawnSystem(Engine &ctx, Entity e, Counter &c);

    int32_t tick;
    Query<Entity, Pos> agentQuery;
    Query<PairInfo> pairQuery;
    Query<SpawnInfo> spawnQuery;
    Query<Entity, SpawnInfo> spawnEntityQuery;
    Query<Counter> counterQuery;
};

class Engine : public CustomContext<Engine, World> {
public:
    using CustomContext::CustomContext;
};

MW_HD void World::moveSystem(Engine &, Pos &p, Vel &v)
{
    for (int32_t k = 0; k < 3; k++) moveAxis(p.v[k], v.v[k]);
}

// One makeTemporary per overlapping pair, e.id < o.id, in agent-query
// order (findOverlappingEntry's loop shape); the pair count goes through
// tmpAlloc scratch and back.
MW_HD void World::pairSystem(Engine &ctx, Entity e, Pos &p, Counter &c)
{
    int32_t *scratch = (int32_t *)ctx.tmpAlloc(64);
    int32_t n = 0;
    ctx.forEach(ctx.data().agentQuery, [&](Entity o, Pos &q) {
        if (e.id < o.id && pairOverlaps(p.v, q.v)) {
            Loc l = ctx.makeTemporary<PairTemp>();
            if (l.valid()) ctx.getDirect<PairInfo>(1, l) = PairInfo { e, o, 0.f, 0 };
            n++;
        }
    });
    if (scratch) scratch[0] = n;
    c.pairsMade = scratch ? scratch[0] : -1;
}

// Cooperative: the 4 lanes of an invocation take one axis each and the
// group's lane 0 sums (dx^2 + dy^2) + dz^2 -- the serial order.
MW_HD void World::pairDistSystem(Engine &ctx, PairInfo &pi)
{
    const Pos &a = ctx.getUnsafe<Pos>(pi.a);
    const Pos &b = ctx.getUnsafe<Pos>(pi.b);
#if defined(__HIP_DEVICE_COMPILE__)
    const int32_t lane = mwGPU::invocationLane<4>();
    const float d = lane < 3 ? a.v[lane] - b.v[lane] : 0.f;
    const float sq = d * d;
    const float s0 = __shfl(sq, 0, 4), s1 = __shfl(sq, 1, 4), s2 = __shfl(sq, 2, 4);
    if (lane == 0) pi.d2 = (s0 + s1) + s2;
#else
    const float dx = a.v[0] - b.v[0], dy = a.v[1] - b.v[1], dz = a.v[2] - b.v[2];
    pi.d2 = (dx * dx + dy * dy) + dz * dz;
#endif
}

MW_HD void World::hitSystem(Engine &ctx, Entity e, Counter &c)
{
    ctx.forEach(ctx.data().pairQuery, [&](PairInfo &pi) {
        if (pi.a == e || pi.b == e) c.hits++;
    });
}

// Per agent: collect its expired spawns (scan of the Spawn table), destroy
// them in serial order -- each may leave a child, made before it is
// destroyed -- destroying every seventh twice; then maybe spawn anew.
MW_HD void World::spawnSystem(Engine &ctx, Entity e, Counter &c)
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
    for (int32_t i = 1; i < n; i++) {               // by serial
        Item x = items[i];
        int32_t j = i - 1;
        while (j >= 0 && items[j].info.serial > x.info.serial) {
            items[j + 1] = items[j];
            j--;
        }
        items[j + 1] = x;
    }
    for (int32_t i = 0; i < n; i++) {
        const SpawnInfo &si = items[i].info;
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

// One-off node, one invocation per world (reference addOneOffNode).  It only
// touches its own world, so it may run inside a world walk (kWorldLocal).
struct StatsNode : NodeBase {
    static constexpr bool kWorldLocal = true;
    MW_HD void run(int32_t world)
    {
#if MW_EXEC_PASS
        Engine ctx = makeContext<Engine>(WorldID { world });
        Stats &st = ctx.getSingleton<Stats>();
        st.numPairs = ctx.numRows<PairTemp>();
        st.numSpawns = ctx.numRows<Spawn>();
        int32_t hits = 0;
        ctx.forEach(ctx.data().counterQuery, [&](Counter &c) { hits += c.hits; });
        st.sumHits = hits;
        float d2 = 0.f;
        ctx.forEach(ctx.data().pairQuery, [&](PairInfo &pi) { d2 += pi.d2; });
        st.sumD2 = d2;
#else
        (void)world;
#endif
    }
};

// Dynamic-count node (reference addDynamicCountNode): numInvocations() is
// read on the device; two lanes per invocation, the first ticks the world.
struct TickNode : NodeBase {
    MW_HD uint32_t numInvocations() const { return (uint32_t)mwNumWorlds; }
    MW_HD void run(int32_t world)
    {
#if MW_EXEC_PASS
        if (mwGPU::invocationLane<2>() != 0) return;
        Engine ctx = makeContext<Engine>(WorldID { world });
        ctx.data().tick += 1;
        ctx.getSingleton<Stats>().tick = ctx.data().tick;
        ctx.getSingleton<Stats>().dynTicks += 1;
#else
        (void)world;
#endif
    }
};

void World::registerTypes(ECSRegistry &reg, const Config &cfg)
{
    reg.registerComponent<Pos>();
    reg.registerComponent<Vel>();
    reg.registerComponent<Counter>();
    reg.registerComponent<PairInfo>();
    reg.registerComponent<SpawnInfo>();
    reg.registerFixedSizeArchetype<Agent>(cfg.numAgents);
    reg.registerFixedSizeArchetype<PairTemp>(kMaxPairs);
    if (cfg.growSpawns) {
        reg.registerArchetype<Spawn>();          // grows past mw_config.default_capacity
    } else {
        reg.registerFixedSizeArchetype<Spawn>(kMaxSpawns);
    }
    reg.registerSingleton<Stats>();
    reg.exportSingleton<Stats>(0);
    reg.exportColumn<Spawn, SpawnInfo>(1);      // packed spawn rows (a growable table's export)
}

void World::setupTasks(TaskGraph::Builder &builder, const Config &)
{
    auto clear = builder.addToGraph<ClearTmpNode<PairTemp>>({});
    auto move = builder.addToGraph<ParallelForNode<Engine, moveSystem, Pos, Vel>>({ clear });
    auto pairs = builder.addToGraph<ParallelForNode<Engine, pairSystem, Entity, Pos, Counter>>({ move });
    auto dist = builder.addToGraph<CustomParallelForNode<Engine, pairDistSystem, 4, 2, PairInfo>>({ pairs });
    auto hits = builder.addToGraph<ParallelForNode<Engine, hitSystem, Entity, Counter>>({ dist });
    auto spawn = builder.addToGraph<ParallelForNode<Engine, spawnSystem, Entity, Counter>>({ hits });
    auto stats = builder.addOneOffNode<StatsNode>({ spawn });
    auto tick = builder.addDynamicCountNode<TickNode>({ stats }, 2);
    builder.addToGraph<ResetTmpAllocNode>({ tick });
}

World::World(Engine &ctx, const Config &cfg, const Init &init)
    : WorldBase(ctx)
{
    tick = 0;
    for (int32_t i = 0; i < cfg.numAgents; i++) {
        Pos p;
        Vel v;
        initAgent((uint32_t)init.worldIndex, (uint32_t)i, p.v, v.v);
        ctx.makeEntityNow<Agent>(p, v, Counter { 0, 0, 0, 0 });
    }
    ctx.getSingleton<Stats>() = Stats { 0, 0, 0, 0, 0.f, 0 };
    agentQuery = ctx.query<Entity, Pos>();
    pairQuery = ctx.query<PairInfo>();
    spawnQuery = ctx.query<SpawnInfo>();
    spawnEntityQuery = ctx.query<Entity, SpawnInfo>();
    counterQuery = ctx.query<Counter>();
}

}

MADRONA_BUILD_MWGPU_ENTRY(EcsOps::Engine, EcsOps::World, EcsOps::Config, EcsOps::Init)
