// "cross_rows" test world (TEST WORKLOAD; see cross_rows_rules.hpp), written
// against this framework's include/madrona API and built OUT OF TREE like
// ecs_ops.hip.  Its ParallelForNode bodies touch other rows (ctx.get of a
// linked cell), carry state from row to row and make / destroy entities, so
// only a world-serial walk reproduces the reference: run it with
// mw_config.serial_nodes = 1, or with Config::perNodeSerial = 1, which builds
// the same graph from WorldSerialForNode.  oracle/ref_cross.cpp is the same
// world on the reference's own ECS.
#include <madrona/mw_gpu_entry.hpp>
#include <madrona/taskgraph.hpp>

#include "cross_rows_rules.hpp"

using namespace madrona;

namespace CrossRows {

using namespace cross_rows;

struct Cell {
    int32_t value;
    float heat;
    Entity next;
    Entity spark;
    uint32_t prefix;
    int32_t pad;
};
struct Spark {
    Entity source;
    int32_t born;
    int32_t energy;
};
struct Stats {
    int32_t tick;
    int32_t cells;
    int32_t sparks;
    uint32_t running;
};

struct CellArch : Archetype<Cell> {};
struct SparkArch : Archetype<Spark> {};

struct Config {
    int32_t numCells;
    int32_t perNodeSerial;      // 1: WorldSerialForNode for the three row nodes;
                                // 2 / 3: the cross-row check's own graphs (one
                                // neighbour-reading row node + tick: 2 reads
                                // Cell const, 3 takes Cell by non-const ref)
};
struct Init {
    int32_t worldIndex;
};

class Engine;

struct World : public WorldBase {
    static void registerTypes(ECSRegistry &reg, const Config &cfg);
    static void setupTasks(TaskGraph::Builder &builder, const Config &cfg);
    World(Engine &ctx, const Config &cfg, const Init &init);

    static MW_HD void flowSystem(Engine &ctx, Entity e, Cell &c);
    static MW_HD void scanSystem(Engine &ctx, Cell &c);
    static MW_HD void churnSystem(Engine &ctx, Entity e, Cell &c);
    static MW_HD void splitSystem(Engine &ctx, Spark &sp);
    static MW_HD void tickSystem(Engine &ctx);
    static MW_HD void peekSystem(Engine &ctx, Entity e, const Cell &c);
    static MW_HD void pokeSystem(Engine &ctx, Entity e, Cell &c);
};

class Engine : public CustomContext<Engine, World> {
public:
    using CustomContext::CustomContext;
};

MW_HD void World::flowSystem(Engine &ctx, Entity e, Cell &c)
{
    ResultRef<Cell> o = ctx.get<Cell>(c.next);
    if (!o.valid()) {
        c.next = e;
        return;
    }
    Cell &oc = o.value();
    flow(c.value, c.heat, oc.value, oc.heat);
}

MW_HD void World::scanSystem(Engine &ctx, Cell &c)
{
    Stats &st = ctx.getSingleton<Stats>();
    c.prefix = st.running;
    st.running = scanStep(st.running, c.value);
    c.value += inject(c.prefix);
}

MW_HD void World::churnSystem(Engine &ctx, Entity e, Cell &c)
{
    Stats &st = ctx.getSingleton<Stats>();
    if (c.spark != Entity::none()) {
        if (dropsSpark(c.value, st.tick)) {
            ctx.destroyEntityNow(c.spark);
            c.spark = Entity::none();
            st.sparks--;
        }
    } else if (makesSpark(c.value) && st.sparks < kMaxSparks) {
        c.spark = ctx.makeEntityNow<SparkArch>(Spark { e, st.tick, c.value });
        st.sparks++;
    }
}

// A spark splits its source cell: the walk is over Sparks, so the Cell
// table it grows is not the one being walked (growing the walked table
// reallocates it under the reference's walk, src/common/table.cpp:44-60).
MW_HD void World::splitSystem(Engine &ctx, Spark &sp)
{
    Stats &st = ctx.getSingleton<Stats>();
    ResultRef<Cell> src = ctx.get<Cell>(sp.source);
    if (!src.valid()) return;
    Cell &c = src.value();
    if (c.value > kSplitValue && st.cells < kMaxCells) {
        const int32_t half = c.value / 2;
        c.value -= half;
        const Entity n = ctx.makeEntityNow<CellArch>(Cell { half, c.heat * 0.5f, sp.source, Entity::none(), 0, 0 });
        // re-resolved: the make may have grown (reallocated) the Cell table
        ctx.get<Cell>(sp.source).value().next = n;
        ctx.getSingleton<Stats>().cells++;
    }
}

MW_HD void World::tickSystem(Engine &ctx)
{
    Stats &st = ctx.getSingleton<Stats>();
    st.tick += 1;
    st.running = 0;
}

// The same neighbour read in a node that only reads Cell (no lane writes a
// Cell row: not a race, must not flag) and in one that may write it (flags).
MW_HD void World::peekSystem(Engine &ctx, Entity, const Cell &c)
{
    (void)ctx.get<Cell>(c.next);
}

MW_HD void World::pokeSystem(Engine &ctx, Entity, Cell &c)
{
    (void)ctx.get<Cell>(c.next);
}

void World::registerTypes(ECSRegistry &reg, const Config &)
{
    reg.registerComponent<Cell>();
    reg.registerComponent<Spark>();
    reg.registerFixedSizeArchetype<CellArch>(kMaxCells);
    reg.registerFixedSizeArchetype<SparkArch>(kMaxSparks);
    reg.registerSingleton<Stats>();
}

template <bool kSerial>
static void setupRowNodes(TaskGraph::Builder &builder)
{
    using FlowNode = std::conditional_t<kSerial, WorldSerialForNode<Engine, World::flowSystem, Entity, Cell>,
                                        ParallelForNode<Engine, World::flowSystem, Entity, Cell>>;
    using ScanNode = std::conditional_t<kSerial, WorldSerialForNode<Engine, World::scanSystem, Cell>,
                                        ParallelForNode<Engine, World::scanSystem, Cell>>;
    using ChurnNode = std::conditional_t<kSerial, WorldSerialForNode<Engine, World::churnSystem, Entity, Cell>,
                                         ParallelForNode<Engine, World::churnSystem, Entity, Cell>>;
    using SplitNode = std::conditional_t<kSerial, WorldSerialForNode<Engine, World::splitSystem, Spark>,
                                         ParallelForNode<Engine, World::splitSystem, Spark>>;
    auto flow_n = builder.addToGraph<FlowNode>({});
    auto scan_n = builder.addToGraph<ScanNode>({ flow_n });
    auto churn_n = builder.addToGraph<ChurnNode>({ scan_n });
    auto split_n = builder.addToGraph<SplitNode>({ churn_n });
    builder.addToGraph<PerWorldNode<Engine, World::tickSystem>>({ split_n });
}

void World::setupTasks(TaskGraph::Builder &builder, const Config &cfg)
{
    if (cfg.perNodeSerial == 2 || cfg.perNodeSerial == 3) {
        auto peek = cfg.perNodeSerial == 2
                        ? builder.addToGraph<ParallelForNode<Engine, World::peekSystem, Entity, Cell>>({})
                        : builder.addToGraph<ParallelForNode<Engine, World::pokeSystem, Entity, Cell>>({});
        builder.addToGraph<PerWorldNode<Engine, World::tickSystem>>({ peek });
    } else if (cfg.perNodeSerial) {
        setupRowNodes<true>(builder);
    } else {
        setupRowNodes<false>(builder);
    }
}

World::World(Engine &ctx, const Config &cfg, const Init &init)
    : WorldBase(ctx)
{
    Entity cells[kMaxCells];
    const int32_t n = cfg.numCells < kMaxCells ? cfg.numCells : kMaxCells;
    for (int32_t i = 0; i < n; i++) {
        int32_t v;
        float h;
        initCell((uint32_t)init.worldIndex, (uint32_t)i, v, h);
        cells[i] = ctx.makeEntityNow<CellArch>(Cell { v, h, Entity::none(), Entity::none(), 0, 0 });
    }
    for (int32_t i = 0; i < n; i++) ctx.getUnsafe<Cell>(cells[i]).next = cells[linkTarget(i, n)];
    ctx.getSingleton<Stats>() = Stats { 0, n, 0, 0 };
}

}

MADRONA_BUILD_MWGPU_ENTRY(CrossRows::Engine, CrossRows::World, CrossRows::Config, CrossRows::Init)
