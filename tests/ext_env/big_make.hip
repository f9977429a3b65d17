// "big_make" test world (TEST WORKLOAD, not product code), built OUT OF TREE
// like ecs_ops.hip.  One ParallelForNode walks a Cell table of more rows per
// world than the row-ordered make path covers (kMakeTurnWaves = 64 waves =
// 4096 rows), and some of its rows makeEntityNow a Mark; a second node
// destroys the marks after two ticks.  Waves 0..63 of a world take IDs in
// row order (their turn marks), waves 64.. through the per-world ID-store
// lock alone; both paths must hand out unique IDs (the ordered
// path now takes the same lock after its turn).
#include <madrona/mw_gpu_entry.hpp>
#include <madrona/taskgraph.hpp>

using namespace madrona;

namespace BigMake {

inline constexpr int32_t kMaxCells = 6144;
inline constexpr int32_t kMaxMarks = 1024;

struct Cell {
    int32_t k;
    int32_t made;       // marks this cell has made
    Entity mark;        // the last one
};
struct Mark {
    Entity source;
    int32_t born;
    int32_t k;
};
struct Stats {
    int32_t tick;
};

struct CellArch : Archetype<Cell> {};
struct MarkArch : Archetype<Mark> {};

struct Config {
    int32_t numCells;
};
struct Init {
    int32_t worldIndex;
};

class Engine;

struct World : public WorldBase {
    static void registerTypes(ECSRegistry &reg, const Config &cfg);
    static void setupTasks(TaskGraph::Builder &builder, const Config &cfg);
    World(Engine &ctx, const Config &cfg, const Init &init);

    static MW_HD void dropSystem(Engine &ctx, Entity e, Mark &m);
    static MW_HD void makeSystem(Engine &ctx, Entity e, Cell &c);
    static MW_HD void tickSystem(Engine &ctx);
};

class Engine : public CustomContext<Engine, World> {
public:
    using CustomContext::CustomContext;
};

// same rule in tests/test_big_make_gpu.py
MW_HD inline bool makes(int32_t k, int32_t tick)
{
    return ((k * 7 + tick * 13) % 23) == 0;
}

MW_HD void World::dropSystem(Engine &ctx, Entity e, Mark &m)
{
    if (ctx.getSingleton<Stats>().tick - m.born >= 2) ctx.destroyEntityNow(e);
}

MW_HD void World::makeSystem(Engine &ctx, Entity e, Cell &c)
{
    const int32_t tick = ctx.getSingleton<Stats>().tick;
    if (makes(c.k, tick)) {
        c.mark = ctx.makeEntityNow<MarkArch>(Mark { e, tick, c.k });
        c.made += 1;
    }
}

MW_HD void World::tickSystem(Engine &ctx)
{
    ctx.getSingleton<Stats>().tick += 1;
}

void World::registerTypes(ECSRegistry &reg, const Config &)
{
    reg.registerComponent<Cell>();
    reg.registerComponent<Mark>();
    reg.registerFixedSizeArchetype<CellArch>(kMaxCells);
    reg.registerFixedSizeArchetype<MarkArch>(kMaxMarks);
    reg.registerSingleton<Stats>();
}

void World::setupTasks(TaskGraph::Builder &builder, const Config &)
{
    auto drop = builder.addToGraph<ParallelForNode<Engine, World::dropSystem, Entity, Mark>>({});
    auto make = builder.addToGraph<ParallelForNode<Engine, World::makeSystem, Entity, Cell>>({ drop });
    builder.addToGraph<PerWorldNode<Engine, World::tickSystem>>({ make });
}

World::World(Engine &ctx, const Config &cfg, const Init &init)
    : WorldBase(ctx)
{
    const int32_t n = cfg.numCells < kMaxCells ? cfg.numCells : kMaxCells;
    for (int32_t i = 0; i < n; i++) {
        ctx.makeEntityNow<CellArch>(Cell { i + init.worldIndex, 0, Entity::none() });
    }
    ctx.getSingleton<Stats>() = Stats { 0 };
}

}

MADRONA_BUILD_MWGPU_ENTRY(BigMake::Engine, BigMake::World, BigMake::Config, BigMake::Init)
