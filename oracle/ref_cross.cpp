// Reference harness, "cross_rows" world (TEST INFRASTRUCTURE ONLY).
//
// The world of tests/ext_env/cross_rows.hip written against the REFERENCE's
// own API and compiled with the untouched reference sources (src/core,
// src/common) by oracle/Makefile.ref into oracle/_ref/libmadrona_ref_cross.so,
// single-world mode (one StateManager + StateCache + TaskGraph per world).
// ParallelForNode walks a world's rows serially (include/madrona/
// taskgraph.inl:63-71, state.inl:387-396), so a row sees every write of the
// rows before it and makeEntityNow / destroyEntityNow act immediately
// (state.inl:398-472, src/core/state.cpp:181-202).  tests/test_cross_rows*.py
// compare the framework's world-serial mode against this.

#include <madrona/taskgraph.hpp>
#include <madrona/custom_context.hpp>
#include <madrona/state.hpp>

#include "core/worker_init.hpp"
#include "../tests/ext_env/cross_rows_rules.hpp"

#include <new>
#include <vector>

using namespace madrona;
using namespace cross_rows;

namespace refcross {

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

class Engine;

struct World : public WorldBase {
    World(Engine &ctx, int32_t num_cells, int32_t world_index);
    Query<Entity, Cell> cellQuery;
    Query<Entity, Spark> sparkQuery;
};

class Engine : public CustomContext<Engine, World> {
public:
    using CustomContext::CustomContext;
};

static void flowSystem(Engine &ctx, Entity e, Cell &c)
{
    ResultRef<Cell> o = ctx.get<Cell>(c.next);
    if (!o.valid()) {
        c.next = e;
        return;
    }
    Cell &oc = o.value();
    flow(c.value, c.heat, oc.value, oc.heat);
}

static void scanSystem(Engine &ctx, Cell &c)
{
    Stats &st = ctx.getSingleton<Stats>();
    c.prefix = st.running;
    st.running = scanStep(st.running, c.value);
    c.value += inject(c.prefix);
}

static void churnSystem(Engine &ctx, Entity e, Cell &c)
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

static void splitSystem(Engine &ctx, Spark &sp)
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

struct TickNode : NodeBase {
    static TaskGraph::NodeID addToGraph(Context &, TaskGraph::Builder &builder,
                                        Span<const TaskGraph::NodeID> deps)
    {
        return builder.addDefaultNode<TickNode>(deps);
    }
    void run(Context *ctx_base)
    {
        Engine &ctx = *static_cast<Engine *>(ctx_base);
        Stats &st = ctx.getSingleton<Stats>();
        st.tick += 1;
        st.running = 0;
    }
};

static void registerTypes(ECSRegistry &reg)
{
    reg.registerComponent<Cell>();
    reg.registerComponent<Spark>();
    reg.registerArchetype<CellArch>();
    reg.registerArchetype<SparkArch>();
    reg.registerSingleton<Stats>();
}

static void setupTasks(TaskGraph::Builder &b)
{
    auto flow_n = b.addToGraph<ParallelForNode<Engine, flowSystem, Entity, Cell>>({});
    auto scan_n = b.addToGraph<ParallelForNode<Engine, scanSystem, Cell>>({ flow_n });
    auto churn_n = b.addToGraph<ParallelForNode<Engine, churnSystem, Entity, Cell>>({ scan_n });
    auto split_n = b.addToGraph<ParallelForNode<Engine, splitSystem, Spark>>({ churn_n });
    b.addToGraph<TickNode>({ split_n });
}

World::World(Engine &ctx, int32_t num_cells, int32_t world_index)
    : WorldBase(ctx)
{
    std::vector<Entity> cells(num_cells);
    for (int32_t i = 0; i < num_cells; i++) {
        int32_t v;
        float h;
        initCell((uint32_t)world_index, (uint32_t)i, v, h);
        cells[i] = ctx.makeEntityNow<CellArch>(Cell { v, h, Entity::none(), Entity::none(), 0, 0 });
    }
    for (int32_t i = 0; i < num_cells; i++) {
        ctx.getUnsafe<Cell>(cells[i]).next = cells[linkTarget(i, num_cells)];
    }
    ctx.getSingleton<Stats>() = Stats { 0, num_cells, 0, 0 };
    cellQuery = ctx.query<Entity, Cell>();
    sparkQuery = ctx.query<Entity, Spark>();
}

struct RefWorld {
    StateManager sm;
    StateCache sc;
    World *world;
    Engine *ctx;
    TaskGraph *graph;
};

}

using namespace refcross;

extern "C" {

struct RefCrossCell {
    uint32_t gen;
    int32_t id;
    Cell cell;
};

struct RefCrossSpark {
    uint32_t gen;
    int32_t id;
    Spark spark;
};

MADRONA_EXPORT void *ref_cross_create(int32_t num_worlds, int32_t num_cells, int32_t first_world_index)
{
    auto *v = new std::vector<RefWorld *>();
    for (int32_t w = 0; w < num_worlds; w++) {
        auto *rw = new RefWorld {};
        ECSRegistry reg(&rw->sm, nullptr);
        registerTypes(reg);
        rw->world = (World *)::operator new(sizeof(World));
        rw->ctx = new Engine(rw->world, WorkerInit { &rw->sm, &rw->sc });
        new (rw->world) World(*rw->ctx, num_cells, first_world_index + w);
        TaskGraph::Builder builder(*rw->ctx);
        setupTasks(builder);
        rw->graph = new TaskGraph(builder.build());
        v->push_back(rw);
    }
    return v;
}

MADRONA_EXPORT void ref_cross_step(void *handle, int32_t num_steps)
{
    auto *v = (std::vector<RefWorld *> *)handle;
    for (int32_t s = 0; s < num_steps; s++) {
        for (RefWorld *rw : *v) rw->graph->run(rw->ctx);
    }
}

MADRONA_EXPORT int32_t ref_cross_read_cells(void *handle, int32_t world, RefCrossCell *out, int32_t cap)
{
    RefWorld *rw = (*(std::vector<RefWorld *> *)handle)[world];
    int32_t n = 0;
    rw->ctx->forEach(rw->world->cellQuery, [&](Entity e, Cell &c) {
        if (n < cap) out[n] = RefCrossCell { e.gen, e.id, c };
        n++;
    });
    return n;
}

MADRONA_EXPORT int32_t ref_cross_read_sparks(void *handle, int32_t world, RefCrossSpark *out, int32_t cap)
{
    RefWorld *rw = (*(std::vector<RefWorld *> *)handle)[world];
    int32_t n = 0;
    rw->ctx->forEach(rw->world->sparkQuery, [&](Entity e, Spark &s) {
        if (n < cap) out[n] = RefCrossSpark { e.gen, e.id, s };
        n++;
    });
    return n;
}

MADRONA_EXPORT void ref_cross_read_stats(void *handle, int32_t world, Stats *out)
{
    RefWorld *rw = (*(std::vector<RefWorld *> *)handle)[world];
    *out = rw->ctx->getSingleton<Stats>();
}

}
