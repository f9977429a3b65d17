// "fantasy_vs" environment (BASELINE.json configs[4]):
// dragons (casters) and knights (archers) damage each other; dead entities
// are destroyed every tick, which stresses entity create / destroy, ID reuse
// and row compaction.  Restated from the reference's job-API example
// (examples/fantasy_vs/fvs.cpp:111-240, fvs.hpp) onto the TaskGraph API:
//   actionSelect  ParallelForNode<Entity, Position, Action>   (fvs.cpp:111-151)
//   caster        ParallelForNode<Entity, Action, Mana>       (fvs.cpp:153-190;
//                 a blast's scan of every Position / Health row is shared by
//                 the lanes of the caster's wave)
//   archer        ParallelForNode<Entity, Action, Quiver>     (fvs.cpp:192-214)
//   cleanup       ParallelForNode<Entity, Health> marks the dead, a
//                 PerWorldNode makes their trackers, a ParallelForNode over
//                 the trackers destroys them (ordered commit), a PerWorldNode
//                 clears the trackers -- fvs.cpp:224-239 (see below)
// The reference draws from a racy thread_local mt19937 inside systems; here
// every draw is a counter-based hash of (world, entity id, tick, draw index)
// (SURVEY.md §8d), so any executor (this one, oracle/fvs_oracle.cpp,
// oracle/ref_fvs.cpp on the reference ECS) produces the same run.  Kept
// reference quirks: a move clamps z from the new x (fvs.cpp:136), damage is
// applied to an integer hp (std::atomic_int, fvs.hpp:24-26).
#include <madrona/math.hpp>
#include <madrona/mw_gpu.hpp>

#include "../runtime/env_registry.hpp"
#include "../../../include/madrona_mw.h"
#include "fvs_rules.hpp"

#include <cstring>
#include <random>

using namespace madrona;
using namespace madrona::math;

namespace FantasyVS {

using namespace fvs_rules;

struct Position : Vector3 {};

struct alignas(64) Health {                    // alignas(MADRONA_CACHE_LINE)
    int32_t hp;
};

struct Mana {
    float mp;
};

struct Quiver {
    int32_t numArrows;
};

struct Action {
    float remainingTime;
};

struct CleanupEntity : Entity {};

struct Dragon : Archetype<Position, Health, Action, Mana> {};
struct Knight : Archetype<Position, Health, Action, Quiver> {};
struct CleanupTracker : Archetype<CleanupEntity> {};

struct Config {
    mw_fvs_config c;
};

class Engine;

struct Game : public WorldBase {
    static void registerTypes(ECSRegistry &reg, const Config &cfg)
    {
        reg.registerComponent<Position>();
        reg.registerComponent<Health>();
        reg.registerComponent<Action>();
        reg.registerComponent<Mana>();
        reg.registerComponent<Quiver>();
        reg.registerComponent<CleanupEntity>();
        reg.registerFixedSizeArchetype<Dragon>(cfg.c.num_dragons);
        reg.registerFixedSizeArchetype<Knight>(cfg.c.num_knights);
        reg.registerFixedSizeArchetype<CleanupTracker>(cfg.c.num_dragons + cfg.c.num_knights);
        // the reference example exports nothing (no learner hand-off)
    }

    static void setupTasks(TaskGraph::Builder &builder, const Config &)
    {
        auto act = builder.addToGraph<
            ParallelForNode<Engine, actionSelectSystem, Entity, Position, Action>>({});
        auto cast = builder.addToGraph<
            ParallelForNode<Engine, casterSystem, Entity, Action, Mana>>({ act });
        auto shoot = builder.addToGraph<
            ParallelForNode<Engine, archerSystem, Entity, Action, Quiver>>({ act });
        auto mark = builder.addToGraph<
            ParallelForNode<Engine, markDeadSystem, Entity, Health>>({ cast, shoot });
        auto track = builder.addToGraph<PerWorldNode<Engine, trackDeadSystem>>({ mark });
        auto kill = builder.addToGraph<
            ParallelForNode<Engine, destroyTrackedSystem, CleanupEntity>>({ track });
        builder.addToGraph<PerWorldNode<Engine, finishTickSystem>>({ kill });
    }

    Game(Engine &ctx, const Config &cfg, const mw_fvs_init &init);

    static MW_HD void actionSelectSystem(Engine &ctx, Entity &e, Position &pos, Action &action);
    static MW_HD void casterSystem(Engine &ctx, Entity &e, Action &action, Mana &mana);
    static MW_HD void archerSystem(Engine &ctx, Entity &e, Action &action, Quiver &quiver);
    static MW_HD void markDeadSystem(Engine &ctx, Entity &e, Health &h);
    static MW_HD void trackDeadSystem(Engine &ctx);
    static MW_HD void destroyTrackedSystem(Engine &ctx, CleanupEntity &c);
    static MW_HD void finishTickSystem(Engine &ctx);

    // Entities found dead by markDeadSystem this tick, in arbitrary order;
    // trackDeadSystem restores the reference's query order (archetype, row).
    static constexpr int32_t kMaxDead = 512;
    struct Dead {
        Entity e;
        Loc loc;
    };
    int32_t numDead;
    Dead dead[kMaxDead];

    uint32_t worldSeed;                  // global world index (shard-independent draws)
    uint32_t tickCount;
    AABB worldBounds;
    int32_t dragonArch;
    int32_t dragonHealthCol;
    Query<Position, Health> healthQuery;
    Query<Entity, Health> cleanupQuery;
};

class Engine : public CustomContext<Engine, Game> {
public:
    using CustomContext::CustomContext;
};

MW_HD static inline void damage(Health &h, int32_t amount)
{
#if defined(__HIP_DEVICE_COMPILE__)
    atomicSub(&h.hp, amount);          // casters / archers of a world run concurrently
#else
    h.hp -= amount;
#endif
}

MW_HD void Game::actionSelectSystem(Engine &ctx, Entity &e, Position &pos, Action &action)
{                                                          // fvs.cpp:111-151
    const Game &g = ctx.data();
    if (action.remainingTime > 0) {
        action.remainingTime -= kDeltaT;
        return;
    }
    const Draw d { g.worldSeed, (uint32_t)e.id, g.tickCount };
    if (d.uniform(kDrawMoveProb) <= kMoveCutoff) {
        Vector3 new_pos = pos + Vector3 {
            d.uniform(kDrawMoveX, -1.f, 1.f),
            d.uniform(kDrawMoveY, -1.f, 1.f),
            d.uniform(kDrawMoveZ, -1.f, 1.f),
        };
        new_pos.x = clampRef(new_pos.x, g.worldBounds.pMin.x, g.worldBounds.pMax.x);
        new_pos.y = clampRef(new_pos.y, g.worldBounds.pMin.y, g.worldBounds.pMax.y);
        new_pos.z = clampRef(new_pos.x, g.worldBounds.pMin.z, g.worldBounds.pMax.z);
        Vector3 pos_delta = new_pos - pos;
        pos = Position { new_pos };
        action.remainingTime = pos_delta.length() / kMoveSpeed;
    }
}

// A blast tests every Position / Health row of the world (250 at the
// benchmark size) against its radius.  A dragon casts about once per 1200
// ticks, so one lane per dragon keeps the common path cheap, but a caster's
// serial scan set the kernel's length (a chain of ~250 dependent cache
// reads).  On the device the active lanes of the caster's wave share each
// blast's scan; damage is an integer atomic subtraction, so every hp ends as
// after the reference's serial scan.
MW_HD static inline void blast(Engine &ctx, const Game &g, int32_t w, const Vector3 &target, int32_t first,
                               int32_t stride)
{
    StateView &st = ctx.state();
    for (int32_t a = 0; a < g.healthQuery.numArchetypes; a++) {
        const int32_t arch = g.healthQuery.archetypes[a];
        const Position *pos = st.column<Position>(arch, g.healthQuery.cols[a][0], w);
        Health *hp = st.column<Health>(arch, g.healthQuery.cols[a][1], w);
        const int32_t n = st.arch[arch].numRows[w];
        // four rows' positions loaded before any damage is applied (the
        // atomics would otherwise order each row's load after the last one)
        for (int32_t r0 = first; r0 < n; r0 += 4 * stride) {
            Vector3 p[4];
#pragma unroll
            for (int32_t k = 0; k < 4; k++) {
                const int32_t r = r0 + k * stride;
                if (r < n) p[k] = rowRef(pos, r);
            }
#pragma unroll
            for (int32_t k = 0; k < 4; k++) {
                const int32_t r = r0 + k * stride;
                if (r < n && target.distance(p[k]) <= kBlastRadius) damage(rowRef(hp, r), kBlastDamage);
            }
        }
    }
}

MW_HD void Game::casterSystem(Engine &ctx, Entity &e, Action &action, Mana &mana)
{                                                          // fvs.cpp:153-190
    const Game &g = ctx.data();
    mana.mp += kManaRegenRate * kDeltaT;
    const bool cast = !(action.remainingTime > 0) && !(mana.mp < kCastCost);
    Vector3 target {};
    if (cast) {
        mana.mp -= kCastCost;
        const Draw d { g.worldSeed, (uint32_t)e.id, g.tickCount };
        target = Vector3 {
            d.uniform(kDrawTargetX, g.worldBounds.pMin.x, g.worldBounds.pMax.x),
            d.uniform(kDrawTargetY, g.worldBounds.pMin.y, g.worldBounds.pMax.y),
            d.uniform(kDrawTargetZ, g.worldBounds.pMin.z, g.worldBounds.pMax.z),
        };
        action.remainingTime = kCastTime;
    }
    const int32_t w = ctx.worldID().idx;
#if defined(__HIP_DEVICE_COMPILE__)
    // every active lane of the wave helps with each of its casters' blasts
    const uint64_t active = __ballot(1);
    const int32_t rank = __popcll(active & ((1ull << __lane_id()) - 1));
    const int32_t lanes = __popcll(active);
    uint64_t casters = __ballot(cast);
    while (casters) {
        const int32_t src = __builtin_ctzll(casters);
        casters &= casters - 1;
        const Vector3 t { __shfl(target.x, src), __shfl(target.y, src), __shfl(target.z, src) };
        blast(ctx, g, __shfl(w, src), t, rank, lanes);
    }
#elif !defined(__HIPCC__)
    if (cast) blast(ctx, g, w, target, 0, 1);
#endif
}

MW_HD void Game::archerSystem(Engine &ctx, Entity &e, Action &action, Quiver &quiver)
{                                                          // fvs.cpp:192-214
    const Game &g = ctx.data();
    if (action.remainingTime > 0 || quiver.numArrows == 0) return;
    StateView &st = ctx.state();
    const int32_t w = ctx.worldID().idx;
    const int32_t num_dragons = st.arch[g.dragonArch].numRows[w];
    if (num_dragons > 0) {            // the reference's uniform_int_distribution(0, -1) is UB
        const Draw d { g.worldSeed, (uint32_t)e.id, g.tickCount };
        const uint32_t idx = d.index(kDrawDragon, (uint32_t)num_dragons);
        damage(rowRef(st.column<Health>(g.dragonArch, g.dragonHealthCol, w), idx), kArrowDamage);
    }
    quiver.numArrows -= 1;
    action.remainingTime = kShootTime;
}

// The reference's cleanup (fvs.cpp:224-239) walks cleanupQuery serially and
// makes a CleanupTracker for every entity with hp <= 0, destroys every
// tracked entity in tracker order, then clears the trackers.  Here:
//   markDead     every row checks itself in parallel (atomics into a list);
//   trackDead    one lane per world sorts the (few) hits back into the
//                walk's order -- query archetype, then row -- and makes the
//                trackers (the same IDs as the reference's serial walk);
//   destroy      a row-parallel node over the trackers: each lane's
//                destroyEntityNow is deferred and the executor's ordered
//                commit replays them in tracker order -- the reference's
//                swap-remove sequence on row indices in LDS, the row moves
//                of every column spread over the world's block, ID releases
//                in order (wave-parallel compaction);
//   finishTick   clears the trackers (bulk ID release) and ticks.
MW_HD void Game::markDeadSystem(Engine &ctx, Entity &e, Health &h)
{
    if (h.hp > 0) return;
    Game &g = ctx.data();
#if defined(__HIP_DEVICE_COMPILE__)
    const int32_t slot = atomicAdd(&g.numDead, 1);
#else
    const int32_t slot = g.numDead++;
#endif
    if (slot < kMaxDead) g.dead[slot] = Dead { e, ctx.getLoc(e) };
}

MW_HD void Game::trackDeadSystem(Engine &ctx)
{
    Game &g = ctx.data();
    const int32_t n = g.numDead < kMaxDead ? g.numDead : kMaxDead;
    if (g.numDead > kMaxDead) ctx.state().errorFlags[ctx.worldID().idx] |= 2;
    for (int32_t i = 1; i < n; i++) {                     // insertion sort by (archetype, row)
        const Dead d = g.dead[i];
        int32_t j = i - 1;
        while (j >= 0 && (g.dead[j].loc.archetype > d.loc.archetype ||
                          (g.dead[j].loc.archetype == d.loc.archetype &&
                           g.dead[j].loc.row > d.loc.row))) {
            g.dead[j + 1] = g.dead[j];
            j--;
        }
        g.dead[j + 1] = d;
    }
    for (int32_t i = 0; i < n; i++) ctx.makeEntityNow<CleanupTracker>(CleanupEntity { g.dead[i].e });
    g.numDead = 0;
}

MW_HD void Game::destroyTrackedSystem(Engine &ctx, CleanupEntity &c)
{
    ctx.destroyEntityNow(c);
}

MW_HD void Game::finishTickSystem(Engine &ctx)
{
    ctx.clearArchetype<CleanupTracker>();
    ctx.data().tickCount += 1;
}

Game::Game(Engine &ctx, const Config &cfg, const mw_fvs_init &init)
    : WorldBase(ctx)
{                                                          // fvs.cpp:42-109
    worldSeed = (uint32_t)init.world_index;
    tickCount = 0;
    numDead = 0;
    worldBounds = AABB { { -10, -10, 0 }, { 10, 10, 10 } };
    for (int32_t i = 0; i < cfg.c.num_dragons; i++) {
        ctx.makeEntityNow<Dragon>(
            Position { Vector3 { init.dragon_pos[3 * i], init.dragon_pos[3 * i + 1],
                                 init.dragon_pos[3 * i + 2] } },
            Health { kDragonHP }, Action { 0.f }, Mana { init.dragon_mana[i] });
    }
    for (int32_t i = 0; i < cfg.c.num_knights; i++) {
        ctx.makeEntityNow<Knight>(
            Position { Vector3 { init.knight_pos[3 * i], init.knight_pos[3 * i + 1],
                                 init.knight_pos[3 * i + 2] } },
            Health { kKnightHP }, Action { 0.f }, Quiver { init.knight_arrows[i] });
    }
    StateView &st = ctx.state();
    dragonArch = st.findArchetype(typeKey<Dragon>());
    dragonHealthCol = st.findColumn(dragonArch, typeKey<Health>());
    healthQuery = ctx.query<Position, Health>();
    cleanupQuery = ctx.query<Entity, Health>();
}

using Exec = TaskGraphExecutor<Engine, Game, Config, mw_fvs_init>;

static Executor *create(const ExecConfig &ecfg, const void *user_cfg, size_t cfg_bytes,
                        const void *inits, size_t init_stride)
{
    if (cfg_bytes != sizeof(mw_fvs_config)) {
        throw std::runtime_error("fantasy_vs: user config size mismatch");
    }
    Config cfg;
    memcpy(&cfg.c, user_cfg, sizeof(cfg.c));
    if (cfg.c.num_dragons < 0 || cfg.c.num_knights < 0) {
        throw std::runtime_error("fantasy_vs: negative entity counts");
    }
    std::vector<mw_fvs_init> init_vec(ecfg.numWorlds);
    for (int32_t w = 0; w < ecfg.numWorlds; w++) {
        memcpy(&init_vec[w], (const char *)inits + (size_t)w * init_stride, sizeof(mw_fvs_init));
    }
    return new Exec(ecfg, cfg, init_vec.data());
}

static EnvRegistration reg("fantasy_vs", &create);

}

// Initial state (fvs.cpp:88-108): one mt19937 drawn serially over worlds;
// per dragon x, y, z then mana ~ U[0, 50); per knight x, y, z then arrows ~
// U{20..40}.  first_world selects a shard of the serial sequence.
extern "C" void mw_gen_fvs_inits(int32_t first_world, int32_t num_worlds, int32_t num_dragons,
                                 int32_t num_knights, uint32_t seed, float *dragon_pos,
                                 float *dragon_mana, float *knight_pos, int32_t *knight_arrows)
{
    std::mt19937 gen(seed);
    std::uniform_real_distribution<float> xd(-10.f, 10.f), yd(-10.f, 10.f), zd(0.f, 10.f);
    std::uniform_real_distribution<float> mp(0.f, 50.f);
    std::uniform_int_distribution<int> arrows(20, 40);
    for (int64_t w = 0; w < (int64_t)first_world + num_worlds; w++) {
        const bool keep = w >= first_world;
        const int64_t o = w - first_world;
        for (int64_t i = 0; i < num_dragons; i++) {
            float x = xd(gen), y = yd(gen), z = zd(gen), m = mp(gen);
            if (!keep) continue;
            float *p = dragon_pos + (o * num_dragons + i) * 3;
            p[0] = x; p[1] = y; p[2] = z;
            dragon_mana[o * num_dragons + i] = m;
        }
        for (int64_t i = 0; i < num_knights; i++) {
            float x = xd(gen), y = yd(gen), z = zd(gen);
            int a = arrows(gen);
            if (!keep) continue;
            float *p = knight_pos + (o * num_knights + i) * 3;
            p[0] = x; p[1] = y; p[2] = z;
            knight_arrows[o * num_knights + i] = a;
        }
    }
}
