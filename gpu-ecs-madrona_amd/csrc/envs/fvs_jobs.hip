// "fantasy_vs_jobs": examples/fantasy_vs as the reference wrote it, against
// the job API (ctx.parallelFor / ctx.submit / ctx.archetype<A>() /
// ctx.currentJobID(), fvs.cpp:111-292), run through this framework's Context
// job API (include/madrona/context.hpp): the game loop is a PerWorldNode and
// each world's jobs run on the lane that owns the world, in submission order
// (SURVEY.md §8(f)-2).  Edits from the reference source, all forced by the
// device or by determinism:
//   1. the racy thread_local mt19937 draws become the counter-based Draw of
//      fvs_rules.hpp keyed by the entity, so the row queries gain an Entity
//      column (the TaskGraph restatement, fvs.hip, does the same);
//   2. lambdas capturing `this` take the world from ctx.game() (a device
//      lane has no host `this`), and the world's constants are fvs_rules';
//   3. the win / tick printf's are dropped (every world, every step);
//   4. no uniform_int_distribution(0, -1) when no dragon is left (UB).
// Same tables, IDs and draws as fvs.hip and oracle/fvs_oracle.cpp, so the
// three agree bit for bit while both sides have entities left (after that
// this loop stops ticking, as the reference's gameLoop does).
#include <madrona/math.hpp>
#include <madrona/mw_gpu.hpp>

#include "../runtime/env_registry.hpp"
#include "../../../include/madrona_mw.h"
#include "fvs_rules.hpp"

#include <cstring>

using namespace madrona;
using namespace madrona::math;

namespace FantasyVSJobs {

using namespace fvs_rules;

struct Position : Vector3 {};

struct alignas(64) Health {                    // std::atomic_int hp, alignas(MADRONA_CACHE_LINE)
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
    }

    // Game::entry (fvs.cpp:290-300) starts gameLoop once; the loop's body is
    // the job the step graph replays.
    static void setupTasks(TaskGraph::Builder &builder, const Config &)
    {
        builder.addToGraph<PerWorldNode<Engine, entry>>({});
    }

    Game(Engine &ctx, const Config &cfg, const mw_fvs_init &init);

    static MW_HD void entry(Engine &ctx);
    MW_HD void tick(Engine &ctx);
    MW_HD void gameLoop(Engine &ctx);

    uint32_t worldSeed;                  // global world index (shard-independent draws)
    uint32_t tickCount;
    AABB worldBounds;

    Query<Entity, Position, Action> actionQuery;
    Query<Entity, Action, Mana> casterQuery;
    Query<Entity, Action, Quiver> archerQuery;
    Query<Position, Health> healthQuery;
    Query<Entity, Health> cleanupQuery;
};

class Engine : public CustomContext<Engine, Game> {
public:
    using CustomContext::CustomContext;
    MW_INLINE Game &game() { return data(); }
};

MW_HD static inline Vector3 randomPosition(const AABB &bounds, const Draw &d)
{                                                          // fvs.cpp:28-39
    return Vector3 {
        d.uniform(kDrawTargetX, bounds.pMin.x, bounds.pMax.x),
        d.uniform(kDrawTargetY, bounds.pMin.y, bounds.pMax.y),
        d.uniform(kDrawTargetZ, bounds.pMin.z, bounds.pMax.z),
    };
}

MW_HD static JobID actionSelectSystem(Engine &ctx)
{                                                          // fvs.cpp:111-151
    return ctx.parallelFor(ctx.game().actionQuery, [](Engine &ctx, Entity e, Position &pos,
                                                      Action &action) {
        const Game &game = ctx.game();

        if (action.remainingTime > 0) {
            action.remainingTime -= kDeltaT;
            return;
        }

        const Draw d { game.worldSeed, (uint32_t)e.id, game.tickCount };

        if (d.uniform(kDrawMoveProb) <= kMoveCutoff) {
            ctx.submit([&pos, &action, d](Engine &ctx) {
                const AABB &world_bounds = ctx.game().worldBounds;

                // Move
                Vector3 new_pos = pos + Vector3 {
                    d.uniform(kDrawMoveX, -1.f, 1.f),
                    d.uniform(kDrawMoveY, -1.f, 1.f),
                    d.uniform(kDrawMoveZ, -1.f, 1.f),
                };

                new_pos.x = clampRef(new_pos.x, world_bounds.pMin.x, world_bounds.pMax.x);
                new_pos.y = clampRef(new_pos.y, world_bounds.pMin.y, world_bounds.pMax.y);
                new_pos.z = clampRef(new_pos.x, world_bounds.pMin.z, world_bounds.pMax.z);

                Vector3 pos_delta = new_pos - pos;
                pos = Position { new_pos };

                action.remainingTime = pos_delta.length() / kMoveSpeed;
            });
        }
    });
}

MW_HD static JobID casterSystem(Engine &ctx, JobID action_job)
{                                                          // fvs.cpp:153-190
    return ctx.parallelFor(ctx.game().casterQuery, [](Engine &ctx, Entity e, Action &action,
                                                      Mana &mana) {
        const Game &game = ctx.game();

        mana.mp += kManaRegenRate * kDeltaT;

        if (action.remainingTime > 0) {
            return;
        }

        if (mana.mp < kCastCost) {
            return;
        }

        mana.mp -= kCastCost;

        const Draw d { game.worldSeed, (uint32_t)e.id, game.tickCount };
        auto target_pos = randomPosition(game.worldBounds, d);

        ctx.parallelFor(game.healthQuery, [target_pos](Engine &, const Position &pos,
                                                       Health &health) {
            if (target_pos.distance(pos) <= kBlastRadius) {
                health.hp -= kBlastDamage;
            }
        });

        action.remainingTime = kCastTime;
    }, true, action_job);
}

MW_HD static JobID archerSystem(Engine &ctx, JobID action_job)
{                                                          // fvs.cpp:192-214
    return ctx.parallelFor(ctx.game().archerQuery, [](Engine &ctx, Entity e, Action &action,
                                                      Quiver &quiver) {
        if (action.remainingTime > 0 || quiver.numArrows == 0) {
            return;
        }

        auto dragons = ctx.archetype<Dragon>();
        uint32_t num_dragons = dragons.size();

        if (num_dragons > 0) {
            const Game &game = ctx.game();
            const Draw d { game.worldSeed, (uint32_t)e.id, game.tickCount };
            uint32_t dragon_idx = d.index(kDrawDragon, num_dragons);
            Health &dragon_health = dragons.get<Health>(dragon_idx);
            dragon_health.hp -= kArrowDamage;
        }

        quiver.numArrows -= 1;
        action.remainingTime = kShootTime;
    }, true, action_job);
}

MW_HD void Game::tick(Engine &ctx)
{                                                          // fvs.cpp:216-240
    JobID init_action_job = actionSelectSystem(ctx);

    JobID cast_job = casterSystem(ctx, init_action_job);

    JobID archer_job = archerSystem(ctx, init_action_job);

    ctx.submit([](Engine &ctx) {
        Game &game = ctx.game();
        ctx.forEach(game.cleanupQuery, [&ctx](Entity e, Health &health) {
            if (health.hp <= 0) {
                ctx.makeEntityNow<CleanupTracker>(CleanupEntity { e });
            }
        });

        auto cleanup_tracker = ctx.archetype<CleanupTracker>();
        auto cleanup_entities = cleanup_tracker.component<CleanupEntity>();
        for (int i = 0, n = cleanup_tracker.size(); i < n; i++) {
            ctx.destroyEntityNow(cleanup_entities[i]);
        }

        ctx.clearArchetype<CleanupTracker>();
    }, true, cast_job, archer_job);
}

MW_HD void Game::gameLoop(Engine &ctx)
{                                                          // fvs.cpp:242-271
    ctx.submit([](Engine &ctx) {
        Game &game = ctx.game();
        auto dragons = ctx.archetype<Dragon>();
        auto knights = ctx.archetype<Knight>();

        if (dragons.size() == 0) {          // "Knights win!"
            return;
        }

        if (knights.size() == 0) {          // "Dragons win!"
            return;
        }

        game.tick(ctx);

        game.tickCount += 1;

        // Queues the loop again behind the current job: the next step.
        game.gameLoop(ctx);
    }, /* not a child of the current job */ false, ctx.currentJobID());
}

MW_HD void Game::entry(Engine &ctx)
{
    ctx.game().gameLoop(ctx);
}

Game::Game(Engine &ctx, const Config &cfg, const mw_fvs_init &init)
    : WorldBase(ctx)
{                                                          // fvs.cpp:42-109
    worldSeed = (uint32_t)init.world_index;
    tickCount = 0;
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
    actionQuery = ctx.query<Entity, Position, Action>();
    casterQuery = ctx.query<Entity, Action, Mana>();
    archerQuery = ctx.query<Entity, Action, Quiver>();
    healthQuery = ctx.query<Position, Health>();
    cleanupQuery = ctx.query<Entity, Health>();
}

using Exec = TaskGraphExecutor<Engine, Game, Config, mw_fvs_init>;

static Executor *create(const ExecConfig &ecfg, const void *user_cfg, size_t cfg_bytes,
                        const void *inits, size_t init_stride)
{
    if (cfg_bytes != sizeof(mw_fvs_config)) {
        throw std::runtime_error("fantasy_vs_jobs: user config size mismatch");
    }
    Config cfg;
    memcpy(&cfg.c, user_cfg, sizeof(cfg.c));
    if (cfg.c.num_dragons < 0 || cfg.c.num_knights < 0) {
        throw std::runtime_error("fantasy_vs_jobs: negative entity counts");
    }
    std::vector<mw_fvs_init> init_vec(ecfg.numWorlds);
    for (int32_t w = 0; w < ecfg.numWorlds; w++) {
        memcpy(&init_vec[w], (const char *)inits + (size_t)w * init_stride, sizeof(mw_fvs_init));
    }
    return new Exec(ecfg, cfg, init_vec.data());
}

static EnvRegistration reg("fantasy_vs_jobs", &create);

}
