// ORACLE (test infrastructure only) — serial CPU restatement of the
// fantasy_vs tick on a restated single-world ECS:
//   * entity store: orc_idmap.hpp (reference id_map_impl.inl);
//   * tables: append on makeEntityNow (reference state.inl:398-449),
//     swap-remove + moved-entity remap on destroyEntityNow
//     (src/core/state.cpp:181-202, table.cpp:64-76), bulkFree on
//     clearArchetype of a non-temporary archetype (state.cpp:565-581);
//   * systems: examples/fantasy_vs/fvs.cpp:111-240 (Game::tick) with the
//     counter-based draws of gpu-ecs-madrona_amd/csrc/envs/fvs_rules.hpp.
// Archetype / query order follows registration: Dragon (0), Knight (1),
// CleanupTracker (2).  Pinned against the reference ECS by
// oracle/ref_fvs.cpp (tests/test_fvs_oracle.py).

#include "orc_idmap.hpp"
#include "../gpu-ecs-madrona_amd/csrc/envs/fvs_rules.hpp"

#include <cmath>
#include <cstdint>
#include <cstring>
#include <random>
#include <vector>

using namespace orc;
using namespace fvs_rules;

namespace {

struct V3 {
    float x, y, z;
    V3 operator+(V3 o) const { return { x + o.x, y + o.y, z + o.z }; }
    V3 operator-(V3 o) const { return { x - o.x, y - o.y, z - o.z }; }
    float length2() const { return x * x + y * y + z * z; }
    float length() const { return sqrtf(length2()); }
    float distance(V3 o) const { return (*this - o).length(); }
};

struct Table {
    std::vector<Entity> ent;
    std::vector<V3> pos;
    std::vector<int32_t> hp;
    std::vector<float> remaining;
    std::vector<uint32_t> extra;   // Mana (float bits) or Quiver (int)

    int32_t size() const { return (int32_t)ent.size(); }
    int32_t append(Entity e, V3 p, int32_t h, float r, uint32_t x)
    {
        ent.push_back(e); pos.push_back(p); hp.push_back(h);
        remaining.push_back(r); extra.push_back(x);
        return size() - 1;
    }
    // Table::removeRow: the last row moves into `row`; true if one moved
    bool removeRow(int32_t row)
    {
        const int32_t last = size() - 1;
        const bool moved = row != last;
        if (moved) {
            ent[row] = ent[last]; pos[row] = pos[last]; hp[row] = hp[last];
            remaining[row] = remaining[last]; extra[row] = extra[last];
        }
        ent.pop_back(); pos.pop_back(); hp.pop_back(); remaining.pop_back(); extra.pop_back();
        return moved;
    }
};

enum : uint32_t { kDragon = 0, kKnight = 1, kTracker = 2 };

struct World {
    IDMap ids;
    IDMap::Cache cache;           // the world's StateCache
    Table tables[2];
    std::vector<Entity> tracker;  // CleanupTracker rows (CleanupEntity column)
    std::vector<Entity> trackerIds;
    uint32_t seed = 0;
    uint32_t tick = 0;
};

struct Fvs {
    int32_t numDragons, numKnights;
    std::vector<World> worlds;
};

static uint32_t fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float bitsf(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static float clampRef3(float v, float lo, float hi) { return clampRef(v, lo, hi); }

static const V3 kMin { -10, -10, 0 }, kMax { 10, 10, 10 };

static void makeEntity(World &w, uint32_t arch, V3 p, int32_t hp, float r, uint32_t x)
{
    Entity e = w.ids.acquireID(w.cache);
    int32_t row = w.tables[arch].append(e, p, hp, r, x);
    w.ids.ref(e.id) = Loc { arch, row };
}

static void destroyEntity(World &w, Entity e)
{
    Loc loc = w.ids.lookup(e);
    if (loc.archetype == 0xFFFFFFFFu) return;
    Table &t = w.tables[loc.archetype];
    if (t.removeRow(loc.row)) w.ids.ref(t.ent[loc.row].id).row = loc.row;
    w.ids.releaseID(w.cache, e.id);
}

static void tick(World &w)
{
    // actionSelect (fvs.cpp:111-151) over (Entity, Position, Action)
    for (uint32_t a : { kDragon, kKnight }) {
        Table &t = w.tables[a];
        for (int32_t r = 0; r < t.size(); r++) {
            float &rem = t.remaining[r];
            if (rem > 0) { rem -= kDeltaT; continue; }
            const Draw d { w.seed, (uint32_t)t.ent[r].id, w.tick };
            if (d.uniform(kDrawMoveProb) <= kMoveCutoff) {
                V3 &pos = t.pos[r];
                V3 np = pos + V3 { d.uniform(kDrawMoveX, -1.f, 1.f), d.uniform(kDrawMoveY, -1.f, 1.f),
                                   d.uniform(kDrawMoveZ, -1.f, 1.f) };
                np.x = clampRef3(np.x, kMin.x, kMax.x);
                np.y = clampRef3(np.y, kMin.y, kMax.y);
                np.z = clampRef3(np.x, kMin.z, kMax.z);
                V3 delta = np - pos;
                pos = np;
                rem = delta.length() / kMoveSpeed;
            }
        }
    }
    // caster (fvs.cpp:153-190) over (Entity, Action, Mana): dragons
    {
        Table &t = w.tables[kDragon];
        for (int32_t r = 0; r < t.size(); r++) {
            float mp = bitsf(t.extra[r]);
            mp += kManaRegenRate * kDeltaT;
            t.extra[r] = fbits(mp);
            if (t.remaining[r] > 0) continue;
            if (mp < kCastCost) continue;
            mp -= kCastCost;
            t.extra[r] = fbits(mp);
            const Draw d { w.seed, (uint32_t)t.ent[r].id, w.tick };
            const V3 target { d.uniform(kDrawTargetX, kMin.x, kMax.x),
                              d.uniform(kDrawTargetY, kMin.y, kMax.y),
                              d.uniform(kDrawTargetZ, kMin.z, kMax.z) };
            for (uint32_t a : { kDragon, kKnight }) {
                Table &o = w.tables[a];
                for (int32_t k = 0; k < o.size(); k++) {
                    if (target.distance(o.pos[k]) <= kBlastRadius) o.hp[k] -= kBlastDamage;
                }
            }
            t.remaining[r] = kCastTime;
        }
    }
    // archer (fvs.cpp:192-214) over (Entity, Action, Quiver): knights
    {
        Table &t = w.tables[kKnight];
        Table &dr = w.tables[kDragon];
        for (int32_t r = 0; r < t.size(); r++) {
            int32_t arrows = (int32_t)t.extra[r];
            if (t.remaining[r] > 0 || arrows == 0) continue;
            if (dr.size() > 0) {
                const Draw d { w.seed, (uint32_t)t.ent[r].id, w.tick };
                dr.hp[d.index(kDrawDragon, (uint32_t)dr.size())] -= kArrowDamage;
            }
            t.extra[r] = (uint32_t)(arrows - 1);
            t.remaining[r] = kShootTime;
        }
    }
    // cleanup (fvs.cpp:224-239)
    for (uint32_t a : { kDragon, kKnight }) {
        Table &t = w.tables[a];
        for (int32_t r = 0; r < t.size(); r++) {
            if (t.hp[r] <= 0) {
                Entity te = w.ids.acquireID(w.cache);          // makeEntityNow<CleanupTracker>
                w.ids.ref(te.id) = Loc { kTracker, (int32_t)w.tracker.size() };
                w.tracker.push_back(t.ent[r]);
                w.trackerIds.push_back(te);
            }
        }
    }
    for (Entity e : w.tracker) destroyEntity(w, e);
    w.ids.bulkRelease(w.cache, w.trackerIds.data(), (int32_t)w.trackerIds.size());
    w.tracker.clear();
    w.trackerIds.clear();
    w.tick += 1;
}

}

extern "C" {

struct OrcFvsRow {
    uint32_t gen;
    int32_t id;
    float pos[3];
    int32_t hp;
    float remaining;
    uint32_t extra;
};

void *orc_fvs_create(int32_t num_worlds, int32_t num_dragons, int32_t num_knights,
                     const float *dragon_pos, const float *dragon_mana,
                     const float *knight_pos, const int32_t *knight_arrows,
                     int32_t first_world_index)
{
    auto *f = new Fvs {};
    f->numDragons = num_dragons;
    f->numKnights = num_knights;
    f->worlds.resize(num_worlds);
    for (int32_t w = 0; w < num_worlds; w++) {
        World &wd = f->worlds[w];
        wd.seed = (uint32_t)(first_world_index + w);
        for (int32_t i = 0; i < num_dragons; i++) {
            const float *p = dragon_pos + ((size_t)w * num_dragons + i) * 3;
            makeEntity(wd, kDragon, V3 { p[0], p[1], p[2] }, kDragonHP, 0.f,
                       fbits(dragon_mana[(size_t)w * num_dragons + i]));
        }
        for (int32_t i = 0; i < num_knights; i++) {
            const float *p = knight_pos + ((size_t)w * num_knights + i) * 3;
            makeEntity(wd, kKnight, V3 { p[0], p[1], p[2] }, kKnightHP, 0.f,
                       (uint32_t)knight_arrows[(size_t)w * num_knights + i]);
        }
    }
    return f;
}

void orc_fvs_step(void *handle, int32_t num_ticks)
{
    auto *f = (Fvs *)handle;
    for (int32_t s = 0; s < num_ticks; s++) {
        for (World &w : f->worlds) tick(w);
    }
}

int32_t orc_fvs_read(void *handle, int32_t world, int32_t arch, OrcFvsRow *out, int32_t cap)
{
    auto *f = (Fvs *)handle;
    const Table &t = f->worlds[world].tables[arch];
    const int32_t n = t.size() < cap ? t.size() : cap;
    for (int32_t r = 0; r < n; r++) {
        out[r] = OrcFvsRow { t.ent[r].gen, t.ent[r].id, { t.pos[r].x, t.pos[r].y, t.pos[r].z },
                             t.hp[r], t.remaining[r], t.extra[r] };
    }
    return t.size();
}

void orc_fvs_destroy(void *handle) { delete (Fvs *)handle; }

// Initial state of examples/fantasy_vs/fvs.cpp:88-108: one mt19937 drawn
// serially over worlds; per dragon x, y, z (randomPosition, :28-39) and mana
// U[0, 50); per knight x, y, z and arrows U{20..40}.
void orc_gen_fvs_inits(int32_t num_worlds, int32_t nd, int32_t nk, uint32_t seed,
                       float *dpos, float *dmana, float *kpos, int32_t *karrows)
{
    std::mt19937 gen(seed);
    std::uniform_real_distribution<float> xd(-10.f, 10.f), yd(-10.f, 10.f), zd(0.f, 10.f);
    std::uniform_real_distribution<float> mp(0.f, 50.f);
    std::uniform_int_distribution<int> arrows(20, 40);
    for (int64_t w = 0; w < num_worlds; w++) {
        for (int64_t i = 0; i < nd; i++) {
            float *p = dpos + (w * nd + i) * 3;
            p[0] = xd(gen); p[1] = yd(gen); p[2] = zd(gen);
            dmana[w * nd + i] = mp(gen);
        }
        for (int64_t i = 0; i < nk; i++) {
            float *p = kpos + (w * nk + i) * 3;
            p[0] = xd(gen); p[1] = yd(gen); p[2] = zd(gen);
            karrows[w * nk + i] = arrows(gen);
        }
    }
}

}
