// ECS state for the MI355X framework.
//
// Reference interface: include/madrona/state.hpp:109-134 (ECSRegistry),
// :137-397 (StateManager), include/madrona/impl/id_map_impl.inl (IDMap).
//
// MI355X layout: ONE arena per executor.  Every archetype has a fixed row
// capacity per world and every column is a [world][capacity] slab, so a
// column for all worlds is one contiguous SoA array:
//
//     element(world w, row r) = cols[c] + (w * capacity + r) * colBytes[c]
//
// Column 0 is the Entity column; user components start at column 1 (the
// reference single-world / GPU layout, physics Cols 1..12).  The same
// StateView struct describes the host mirror (used while worlds are built on
// the host) and the device arena (used by every kernel), so host and device
// code paths share one implementation.
#pragma once

#include <madrona/ecs.hpp>

#include <cassert>
#include <cstring>
#include <type_traits>
#include <utility>

namespace madrona {

inline constexpr int32_t kMaxArchetypes = 64;
inline constexpr int32_t kMaxColumns = 24;
inline constexpr int32_t kIDsPerCache = 64;            // id_map.hpp:134

// ---------------------------------------------------------------------------
// Compile-time type keys: FNV-1a of the clang type spelling.  Identical on the
// host and device passes of hipcc, so device code can resolve a component's
// column without any runtime registration hand-off.
// ---------------------------------------------------------------------------
namespace detail {
constexpr MW_INLINE uint64_t fnv1a(const char *s)
{
    uint64_t h = 1469598103934665603ull;
    while (*s) {
        h ^= (uint64_t)(unsigned char)*s++;
        h *= 1099511628211ull;
    }
    return h;
}

template <typename T>
constexpr MW_INLINE uint64_t typeKeyImpl()
{
    return fnv1a(__PRETTY_FUNCTION__);
}
}

template <typename T>
constexpr MW_INLINE uint64_t typeKey()
{
    return detail::typeKeyImpl<std::remove_cv_t<std::remove_reference_t<T>>>();
}

// ---------------------------------------------------------------------------
// Entity ID store: per-world restatement of the reference IDMap
// (id_map_impl.inl:17-332).  Each world owns a node array of idsPerWorld
// entries and a header; expansion hands out the next 64-ID block.
// ---------------------------------------------------------------------------
struct IDCache {
    int32_t freeHead;
    int32_t numFree;
    int32_t overflowHead;
    int32_t numOverflow;
};

struct IDNode {
    Loc val;          // aliased by {subNext, globalNext} while free
    uint32_t gen;
};

struct IDMapState {
    int32_t globalHead;
    int32_t numIDs;
    IDCache worldCache;
    IDCache initCache;
    int32_t lock;         // row-parallel makeEntityNow (Context::lockedAcquire)
    int32_t pad;
};

struct IDMapView {
    IDNode *nodes;
    IDMapState *st;
    int32_t capacity;
    int32_t *errorFlag;

    MW_INLINE int32_t &subNext(int32_t id) { return *(int32_t *)&nodes[id].val.archetype; }
    MW_INLINE int32_t &globalNext(int32_t id) { return nodes[id].val.row; }

    MW_INLINE Entity assignCached(int32_t *head)
    {
        int32_t new_id = *head;
        int32_t num_contiguous = globalNext(new_id);
        if (num_contiguous == 1) {
            *head = subNext(new_id);
        } else {
            int32_t next_free = new_id + 1;
            subNext(next_free) = subNext(new_id);
            globalNext(next_free) = num_contiguous - 1;
            nodes[next_free].gen = 0;
            *head = next_free;
        }
        return Entity { nodes[new_id].gen, new_id };
    }

    MW_INLINE Entity acquire(IDCache &cache)
    {
        if (cache.numOverflow > 0) {
            cache.numOverflow -= 1;
            return assignCached(&cache.overflowHead);
        }
        if (cache.numFree > 0) {
            cache.numFree -= 1;
            return assignCached(&cache.freeHead);
        }
        if (st->globalHead != -1) {
            int32_t free_ids = st->globalHead;
            st->globalHead = globalNext(free_ids);
            globalNext(free_ids) = 1;
            cache.freeHead = free_ids;
            cache.numFree = kIDsPerCache - 1;
            return assignCached(&cache.freeHead);
        }
        int32_t block_start = st->numIDs;
        if (block_start + kIDsPerCache > capacity) {
            *errorFlag |= 1;
            return Entity::none();
        }
        st->numIDs += kIDsPerCache;
        nodes[block_start].gen = 0;
        subNext(block_start + 1) = -1;
        globalNext(block_start + 1) = kIDsPerCache - 1;
        nodes[block_start + 1].gen = 0;
        cache.freeHead = block_start + 1;
        cache.numFree = kIDsPerCache - 1;
        return Entity { 0, block_start };
    }

    MW_INLINE void release(IDCache &cache, int32_t id)
    {
        nodes[id].gen += 1;
        globalNext(id) = 1;
        if (cache.numFree < kIDsPerCache) {
            subNext(id) = cache.freeHead;
            cache.freeHead = id;
            cache.numFree += 1;
            return;
        }
        if (cache.numOverflow < kIDsPerCache) {
            subNext(id) = cache.overflowHead;
            cache.overflowHead = id;
            cache.numOverflow += 1;
        }
        if (cache.numOverflow == kIDsPerCache) {
            globalNext(cache.overflowHead) = st->globalHead;
            st->globalHead = cache.overflowHead;
            cache.overflowHead = -1;
            cache.numOverflow = 0;
        }
    }

    MW_INLINE void bulkRelease(IDCache &cache, const Entity *keys, int32_t num_keys)
    {
        if (num_keys <= 0) return;
        int32_t base_idx;
        int32_t num_remaining = 0;
        int32_t global_tail = -1;
        auto link = [&](int32_t idx) {
            int32_t cur = keys[idx].id;
            nodes[cur].gen += 1;
            subNext(cur) = keys[idx + 1].id;
            globalNext(cur) = 1;
        };
        for (base_idx = 0; base_idx < num_keys; base_idx += kIDsPerCache) {
            num_remaining = num_keys - base_idx;
            if (num_remaining < kIDsPerCache) break;
            int32_t head_id = keys[base_idx].id;
            for (int32_t s = 0; s < kIDsPerCache; s++) link(base_idx + s);
            int32_t last = keys[base_idx + kIDsPerCache - 1].id;
            nodes[last].gen += 1;
            subNext(last) = -1;
            globalNext(last) = 1;
            if (global_tail != -1) globalNext(global_tail) = head_id;
            global_tail = head_id;
        }
        if (num_remaining != kIDsPerCache) {
            int32_t start_id = keys[base_idx].id;
            for (int32_t idx = base_idx; idx < num_keys - 1; idx++) link(idx);
            int32_t tail = keys[num_keys - 1].id;
            nodes[tail].gen += 1;
            globalNext(tail) = 1;
            subNext(tail) = cache.overflowHead;
            int32_t num_from_overflow = kIDsPerCache - num_remaining;
            if (cache.numOverflow < num_from_overflow) {
                cache.overflowHead = start_id;
                cache.numOverflow += num_remaining;
            } else {
                int32_t next_id = cache.overflowHead;
                int32_t overflow_node = -1;
                for (int32_t i = 0; i < num_from_overflow; i++) {
                    overflow_node = next_id;
                    next_id = subNext(overflow_node);
                }
                subNext(overflow_node) = -1;
                cache.overflowHead = next_id;
                cache.numOverflow -= num_from_overflow;
                if (global_tail != -1) globalNext(global_tail) = start_id;
                global_tail = start_id;
            }
        }
        if (global_tail == -1) return;
        globalNext(global_tail) = st->globalHead;
        st->globalHead = keys[0].id;
    }

    MW_INLINE Loc lookup(Entity e) const
    {
        if (e.id < 0 || e.id >= st->numIDs) return Loc::none();
        const IDNode &n = nodes[e.id];
        if (n.gen != e.gen) return Loc::none();
        return n.val;
    }
};

// ---------------------------------------------------------------------------
// Per-world error bits raised by the engine (StateView::errorFlags; the
// physics module's bits live in csrc/physics/physics_impl.hpp, bits 0..15).
// ---------------------------------------------------------------------------
inline constexpr int32_t kErrFlagJobDropped = 1 << 16;     // deferred job queue full / closure too big
inline constexpr int32_t kErrFlagTmpAllocFull = 1 << 17;   // per-world tmpAlloc arena exhausted
inline constexpr int32_t kErrFlagDeferredFull = 1 << 18;   // deferred destroy log full
inline constexpr int32_t kErrFlagRowParallelOp = 1 << 19;  // op not available in a row-parallel node
inline constexpr int32_t kErrFlagCommitLimit = 1 << 20;    // archetype too large for the ordered commit
inline constexpr int32_t kErrFlagMakeOrder = 1 << 22;      // a row-parallel make gave up waiting for its turn
inline constexpr int32_t kErrFlagCrossRow = 1 << 23;       // row-parallel get/getUnsafe of a query component at another row

// Ordered structural commit (see Context, row-parallel mode): an append key
// orders a row made by a row-parallel lane exactly where the reference's
// world-serial row walk would have made it: [63:32] the lane's row key
// (query archetype << 24 | row), [31:16] the lane's per-row sequence number,
// [15:0] free for the commit's sort.  kNoAppendKey marks settled rows.
inline constexpr uint64_t kNoAppendKey = ~0ull;
inline constexpr uint32_t kSerialRowKey = 0xFFFF'FFFFu;

// Exact type keys of the query components a row-parallel node writes
// (Context::setRowParallel / checkCrossRow); at most kMaxRowWriteKeys are
// tracked -- a node writing more sets `all`, and then every cross-row get
// counts as racing (conservative: flagged rather than left unchecked).
inline constexpr int32_t kMaxRowWriteKeys = 8;
struct RowWriteKeys {
    uint64_t key[kMaxRowWriteKeys];
    int32_t n;
    bool all;

    // constant indices only (no loop the backend could leave in scratch)
    template <size_t... Is>
    MW_INLINE bool hasImpl(uint64_t k, std::index_sequence<Is...>) const
    {
        return (((int32_t)Is < n && key[Is] == k) || ...);
    }
    MW_INLINE bool has(uint64_t k) const
    {
        return all || hasImpl(k, std::make_index_sequence<kMaxRowWriteKeys> {});
    }
};

// Destroy requested by a row-parallel lane; applied by the commit after the
// node, in key order (= the reference's serial destroy order).
struct DeferredDestroy {
    uint64_t key;
    Entity e;
};

// ---------------------------------------------------------------------------
// Arena view (host mirror and device arena share this layout)
// ---------------------------------------------------------------------------
inline constexpr uint32_t kArchTemporary = 1;     // rows have no entity IDs
inline constexpr uint32_t kArchModuleRows = 2;    // rows written by a module's own kernels
inline constexpr uint32_t kArchSingleton = 4;     // exactly one row per world, always
inline constexpr uint32_t kArchGrowable = 8;      // registerArchetype table: the executor grows it

struct ArchetypeView {
    int32_t numColumns;
    int32_t capacity;          // rows per world
    uint32_t flags;            // kArchTemporary | kArchModuleRows
    int32_t *numRows;          // [numWorlds]
    uint64_t *appendKeys;      // [numWorlds][capacity] device only (null: no row-parallel appends)
    int32_t *pendingRows;      // [numWorlds] rows appended by the running row-parallel node
    char *cols[kMaxColumns];
    uint32_t colBytes[kMaxColumns];
    uint64_t colKeys[kMaxColumns];
};

inline constexpr int32_t kMakeTurnSlots = 8;     // = kMaxQueryArchetypes (context.hpp)
inline constexpr int32_t kCommitMaxRows = 4096;  // ordered-commit table limit
inline constexpr int32_t kMakeTurnWaves = 64;    // waves per world with ordered makes

struct StateView {
    int32_t numWorlds;
    int32_t numArchetypes;
    int32_t idsPerWorld;
    uint32_t worldDataStride;
    IDNode *idNodes;            // [numWorlds][idsPerWorld]
    IDMapState *idState;        // [numWorlds]
    char *worldData;            // [numWorlds][worldDataStride]
    int32_t *errorFlags;        // [numWorlds]  bit0 ID store full, bit1 table full, kErrFlag*
    // Ordered structural commit of row-parallel nodes (device only; null
    // on the host mirror, whose contexts are world-serial).
    uint64_t *appendDirty;      // [numWorlds] archetypes appended to by the running node
    int32_t *deferCount;        // [numWorlds] deferred destroys of the running node
    DeferredDestroy *deferLog;  // [numWorlds][deferCap]
    int32_t deferCap;
    // Waves of the running row-parallel node that have finished their rows:
    // per (query archetype, world, wave covering the world) the node's epoch
    // once the wave is done.  A wave's makeEntityNow calls wait until every
    // lower wave of the world is done, so IDs are taken in row order
    // (Context::lockedAcquire).  The ordered commit after each node advances
    // the epoch, so nothing is ever reset.
    int32_t *makeTurn;          // [kMakeTurnSlots][numWorlds][kMakeTurnWaves]
    int32_t *makeEpoch;         // [1]
    // Ordered-commit shape (madrona/commit.hpp): rows per world the index
    // arrays hold, the key sorts' sizes, the widest column.
    int32_t commitCapMax;
    int32_t commitSortA;
    int32_t commitSortO;
    uint32_t commitColMax;
    // Per-world bump allocator (Context::tmpAlloc, reference
    // StateManager::tmpAlloc, src/core/state.cpp:584-602): 256-byte
    // granules, reset by ResetTmpAllocNode.
    uint32_t tmpBytesPerWorld;
    char *tmpArena;             // [numWorlds][tmpBytesPerWorld]
    uint32_t *tmpOffset;        // [numWorlds]
    // Past a world's arena the reference chains another block
    // (TmpAllocator::alloc, src/core/state.cpp:95-114).  Device: a bump pool
    // shared by every world, reset with the arenas by ResetTmpAllocNode; host
    // (CPU back end, world construction): per-world heap blocks
    // (hostTmpOverflow*).  Null / 0: no chaining, exhaustion is flagged.
    char *tmpPool;                       // [tmpPoolBytes] device only
    uint64_t tmpPoolBytes;
    unsigned long long *tmpPoolOffset;   // device only
    void *hostTmpOverflow;               // host only
    uint64_t archKeys[kMaxArchetypes];
    ArchetypeView arch[kMaxArchetypes];

    MW_INLINE IDMapView ids(int32_t world)
    {
        return IDMapView {
            idNodes + (size_t)world * idsPerWorld,
            idState + world,
            idsPerWorld,
            errorFlags + world,
        };
    }

    template <typename T>
    MW_INLINE T *column(uint32_t archetype, int32_t col, int32_t world)
    {
        const ArchetypeView &a = arch[archetype];
        return (T *)(a.cols[col] + (size_t)world * a.capacity * a.colBytes[col]);
    }

    MW_INLINE int32_t findColumn(uint32_t archetype, uint64_t key) const
    {
        const ArchetypeView &a = arch[archetype];
        for (int32_t c = 0; c < a.numColumns; c++) {
            if (a.colKeys[c] == key) return c;
        }
        return -1;
    }

    MW_INLINE int32_t findArchetype(uint64_t key) const
    {
        for (int32_t i = 0; i < numArchetypes; i++) {
            if (archKeys[i] == key) return i;
        }
        return -1;
    }

    // Row-parallel append (device): a row at the end of the world's table,
    // tagged with the caller's append key; the node's commit moves it to its
    // serial position.  -1 when the table is full or the archetype takes no
    // row-parallel appends.
    MW_INLINE int32_t appendRowParallel(uint32_t archetype, int32_t world, uint64_t key)
    {
#if defined(__HIP_DEVICE_COMPILE__)
        ArchetypeView &a = arch[archetype];
        if (!a.appendKeys) {
            atomicOr(errorFlags + world, kErrFlagRowParallelOp);
            return -1;
        }
        const unsigned long long bit = 1ull << archetype;
        if (!(appendDirty[world] & bit)) {
            atomicOr((unsigned long long *)(appendDirty + world), bit);
        }
        // The row count itself stays put until the commit, so every lane of
        // the node sees the tables as they were when it started (rows made
        // by other lanes are not visible, as destroyed rows stay visible).
        const int32_t row = a.numRows[world] + atomicAdd(a.pendingRows + world, 1);
        if (row >= a.capacity) {
            atomicOr(errorFlags + world, 2);
            return -1;
        }
        a.appendKeys[(size_t)world * a.capacity + row] = key;
        return row;
#else
        (void)key;
        return addRow(archetype, world);
#endif
    }

    // Append a row (no entity) from a world-serial context (host, or one
    // lane owning the world).
    MW_INLINE int32_t addRow(uint32_t archetype, int32_t world)
    {
        ArchetypeView &a = arch[archetype];
        int32_t row = a.numRows[world];
        if (row >= a.capacity) {
            errorFlags[world] |= 2;
            return -1;
        }
        a.numRows[world] = row + 1;
        return row;
    }

    // Swap-remove a row (Table::removeRow, src/common/table.cpp:64-76);
    // returns true if the last row moved into `row`.
    MW_INLINE bool removeRow(uint32_t archetype, int32_t world, int32_t row)
    {
        ArchetypeView &a = arch[archetype];
        int32_t from = --a.numRows[world];
        if (from == row) return false;
        for (int32_t c = 0; c < a.numColumns; c++) {
            uint32_t nb = a.colBytes[c];
            char *base = a.cols[c] + (size_t)world * a.capacity * nb;
            memcpy(base + (size_t)row * nb, base + (size_t)from * nb, nb);
        }
        return true;
    }
};

// Chained tmpAlloc blocks of the host view (state.cpp): a block of `bytes`
// for `world` (null when chaining is off), and the release of the world's
// blocks at its tmpAlloc reset.
void *hostTmpOverflowAlloc(StateView &v, int32_t world, uint64_t bytes);
void hostTmpOverflowReset(StateView &v, int32_t world);

// ---------------------------------------------------------------------------
// Host-side registry (StateManager); implementation in csrc/runtime/state.cpp
// ---------------------------------------------------------------------------
struct TypeDesc {
    uint64_t key;
    uint32_t numBytes;
    uint32_t alignment;
    const char *name;
};

class StateManager;

// Module-owned device state (e.g. the physics BVH / contact slabs) that is
// built on the host during world construction and uploaded with the arena.
class StateExtension {
public:
    virtual ~StateExtension() = default;
    virtual void upload(void *stream) = 0;
    // After a table growth (StateManager::growArchetype): slabs the
    // extension cached from the device view may have moved (the entity ID
    // store grows with the tables that take entities).  Called before the
    // executor re-captures the step.
    virtual void stateResized() {}
    // At every executor synchronisation (the stream is idle), with the
    // number of steps run so far: true when the extension changed how its
    // nodes launch and the step must be re-captured.
    virtual bool poll(void *stream, int64_t steps)
    {
        (void)stream; (void)steps;
        return false;
    }
};

class ECSRegistry {
public:
    ECSRegistry(StateManager *state_mgr, void **export_ptrs);

    template <typename ComponentT> void registerComponent();
    template <typename ArchetypeT> void registerArchetype();
    template <typename ArchetypeT> void registerFixedSizeArchetype(CountT max_num_entities);
    template <typename SingletonT> void registerSingleton();
    template <typename ArchetypeT, typename ComponentT> void exportColumn(int32_t slot);
    template <typename SingletonT> void exportSingleton(int32_t slot);

    StateManager &stateManager() { return *state_mgr_; }

private:
    StateManager *state_mgr_;
    void **export_ptrs_;
};

template <typename SingletonT>
struct SingletonArchetype : public madrona::Archetype<SingletonT> {};

namespace detail {
template <typename Base> struct ArchetypeComponents;
template <typename... Cs>
struct ArchetypeComponents<Archetype<Cs...>> {
    static constexpr int32_t count = sizeof...(Cs);
    static void descs(TypeDesc *out)
    {
        int32_t i = 0;
        ((out[i++] = TypeDesc { typeKey<Cs>(), (uint32_t)sizeof(Cs),
                                (uint32_t)alignof(Cs), __PRETTY_FUNCTION__ }), ...);
    }
};
}

class StateManager {
public:
    struct Config {
        int32_t numWorlds;
        int32_t defaultCapacity;     // rows per world for registerArchetype
        int32_t tmpAllocBytesPerWorld = 0;   // Context::tmpAlloc arena per world
        int32_t deferCap = 256;              // deferred destroys per world per node
        int64_t tmpPoolBytes = 0;            // chained tmpAlloc pool (device bytes;
                                             // host: > 0 enables the heap blocks)
    };

    explicit StateManager(const Config &cfg);
    ~StateManager();

    // registration (order defines component / archetype IDs, as in the reference)
    uint32_t registerComponentDesc(const TypeDesc &desc);
    uint32_t registerArchetypeDesc(uint64_t key, const char *name, const TypeDesc *comps,
                                   int32_t num_comps, int32_t capacity, bool temporary);
    void registerSingletonDesc(uint64_t archetype_key);
    void setCapacityHint(uint64_t archetype_key, int32_t capacity);
    int32_t capacityHint(uint64_t archetype_key) const;
    void setTemporary(uint64_t archetype_key);
    // Rows of this archetype are written by a module's own kernels (e.g. the
    // physics candidate list): no row-parallel append keys are kept for it.
    void setModuleRows(uint64_t archetype_key);
    // A module keeps pointers into this archetype's slabs (physics bodies):
    // its capacity stays fixed.
    void pinCapacity(int32_t archetype);

    // Table growth (reference Table::addRow, src/common/table.cpp:44-61: x2
    // when a per-world table is full).  Tables registered with
    // registerArchetype (no fixed size) are growable; the executor grows one
    // between steps, at its high-water mark, to `new_capacity` rows per
    // world: every column slab (and the append keys) is re-strided from
    // [world][capacity] to [world][new_capacity], the entity ID store and the
    // ordered-commit shape are resized with it, and the device view is
    // re-uploaded.  The caller re-captures anything that baked capacities in.
    bool growable(int32_t archetype) const;
    void growArchetype(int32_t archetype, int32_t new_capacity, void *stream);

    template <typename ComponentT>
    uint32_t registerComponent()
    {
        return registerComponentDesc(TypeDesc { typeKey<ComponentT>(), (uint32_t)sizeof(ComponentT),
                                                (uint32_t)alignof(ComponentT), __PRETTY_FUNCTION__ });
    }

    template <typename ArchetypeT>
    uint32_t registerArchetype(int32_t capacity = 0)
    {
        using Comps = detail::ArchetypeComponents<typename ArchetypeT::Base>;
        TypeDesc descs[kMaxColumns];
        Comps::descs(descs);
        return registerArchetypeDesc(typeKey<ArchetypeT>(), __PRETTY_FUNCTION__, descs,
                                     Comps::count, capacity, false);
    }

    template <typename SingletonT>
    void registerSingleton()
    {
        registerComponent<SingletonT>();
        registerArchetype<SingletonArchetype<SingletonT>>(1);
        registerSingletonDesc(typeKey<SingletonArchetype<SingletonT>>());
    }

    template <typename ArchetypeT>
    int32_t archetypeID() const { return archetypeIndex(typeKey<ArchetypeT>()); }

    int32_t archetypeIndex(uint64_t key) const;
    int32_t numArchetypes() const;

    // Export registration: slot -> (archetype, column).
    void registerExport(int32_t slot, uint64_t archetype_key, uint64_t component_key);
    struct ExportDesc { int32_t slot, archetype, column; uint32_t bytes; };
    const ExportDesc *exports(int32_t *num) const;

    // Layout: after registerTypes, allocate the host mirror and create the
    // singleton entities (in registration order, from the init cache).
    void finalizeLayout(uint32_t world_data_bytes, uint32_t world_data_align);
    bool finalized() const;

    StateView &hostView();
    const StateView &hostViewConst() const;

    // Device arena: allocate + copy the host mirror (executor calls this).
    void uploadToDevice(void *stream);
    StateView *deviceView() const;        // device pointer to the StateView
    const StateView &deviceViewHost() const;  // host copy of the device view
    void downloadFromDevice(void *stream);

    // Query resolution: archetypes containing all component keys (Entity key
    // maps to column 0).  Fills (archetype, col...) tuples; returns count.
    int32_t resolveQuery(const uint64_t *keys, int32_t num_keys,
                         int32_t *out_archetypes, int32_t *out_cols, int32_t max_out) const;

    int32_t numWorlds() const;

    void setExtension(const char *name, StateExtension *ext);   // takes ownership
    StateExtension *getExtension(const char *name) const;
    // StateExtension::poll of every extension; true if any asked for a
    // re-capture of the step
    bool pollExtensions(void *stream, int64_t steps);

    struct Impl;
private:
    Impl *impl_;
};

template <typename ComponentT>
void ECSRegistry::registerComponent() { state_mgr_->registerComponent<ComponentT>(); }

template <typename ArchetypeT>
void ECSRegistry::registerArchetype()
{
    state_mgr_->registerArchetype<ArchetypeT>(state_mgr_->capacityHint(typeKey<ArchetypeT>()));
}

template <typename ArchetypeT>
void ECSRegistry::registerFixedSizeArchetype(CountT max_num_entities)
{
    assert(max_num_entities > 0);
    state_mgr_->registerArchetype<ArchetypeT>((int32_t)max_num_entities);
}

template <typename SingletonT>
void ECSRegistry::registerSingleton() { state_mgr_->registerSingleton<SingletonT>(); }

template <typename ArchetypeT, typename ComponentT>
void ECSRegistry::exportColumn(int32_t slot)
{
    state_mgr_->registerExport(slot, typeKey<ArchetypeT>(), typeKey<ComponentT>());
    if (export_ptrs_) export_ptrs_[slot] = nullptr;
}

template <typename SingletonT>
void ECSRegistry::exportSingleton(int32_t slot)
{
    exportColumn<SingletonArchetype<SingletonT>, SingletonT>(slot);
}

}
