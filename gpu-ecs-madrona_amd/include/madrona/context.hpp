// Per-world context (reference include/madrona/context.hpp:17-159,
// context.inl, custom_context.hpp).  One Context type serves both sides:
//   * host, while WorldT constructors build the initial state into the
//     arena's host mirror (IDs are computed exactly as the reference's
//     single-world executor would, SURVEY.md §8c entity-ID rule);
//   * device, inside every kernel, one Context per (world, lane).
// Structural mutation has two modes on the device:
//   * world-serial (one lane owns the world: PerWorldNode, one-off nodes,
//     the host): makeEntityNow / destroyEntityNow / makeTemporary / clear act
//     immediately, exactly as the reference's StateManager does;
//   * row-parallel (ParallelForNode / CustomParallelForNode lanes, where the
//     reference walks the world's rows serially, taskgraph.inl:63-71): a
//     lane's makeTemporary / makeEntityNow appends its row atomically and
//     tags it with an append key (the lane's row, then its call count); a
//     destroyEntityNow is logged with its key.  After the node the executor's
//     ordered commit (csrc/runtime/executor.hip) sorts each world's appended
//     rows and deferred destroys by key and replays them in that order --
//     rows land where the reference's serial walk puts them, swap-removes
//     happen in its order, moved entities are remapped.  Entity IDs made by
//     row-parallel lanes come from the world's ID store in row order
//     (lockedAcquire): deterministic, and the reference's IDs when each row
//     makes at most one entity; clearArchetype is world-serial only.
#pragma once

#include <madrona/state.hpp>

#include <new>
#include <tuple>
#include <utility>

namespace madrona {

struct WorkerInit {
    StateView *state;
    int32_t worldIdx;
    StateManager *mgr;     // host only (query resolution); null on device
};

template <typename T>
class ResultRef {
public:
    MW_INLINE ResultRef(T *ptr) : ptr_(ptr) {}
    MW_INLINE T &value() { return *ptr_; }
    MW_INLINE bool valid() const { return ptr_ != nullptr; }
private:
    T *ptr_;
};

inline constexpr int32_t kMaxQueryArchetypes = 8;
static_assert(kMaxQueryArchetypes == kMakeTurnSlots);
inline constexpr int32_t kMaxQueryComponents = 12;

// A resolved query: matching archetypes and the column of each component.
// Plain data, so a Query built on the host (e.g. stored in world data) is
// valid inside kernels.
template <typename... ComponentTs>
struct Query {
    int32_t numArchetypes = 0;
    int32_t archetypes[kMaxQueryArchetypes];
    int32_t cols[kMaxQueryArchetypes][sizeof...(ComponentTs) > 0 ? sizeof...(ComponentTs) : 1];

    static Query resolve(const StateManager &mgr);
};

// ---------------------------------------------------------------------------
// Job API (reference include/madrona/context.hpp:88-114, job.hpp:29-34,
// query.hpp:60-105).  The reference snapshot's job system is dead code
// (SURVEY.md Q2), but examples/collisions and examples/fantasy_vs are written
// against it.  Here a job runs where it is submitted, on the lane that owns
// the world: submit(fn) calls fn(ctx) and parallelFor(query, fn) walks the
// world's matching rows in query order -- one valid schedule of the
// reference's dependency graph, since every dependency names an earlier
// submission.  A non-child job submitted from inside a job runs after the
// outermost running job returns, except a job re-queueing itself while it
// runs (the examples' `submit(loop, false, currentJobID())`): that is the
// next tick, i.e. the next replay of the step graph.  The loop is hosted by
// a PerWorldNode (csrc/envs/fvs_jobs.hip, collisions_jobs.hip).
// ---------------------------------------------------------------------------
struct JobID {
    uint32_t gen;
    int32_t id;
    static constexpr JobID none() { return JobID { 0, -1 }; }
};

// A non-child job submitted from inside a job runs after the outermost job
// of the lane returns (the reference runs it once its parent finishes); its
// closure is kept by value in the submitting context.
inline constexpr int32_t kMaxDeferredJobs = 4;
inline constexpr int32_t kDeferredJobBytes = 64;
inline constexpr int32_t kMaxJobDepth = 8;

template <typename ComponentT>
class ComponentRef {
public:
    MW_INLINE ComponentRef(ComponentT *col, const int32_t *num_rows) : col_(col), n_(num_rows) {}
    MW_INLINE ComponentT &operator[](uint32_t row) const { return col_[row]; }
    MW_INLINE ComponentT *data() const { return col_; }
    MW_INLINE uint32_t size() const { return (uint32_t)*n_; }
    MW_INLINE ComponentT *begin() const { return col_; }
    MW_INLINE ComponentT *end() const { return col_ + size(); }
private:
    ComponentT *col_;
    const int32_t *n_;      // live row count, as the reference reads tbl_->numRows()
};

template <typename ArchetypeT>
class ArchetypeRef {
public:
    MW_INLINE ArchetypeRef(StateView *st, int32_t world)
        : st_(st), arch_(st->findArchetype(typeKey<ArchetypeT>())), world_(world)
    {}
    template <typename ComponentT>
    MW_INLINE ComponentRef<ComponentT> component() const
    {
        const int32_t col = st_->findColumn(arch_, typeKey<std::remove_const_t<ComponentT>>());
        return ComponentRef<ComponentT>(
            st_->column<std::remove_const_t<ComponentT>>(arch_, col, world_),
            st_->arch[arch_].numRows + world_);
    }
    template <typename ComponentT>
    MW_INLINE ComponentT &get(uint32_t idx) const { return component<ComponentT>()[idx]; }
    MW_INLINE uint32_t size() const { return (uint32_t)st_->arch[arch_].numRows[world_]; }
private:
    StateView *st_;
    int32_t arch_;
    int32_t world_;
};

namespace detail {
// The context type a job function takes first (Engine &ctx, ...).
template <typename F>
struct JobFnTraits : JobFnTraits<decltype(&std::remove_reference_t<F>::operator())> {};
template <typename C, typename R, typename A0, typename... A>
struct JobFnTraits<R (C::*)(A0, A...) const> {
    using Ctx = std::remove_cv_t<std::remove_reference_t<A0>>;
};
template <typename C, typename R, typename A0, typename... A>
struct JobFnTraits<R (C::*)(A0, A...)> {
    using Ctx = std::remove_cv_t<std::remove_reference_t<A0>>;
};
}

class Context {
public:
    MW_INLINE Context(WorldBase *world_data, const WorkerInit &init)
        : data_(world_data), state_(init.state), world_(init.worldIdx), mgr_(init.mgr)
    {}

    // Row-parallel mode (set by the row-parallel node kernels): the lane's
    // position in the reference's serial walk, (query archetype << 24) | row,
    // the archetype the lane's row lives in and the exact type keys of the
    // query components the node's function takes by non-const reference
    // (rowWriteKeys): get / getUnsafe of one of those components at another
    // row reads or writes a row another lane of the launch is writing -- an
    // access the serial walk would order and the row-parallel launch does
    // not -- so it raises kErrFlagCrossRow.  Components the node only reads
    // are not flagged (no lane writes them through the query).
    MW_INLINE void setRowParallel(uint32_t row_key, int32_t own_arch, const RowWriteKeys &keys)
    {
        rowKey_ = row_key;
        seq_ = 0;
        ownArch_ = own_arch;
        writeKeys_ = keys;
    }
    MW_INLINE void setRowParallel(uint32_t row_key)
    {
        rowKey_ = row_key;
        seq_ = 0;
        ownArch_ = -1;
        writeKeys_.n = 0;
    }
    // The lane's wave index among the waves covering this world's rows, the
    // world's finished-wave marks (StateView::makeTurn) and the node's epoch.
    MW_INLINE void setMakeTurn(int32_t *marks, int32_t chunk, int32_t epoch)
    {
        turn_ = marks;
        turnChunk_ = chunk;
        turnEpoch_ = epoch;
    }
    MW_INLINE bool madeEntities() const { return made_; }
    MW_INLINE bool rowParallel() const { return rowKey_ != kSerialRowKey; }

    template <typename ArchetypeT, typename... Args>
    MW_INLINE Entity makeEntityNow(Args &&...args);
    MW_INLINE void destroyEntityNow(Entity e);
    template <typename ArchetypeT>
    MW_INLINE Loc makeTemporary();

    MW_INLINE Loc getLoc(Entity e) const { return state_->ids(world_).lookup(e); }

    template <typename ComponentT> MW_INLINE ResultRef<ComponentT> get(Entity e);
    template <typename ComponentT> MW_INLINE ResultRef<ComponentT> get(Loc l);
    template <typename ComponentT> MW_INLINE ComponentT &getUnsafe(Entity e) { return getUnsafe<ComponentT>(e.id); }
    template <typename ComponentT> MW_INLINE ComponentT &getUnsafe(int32_t e_id);
    template <typename ComponentT> MW_INLINE ComponentT &getUnsafe(Loc l);
    template <typename ComponentT>
    MW_INLINE ComponentT &getDirect(int32_t column_idx, Loc loc)
    {
        return rowRef(state_->column<ComponentT>(loc.archetype, column_idx, world_), loc.row);
    }
    template <typename SingletonT> MW_INLINE SingletonT &getSingleton();

    template <typename ArchetypeT> MW_INLINE void clearArchetype() { clear(state_->findArchetype(typeKey<ArchetypeT>()), false); }
    template <typename ArchetypeT> MW_INLINE void clearTemporaries() { clear(state_->findArchetype(typeKey<ArchetypeT>()), true); }

    template <typename... ComponentTs> Query<ComponentTs...> query();
    template <typename... ComponentTs, typename Fn>
    MW_INLINE void forEach(const Query<ComponentTs...> &q, Fn &&fn);
    template <typename Fn, size_t... Is, typename... Ts>
    MW_INLINE void forEachRows(int32_t arch, const int32_t *cols, int32_t n, Fn &fn,
                               std::index_sequence<Is...>, Ts *...);
    template <typename... ComponentTs>
    MW_INLINE uint32_t numMatches(const Query<ComponentTs...> &q);

    template <typename ArchetypeT> MW_INLINE int32_t numRows()
    {
        return state_->arch[state_->findArchetype(typeKey<ArchetypeT>())].numRows[world_];
    }

    // Job API (see above).
    template <typename ArchetypeT>
    MW_INLINE ArchetypeRef<ArchetypeT> archetype() { return ArchetypeRef<ArchetypeT>(state_, world_); }
    template <typename Fn, typename... DepTs>
    MW_INLINE JobID submit(Fn &&fn, bool is_child = true, DepTs &&...dependencies);
    template <typename... ComponentTs, typename Fn, typename... DepTs>
    MW_INLINE JobID parallelFor(const Query<ComponentTs...> &query, Fn &&fn, bool is_child = true,
                                DepTs &&...dependencies);
    MW_INLINE JobID currentJobID() const { return jobDepth_ > 0 ? JobID { 0, jobDepth_ } : JobID::none(); }

    MW_INLINE void *tmpAlloc(uint64_t num_bytes);
    MW_INLINE void resetTmpAlloc();

    MW_INLINE WorldID worldID() const { return WorldID { world_ }; }
    MW_INLINE WorldBase &data() { return rowRef(data_, 0); }
    MW_INLINE StateView &state() { return *state_; }

    // registration forwarding used by some reference examples' ctors
    template <typename ComponentT> void registerComponent() {}
    template <typename ArchetypeT> void registerArchetype() {}

protected:
    MW_INLINE void clear(int32_t archetype, bool is_temporary);
    MW_INLINE uint64_t nextAppendKey() { return ((uint64_t)rowKey_ << 32) | ((uint64_t)(seq_++ & 0xFFFFu) << 16); }
    MW_INLINE Entity lockedAcquire(int32_t arch, int32_t row);
    MW_INLINE void raiseFlag(int32_t bit);
    template <typename ComponentT> MW_INLINE void checkCrossRow(Loc loc);
    template <typename Fn> MW_INLINE void runJob(Fn &fn);
    MW_INLINE void drainDeferredJobs();
    MW_INLINE bool jobRunning(uint64_t key) const
    {
        for (int32_t i = 0; i < jobDepth_ && i < kMaxJobDepth; i++) {
            if (jobKeys_[i] == key) return true;
        }
        return false;
    }

    WorldBase *data_;
    StateView *state_;
    int32_t world_;
    StateManager *mgr_;
    uint32_t rowKey_ = kSerialRowKey;
    uint32_t seq_ = 0;
    int32_t ownArch_ = -1;
    RowWriteKeys writeKeys_ {};
    int32_t *turn_ = nullptr;
    int32_t turnChunk_ = 0;
    int32_t turnEpoch_ = 0;
    bool made_ = false;
    int32_t jobDepth_ = 0;      // nesting of the job being run (0: none)
    // Job API bookkeeping (only touched by job-API worlds).
    uint64_t jobKeys_[kMaxJobDepth];
    int32_t numDeferredJobs_ = 0;
    struct DeferredJob {
        void (*run)(Context &, void *);
        alignas(16) char bytes[kDeferredJobBytes];
    } deferredJobs_[kMaxDeferredJobs];
};

template <typename ContextT, typename DataT>
class CustomContext : public Context {
public:
    MW_INLINE CustomContext(DataT *world_data, const WorkerInit &init)
        : Context(world_data, init)
    {}
    MW_INLINE DataT &data() const { return rowRef(static_cast<DataT *>(data_), 0); }

    using WorldDataT = DataT;
};

// ---------------------------------------------------------------------------
// Row-parallel makeEntityNow: the world's ID store is serial
// (id_map_impl.inl:69-182), so lanes take it one at a time, in row order:
// the lanes of a wave in lane order, and a wave only once every lower wave
// covering the world's rows has finished (StateView::makeTurn: each wave
// marks itself done with the node's epoch -- a count would also count higher
// waves that finished first).  The IDs are therefore the same run to run,
// and the reference's when every row makes at most one entity and the node
// walks one row per invocation (its serial walk hands them out in row
// order).  With items_per_invocation = k > 1 a wave's lanes take IDs in
// lockstep per item -- rows 0, k, 2k, ... first, then 1, k + 1, ... -- so
// the IDs are deterministic but not in row order; the rows themselves still
// land in the reference's order (the ordered commit sorts the append keys).
// Lower waves are dispatched before
// higher ones and never wait on them, so the wait always ends.  Without the
// marks (other callers, worlds past kMakeTurnWaves waves) waves go through
// the per-world lock alone.  The ordered path takes the same lock after its
// turn: a world whose walked table spans more than kMakeTurnWaves waves
// mixes ordered and unordered waves, and a turn wait that timed out must
// still not race another wave inside the ID store.
MW_INLINE bool lowerWavesDone(const int32_t *marks, int32_t chunk, int32_t epoch)
{
#if defined(__HIP_DEVICE_COMPILE__)
    for (int32_t i = 0; i < chunk; i++) {
        if (__hip_atomic_load(marks + i, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != epoch) return false;
    }
    return true;
#else
    (void)marks; (void)chunk; (void)epoch;
    return true;
#endif
}

MW_INLINE Entity Context::lockedAcquire(int32_t arch, int32_t row)
{
    IDMapView ids = state_->ids(world_);
#if defined(__HIP_DEVICE_COMPILE__)
    Entity e = Entity::none();
    const uint32_t lane = __lane_id();
    uint64_t pending = __ballot(1);
    while (pending) {
        const uint32_t leader = (uint32_t)__builtin_ctzll(pending);
        if (lane == leader) {
            if (turn_) {
                // bounded: a wait that never ends is flagged and the ID taken
                uint32_t spins = 0;
                while (!lowerWavesDone(turn_, turnChunk_, turnEpoch_)) {
                    __builtin_amdgcn_s_sleep(2);
                    if (++spins == (1u << 20)) {
                        atomicOr(state_->errorFlags + world_, kErrFlagMakeOrder);
                        break;
                    }
                }
                made_ = true;
            }
            while (atomicCAS(&ids.st->lock, 0, 1) != 0) __builtin_amdgcn_s_sleep(2);
            __threadfence();
            e = ids.acquire(ids.st->worldCache);
            if (e.id >= 0) ids.nodes[e.id].val = Loc { (uint32_t)arch, row };
            __threadfence();
            atomicExch(&ids.st->lock, 0);
        }
        pending &= pending - 1;
    }
    return e;
#else
    Entity e = ids.acquire(ids.st->worldCache);
    if (e.id >= 0) ids.nodes[e.id].val = Loc { (uint32_t)arch, row };
    return e;
#endif
}

template <typename ArchetypeT, typename... Args>
MW_INLINE Entity Context::makeEntityNow(Args &&...args)
{                                              // state.inl:398-449
    int32_t arch = state_->findArchetype(typeKey<ArchetypeT>());
    auto construct_row = [&](int32_t row) {
        int32_t col = 1;
        auto construct = [&](auto &&arg) {
            using T = std::remove_cv_t<std::remove_reference_t<decltype(arg)>>;
            new (&rowRef(state_->column<T>(arch, col, world_), row)) T(std::forward<decltype(arg)>(arg));
            col++;
        };
        (construct(std::forward<Args>(args)), ...);
    };
    if (rowParallel()) {
        const int32_t row = state_->appendRowParallel(arch, world_, nextAppendKey());
        if (row < 0) return Entity::none();
        Entity e = lockedAcquire(arch, row);
        // a row whose ID could not be acquired keeps Entity::none(); the
        // commit drops it
        rowRef(state_->column<Entity>(arch, 0, world_), row) = e;
        if (e.id >= 0) construct_row(row);
        return e;
    }
    IDMapView ids = state_->ids(world_);
    Entity e = ids.acquire(ids.st->worldCache);
    int32_t row = state_->addRow(arch, world_);
    if (row < 0 || e.id < 0) return Entity::none();
    rowRef(state_->column<Entity>(arch, 0, world_), row) = e;
    construct_row(row);
    ids.nodes[e.id].val = Loc { (uint32_t)arch, row };
    return e;
}

MW_INLINE void Context::destroyEntityNow(Entity e)
{                                              // src/core/state.cpp:181-202
    if (rowParallel()) {
#if defined(__HIP_DEVICE_COMPILE__)
        const int32_t i = atomicAdd(state_->deferCount + world_, 1);
        if (i >= state_->deferCap) {
            atomicOr(state_->errorFlags + world_, kErrFlagDeferredFull);
            return;
        }
        state_->deferLog[(size_t)world_ * state_->deferCap + i] = DeferredDestroy { nextAppendKey(), e };
        return;
#endif
    }
    IDMapView ids = state_->ids(world_);
    Loc loc = ids.lookup(e);
    if (!loc.valid()) return;
    bool moved = state_->removeRow(loc.archetype, world_, loc.row);
    if (moved) {
        Entity m = rowRef(state_->column<Entity>(loc.archetype, 0, world_), loc.row);
        ids.nodes[m.id].val.row = loc.row;
    }
    ids.release(ids.st->worldCache, e.id);
}

template <typename ArchetypeT>
MW_INLINE Loc Context::makeTemporary()
{                                              // state.inl:451-463
    int32_t arch = state_->findArchetype(typeKey<ArchetypeT>());
    int32_t row = rowParallel() ? state_->appendRowParallel(arch, world_, nextAppendKey())
                                : state_->addRow(arch, world_);
    if (row < 0) return Loc::none();
    return Loc { (uint32_t)arch, row };
}

// A world's error bit; row-parallel lanes of one world set bits concurrently.
MW_INLINE void Context::raiseFlag(int32_t bit)
{
#if defined(__HIP_DEVICE_COMPILE__)
    atomicOr(state_->errorFlags + world_, bit);
#else
    state_->errorFlags[world_] |= bit;
#endif
}

MW_INLINE void Context::clear(int32_t arch, bool is_temporary)
{                                              // src/core/state.cpp:565-581
    if (rowParallel()) {
        // a clear inside a row walk has no per-row order to keep: use a
        // ClearTmpNode or a world-serial node
        raiseFlag(kErrFlagRowParallelOp);
        return;
    }
    if (!is_temporary) {
        IDMapView ids = state_->ids(world_);
        ids.bulkRelease(ids.st->worldCache, state_->column<Entity>(arch, 0, world_),
                        state_->arch[arch].numRows[world_]);
    }
    state_->arch[arch].numRows[world_] = 0;
}

// Per-world bump allocator (reference TmpAllocator::alloc,
// src/core/state.cpp:95-114: 256-byte granules); row-parallel lanes bump
// the world's offset atomically.  Past the world's arena an allocation is
// chained (the reference allocates another block): from the device pool
// shared by all worlds, or a host heap block; only when that is exhausted
// (or off) does tmpAlloc return null and raise kErrFlagTmpAllocFull.
MW_INLINE void *Context::tmpAlloc(uint64_t num_bytes)
{
    const uint64_t bytes = (num_bytes + 255) & ~uint64_t(255);
    if (bytes == 0) return nullptr;
    if (state_->tmpArena && bytes <= state_->tmpBytesPerWorld) {
        uint32_t off;
#if defined(__HIP_DEVICE_COMPILE__)
        if (rowParallel()) {
            off = atomicAdd(state_->tmpOffset + world_, (uint32_t)bytes);
        } else
#endif
        {
            off = state_->tmpOffset[world_];
            if ((uint64_t)off + bytes <= state_->tmpBytesPerWorld) state_->tmpOffset[world_] = off + (uint32_t)bytes;
        }
        if ((uint64_t)off + bytes <= state_->tmpBytesPerWorld) {
            return state_->tmpArena + (size_t)world_ * state_->tmpBytesPerWorld + off;
        }
    }
#if defined(__HIP_DEVICE_COMPILE__)
    if (state_->tmpPool) {
        const unsigned long long off = atomicAdd(state_->tmpPoolOffset, (unsigned long long)bytes);
        if (off + bytes <= state_->tmpPoolBytes) return state_->tmpPool + off;
    }
#else
    if (void *p = hostTmpOverflowAlloc(*state_, world_, bytes)) return p;
#endif
    raiseFlag(kErrFlagTmpAllocFull);
    return nullptr;
}

// The world's arena (device: its pool blocks are reclaimed at the next
// ResetTmpAllocNode, which resets every world at once).
MW_INLINE void Context::resetTmpAlloc()
{                                              // src/core/state.cpp:116-127
    if (state_->tmpOffset) state_->tmpOffset[world_] = 0;
#if !defined(__HIP_DEVICE_COMPILE__)
    hostTmpOverflowReset(*state_, world_);
#endif
}

namespace detail {
// Parameter list of a node function (a plain function pointer
// `void (*)(Ctx &, Cs &...)`); other callables are not introspected.
template <typename F> struct NodeFnSig { static constexpr bool known = false; };
template <typename R, typename C, typename... Ps>
struct NodeFnSig<R (*)(C, Ps...)> {
    static constexpr bool known = true;
    template <size_t I> using Param = std::tuple_element_t<I, std::tuple<Ps...>>;
};
template <typename T> inline constexpr bool kMutRef = false;
template <typename T> inline constexpr bool kMutRef<T &> = !std::is_const_v<T>;

template <auto Fn, size_t I, typename ComponentT>
constexpr bool nodeWrites()
{
    using Sig = NodeFnSig<decltype(Fn)>;
    if constexpr (std::is_same_v<std::remove_cv_t<ComponentT>, Entity> ||
                  std::is_const_v<ComponentT>) {
        return false;
    } else if constexpr (Sig::known) {
        return kMutRef<typename Sig::template Param<I>>;
    } else {
        return true;     // unknown signature: every non-const query component
    }
}
}

// The exact type keys of the query components a row node's function may
// write (non-const reference parameters), for Context::checkCrossRow.
template <auto Fn, typename... ComponentTs, size_t... Is>
constexpr RowWriteKeys rowWriteKeysImpl(std::index_sequence<Is...>)
{
    RowWriteKeys r {};
    ((detail::nodeWrites<Fn, Is, ComponentTs>()
          ? (r.n < kMaxRowWriteKeys ? (void)(r.key[r.n++] = typeKey<ComponentTs>()) : (void)(r.all = true))
          : (void)0),
     ...);
    return r;
}

template <auto Fn, typename... ComponentTs>
constexpr RowWriteKeys rowWriteKeys()
{
    return rowWriteKeysImpl<Fn, ComponentTs...>(std::index_sequence_for<ComponentTs...> {});
}

template <typename ComponentT>
MW_INLINE void Context::checkCrossRow(Loc loc)
{
#if defined(__HIP_DEVICE_COMPILE__)
    // Another lane of the same launch owns that row and may be writing it
    // (the reference walks the world's rows serially, taskgraph.inl:63-71):
    // flag it so an unported world fails loudly instead of racing.
    if (writeKeys_.has(typeKey<ComponentT>()) && rowParallel() &&
        ((int32_t)loc.archetype != ownArch_ || loc.row != (int32_t)(rowKey_ & 0xFFFFFFu))) {
        raiseFlag(kErrFlagCrossRow);
    }
#else
    (void)loc;
#endif
}

template <typename ComponentT>
MW_INLINE ResultRef<ComponentT> Context::get(Loc loc)
{
    checkCrossRow<ComponentT>(loc);
    int32_t col = state_->findColumn(loc.archetype, typeKey<ComponentT>());
    if (col < 0) return ResultRef<ComponentT>(nullptr);
    return ResultRef<ComponentT>(&rowRef(state_->column<ComponentT>(loc.archetype, col, world_), loc.row));
}

template <typename ComponentT>
MW_INLINE ResultRef<ComponentT> Context::get(Entity e)
{
    Loc loc = getLoc(e);
    if (!loc.valid()) return ResultRef<ComponentT>(nullptr);
    return get<ComponentT>(loc);
}

template <typename ComponentT>
MW_INLINE ComponentT &Context::getUnsafe(int32_t e_id)
{
    Loc loc = state_->ids(world_).nodes[e_id].val;
    return getUnsafe<ComponentT>(loc);
}

template <typename ComponentT>
MW_INLINE ComponentT &Context::getUnsafe(Loc loc)
{
    checkCrossRow<ComponentT>(loc);
    int32_t col = state_->findColumn(loc.archetype, typeKey<ComponentT>());
    return rowRef(state_->column<ComponentT>(loc.archetype, col, world_), loc.row);
}

template <typename SingletonT>
MW_INLINE SingletonT &Context::getSingleton()
{
    int32_t arch = state_->findArchetype(typeKey<SingletonArchetype<SingletonT>>());
    return rowRef(state_->column<SingletonT>(arch, 1, world_), 0);
}

template <typename... ComponentTs, typename Fn>
MW_INLINE void Context::forEach(const Query<ComponentTs...> &q, Fn &&fn)
{                                              // state.inl:358-396
    for (int32_t a = 0; a < q.numArchetypes; a++) {
        const int32_t arch = q.archetypes[a];
        const int32_t n = state_->arch[arch].numRows[world_];
        forEachRows(arch, q.cols[a], n, fn, std::index_sequence_for<ComponentTs...> {},
                    (std::remove_const_t<ComponentTs> *)nullptr...);
    }
}

template <typename Fn, size_t... Is, typename... Ts>
MW_INLINE void Context::forEachRows(int32_t arch, const int32_t *cols, int32_t n, Fn &fn,
                                    std::index_sequence<Is...>, Ts *...)
{
    // column i of the query is cols[i] (the pack is expanded by index, so the
    // column binding does not depend on argument evaluation order)
    auto ptrs = std::make_tuple(state_->column<Ts>(arch, cols[Is], world_)...);
    // unrolled so a device lane keeps several rows' loads in flight
#pragma unroll 4
    for (int32_t r = 0; r < n; r++) {
        fn(rowRef(std::get<Is>(ptrs), r)...);
    }
}

template <typename Fn>
MW_INLINE void Context::runJob(Fn &fn)
{
    using CtxT = typename detail::JobFnTraits<Fn>::Ctx;
    if (jobDepth_ < kMaxJobDepth) jobKeys_[jobDepth_] = typeKey<Fn>();
    jobDepth_++;
    fn(static_cast<CtxT &>(*this));
    jobDepth_--;
    if (jobDepth_ == 0) drainDeferredJobs();
}

MW_INLINE void Context::drainDeferredJobs()
{
    // FIFO; a drained job may defer more (it runs at depth 0, so those run
    // when it returns)
    for (int32_t i = 0; i < numDeferredJobs_; i++) {
        DeferredJob job = deferredJobs_[i];
        deferredJobs_[i].run = nullptr;
        job.run(*this, job.bytes);
    }
    numDeferredJobs_ = 0;
}

template <typename Fn, typename... DepTs>
MW_INLINE JobID Context::submit(Fn &&fn, bool is_child, DepTs &&...)
{
    using FnT = std::remove_cv_t<std::remove_reference_t<Fn>>;
    if (!is_child && jobDepth_ > 0) {
        // The examples' loop re-queues itself behind the running job
        // (`submit(loop, false, currentJobID())`): that is the next tick,
        // i.e. the next replay of the step graph.
        if (jobRunning(typeKey<FnT>())) return JobID::none();
        // Any other non-child job runs after the outermost job returns.
        if constexpr (sizeof(FnT) <= kDeferredJobBytes && alignof(FnT) <= 16 &&
                      std::is_trivially_copyable_v<FnT>) {
            if (numDeferredJobs_ < kMaxDeferredJobs) {
                DeferredJob &d = deferredJobs_[numDeferredJobs_++];
                memcpy(d.bytes, &fn, sizeof(FnT));
                d.run = [](Context &c, void *bytes) {
                    alignas(FnT) char copy[sizeof(FnT)];
                    memcpy(copy, bytes, sizeof(FnT));
                    c.runJob(*reinterpret_cast<FnT *>(copy));
                };
                return JobID { 0, jobDepth_ + 1 };
            }
        }
        raiseFlag(kErrFlagJobDropped);
        return JobID::none();
    }
    runJob(fn);
    return JobID { 0, jobDepth_ + 1 };
}

template <typename... ComponentTs, typename Fn, typename... DepTs>
MW_INLINE JobID Context::parallelFor(const Query<ComponentTs...> &q, Fn &&fn, bool, DepTs &&...)
{                                              // context.inl:172-289 (#if 0 in the snapshot)
    using CtxT = typename detail::JobFnTraits<Fn>::Ctx;
    if (jobDepth_ < kMaxJobDepth) jobKeys_[jobDepth_] = 0;
    jobDepth_++;
    CtxT &ctx = static_cast<CtxT &>(*this);
    for (int32_t a = 0; a < q.numArchetypes; a++) {
        const int32_t arch = q.archetypes[a];
        const int32_t n = state_->arch[arch].numRows[world_];   // rows at launch
        [&]<size_t... Is>(std::index_sequence<Is...>) {
            auto cols = std::make_tuple(
                state_->column<std::remove_const_t<ComponentTs>>(arch, q.cols[a][Is], world_)...);
            for (int32_t r = 0; r < n; r++) fn(ctx, rowRef(std::get<Is>(cols), r)...);
        }(std::index_sequence_for<ComponentTs...> {});
    }
    jobDepth_--;
    if (jobDepth_ == 0) drainDeferredJobs();
    return JobID { 0, jobDepth_ + 1 };
}

template <typename... ComponentTs>
MW_INLINE uint32_t Context::numMatches(const Query<ComponentTs...> &q)
{
    uint32_t n = 0;
    for (int32_t a = 0; a < q.numArchetypes; a++) n += state_->arch[q.archetypes[a]].numRows[world_];
    return n;
}

template <typename... ComponentTs>
Query<ComponentTs...> Query<ComponentTs...>::resolve(const StateManager &mgr)
{
    Query<ComponentTs...> q;
    constexpr int32_t nc = sizeof...(ComponentTs);
    uint64_t keys[nc > 0 ? nc : 1] = { typeKey<std::remove_const_t<ComponentTs>>()... };
    int32_t archs[kMaxQueryArchetypes];
    int32_t cols[kMaxQueryArchetypes * kMaxQueryComponents];
    q.numArchetypes = mgr.resolveQuery(keys, nc, archs, cols, kMaxQueryArchetypes);
    for (int32_t a = 0; a < q.numArchetypes; a++) {
        q.archetypes[a] = archs[a];
        for (int32_t c = 0; c < nc; c++) q.cols[a][c] = cols[a * kMaxQueryComponents + c];
    }
    return q;
}

template <typename... ComponentTs>
Query<ComponentTs...> Context::query()
{
    return Query<ComponentTs...>::resolve(*mgr_);
}

}
