// TaskGraph for the MI355X framework.
//
// Reference interface: include/madrona/taskgraph.hpp:8-138, taskgraph.inl,
// src/core/taskgraph.cpp:18-122 (Builder::registerNode / build / run).
//
// MI355X design: the graph is built ONCE on the host (all worlds share it, as
// they do in the reference), topologically sorted with the reference's rule
// (registration order, a node waits for earlier dependencies), and every node
// becomes one or more kernel launches that process ALL worlds at once.  The
// whole sorted launch sequence is captured into a hipGraph and replayed per
// step, so a step makes no host round trip.  Node order is preserved per
// world, which is all the reference's per-world serial walk guarantees.
#pragma once

#include <madrona/context.hpp>
#include <madrona/commit.hpp>
#include <madrona/optional.hpp>
#include <madrona/tracing.hpp>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#endif

#include <cstring>
#include <functional>
#include <initializer_list>
#include <memory>
#include <stdexcept>
#include <tuple>
#include <type_traits>
#include <vector>

namespace madrona {

template <typename T>
class Span {
public:
    Span() : ptr_(nullptr), n_(0) {}
    Span(const T *ptr, CountT n) : ptr_(ptr), n_(n) {}
    Span(std::initializer_list<std::remove_const_t<T>> il) : ptr_(il.begin()), n_((CountT)il.size()) {}
    const T *data() const { return ptr_; }
    CountT size() const { return n_; }
    const T *begin() const { return ptr_; }
    const T *end() const { return ptr_ + n_; }
    const T &operator[](CountT i) const { return ptr_[i]; }
private:
    const T *ptr_;
    CountT n_;
};

class Executor;

// ---------------------------------------------------------------------------
// World walk: the persistent megakernel of the reference
// (src/mw/device/megakernel_impl.inl:29-55: each block walks the task graph,
// dispatch(funcID) per node).  A run of consecutive world-local nodes -- row
// nodes over small tables with their ordered commits, world-serial row nodes,
// per-world nodes, fixed-count device nodes -- becomes ONE launch: a wave
// takes a world and calls every node's world function for it in graph order
// (device function pointers: the node kinds of a world are known only when
// setupTasks runs, as the reference's are only known to its NVRTC build).
// Worlds are independent, so the result is that of the per-node launches;
// the launch floors and inter-kernel drains between the nodes go away.
// ---------------------------------------------------------------------------
namespace detail {
inline constexpr int32_t kWalkParamBytes = 240;
inline constexpr int32_t kMaxWalkEntriesPerNode = 2;
struct WalkEntry;
// What a world function gets besides its entry: the device state.
struct WalkCtx {
    StateView *st;
};
using WalkFn = void (*)(const WalkEntry &, const WalkCtx &, int32_t);
// kind: a node's world function, or the ordered-commit point after a
// row-parallel node.
inline constexpr int32_t kWalkCall = 0;
inline constexpr int32_t kWalkCommit = 1;
struct alignas(16) WalkEntry {
    WalkFn fn;                     // device address (same code object as the walk kernels)
    int32_t kind;
    int32_t pad;
    char params[kWalkParamBytes];  // the node's launch arguments
};
static_assert(sizeof(WalkEntry) == 256);
}

// Everything a node's launch function needs.  Captured into a hipGraph, so a
// launch must be a pure function of its node data and this struct.
struct LaunchCtx {
    void *stream;                // hipStream_t
    StateView *devState;         // device pointer
    const StateView *view;       // host copy of the device view
    int32_t numWorlds;
    Executor *exec;
    // Per-node launch configuration (reference MegakernelConfig,
    // src/mw/cuda_exec.cpp:216-222, 1460-1517): blocks per CU for the node's
    // grid-stride / persistent kernels, 0 = the node's own full grid; numCUs
    // = the CUs the grid is sized for.  Set by the executor for each node.
    int32_t blocksPerCU = 0;
    int32_t numCUs = 0;
    // Device copies of the graph's node data blocks (TaskGraph::NodeData,
    // constructNodeData), uploaded once when the graph is set.
    char *nodeData = nullptr;
    // Executor-wide world-serial mode (ExecConfig::serialNodes): every
    // ParallelForNode / CustomParallelForNode walks each world's rows in
    // order on one invocation, as the reference's ParallelForNode::run does.
    int32_t serialNodes = 0;
    // Row nodes whose tables need at most this many lanes per world run one
    // wave per world (parallelForWorldKernel); env
    // MADRONA_MW_WORLD_WAVE_LANES overrides the default (0: never).
    int32_t worldWaveLanes = 256;
    // Row nodes over several small tables launch once for all of them
    // (parallelForWorldMultiKernel); env MADRONA_MW_FUSE_ARCHETYPES=0: one
    // launch per archetype.
    int32_t fuseArchetypes = 1;
    // A second stream of the executor for a node's independent kernels
    // (fork: record forkEvent on `stream`, the side stream waits on it; join:
    // record joinEvent on the side stream, `stream` waits on it).  Inside the
    // step graph's capture this makes parallel branches.  Null (the default;
    // env MADRONA_MW_SIDE_STREAM=1 sets it): every kernel runs on `stream`.
    void *sideStream = nullptr;     // hipStream_t
    void *forkEvent = nullptr;      // hipEvent_t
    void *joinEvent = nullptr;      // hipEvent_t

    // Grid for a grid-stride kernel that needs `blocks` blocks to cover its
    // work in one pass: capped at numCUs x blocksPerCU when configured.
    // The product is formed in 64 bits and is at least one block (the
    // parsers bound blocksPerCU and numCUs, launch_config.hpp).
    uint32_t capGrid(uint32_t blocks) const
    {
        if (blocksPerCU <= 0 || numCUs <= 0) return blocks;
        const uint64_t cap = (uint64_t)numCUs * (uint64_t)blocksPerCU;
        return (uint64_t)blocks < cap ? blocks : (uint32_t)(cap < 0x7fffffffu ? cap : 0x7fffffffu);
    }
    // Grid for a persistent kernel whose default grid is `resident` blocks.
    uint32_t persistentGrid(uint32_t resident) const
    {
        if (blocksPerCU <= 0 || numCUs <= 0) return resident > 0 ? resident : 1;
        const uint64_t g = (uint64_t)numCUs * (uint64_t)blocksPerCU;
        return (uint32_t)(g < 0x7fffffffu ? g : 0x7fffffffu);
    }
};

// The CPU back end (libmadrona_cpu.so, csrc/runtime/cpu_executor.cpp; the
// reference's TaskGraphExecutor, include/madrona/mw_cpu.hpp:53-81) runs the
// same graph on host threads.  A world-local node runs for one world at a
// time (runWorld), so a run of consecutive world-local nodes executes world
// by world on a pinned worker, like the reference's per-world TaskGraph::run
// (src/core/taskgraph.cpp:111-122); a global node (runGlobal: node data
// shared by every world, e.g. addDynamicCountNode) runs once, between them.
class CpuThreadPool;
struct CpuRunCtx {
    StateView *state;            // host arena
    StateManager *mgr;
    int32_t numWorlds;
    char *nodeData;              // host copies of the graph's node data blocks
    CpuThreadPool *pool;
};
using CpuWorldFn = void (*)(void *node, CpuRunCtx &rc, int32_t world);
using CpuGlobalFn = void (*)(void *node, CpuRunCtx &rc);

// Parallel loop over [0, n) on the CPU back end's pinned workers (the
// caller's thread joins in); fn(begin, end) gets contiguous chunks.
void cpuParallelFor(CpuRunCtx &rc, int64_t n, void (*fn)(void *arg, int64_t begin, int64_t end),
                    void *arg);

// Base of every node's data (reference device NodeBase,
// src/mw/device/include/madrona/taskgraph.hpp:23-25).  For nodes whose run()
// executes on the device (addNodeFn / addOneOffNode / addDynamicCountNode)
// the executor fills in the device state before uploading the node data, so
// run() can build a world's context: makeContext<ContextT>(WorldID), the
// analogue of the reference's static TaskGraph::makeContext.
struct NodeBase {
    uint32_t numDynamicInvocations = 0;
    int32_t mwNumWorlds = 0;
    StateView *mwState = nullptr;

#if defined(__HIPCC__)
    template <typename ContextT>
    __device__ inline ContextT makeContext(WorldID world) const;
#else
    template <typename ContextT>
    inline ContextT makeContext(WorldID world) const;
#endif
};

class TaskGraph {
public:
    struct NodeID {
        uint32_t id;
    };
    struct DataID {
        int32_t id;
    };
    template <typename NodeT>
    struct TypedDataID : DataID {};

    // Node data: at most 128 bytes, trivially copyable (the reference
    // memcpy's it into the built graph, src/core/taskgraph.cpp:104-106).
    static inline constexpr uint32_t maxNodeDataBytes = 128;
    struct alignas(maxNodeDataBytes) NodeData {
        char userData[maxNodeDataBytes];
    };

    using LaunchFn = void (*)(void *node, LaunchCtx &lc);

    // How a node runs: kernels (LaunchFn, hipcc builds) and / or on host
    // threads (CPU back end, g++ builds) -- per world or once per step.
    // walk: the node's world-walk entries (at most kMaxWalkEntriesPerNode)
    // and the walk / resume kernels of its code object (kernels[0], [1]), or
    // 0 when the node cannot run inside a walk in this configuration (called
    // before capture).
    using WalkPlanFn = int32_t (*)(void *node, LaunchCtx &lc, detail::WalkEntry *out,
                                   const void **kernels);
    struct NodeFns {
        LaunchFn launch = nullptr;
        CpuWorldFn cpuWorld = nullptr;
        CpuGlobalFn cpuGlobal = nullptr;
        WalkPlanFn walk = nullptr;
    };

    // Node flags: a framework node whose kernels never call Context::tmpAlloc
    // (static constexpr bool kNoTmpAlloc), and ResetTmpAllocNode itself.  A
    // reset with no possibly-allocating node since the previous one is a
    // no-op and is not launched (the physics substeps reset twice each).
    static constexpr uint32_t kNodeNoTmpAlloc = 1;
    static constexpr uint32_t kNodeTmpAllocReset = 2;

    class Builder {
    public:
        explicit Builder(Context &ctx);

        // Node data constructed in place in the graph (reference
        // taskgraph.inl:5-19); shared by every node that names it.
        template <typename NodeT, typename... Args>
        TypedDataID<NodeT> constructNodeData(Args &&...args)
        {
            static_assert(sizeof(NodeT) <= maxNodeDataBytes);
            static_assert(alignof(NodeT) <= maxNodeDataBytes);
            static_assert(std::is_trivially_copyable_v<NodeT>,
                          "node data is copied to the device: it must be trivially copyable");
            datas_.emplace_back();
            new (datas_.back().userData) NodeT(std::forward<Args>(args)...);
            dataIsNodeBase_.push_back(std::is_base_of_v<NodeBase, NodeT>);
            return TypedDataID<NodeT> { DataID { (int32_t)datas_.size() - 1 } };
        }

        template <typename NodeT>
        NodeT &getDataRef(TypedDataID<NodeT> data_id)
        {
            return *(NodeT *)datas_[data_id.id].userData;
        }

        // A node that runs `fn(NodeT *, int32_t invocation_idx)` on the
        // device (reference device taskgraph.inl:41-59).  fixed_num_invocations
        // > 0: that many invocations per world, invocation_idx = world *
        // count + k (count 1: invocation_idx is the world, as every node of
        // the reference snapshot is invoked, megakernel_impl.inl:29-40).
        // 0: node->numDynamicInvocations invocations in total, read on the
        // device when the node runs (set by an earlier node, e.g.
        // addDynamicCountNode's count node).  num_threads_per_invocation
        // lanes call fn for each invocation (a power of two <= 64).
        // Contexts made in run() are world-serial: with more than one
        // invocation per world, at most one of them may mutate the world's
        // structure.
        template <auto fn, typename NodeT>
        NodeID addNodeFn(TypedDataID<NodeT> data, Span<const NodeID> dependencies,
                         Optional<NodeID> parent_node = Optional<NodeID>::none(),
                         uint32_t fixed_num_invocations = 0,
                         uint32_t num_threads_per_invocation = 1);

        // Reference device taskgraph.inl:61-70: NodeT::run(int32_t) over
        // `count` invocations per world.
        template <typename NodeT, int32_t count = 1, typename... Args>
        NodeID addOneOffNode(Span<const NodeID> dependencies, Args &&...args)
        {
            auto data_id = constructNodeData<NodeT>(std::forward<Args>(args)...);
            return addNodeFn<&NodeT::run>(data_id, dependencies, Optional<NodeID>::none(),
                                          (uint32_t)count);
        }

        // Reference device taskgraph.inl:72-95: a one-invocation node stores
        // NodeT::numInvocations() in the node data, then NodeT::run runs over
        // that many invocations (num_threads_per_invocation lanes each).
        template <typename NodeT, typename... Args>
        NodeID addDynamicCountNode(Span<const NodeID> dependencies,
                                   uint32_t num_threads_per_invocation, Args &&...args)
        {
            auto data_id = constructNodeData<NodeT>(std::forward<Args>(args)...);
            NodeID count_node = addNodeFn<&Builder::dynamicCountWrapper<NodeT>>(
                data_id, dependencies, Optional<NodeID>::none(), 0xFFFF'FFFFu);
            return addNodeFn<&NodeT::run>(data_id, { count_node }, Optional<NodeID>::none(), 0,
                                          num_threads_per_invocation);
        }

        // Framework nodes (static launch(NodeT *, LaunchCtx &): their own
        // kernels over all worlds) keep their data on the host; any other
        // NodeT is a device node: constructNodeData + addNodeFn<&NodeT::run>
        // with one invocation per world (reference taskgraph.inl:33-43).
        template <typename NodeT, typename... Args>
        NodeID addDefaultNode(Span<const NodeID> dependencies, Args &&...args)
        {
            if constexpr (requires(NodeT *n, LaunchCtx &lc) { NodeT::launch(n, lc); }) {
                auto data = std::make_shared<NodeT>(std::forward<Args>(args)...);
                uint32_t flags = 0;
                if constexpr (requires { NodeT::kNoTmpAlloc; }) flags |= kNodeNoTmpAlloc;
                if constexpr (requires { NodeT::kTmpAllocReset; }) flags |= kNodeTmpAllocReset;
                NodeFns fns;
                fns.launch = [](void *n, LaunchCtx &lc) { NodeT::launch((NodeT *)n, lc); };
                if constexpr (requires(NodeT *n, LaunchCtx &lc, detail::WalkEntry *e, const void **k) {
                                  NodeT::walkPlan(n, lc, e, k); }) {   // k: const void *[2]
                    fns.walk = [](void *n, LaunchCtx &lc, detail::WalkEntry *e, const void **k) {
                        return NodeT::walkPlan((NodeT *)n, lc, e, k);
                    };
                }
                if constexpr (requires(NodeT *n, CpuRunCtx &rc, int32_t w) { NodeT::runWorld(n, rc, w); }) {
                    fns.cpuWorld = [](void *n, CpuRunCtx &rc, int32_t w) { NodeT::runWorld((NodeT *)n, rc, w); };
                }
                if constexpr (requires(NodeT *n, CpuRunCtx &rc) { NodeT::runGlobal(n, rc); }) {
                    fns.cpuGlobal = [](void *n, CpuRunCtx &rc) { NodeT::runGlobal((NodeT *)n, rc); };
                }
                return registerNode(std::static_pointer_cast<void>(data), fns,
                                    dependencies, NodeT::nodeName(), flags);
            } else {
                auto data_id = constructNodeData<NodeT>(std::forward<Args>(args)...);
                return addNodeFn<&NodeT::run>(data_id, dependencies, Optional<NodeID>::none(), 1);
            }
        }

        // NodeT::addToGraph in either reference form: (Context &, Builder &,
        // deps) (CPU, include/madrona/taskgraph.hpp) or (Builder &, deps)
        // (device, src/mw/device/include/madrona/taskgraph.hpp).
        template <typename NodeT>
        NodeID addToGraph(Span<const NodeID> dependencies)
        {
            if constexpr (requires(Builder &b) { NodeT::addToGraph(b, dependencies); }) {
                return NodeT::addToGraph(*this, dependencies);
            } else {
                return NodeT::addToGraph(*ctx_, *this, dependencies);
            }
        }

        Context &context() { return *ctx_; }
        StateManager &stateManager();
        int32_t worldIDX() const { return 0; }

        TaskGraph build();

    private:
        template <typename NodeT>
        MW_HD static void dynamicCountWrapper(NodeT *node, int32_t)
        {
            node->numDynamicInvocations = (uint32_t)node->numInvocations();
        }

        NodeID registerNode(std::shared_ptr<void> data, NodeFns fns,
                            Span<const NodeID> deps, const char *name, uint32_t flags = 0);

        struct Staged {
            std::shared_ptr<void> data;
            NodeFns fn;
            std::vector<uint32_t> deps;
            const char *name;
            uint32_t flags;
        };

        Context *ctx_;
        std::vector<Staged> staged_;
        std::vector<NodeData> datas_;
        std::vector<uint8_t> dataIsNodeBase_;
    };

    TaskGraph() = default;
    void launch(LaunchCtx &lc) const;
    void launchNode(int32_t i, LaunchCtx &lc) const { nodes_[i].fn.launch(nodes_[i].data.get(), lc); }
    const NodeFns &nodeFns(int32_t i) const { return nodes_[i].fn; }
    void *nodeState(int32_t i) const { return nodes_[i].data.get(); }
    int32_t numNodes() const { return (int32_t)nodes_.size(); }
    const char *nodeName(int32_t i) const { return nodes_[i].name; }
    uint32_t nodeFlags(int32_t i) const { return nodes_[i].flags; }

    // Node data blocks, for the executor to upload (NodeBase-derived blocks
    // get the device state filled in first).
    int32_t numNodeDatas() const { return (int32_t)datas_.size(); }
    const NodeData *nodeDatas() const { return datas_.data(); }
    bool nodeDataIsNodeBase(int32_t i) const { return dataIsNodeBase_[i] != 0; }

private:
    struct Node {
        std::shared_ptr<void> data;
        NodeFns fn;
        const char *name;
        uint32_t flags;
    };
    std::vector<Node> nodes_;
    std::vector<NodeData> datas_;
    std::vector<uint8_t> dataIsNodeBase_;

    friend class Builder;
};

namespace detail {

template <typename C, typename = void>
struct WorldOf {
    using type = WorldBase;
};
template <typename C>
struct WorldOf<C, std::void_t<typename C::WorldDataT>> {
    using type = typename C::WorldDataT;
};

template <int32_t N>
struct ColArgs {
    int32_t c[N > 0 ? N : 1];
};

// A row node's archetypes run by one world-wave launch
// (parallelForWorldMultiKernel): up to kFusedArchetypes of them, in query
// order, each with its query index and column indices.
inline constexpr int32_t kFusedArchetypes = 4;
template <int32_t N>
struct MultiColArgs {
    int32_t n;
    int32_t arch[kFusedArchetypes];
    int32_t queryArch[kFusedArchetypes];
    ColArgs<N> cols[kFusedArchetypes];
};

// Launch helpers (csrc/runtime/executor.hip).
void launchRowKernel(const void *kernel, LaunchCtx &lc, int32_t archetype, int32_t query_arch,
                     int32_t threads_per_invocation, int32_t items_per_invocation,
                     const void *cols, size_t cols_bytes, bool world_waves);
void launchWorldKernel(const void *kernel, LaunchCtx &lc);
void launchNodeFnKernel(const void *kernel, LaunchCtx &lc, void *node_dev, uint32_t fixed_count,
                        uint32_t threads_per_invocation);
// World-serial row walk: one invocation (threads_per_invocation lanes) per
// world; `query` points at the node's Query (a kernel argument by value).
void launchSerialKernel(const void *kernel, LaunchCtx &lc, int32_t threads_per_invocation,
                        const void *query);
// The ordered structural commit of a row-parallel node (see Context): a
// no-op for worlds whose lanes made / destroyed nothing.
void launchStructuralCommit(LaunchCtx &lc);
// Runs `kernel(out_dev)` (one lane) and copies the 8-byte word it stores
// back to the host: the device address of a world function (plan time only,
// never during a capture).
void readDeviceWord(const void *kernel, void *host_out);

template <typename ContextT>
MW_INLINE ContextT worldContext(StateView *st, int32_t w, StateManager *mgr = nullptr)
{
    using WorldT = typename WorldOf<ContextT>::type;
    return ContextT((WorldT *)(st->worldData + (size_t)w * st->worldDataStride),
                    WorkerInit { st, w, mgr });
}

}

#if defined(__HIPCC__)
template <typename ContextT>
__device__ inline ContextT NodeBase::makeContext(WorldID world) const
{
    return detail::worldContext<ContextT>(mwState, world.idx);
}
#else
template <typename ContextT>
inline ContextT NodeBase::makeContext(WorldID world) const
{
    return detail::worldContext<ContextT>(mwState, world.idx);
}
#endif

#if defined(__HIPCC__)
namespace mwGPU {
// Lane within the invocation of a CustomParallelForNode / multi-thread
// node (invocations are aligned groups of threads_per_invocation lanes).
template <int32_t threads_per_invocation>
__device__ inline int32_t invocationLane()
{
    return (int32_t)(threadIdx.x & (threads_per_invocation - 1));
}
}
#else
namespace mwGPU {
// CPU back end: an invocation's lanes run one after another on the worker
// thread, each seeing its own lane index.
namespace detail { inline thread_local int32_t cpuInvocationLane = 0; }
template <int32_t threads_per_invocation>
inline int32_t invocationLane() { return detail::cpuInvocationLane; }
}
#endif

// ---------------------------------------------------------------------------
// Row-parallel node (reference device CustomParallelForNode, taskgraph.hpp:
// 166-182; CPU ParallelForNode, taskgraph.inl:58-71): Fn(ctx, components...)
// for every row of every archetype the query matches, all worlds in one
// launch.  An invocation is a group of threads_per_invocation lanes (a power
// of two <= 64, aligned within the wave) that all call Fn for the same row
// -- a cooperative Fn splits the row's work by mwGPU::invocationLane() --
// and walks items_per_invocation consecutive rows.  Rows of one world are
// contiguous in every column slab, so the lanes read columns coalesced.
// Structural mutation from Fn follows the reference's serial row order
// through the ordered commit (Context, row-parallel mode); with several
// threads per invocation only one lane of the group may mutate.
// ---------------------------------------------------------------------------
namespace detail {

#if defined(__HIPCC__)
template <typename ContextT, auto Fn, typename... ComponentTs, size_t... Is>
__device__ inline void invokeRow(ContextT &ctx, StateView *st, int32_t arch,
                                 const ColArgs<sizeof...(ComponentTs)> &cols,
                                 int32_t w, int32_t r, std::index_sequence<Is...>)
{
    Fn(ctx, rowRef(st->column<std::remove_const_t<ComponentTs>>(arch, cols.c[Is], w), r)...);
}

template <typename ContextT, auto Fn, int32_t threads, int32_t items, typename... ComponentTs>
__global__ void __launch_bounds__(256)
parallelForKernel(const StateView *__restrict__ st_in, int32_t arch, int32_t query_arch,
                  ColArgs<sizeof...(ComponentTs)> cols)
{
    MW_TRACE_BLOCK(arch);
    // The StateView itself is read-only inside a node (only the slabs it
    // points to are written); const + restrict lets the backend treat the
    // column pointers loaded from it as global (no flat accesses).
    StateView *st = const_cast<StateView *>(st_in);
    const int32_t cap = st->arch[arch].capacity;
    const int32_t inv_per_world = (cap + items - 1) / items;
    const int64_t total = (int64_t)st->numWorlds * inv_per_world * threads;
    // grid-stride: one pass with the default grid, several when the node's
    // launch configuration caps the grid (LaunchCtx::capGrid)
    // finished waves per world (row-ordered makeEntityNow, Context::lockedAcquire)
    int32_t *turn = st->makeTurn && query_arch < kMakeTurnSlots
                        ? st->makeTurn + (size_t)query_arch * st->numWorlds * kMakeTurnWaves : nullptr;
    const int32_t epoch = turn ? st->makeEpoch[0] : 0;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t inv = t / threads;
        const int32_t w = (int32_t)(inv / inv_per_world);
        const int32_t first = (int32_t)(inv - (int64_t)w * inv_per_world) * items;
        const int32_t n = st->arch[arch].numRows[w];
        // this wave's index among the waves covering world w
        const int64_t t_w0 = (int64_t)w * inv_per_world * threads;
        const int64_t chunk = (t >> 6) - (t_w0 >> 6);
        int32_t *marks = turn ? turn + (size_t)w * kMakeTurnWaves : nullptr;
        bool made = false;
        if (first < n) {
            ContextT ctx = worldContext<ContextT>(st, w);
            if (marks && chunk < kMakeTurnWaves) ctx.setMakeTurn(marks, (int32_t)chunk, epoch);
#pragma unroll 1
            for (int32_t k = 0; k < items && first + k < n; k++) {
                ctx.setRowParallel(((uint32_t)query_arch << 24) | (uint32_t)(first + k), arch,
                                   rowWriteKeys<Fn, ComponentTs...>());
                invokeRow<ContextT, Fn, ComponentTs...>(ctx, st, arch, cols, w, first + k,
                                                        std::index_sequence_for<ComponentTs...> {});
            }
            made = ctx.madeEntities();
        }
#if !defined(MW_NO_MAKE_TURN_SIGNAL)      // (A/B experiments only: breaks row-ordered makes)
        if (turn) {
            // The wave is done with its rows of each world it covers (the
            // active lanes are a prefix of the wave: t ascends with the
            // lane).  Only a world's later waves wait on the count, so the
            // world's last wave does not signal; release ordering (an L2
            // write-back) only when the wave took IDs the next one must see.
            const int32_t pw = __shfl_up(w, 1, 64);
            const int64_t t_w_last = t_w0 + (int64_t)inv_per_world * threads - 1;
            const bool signal = (__lane_id() == 0 || pw != w) && (t >> 6) < (t_w_last >> 6) &&
                                chunk < kMakeTurnWaves;
            // a plain store of the epoch (no read-modify-write)
            if (__ballot(made) != 0) {
                if (signal) __hip_atomic_store(marks + chunk, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            } else if (signal) {
                __hip_atomic_store(marks + chunk, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
#endif
    }
}

// Small tables (at most LaunchCtx::worldWaveLanes lanes of invocations per
// world, 256 by default): one
// wave per world walks the world's invocations 64 lanes at a time, stopping
// at the world's row count.  Rows of one world never span waves, so
// row-parallel makeEntityNow needs no cross-wave ordering (the wave's lanes
// take IDs in lane order, chunk after chunk), and a sparse table (fantasy_vs'
// cleanup trackers: a few rows of 250) costs one wave per world instead of
// one per 64 rows of capacity.
template <typename ContextT, auto Fn, int32_t threads, int32_t items, typename... ComponentTs>
__global__ void __launch_bounds__(256)
parallelForWorldKernel(const StateView *__restrict__ st_in, int32_t arch, int32_t query_arch,
                       ColArgs<sizeof...(ComponentTs)> cols)
{
    MW_TRACE_BLOCK(arch);
    StateView *st = const_cast<StateView *>(st_in);
    const int32_t cap = st->arch[arch].capacity;
    const int32_t inv_per_world = (cap + items - 1) / items;
    const int32_t lanes_per_world = inv_per_world * threads;
    const int32_t lane = (int32_t)(threadIdx.x & 63);
    const int64_t waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t wv = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; wv < st->numWorlds; wv += waves) {
        const int32_t w = (int32_t)wv;
        const int32_t n = st->arch[arch].numRows[w];
        for (int32_t base = 0; base < lanes_per_world && (base / threads) * items < n; base += 64) {
            const int32_t l = base + lane;
            const int32_t first = (l / threads) * items;
            if (l < lanes_per_world && first < n) {
                ContextT ctx = worldContext<ContextT>(st, w);
#pragma unroll 1
                for (int32_t k = 0; k < items && first + k < n; k++) {
                    ctx.setRowParallel(((uint32_t)query_arch << 24) | (uint32_t)(first + k), arch,
                                       rowWriteKeys<Fn, ComponentTs...>());
                    invokeRow<ContextT, Fn, ComponentTs...>(ctx, st, arch, cols, w, first + k,
                                                            std::index_sequence_for<ComponentTs...> {});
                }
            }
        }
    }
}

// The same for every archetype of the query in one launch (all of them
// small tables): each world's wave walks the archetypes in query order, so a
// world's rows run in the order the per-archetype launches gave them (its
// first archetype's rows, then the next one's), one launch instead of one per
// archetype.
// One world's rows of every archetype of a small-table query, walked by the
// calling wave (all 64 lanes, wave-uniform w): the body of
// parallelForWorldMultiKernel and of the world walk's row entries.
template <typename ContextT, auto Fn, int32_t threads, int32_t items, typename... ComponentTs>
__device__ inline void rowWorldMulti(StateView *st, const MultiColArgs<sizeof...(ComponentTs)> &m,
                                     int32_t w, int32_t lane)
{
    for (int32_t a = 0; a < m.n; a++) {
        const int32_t arch = m.arch[a];
        const int32_t query_arch = m.queryArch[a];
        const int32_t cap = st->arch[arch].capacity;
        const int32_t inv_per_world = (cap + items - 1) / items;
        const int32_t lanes_per_world = inv_per_world * threads;
        const int32_t n = st->arch[arch].numRows[w];
        for (int32_t base = 0; base < lanes_per_world && (base / threads) * items < n; base += 64) {
            const int32_t l = base + lane;
            const int32_t first = (l / threads) * items;
            if (l < lanes_per_world && first < n) {
                ContextT ctx = worldContext<ContextT>(st, w);
#pragma unroll 1
                for (int32_t k = 0; k < items && first + k < n; k++) {
                    ctx.setRowParallel(((uint32_t)query_arch << 24) | (uint32_t)(first + k), arch,
                                       rowWriteKeys<Fn, ComponentTs...>());
                    invokeRow<ContextT, Fn, ComponentTs...>(ctx, st, arch, m.cols[a], w, first + k,
                                                            std::index_sequence_for<ComponentTs...> {});
                }
            }
        }
    }
}

template <typename ContextT, auto Fn, int32_t threads, int32_t items, typename... ComponentTs>
__global__ void __launch_bounds__(256)
parallelForWorldMultiKernel(const StateView *__restrict__ st_in, int32_t, int32_t,
                            MultiColArgs<sizeof...(ComponentTs)> m)
{
    MW_TRACE_BLOCK(m.arch[0]);
    StateView *st = const_cast<StateView *>(st_in);
    const int32_t lane = (int32_t)(threadIdx.x & 63);
    const int64_t waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t wv = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; wv < st->numWorlds; wv += waves) {
        rowWorldMulti<ContextT, Fn, threads, items, ComponentTs...>(st, m, (int32_t)wv, lane);
    }
}
#endif

}

namespace detail {

#if defined(__HIPCC__)
// World-serial walk (reference ParallelForNode::run, taskgraph.inl:63-71;
// the reference's megakernel also runs a world's rows on one thread,
// src/mw/device/megakernel_impl.inl:44-55): invocation = world, its
// threads_per_invocation lanes walk the query's archetypes in order and
// every row in order, rows counted when each archetype's walk starts.  The
// context is world-serial, so structural ops act immediately and entity IDs
// are exactly the reference's; a row sees every write of the rows before it.
template <typename ContextT, auto Fn, int32_t threads, typename... ComponentTs>
__global__ void __launch_bounds__(256)
serialForKernel(const StateView *__restrict__ st_in, Query<ComponentTs...> q)
{
    MW_TRACE_BLOCK(0);
    StateView *st = const_cast<StateView *>(st_in);
    const int64_t total = (int64_t)st->numWorlds * threads;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int32_t w = (int32_t)(t / threads);
        ContextT ctx = worldContext<ContextT>(st, w);
        for (int32_t a = 0; a < q.numArchetypes; a++) {
            const int32_t arch = q.archetypes[a];
            ColArgs<sizeof...(ComponentTs)> cols;
            for (int32_t c = 0; c < (int32_t)sizeof...(ComponentTs); c++) cols.c[c] = q.cols[a][c];
            const int32_t n = st->arch[arch].numRows[w];
#pragma unroll 1
            for (int32_t r = 0; r < n; r++) {
                invokeRow<ContextT, Fn, ComponentTs...>(ctx, st, arch, cols, w, r,
                                                        std::index_sequence_for<ComponentTs...> {});
                if constexpr (threads > 1) {
                    // the group's writes before its next row
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                }
            }
        }
    }
}
#endif

#if defined(__HIPCC__)
// ---------------------------------------------------------------------------
// World walk (see WalkEntry): the kernel and the world functions.  Every
// world function is called by a whole wave (lanes 0..63, wave-uniform w).
// Each translation unit gets its own walk kernel (WalkTU is internal), so a
// run's world functions and the kernel calling them share one code object,
// and the kernel's register budget covers every function it can call.
namespace {
struct WalkTU {};
}

// A world function is called through a pointer, so its arguments arrive in
// vector registers even though every lane passes the same values; reading
// them back through readfirstlane makes them scalar again (uniform
// addresses and loop bounds in SGPRs: fewer VGPRs, scalar loads).
template <typename T>
__device__ inline T *walkUniform(T *p)
{
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (T *)(((uint64_t)hi << 32) | lo);
}

__device__ inline int32_t walkUniform(int32_t x)
{
    return __builtin_amdgcn_readfirstlane(x);
}

// A world function's arguments: under the generated dispatch the function
// inlines into the walk kernel, whose state pointer is its own
// `const __restrict__` argument -- left untouched, the backend keeps it (and
// the column pointers loaded from it) in the global address space and reads
// the state view with scalar loads; an integer round trip through
// readfirstlane would make every such access a flat vector load (measured:
// 4.8x the vector memory reads of the per-node kernels).  Called through a
// pointer, the arguments arrive in VGPRs and walkUniform makes them scalar.
template <typename T>
__device__ inline T walkArg(T x)
{
#if defined(MW_WALK_DISPATCH)
    return x;
#else
    return walkUniform(x);
#endif
}

// How the walk calls an entry's world function.  A world source compiled
// through its generated wrapper (MW_WALK_DISPATCH, tools/gen_walk_dispatch.py,
// the analogue of the reference's generated dispatch() switch) gets
// walkDispatch: direct calls to every world function of this translation
// unit, which inline into the walk kernel.  Otherwise (an out-of-tree world
// built without the generator) the call goes through the device pointer.
#if defined(MW_WALK_DISPATCH)
namespace {
__device__ void walkDispatch(const WalkEntry &e, const WalkCtx &c, int32_t w);
}
#endif
__device__ inline void walkCall(const WalkEntry &e, const WalkCtx &c, int32_t w)
{
#if defined(MW_WALK_DISPATCH)
    walkDispatch(e, c, w);
#else
    e.fn(e, c, w);
#endif
}

// World functions under the generated dispatch inline into the walk kernel;
// MW_WALK_NOINLINE keeps each its own function, called directly (measured
// slower: the caster's row code takes 97 VGPRs under the function ABI
// against 68 inlined, fantasy_vs 63 vs 74 M env-steps/s).
#if defined(MW_WALK_DISPATCH) && defined(MW_WALK_NOINLINE)
#define MW_WALK_FN_ATTR __attribute__((noinline))
#else
#define MW_WALK_FN_ATTR
#endif

__device__ inline void walkSync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// The walk: one wave per block, blocks strided over the worlds; a world's
// entries run in graph order with a wave barrier between them (the next node
// sees every lane's writes).  At a commit point a world whose lanes made or
// destroyed nothing goes on; a world with structural work stops there and
// leaves the entry index in resume[w] for worldResumeKernel.  The commit code
// is not reachable from this kernel, so its register budget is the world
// functions' (the commit alone needs ~120 VGPRs; most nodes of most worlds
// never reach it).
// Waves per SIMD the walk kernel is compiled for (its register budget).
#ifndef MW_WALK_WAVES
#define MW_WALK_WAVES 1
#endif
// Walk profile (experiments only, -DMW_WALK_PROFILE): per entry the summed
// wall-clock ticks (100 MHz) its world function took, over every world and
// launch, and the calls (g_walkProf[64 + i]); the generated wrapper exports
// the reader (mw_debug_walk_profile_<world source>).
#if defined(MW_WALK_PROFILE)
namespace {
__device__ unsigned long long g_walkProf[128];
}
#endif

template <typename Tag>
__global__ void __launch_bounds__(64, MW_WALK_WAVES)
worldWalkKernel(const WalkEntry *__restrict__ entries, int32_t n, const StateView *__restrict__ st_in,
                int32_t *resume)
{
    MW_TRACE_BLOCK(0);
    StateView *st = const_cast<StateView *>(st_in);
    const WalkCtx c { st };
    for (int32_t w = (int32_t)blockIdx.x; w < st->numWorlds; w += (int32_t)gridDim.x) {
#pragma unroll 1
        for (int32_t i = 0; i < n; i++) {
#if defined(MW_WALK_PROFILE)
            const long long t0 = wall_clock64();
#endif
            const WalkEntry &e = entries[i];
            if (e.kind == kWalkCommit) {
                if (commitLoad(st->appendDirty + w) != 0 || commitLoad(st->deferCount + w) != 0) {
                    if (threadIdx.x == 0) resume[w] = i;
                    break;
                }
                continue;
            }
            walkCall(e, c, w);
            walkSync();
#if defined(MW_WALK_PROFILE)
            if (threadIdx.x == 0 && i < 64 && (w & 15) == 0) {   // sampled: 1 world in 16
                atomicAdd(&g_walkProf[i], (unsigned long long)(wall_clock64() - t0));
                atomicAdd(&g_walkProf[64 + i], 1ull);
            }
#endif
        }
    }
}

// The worlds a walk stopped at a commit point: commit (the executor's ordered
// commit, working set in LDS when it fits), then the rest of the
// world's entries, committing again wherever the world is dirty.  Blocks
// (one wave) check 64 worlds per round with one ballot, as the commit kernel
// does; a step where no world stopped costs one pass of loads.
template <typename Tag>
__global__ void __launch_bounds__(64)
worldResumeKernel(const WalkEntry *__restrict__ entries, int32_t n, const StateView *__restrict__ st_in,
                  int32_t *resume, char *scratch, uint64_t per_block, CommitShape shape, uint64_t ws_bytes)
{
    MW_TRACE_BLOCK(0);
    StateView *st = const_cast<StateView *>(st_in);
    // the commit's working set: in this block's dynamic LDS (ws_bytes == 0,
    // as the ordered-commit kernel keeps it), else in its global slab
    extern __shared__ __align__(16) char resume_lds[];
    char *slab = scratch + (size_t)blockIdx.x * per_block;
    char *ws = ws_bytes == 0 ? resume_lds : slab;
    char *moves = slab + ws_bytes;
    const WalkCtx c { st };
    const int32_t lane = (int32_t)(threadIdx.x & 63);
    for (int64_t base = blockIdx.x; base < st->numWorlds; base += (int64_t)gridDim.x * 64) {
        const int64_t mine = base + (int64_t)lane * gridDim.x;
        const bool stopped = mine < st->numWorlds && resume[mine] >= 0;
        for (uint64_t todo = __ballot(stopped); todo != 0; todo &= todo - 1) {
            const int32_t w = (int32_t)(base + (int64_t)__builtin_ctzll(todo) * gridDim.x);
            const int32_t from = resume[w];
            walkSync();
            for (int32_t i = from; i < n; i++) {
                const WalkEntry &e = entries[i];
                if (e.kind == kWalkCommit) {
                    if (shape.capMax > 0 &&
                        (commitLoad(st->appendDirty + w) != 0 || commitLoad(st->deferCount + w) != 0)) {
                        commitWorld(*st, shape, ws, moves, w);
                    }
                } else {
                    walkCall(e, c, w);
                }
                walkSync();
            }
            if (lane == 0) resume[w] = -1;
        }
    }
}

template <typename Tag, auto F>
__global__ void walkFnAddrKernel(WalkFn *out)
{
    *out = F;
}

// Device address of world function F in this translation unit's code object
// (per device: each device loads its own copy of the code object).
template <typename Tag, auto F>
WalkFn walkFnAddr()
{
    static WalkFn cache[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
        throw std::runtime_error("world walk: no current HIP device");
    }
    if (!cache[dev]) readDeviceWord((const void *)&walkFnAddrKernel<Tag, F>, &cache[dev]);
    return cache[dev];
}

template <int32_t N>
struct RowWalkParams {
    MultiColArgs<N> m;
    int32_t serial;
    int32_t threads;
};

// A row node's world: row-parallel lanes over the world's small tables
// (rowWorldMulti, as parallelForWorldMultiKernel), or the world-serial walk
// on threads_per_invocation lanes (serialForKernel's body).
template <typename ContextT, auto Fn, int32_t threads, int32_t items, typename... ComponentTs>
__device__ MW_WALK_FN_ATTR void rowWalkEntry(const WalkEntry &e_in, const WalkCtx &c, int32_t w_in)
{
    const WalkEntry &e = *walkArg(&e_in);
    const int32_t w = walkArg(w_in);
    const auto &p = *reinterpret_cast<const RowWalkParams<sizeof...(ComponentTs)> *>(e.params);
    const int32_t lane = (int32_t)(threadIdx.x & 63);
    StateView *st = walkArg(c.st);
    if (!p.serial) {
        rowWorldMulti<ContextT, Fn, threads, items, ComponentTs...>(st, p.m, w, lane);
        return;
    }
#if defined(MW_WALK_NO_SERIAL)
    return;
#endif
    if (lane >= threads) return;
    ContextT ctx = worldContext<ContextT>(st, w);
    for (int32_t a = 0; a < p.m.n; a++) {
        const int32_t arch = p.m.arch[a];
        const int32_t n = st->arch[arch].numRows[w];
#pragma unroll 1
        for (int32_t r = 0; r < n; r++) {
            invokeRow<ContextT, Fn, ComponentTs...>(ctx, st, arch, p.m.cols[a], w, r,
                                                    std::index_sequence_for<ComponentTs...> {});
            if constexpr (threads > 1) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
        }
    }
}

// PerWorldNode: Fn(ctx) on the world's lane 0 (world-serial context).
template <typename ContextT, auto Fn>
__device__ MW_WALK_FN_ATTR void perWorldWalkEntry(const WalkEntry &, const WalkCtx &c, int32_t w_in)
{
    const int32_t w = walkArg(w_in);
    StateView *st = walkArg(c.st);
    if ((threadIdx.x & 63) != 0) return;
    ContextT ctx = worldContext<ContextT>(st, w);
    Fn(ctx);
}

// addNodeFn with a fixed count per world: the world's invocations w * count
// + k, threads lanes each (nodeFnKernel's numbering).
template <typename NodeT>
struct NodeFnWalkParams {
    NodeT *node;
    uint32_t count;
    uint32_t threads;
};

template <typename NodeT, auto fn>
__device__ MW_WALK_FN_ATTR void nodeFnWalkEntry(const WalkEntry &e_in, const WalkCtx &, int32_t w_in)
{
    const WalkEntry &e = *walkArg(&e_in);
    const int32_t w = walkArg(w_in);
    const auto &p = *reinterpret_cast<const NodeFnWalkParams<NodeT> *>(e.params);
    const int32_t total = (int32_t)(p.count * p.threads);
    for (int32_t base = 0; base < total; base += 64) {
        const int32_t t = base + (int32_t)(threadIdx.x & 63);
        if (t < total) std::invoke(fn, p.node, (int32_t)((int64_t)w * p.count + t / (int32_t)p.threads));
    }
}
#endif

// ParallelForNode / CustomParallelForNode (kSerial = false: row-parallel
// unless the executor runs every node world-serially) and WorldSerialForNode
// (kSerial = true: always world-serial).
template <typename ContextT, auto Fn, int32_t threads_per_invocation, int32_t items_per_invocation,
          bool kSerial, typename... ComponentTs>
class RowForNode : public NodeBase {
    static_assert(threads_per_invocation >= 1 && threads_per_invocation <= 64 &&
                  (threads_per_invocation & (threads_per_invocation - 1)) == 0,
                  "threads_per_invocation: a power of two <= 64 (one wave)");
    static_assert(items_per_invocation >= 1);
public:
    explicit RowForNode(Context &ctx) : query_(ctx.query<ComponentTs...>()) {}

    static TaskGraph::NodeID addToGraph(Context &ctx, TaskGraph::Builder &builder,
                                        Span<const TaskGraph::NodeID> deps)
    {
        return builder.addDefaultNode<RowForNode>(deps, ctx);
    }
    static TaskGraph::NodeID addToGraph(TaskGraph::Builder &builder,
                                        Span<const TaskGraph::NodeID> deps)
    {
        return builder.addDefaultNode<RowForNode>(deps, builder.context());
    }

    static void launch(RowForNode *self, LaunchCtx &lc)
    {
#if defined(__HIPCC__)
        if (kSerial || lc.serialNodes) {
            detail::launchSerialKernel(
                (const void *)&detail::serialForKernel<ContextT, Fn, threads_per_invocation,
                                                       ComponentTs...>,
                lc, threads_per_invocation, &self->query_);
            return;
        }
        // every archetype a small table: one world-wave launch for all
        const int32_t na = self->query_.numArchetypes;
        bool all_small = na >= 2 && na <= kFusedArchetypes && lc.fuseArchetypes;
        int32_t widest = 0;
        for (int32_t a = 0; all_small && a < na; a++) {
            const int32_t arch = self->query_.archetypes[a];
            const int64_t lanes = (int64_t)(lc.view->arch[arch].capacity + items_per_invocation - 1) /
                                  items_per_invocation * threads_per_invocation;
            all_small = lanes <= lc.worldWaveLanes;
            if (lc.view->arch[arch].capacity > lc.view->arch[self->query_.archetypes[widest]].capacity)
                widest = a;
        }
        if (all_small) {
            detail::MultiColArgs<sizeof...(ComponentTs)> m {};
            m.n = na;
            for (int32_t a = 0; a < na; a++) {
                m.arch[a] = self->query_.archetypes[a];
                m.queryArch[a] = a;
                for (int32_t c = 0; c < (int32_t)sizeof...(ComponentTs); c++) {
                    m.cols[a].c[c] = self->query_.cols[a][c];
                }
            }
            detail::launchRowKernel(
                (const void *)&detail::parallelForWorldMultiKernel<
                    ContextT, Fn, threads_per_invocation, items_per_invocation, ComponentTs...>,
                lc, self->query_.archetypes[widest], 0, threads_per_invocation, items_per_invocation,
                &m, sizeof(m), true);
            detail::launchStructuralCommit(lc);
            return;
        }
        for (int32_t a = 0; a < self->query_.numArchetypes; a++) {
            detail::ColArgs<sizeof...(ComponentTs)> cols;
            for (int32_t c = 0; c < (int32_t)sizeof...(ComponentTs); c++) {
                cols.c[c] = self->query_.cols[a][c];
            }
            const int32_t arch = self->query_.archetypes[a];
            const int64_t lanes = (int64_t)(lc.view->arch[arch].capacity + items_per_invocation - 1) /
                                  items_per_invocation * threads_per_invocation;
            const bool world_waves = lanes <= lc.worldWaveLanes;
            const void *kernel =
                world_waves ? (const void *)&detail::parallelForWorldKernel<
                                  ContextT, Fn, threads_per_invocation, items_per_invocation, ComponentTs...>
                            : (const void *)&detail::parallelForKernel<
                                  ContextT, Fn, threads_per_invocation, items_per_invocation, ComponentTs...>;
            detail::launchRowKernel(kernel, lc, arch, a, threads_per_invocation, items_per_invocation,
                                    &cols, sizeof(cols), world_waves);
        }
        detail::launchStructuralCommit(lc);
#else
        (void)self; (void)lc;
#endif
    }

    // World walk: the node's rows (and its ordered commit) for one world at a
    // time, when every archetype of the query is a small table (as for
    // parallelForWorldMultiKernel) or the node is world-serial.
    static int32_t walkPlan(RowForNode *self, LaunchCtx &lc, detail::WalkEntry *out, const void **kernels)
    {
#if defined(__HIPCC__)
        const int32_t na = self->query_.numArchetypes;
        if (na < 1 || na > detail::kFusedArchetypes) return 0;
        const bool serial = kSerial || lc.serialNodes;
        for (int32_t a = 0; a < na && !serial; a++) {
            const int64_t lanes = (int64_t)(lc.view->arch[self->query_.archetypes[a]].capacity +
                                            items_per_invocation - 1) /
                                  items_per_invocation * threads_per_invocation;
            if (lanes > lc.worldWaveLanes) return 0;
        }
        detail::RowWalkParams<sizeof...(ComponentTs)> p {};
        static_assert(sizeof(p) <= detail::kWalkParamBytes, "row walk parameters");
        p.m.n = na;
        for (int32_t a = 0; a < na; a++) {
            p.m.arch[a] = self->query_.archetypes[a];
            p.m.queryArch[a] = a;
            for (int32_t c = 0; c < (int32_t)sizeof...(ComponentTs); c++) p.m.cols[a].c[c] = self->query_.cols[a][c];
        }
        p.serial = serial ? 1 : 0;
        p.threads = threads_per_invocation;
        out[0] = detail::WalkEntry {};
        out[0].fn = detail::walkFnAddr<detail::WalkTU,
                                       &detail::rowWalkEntry<ContextT, Fn, threads_per_invocation,
                                                             items_per_invocation, ComponentTs...>>();
        memcpy(out[0].params, &p, sizeof(p));
        kernels[0] = (const void *)&detail::worldWalkKernel<detail::WalkTU>;
        kernels[1] = (const void *)&detail::worldResumeKernel<detail::WalkTU>;
        if (serial) return 1;
        out[1] = detail::WalkEntry {};
        out[1].kind = detail::kWalkCommit;
        return 2;
#else
        (void)self; (void)lc; (void)out; (void)kernels;
        return 0;
#endif
    }

#if !defined(__HIPCC__)
    // CPU back end: the reference's ParallelForNode::run (taskgraph.inl:
    // 63-71) -- the world's matching rows in query order, rows counted when
    // each archetype's walk starts, structural ops immediate (world-serial).
    // A cooperative Fn runs once per invocation lane, lanes in order.
    [[gnu::flatten]] static void runWorld(RowForNode *self, CpuRunCtx &rc, int32_t w)
    {
        ContextT ctx = detail::worldContext<ContextT>(rc.state, w, rc.mgr);
        StateView *st = rc.state;
        for (int32_t a = 0; a < self->query_.numArchetypes; a++) {
            const int32_t arch = self->query_.archetypes[a];
            const int32_t n = st->arch[arch].numRows[w];
            const int32_t *cols = self->query_.cols[a];
            [&]<size_t... Is>(std::index_sequence<Is...>) {
                // the world's column bases, once per archetype (Fn's stores
                // could alias the StateView, so the loop would reload them)
                const auto bases = std::make_tuple(
                    st->column<std::remove_const_t<ComponentTs>>(arch, cols[Is], w)...);
                for (int32_t r = 0; r < n; r++) {
                    if constexpr (threads_per_invocation == 1) {
                        Fn(ctx, std::get<Is>(bases)[r]...);
                    } else {
                        for (int32_t t = 0; t < threads_per_invocation; t++) {
                            mwGPU::detail::cpuInvocationLane = t;
                            Fn(ctx, std::get<Is>(bases)[r]...);
                        }
                    }
                }
            }(std::index_sequence_for<ComponentTs...> {});
        }
        mwGPU::detail::cpuInvocationLane = 0;
    }
#endif

    static const char *nodeName()
    {
        if (kSerial) return "WorldSerialForNode";
        return threads_per_invocation == 1 && items_per_invocation == 1 ? "ParallelForNode"
                                                                        : "CustomParallelForNode";
    }

    Query<ComponentTs...> query_;
};

}

template <typename ContextT, auto Fn, int32_t threads_per_invocation, int32_t items_per_invocation,
          typename... ComponentTs>
using CustomParallelForNode = detail::RowForNode<ContextT, Fn, threads_per_invocation,
                                                 items_per_invocation, false, ComponentTs...>;

// Reference device taskgraph.hpp:184-186 (the CPU class of the same name
// walks rows serially; the commit keeps its structural order).
template <typename ContextT, auto Fn, typename... ComponentTs>
using ParallelForNode = CustomParallelForNode<ContextT, Fn, 1, 1, ComponentTs...>;

// A ParallelForNode that always runs world-serially: for bodies whose result
// depends on the reference's row order beyond structural ops -- a row that
// reads or writes another row's components (ctx.get<T>(other)) which this
// node also writes, state carried from row to row through world data, or
// entity IDs that must equal the reference's.
template <typename ContextT, auto Fn, typename... ComponentTs>
using WorldSerialForNode = detail::RowForNode<ContextT, Fn, 1, 1, true, ComponentTs...>;

// ---------------------------------------------------------------------------
// Device nodes of addNodeFn (run(int32_t invocation_idx) on the device).
// ---------------------------------------------------------------------------
namespace detail {

#if defined(__HIPCC__)
// fixed_count > 0: fixed_count invocations per world; 0: the node's
// numDynamicInvocations in total; 0xFFFFFFFF: one invocation (the dynamic
// count node).
template <typename NodeT, auto fn>
__global__ void __launch_bounds__(256)
nodeFnKernel(NodeT *node, uint32_t fixed_count, uint32_t threads)
{
    MW_TRACE_BLOCK(0);
    int64_t total;
    if (fixed_count == 0xFFFF'FFFFu) {
        total = 1;
    } else if (fixed_count > 0) {
        total = (int64_t)node->mwNumWorlds * fixed_count;
    } else {
        total = (int64_t)__hip_atomic_load(&node->numDynamicInvocations, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    }
    total *= threads;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        std::invoke(fn, node, (int32_t)(t / threads));
    }
}
#endif

}

template <auto fn, typename NodeT>
TaskGraph::NodeID TaskGraph::Builder::addNodeFn(TypedDataID<NodeT> data,
                                                Span<const NodeID> dependencies,
                                                Optional<NodeID> parent_node,
                                                uint32_t fixed_num_invocations,
                                                uint32_t num_threads_per_invocation)
{
    static_assert(std::is_base_of_v<NodeBase, NodeT>, "device nodes derive from NodeBase");
    (void)parent_node;   // children run as ordinary nodes, in dependency order
    if (num_threads_per_invocation == 0 || num_threads_per_invocation > 64 ||
        (num_threads_per_invocation & (num_threads_per_invocation - 1)) != 0) {
        throw std::runtime_error("addNodeFn: num_threads_per_invocation must be a power of two <= 64");
    }
    struct Desc {
        int32_t dataIdx;
        uint32_t fixedCount;
        uint32_t threads;
    };
    auto desc = std::make_shared<Desc>(Desc { data.id, fixed_num_invocations,
                                              num_threads_per_invocation });
    NodeFns fns;
    fns.launch = [](void *d, LaunchCtx &lc) {
#if defined(__HIPCC__)
        const Desc &dd = *(const Desc *)d;
        void *node = lc.nodeData + (size_t)dd.dataIdx * maxNodeDataBytes;
        detail::launchNodeFnKernel((const void *)&detail::nodeFnKernel<NodeT, fn>, lc, node,
                                   dd.fixedCount, dd.threads);
#else
        (void)d; (void)lc;
#endif
    };
#if defined(__HIPCC__)
    // A device node joins a world walk only when it declares itself
    // world-local (static constexpr bool kWorldLocal = true: invocation
    // w * count + k touches world w only).  The per-node launch orders the
    // node after every world of the previous node; the walk does not, so a
    // node reading another world's state, or state other nodes accumulate
    // across worlds, must stay out of it (the default).
    constexpr bool world_local = [] {
        if constexpr (requires { NodeT::kWorldLocal; }) return (bool)NodeT::kWorldLocal;
        else return false;
    }();
    if (world_local && fixed_num_invocations > 0 && fixed_num_invocations != 0xFFFF'FFFFu) {
        fns.walk = [](void *d, LaunchCtx &lc, detail::WalkEntry *out, const void **kernels) -> int32_t {
            const Desc &dd = *(const Desc *)d;
            detail::NodeFnWalkParams<NodeT> p { (NodeT *)(lc.nodeData + (size_t)dd.dataIdx * maxNodeDataBytes),
                                                dd.fixedCount, dd.threads };
            static_assert(sizeof(p) <= detail::kWalkParamBytes);
            out[0] = detail::WalkEntry {};
            out[0].fn = detail::walkFnAddr<detail::WalkTU, &detail::nodeFnWalkEntry<NodeT, fn>>();
            memcpy(out[0].params, &p, sizeof(p));
            kernels[0] = (const void *)&detail::worldWalkKernel<detail::WalkTU>;
            kernels[1] = (const void *)&detail::worldResumeKernel<detail::WalkTU>;
            return 1;
        };
    }
#endif
#if !defined(__HIPCC__)
    // CPU back end.  A fixed count per world is world-local (invocation
    // world * count + k, k in order, each by every one of its lanes in
    // turn); the single count invocation and a dynamic count (invocations
    // over all worlds, read from the node data) run once per step.
    if (fixed_num_invocations > 0 && fixed_num_invocations != 0xFFFF'FFFFu) {
        fns.cpuWorld = [](void *d, CpuRunCtx &rc, int32_t w) {
            const Desc &dd = *(const Desc *)d;
            NodeT *node = (NodeT *)(rc.nodeData + (size_t)dd.dataIdx * maxNodeDataBytes);
            for (uint32_t k = 0; k < dd.fixedCount; k++) {
                for (uint32_t t = 0; t < dd.threads; t++) {
                    mwGPU::detail::cpuInvocationLane = (int32_t)t;
                    std::invoke(fn, node, (int32_t)((int64_t)w * dd.fixedCount + k));
                }
            }
            mwGPU::detail::cpuInvocationLane = 0;
        };
    } else {
        fns.cpuGlobal = [](void *d, CpuRunCtx &rc) {
            const Desc &dd = *(const Desc *)d;
            NodeT *node = (NodeT *)(rc.nodeData + (size_t)dd.dataIdx * maxNodeDataBytes);
            if (dd.fixedCount == 0xFFFF'FFFFu) {
                for (uint32_t t = 0; t < dd.threads; t++) {
                    mwGPU::detail::cpuInvocationLane = (int32_t)t;
                    std::invoke(fn, node, 0);
                }
                mwGPU::detail::cpuInvocationLane = 0;
                return;
            }
            struct Arg { NodeT *node; uint32_t threads; } arg { node, dd.threads };
            cpuParallelFor(rc, (int64_t)node->numDynamicInvocations,
                           [](void *a, int64_t b, int64_t e) {
                               Arg &ar = *(Arg *)a;
                               for (int64_t i = b; i < e; i++) {
                                   for (uint32_t t = 0; t < ar.threads; t++) {
                                       mwGPU::detail::cpuInvocationLane = (int32_t)t;
                                       std::invoke(fn, ar.node, (int32_t)i);
                                   }
                               }
                               mwGPU::detail::cpuInvocationLane = 0;
                           }, &arg);
        };
    }
#endif
    return registerNode(std::static_pointer_cast<void>(desc), fns, dependencies, "NodeFn");
}

// ---------------------------------------------------------------------------
// Per-world node: Fn(ContextT &) once per world, worlds in parallel (one lane
// each).  The reference runs every node once per world (taskgraph.cpp:
// 111-122); this is its general custom-node form: the lane owns its world, so
// structural mutation acts immediately (world-serial mode).
// ---------------------------------------------------------------------------
namespace detail {
#if defined(__HIPCC__)
template <typename ContextT, auto Fn>
__global__ void __launch_bounds__(64) perWorldKernel(const StateView *__restrict__ st_in)
{
    MW_TRACE_BLOCK(0);
    StateView *st = const_cast<StateView *>(st_in);
    for (int32_t w = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x); w < st->numWorlds;
         w += (int32_t)(gridDim.x * blockDim.x)) {
        ContextT ctx = worldContext<ContextT>(st, w);
        Fn(ctx);
    }
}
#endif
}

template <typename ContextT, auto Fn>
class PerWorldNode : public NodeBase {
public:
    static TaskGraph::NodeID addToGraph(Context &, TaskGraph::Builder &builder,
                                        Span<const TaskGraph::NodeID> deps)
    {
        return builder.addDefaultNode<PerWorldNode>(deps);
    }

    static void launch(PerWorldNode *, LaunchCtx &lc)
    {
#if defined(__HIPCC__)
        detail::launchWorldKernel((const void *)&detail::perWorldKernel<ContextT, Fn>, lc);
#else
        (void)lc;
#endif
    }
    static int32_t walkPlan(PerWorldNode *, LaunchCtx &, detail::WalkEntry *out, const void **kernels)
    {
#if defined(__HIPCC__)
        out[0] = detail::WalkEntry {};
        out[0].fn = detail::walkFnAddr<detail::WalkTU, &detail::perWorldWalkEntry<ContextT, Fn>>();
        kernels[0] = (const void *)&detail::worldWalkKernel<detail::WalkTU>;
        kernels[1] = (const void *)&detail::worldResumeKernel<detail::WalkTU>;
        return 1;
#else
        (void)out; (void)kernels;
        return 0;
#endif
    }
#if !defined(__HIPCC__)
    static void runWorld(PerWorldNode *, CpuRunCtx &rc, int32_t w)
    {
        ContextT ctx = detail::worldContext<ContextT>(rc.state, w, rc.mgr);
        Fn(ctx);
    }
#endif

    static const char *nodeName() { return "PerWorldNode"; }
};

// Clear a temporary archetype in every world (taskgraph.inl:94-104).
void launchClearRows(LaunchCtx &lc, int32_t archetype);
// Reset every world's tmpAlloc arena (taskgraph.inl:83-86).
void launchResetTmpAlloc(LaunchCtx &lc);

template <typename ArchetypeT>
class ClearTmpNode : public NodeBase {
public:
    explicit ClearTmpNode(Context &ctx)
        : archetype_(ctx.state().findArchetype(typeKey<ArchetypeT>()))
    {}
    static TaskGraph::NodeID addToGraph(Context &ctx, TaskGraph::Builder &builder,
                                        Span<const TaskGraph::NodeID> deps)
    {
        return builder.addDefaultNode<ClearTmpNode>(deps, ctx);
    }
    static TaskGraph::NodeID addToGraph(TaskGraph::Builder &builder,
                                        Span<const TaskGraph::NodeID> deps)
    {
        return builder.addDefaultNode<ClearTmpNode>(deps, builder.context());
    }
    static void launch(ClearTmpNode *self, LaunchCtx &lc) { launchClearRows(lc, self->archetype_); }
    static void runWorld(ClearTmpNode *self, CpuRunCtx &rc, int32_t w)
    {                                              // clearTemporaries: numRows = 0
        rc.state->arch[self->archetype_].numRows[w] = 0;
    }
    static const char *nodeName() { return "ClearTmpNode"; }
    static constexpr bool kNoTmpAlloc = true;

    int32_t archetype_;
};

class ResetTmpAllocNode : public NodeBase {
public:
    static TaskGraph::NodeID addToGraph(Context &, TaskGraph::Builder &builder,
                                        Span<const TaskGraph::NodeID> deps)
    {
        return builder.addDefaultNode<ResetTmpAllocNode>(deps);
    }
    static TaskGraph::NodeID addToGraph(TaskGraph::Builder &builder,
                                        Span<const TaskGraph::NodeID> deps)
    {
        return builder.addDefaultNode<ResetTmpAllocNode>(deps);
    }
    static void launch(ResetTmpAllocNode *, LaunchCtx &lc) { launchResetTmpAlloc(lc); }
    static void runWorld(ResetTmpAllocNode *, CpuRunCtx &rc, int32_t w)
    {
        if (rc.state->tmpOffset) rc.state->tmpOffset[w] = 0;
        hostTmpOverflowReset(*rc.state, w);
    }
    static const char *nodeName() { return "ResetTmpAllocNode"; }
    static constexpr bool kNoTmpAlloc = true;
    static constexpr bool kTmpAllocReset = true;
};

}
