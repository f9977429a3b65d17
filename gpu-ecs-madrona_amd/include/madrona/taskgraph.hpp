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
#include <madrona/tracing.hpp>

#include <initializer_list>
#include <memory>
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

struct NodeBase {};

class TaskGraph {
public:
    struct NodeID {
        uint32_t id;
    };

    using LaunchFn = void (*)(void *node, LaunchCtx &lc);

    class Builder {
    public:
        explicit Builder(Context &ctx);

        template <typename NodeT, typename... Args>
        NodeID addDefaultNode(Span<const NodeID> dependencies, Args &&...args)
        {
            auto data = std::make_shared<NodeT>(std::forward<Args>(args)...);
            return registerNode(std::static_pointer_cast<void>(data),
                                [](void *n, LaunchCtx &lc) { NodeT::launch((NodeT *)n, lc); },
                                dependencies, NodeT::nodeName());
        }

        template <typename NodeT>
        NodeID addToGraph(Span<const NodeID> dependencies)
        {
            return NodeT::addToGraph(*ctx_, *this, dependencies);
        }

        Context &context() { return *ctx_; }
        StateManager &stateManager();

        TaskGraph build();

    private:
        NodeID registerNode(std::shared_ptr<void> data, LaunchFn fn,
                            Span<const NodeID> deps, const char *name);

        struct Staged {
            std::shared_ptr<void> data;
            LaunchFn fn;
            std::vector<uint32_t> deps;
            const char *name;
        };

        Context *ctx_;
        std::vector<Staged> staged_;
    };

    TaskGraph() = default;
    void launch(LaunchCtx &lc) const;
    void launchNode(int32_t i, LaunchCtx &lc) const { nodes_[i].fn(nodes_[i].data.get(), lc); }
    int32_t numNodes() const { return (int32_t)nodes_.size(); }
    const char *nodeName(int32_t i) const { return nodes_[i].name; }

private:
    struct Node {
        std::shared_ptr<void> data;
        LaunchFn fn;
        const char *name;
    };
    std::vector<Node> nodes_;

    friend class Builder;
};

// ---------------------------------------------------------------------------
// Generic row-parallel node: one lane per (world, row) of every archetype the
// query matches; all worlds in one launch.  Rows of one world are contiguous
// in every column slab, so lanes read columns fully coalesced.
// ---------------------------------------------------------------------------
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

void launchRowKernel(const void *kernel, LaunchCtx &lc, int32_t archetype,
                     const void *args, size_t args_bytes);

#if defined(__HIPCC__)
template <typename ContextT, auto Fn, typename... ComponentTs, size_t... Is>
__device__ inline void invokeRow(ContextT &ctx, StateView *st, int32_t arch,
                                 const ColArgs<sizeof...(ComponentTs)> &cols,
                                 int32_t w, int32_t r, std::index_sequence<Is...>)
{
    Fn(ctx, rowRef(st->column<std::remove_const_t<ComponentTs>>(arch, cols.c[Is], w), r)...);
}

template <typename ContextT, auto Fn, typename... ComponentTs>
__global__ void __launch_bounds__(256)
parallelForKernel(const StateView *__restrict__ st_in, int32_t arch,
                  ColArgs<sizeof...(ComponentTs)> cols)
{
    MW_TRACE_BLOCK(arch);
    // The StateView itself is read-only inside a node (only the slabs it
    // points to are written); const + restrict lets the backend treat the
    // column pointers loaded from it as global (no flat accesses).
    StateView *st = const_cast<StateView *>(st_in);
    const int32_t cap = st->arch[arch].capacity;
    const int64_t total = (int64_t)st->numWorlds * cap;
    // grid-stride: one pass with the default grid, several when the node's
    // launch configuration caps the grid (LaunchCtx::capGrid)
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int32_t w = (int32_t)(t / cap);
        const int32_t r = (int32_t)(t - (int64_t)w * cap);
        if (r >= st->arch[arch].numRows[w]) continue;
        using WorldT = typename WorldOf<ContextT>::type;
        ContextT ctx((WorldT *)(st->worldData + (size_t)w * st->worldDataStride),
                     WorkerInit { st, w, nullptr });
        invokeRow<ContextT, Fn, ComponentTs...>(ctx, st, arch, cols, w, r,
                                                std::index_sequence_for<ComponentTs...> {});
    }
}
#endif

}

template <typename ContextT, auto Fn, typename... ComponentTs>
class ParallelForNode : public NodeBase {
public:
    explicit ParallelForNode(Context &ctx);

    static TaskGraph::NodeID addToGraph(Context &ctx, TaskGraph::Builder &builder,
                                        Span<const TaskGraph::NodeID> deps)
    {
        return builder.addDefaultNode<ParallelForNode>(deps, ctx);
    }

    static void launch(ParallelForNode *self, LaunchCtx &lc)
    {
#if defined(__HIPCC__)
        for (int32_t a = 0; a < self->query_.numArchetypes; a++) {
            detail::ColArgs<sizeof...(ComponentTs)> cols;
            for (int32_t c = 0; c < (int32_t)sizeof...(ComponentTs); c++) {
                cols.c[c] = self->query_.cols[a][c];
            }
            detail::launchRowKernel(
                (const void *)&detail::parallelForKernel<ContextT, Fn, ComponentTs...>,
                lc, self->query_.archetypes[a], &cols, sizeof(cols));
        }
#else
        (void)self; (void)lc;
#endif
    }

    static const char *nodeName() { return "ParallelForNode"; }

    Query<ComponentTs...> query_;
};

template <typename ContextT, auto Fn, typename... ComponentTs>
ParallelForNode<ContextT, Fn, ComponentTs...>::ParallelForNode(Context &ctx)
    : query_(ctx.query<ComponentTs...>())
{}

// ---------------------------------------------------------------------------
// Per-world node: Fn(ContextT &) once per world, worlds in parallel (one lane
// each).  The reference runs every node once per world (taskgraph.cpp:
// 111-122); this is its general custom-node form, and the place for
// structural mutation (makeEntityNow / destroyEntityNow / clearArchetype),
// which must not race with other lanes of the same world.
// ---------------------------------------------------------------------------
namespace detail {
void launchWorldKernel(const void *kernel, LaunchCtx &lc);

#if defined(__HIPCC__)
template <typename ContextT, auto Fn>
__global__ void __launch_bounds__(64) perWorldKernel(const StateView *__restrict__ st_in)
{
    MW_TRACE_BLOCK(0);
    StateView *st = const_cast<StateView *>(st_in);
    for (int32_t w = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x); w < st->numWorlds;
         w += (int32_t)(gridDim.x * blockDim.x)) {
        using WorldT = typename WorldOf<ContextT>::type;
        ContextT ctx((WorldT *)(st->worldData + (size_t)w * st->worldDataStride),
                     WorkerInit { st, w, nullptr });
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

    static const char *nodeName() { return "PerWorldNode"; }
};

// Clear a temporary archetype in every world (taskgraph.inl:94-104).
void launchClearRows(LaunchCtx &lc, int32_t archetype);

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
    static void launch(ClearTmpNode *self, LaunchCtx &lc) { launchClearRows(lc, self->archetype_); }
    static const char *nodeName() { return "ClearTmpNode"; }

    int32_t archetype_;
};

// The per-world bump allocator has no device state in this design (physics
// scratch lives in module-owned slabs), so the node is a scheduling marker.
class ResetTmpAllocNode : public NodeBase {
public:
    static TaskGraph::NodeID addToGraph(Context &, TaskGraph::Builder &builder,
                                        Span<const TaskGraph::NodeID> deps)
    {
        return builder.addDefaultNode<ResetTmpAllocNode>(deps);
    }
    static void launch(ResetTmpAllocNode *, LaunchCtx &) {}
    static const char *nodeName() { return "ResetTmpAllocNode"; }
};

}
