// TaskGraph::Builder / build (reference src/core/taskgraph.cpp:18-122),
// shared by the gfx950 library and the CPU back end.
#include <madrona/taskgraph.hpp>

#include <stdexcept>
#include <vector>

namespace madrona {

// ---------------------------------------------------------------------------
// TaskGraph
// ---------------------------------------------------------------------------
TaskGraph::Builder::Builder(Context &ctx) : ctx_(&ctx) {}

StateManager &TaskGraph::Builder::stateManager()
{
    // The host context always carries the StateManager (WorkerInit::mgr).
    struct Peek : Context { StateManager *mgr() { return mgr_; } };
    return *static_cast<Peek *>(ctx_)->mgr();
}

TaskGraph::NodeID TaskGraph::Builder::registerNode(std::shared_ptr<void> data, NodeFns fn,
                                                   Span<const NodeID> deps, const char *name,
                                                   uint32_t flags)
{                                               // taskgraph.cpp:18-44
    Staged s;
    s.data = std::move(data);
    s.fn = fn;
    s.name = name;
    s.flags = flags;
    for (const NodeID &d : deps) s.deps.push_back(d.id);
    staged_.push_back(std::move(s));
    return NodeID { (uint32_t)staged_.size() - 1 };
}

TaskGraph TaskGraph::Builder::build()
{                                               // taskgraph.cpp:46-109
    TaskGraph g;
    const size_t n = staged_.size();
    if (n == 0) {                               // the reference segfaults here
        g.datas_ = datas_;
        g.dataIsNodeBase_ = dataIsNodeBase_;
        return g;
    }
    std::vector<bool> queued(n, false);
    if (!staged_[0].deps.empty()) throw std::runtime_error("first node has dependencies");
    g.nodes_.push_back(Node { staged_[0].data, staged_[0].fn, staged_[0].name, staged_[0].flags });
    queued[0] = true;
    size_t remaining = n - 1;
    while (remaining > 0) {
        size_t cur;
        for (cur = 0; queued[cur]; cur++) {}
        bool ok = true;
        for (uint32_t d : staged_[cur].deps) {
            if (d >= n || !queued[d]) { ok = false; break; }
        }
        // The reference spins forever here; report the bad dependency instead.
        if (!ok) throw std::runtime_error("taskgraph: node depends on a later node");
        queued[cur] = true;
        g.nodes_.push_back(Node { staged_[cur].data, staged_[cur].fn, staged_[cur].name,
                                  staged_[cur].flags });
        remaining--;
    }
    g.datas_ = datas_;
    g.dataIsNodeBase_ = dataIsNodeBase_;
    return g;
}

void TaskGraph::launch(LaunchCtx &lc) const
{
    for (const Node &nd : nodes_) nd.fn.launch(nd.data.get(), lc);
}

}
