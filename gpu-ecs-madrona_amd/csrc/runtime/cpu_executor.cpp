// CPU back end of the executor (libmadrona_cpu.so): the reference's
// TaskGraphExecutor / ThreadPoolExecutor (include/madrona/mw_cpu.hpp:20-81,
// mw_cpu.inl:8-58, src/mw/cpu_exec.cpp:31-284) over the same world sources,
// graph and C ABI as the gfx950 library.
//
// The arena is the StateManager's host mirror (state.cpp, MW_CPU_BACKEND).
// A step runs the sorted graph world by world: consecutive world-local nodes
// (runWorld) form a segment that one pinned worker runs for a world at a
// time -- the reference's per-world TaskGraph::run (src/core/taskgraph.cpp:
// 111-122) -- and a global node (runGlobal) runs between segments.  Worlds
// are handed out by an atomic counter; every world runs its nodes in graph
// order with world-serial structural mutation, so results do not depend on
// the worker count.  Exports are packed after each step ([world-major, row],
// src/core/state.cpp:489-563).
#include <madrona/mw_gpu.hpp>

#include <sched.h>
#include <pthread.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace madrona {

// ---------------------------------------------------------------------------
// Thread pool: one worker per core of the affinity mask, pinned 1:1 (the
// reference pins its workers the same way, src/mw/cpu_exec.cpp:56-93); the
// calling thread works too and is left unpinned.
// ---------------------------------------------------------------------------
class CpuThreadPool {
public:
    explicit CpuThreadPool(int32_t num_threads)
    {
        cpu_set_t mask;
        CPU_ZERO(&mask);
        std::vector<int> cpus;
        if (sched_getaffinity(0, sizeof(mask), &mask) == 0) {
            for (int c = 0; c < CPU_SETSIZE; c++) {
                if (CPU_ISSET(c, &mask)) cpus.push_back(c);
            }
        }
        if (num_threads <= 0) num_threads = std::max<int32_t>(1, (int32_t)cpus.size());
        numThreads_ = num_threads;
        for (int32_t t = 1; t < num_threads; t++) {
            threads_.emplace_back([this, t] { workerLoop(t); });
            if (!cpus.empty()) {
                cpu_set_t one;
                CPU_ZERO(&one);
                CPU_SET(cpus[t % cpus.size()], &one);
                pthread_setaffinity_np(threads_.back().native_handle(), sizeof(one), &one);
            }
        }
    }

    ~CpuThreadPool()
    {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
            gen_++;
        }
        cv_.notify_all();
        for (auto &t : threads_) t.join();
    }

    int32_t numThreads() const { return numThreads_; }

    // fn(arg, begin, end) over [0, n) in chunks of `chunk`.
    void parallelFor(int64_t n, int64_t chunk, void (*fn)(void *, int64_t, int64_t), void *arg)
    {
        if (n <= 0) return;
        if (numThreads_ == 1 || n <= chunk) {
            fn(arg, 0, n);
            return;
        }
        {
            std::lock_guard<std::mutex> lk(m_);
            job_ = Job { fn, arg, n, std::max<int64_t>(chunk, 1) };
            next_.store(0, std::memory_order_relaxed);
            active_ = (int32_t)threads_.size();
            gen_++;
        }
        cv_.notify_all();
        work();
        std::unique_lock<std::mutex> lk(m_);
        done_.wait(lk, [this] { return active_ == 0; });
    }

private:
    struct Job {
        void (*fn)(void *, int64_t, int64_t);
        void *arg;
        int64_t n;
        int64_t chunk;
    };

    void work()
    {
        const Job j = job_;
        while (true) {
            const int64_t b = next_.fetch_add(j.chunk, std::memory_order_relaxed);
            if (b >= j.n) break;
            j.fn(j.arg, b, std::min(j.n, b + j.chunk));
        }
    }

    void workerLoop(int32_t)
    {
        uint64_t seen = 0;
        while (true) {
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
                if (stop_) return;
            }
            work();
            {
                std::lock_guard<std::mutex> lk(m_);
                if (--active_ == 0) done_.notify_one();
            }
        }
    }

    int32_t numThreads_ = 1;
    std::vector<std::thread> threads_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    uint64_t gen_ = 0;
    bool stop_ = false;
    int32_t active_ = 0;
    Job job_ {};
    std::atomic<int64_t> next_ { 0 };
};

// Kernel-launch entry points of the framework nodes (executor.hip); the CPU
// back end runs those nodes through runWorld and never launches.
void launchClearRows(LaunchCtx &, int32_t)
{
    throw std::runtime_error("launchClearRows: no kernels on the CPU back end");
}

void launchResetTmpAlloc(LaunchCtx &)
{
    throw std::runtime_error("launchResetTmpAlloc: no kernels on the CPU back end");
}

void cpuParallelFor(CpuRunCtx &rc, int64_t n, void (*fn)(void *, int64_t, int64_t), void *arg)
{
    const int64_t chunk = std::max<int64_t>(1, n / ((int64_t)rc.pool->numThreads() * 8));
    rc.pool->parallelFor(n, chunk, fn, arg);
}

// ---------------------------------------------------------------------------
// Executor
// ---------------------------------------------------------------------------
struct CpuExport {
    int32_t slot, archetype, column;
    uint32_t bytes;
    std::vector<char> buf;
    int64_t rows = 0;
};

struct Executor::Impl {
    ExecConfig cfg;
    std::unique_ptr<StateManager> mgr;
    std::unique_ptr<CpuThreadPool> pool;
    TaskGraph graph;
    std::vector<TaskGraph::NodeData> nodeData;     // host copies (NodeBase filled in)
    struct Segment {
        bool global;
        std::vector<int32_t> nodes;
    };
    std::vector<Segment> segs;
    std::vector<CpuExport> exports;
    // timing of one node kind (setTimedNode / timeNode): wall time of every
    // run of that node, summed over worlds
    std::string timedName;
    int32_t timedIndex = -1;        // setTimedNodeIndex: one node only
    bool timedMatch(int32_t n) const
    {
        if (timedIndex >= 0) return n == timedIndex;
        return !timedName.empty() && timedName == graph.nodeName(n);
    }
    std::atomic<int64_t> timedNs { 0 };
    int64_t timedLaunches = 0;
};

Executor::Executor(const ExecConfig &cfg) : impl_(new Impl)
{
    impl_->cfg = cfg;
    impl_->mgr.reset(new StateManager(StateManager::Config {
        cfg.numWorlds, cfg.defaultCapacity,
        cfg.tmpAllocBytesPerWorld >= 0 ? cfg.tmpAllocBytesPerWorld : kDefaultTmpAllocBytes,
        cfg.maxDeferredPerWorld > 0 ? cfg.maxDeferredPerWorld : kDefaultDeferredPerWorld,
        cfg.tmpPoolBytes >= 0 ? cfg.tmpPoolBytes
                              : defaultTmpPoolBytes(cfg.numWorlds, cfg.tmpAllocBytesPerWorld >= 0
                                                                       ? cfg.tmpAllocBytesPerWorld
                                                                       : kDefaultTmpAllocBytes) }));
    impl_->pool.reset(new CpuThreadPool(cfg.numWorkers));
}

Executor::~Executor()
{
    impl_->pool.reset();
    impl_->mgr.reset();
}

StateManager &Executor::stateManager() { return *impl_->mgr; }
ECSRegistry Executor::registry() { return ECSRegistry(impl_->mgr.get(), nullptr); }
int32_t Executor::numWorlds() const { return impl_->cfg.numWorlds; }
void *Executor::stream() const { return nullptr; }
const void *Executor::commitArgs() const { return nullptr; }

void Executor::finalizeRegistration(uint32_t world_bytes, uint32_t world_align)
{
    impl_->mgr->finalizeLayout(world_bytes, world_align);
}

Context Executor::makeHostContext(int32_t world)
{
    return Context((WorldBase *)hostWorldData(world),
                   WorkerInit { &impl_->mgr->hostView(), world, impl_->mgr.get() });
}

char *Executor::hostWorldData(int32_t world)
{
    StateView &v = impl_->mgr->hostView();
    return v.worldData + (size_t)world * v.worldDataStride;
}

namespace {
void packExports(Executor::Impl &I);
}

void Executor::uploadState()
{
    impl_->mgr->uploadToDevice(nullptr);
    int32_t num_exports = 0;
    const StateManager::ExportDesc *ex = impl_->mgr->exports(&num_exports);
    const StateView &v = impl_->mgr->hostView();
    for (int32_t i = 0; i < num_exports; i++) {
        CpuExport b;
        b.slot = ex[i].slot;
        b.archetype = ex[i].archetype;
        b.column = ex[i].column;
        b.bytes = ex[i].bytes;
        b.buf.assign((size_t)v.numWorlds * v.arch[b.archetype].capacity * b.bytes, 0);
        impl_->exports.push_back(std::move(b));
    }
    packExports(*impl_);                 // the initial state's rows (as the GPU executor)
}

void Executor::setGraph(TaskGraph &&graph)
{
    Impl &I = *impl_;
    I.graph = std::move(graph);
    const TaskGraph &g = I.graph;
    I.nodeData.assign(g.nodeDatas(), g.nodeDatas() + g.numNodeDatas());
    for (int32_t i = 0; i < g.numNodeDatas(); i++) {
        if (!g.nodeDataIsNodeBase(i)) continue;
        NodeBase *nb = (NodeBase *)I.nodeData[i].userData;
        nb->mwState = &I.mgr->hostView();
        nb->mwNumWorlds = I.cfg.numWorlds;
    }
    I.segs.clear();
    for (int32_t i = 0; i < g.numNodes(); i++) {
        const TaskGraph::NodeFns &f = g.nodeFns(i);
        if (!f.cpuWorld && !f.cpuGlobal) {
            throw std::runtime_error(std::string("CPU executor: node ") + g.nodeName(i) +
                                     " has no CPU implementation");
        }
        const bool global = f.cpuWorld == nullptr;
        if (I.segs.empty() || global || I.segs.back().global) I.segs.push_back({ global, {} });
        I.segs.back().nodes.push_back(i);
    }
}

namespace {

struct StepArg {
    Executor::Impl *I;
    CpuRunCtx *rc;
    const std::vector<int32_t> *nodes;
    const std::vector<uint8_t> *timed;       // per node of the segment: time it
};

void runWorlds(void *a, int64_t begin, int64_t end)
{
    StepArg &s = *(StepArg *)a;
    const TaskGraph &g = s.I->graph;
    for (int64_t w = begin; w < end; w++) {
        for (size_t k = 0; k < s.nodes->size(); k++) {
            const int32_t n = (*s.nodes)[k];
            const TaskGraph::NodeFns &f = g.nodeFns(n);
            if (s.timed && (*s.timed)[k]) {
                const auto t0 = std::chrono::steady_clock::now();
                f.cpuWorld(g.nodeState(n), *s.rc, (int32_t)w);
                const auto t1 = std::chrono::steady_clock::now();
                s.I->timedNs.fetch_add(
                    std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count(),
                    std::memory_order_relaxed);
            } else {
                f.cpuWorld(g.nodeState(n), *s.rc, (int32_t)w);
            }
        }
    }
}

void packExports(Executor::Impl &I)
{                                              // src/core/state.cpp:489-563
    StateView &v = I.mgr->hostView();
    for (CpuExport &b : I.exports) {
        const ArchetypeView &av = v.arch[b.archetype];
        int64_t off = 0;
        for (int32_t w = 0; w < v.numWorlds; w++) {
            const int64_t n = av.numRows[w];
            memcpy(b.buf.data() + off * b.bytes,
                   av.cols[b.column] + (size_t)w * av.capacity * b.bytes, (size_t)n * b.bytes);
            off += n;
        }
        b.rows = off;
    }
}

}

// Table growth between steps (the GPU executor's growTables, at every
// step here: the CPU back end steps synchronously): a growable table past
// half its capacity in any world doubles until at most half full.
static void growTables(Executor::Impl &I)
{
    StateView &v = I.mgr->hostView();
    for (int32_t a = 0; a < v.numArchetypes; a++) {
        if (!(v.arch[a].flags & kArchGrowable) || !I.mgr->growable(a)) continue;
        int32_t m = 0;
        for (int32_t w = 0; w < v.numWorlds; w++) m = std::max(m, v.arch[a].numRows[w]);
        const int32_t cap = v.arch[a].capacity;
        if ((int64_t)m * 2 <= cap) continue;
        int64_t nc = std::max(cap, 1);
        while ((int64_t)m * 2 > nc) nc *= 2;
        if (nc > (1 << 28)) throw std::runtime_error("table growth past 2^28 rows per world");
        I.mgr->growArchetype(a, (int32_t)nc, nullptr);
        for (CpuExport &b : I.exports) {
            if (b.archetype == a) b.buf.resize((size_t)v.numWorlds * nc * b.bytes, 0);
        }
    }
}

void Executor::runAsync()
{
    Impl &I = *impl_;
    CpuRunCtx rc { &I.mgr->hostView(), I.mgr.get(), I.cfg.numWorlds,
                   I.nodeData.empty() ? nullptr : (char *)I.nodeData.data(), I.pool.get() };
    const bool timing = !I.timedName.empty();
    for (const Impl::Segment &sg : I.segs) {
        if (sg.global) {
            const int32_t n = sg.nodes[0];
            const auto t0 = std::chrono::steady_clock::now();
            I.graph.nodeFns(n).cpuGlobal(I.graph.nodeState(n), rc);
            if (timing && I.timedMatch(n)) {
                I.timedNs += std::chrono::duration_cast<std::chrono::nanoseconds>(
                    std::chrono::steady_clock::now() - t0).count();
                I.timedLaunches++;
            }
            continue;
        }
        std::vector<uint8_t> timed;
        if (timing) {
            for (int32_t n : sg.nodes) {
                timed.push_back(I.timedMatch(n));
                I.timedLaunches += timed.back();
            }
        }
        StepArg arg { &I, &rc, &sg.nodes, timing ? &timed : nullptr };
        I.pool->parallelFor(I.cfg.numWorlds, 1, runWorlds, &arg);
    }
    packExports(I);
    growTables(I);
}

// Several steps world-major (every node world-local): each world runs n
// steps on one worker, then the exports are packed once -- the same states
// as n single steps, since worlds never read each other.
void Executor::runSteps(int32_t n)
{
    Impl &I = *impl_;
    if (n <= 0) return;
    const bool world_local = I.segs.size() == 1 && !I.segs[0].global;
    // growable tables grow between any two steps: one step at a time
    bool growable = false;
    const StateView &hv = I.mgr->hostView();
    for (int32_t a = 0; a < hv.numArchetypes; a++) growable |= I.mgr->growable(a);
    if (n == 1 || !world_local || !I.timedName.empty() || growable) {
        for (int32_t i = 0; i < n; i++) runAsync();
        return;
    }
    CpuRunCtx rc { &I.mgr->hostView(), I.mgr.get(), I.cfg.numWorlds,
                   I.nodeData.empty() ? nullptr : (char *)I.nodeData.data(), I.pool.get() };
    struct MultiArg {
        StepArg step;
        int32_t steps;
    } arg { StepArg { &I, &rc, &I.segs[0].nodes, nullptr }, n };
    // runs of neighbouring worlds per claim: a world's rows share cache lines
    // with its neighbours' at the edges of every column slab, and two
    // workers stepping neighbours n times each would trade those lines
    const int64_t chunk = std::max<int64_t>(1, I.cfg.numWorlds / (16 * (int64_t)I.pool->numThreads()));
    I.pool->parallelFor(I.cfg.numWorlds, chunk, [](void *a, int64_t begin, int64_t end) {
        MultiArg &m = *(MultiArg *)a;
        for (int64_t w = begin; w < end; w++) {
            for (int32_t s = 0; s < m.steps; s++) runWorlds(&m.step, w, w + 1);
        }
    }, &arg);
    packExports(I);
    growTables(I);
}

void Executor::sync() {}

void Executor::run() { runAsync(); }

void *Executor::getExported(int32_t slot, int64_t *num_rows)
{
    for (CpuExport &b : impl_->exports) {
        if (b.slot == slot) {
            if (num_rows) *num_rows = b.rows;
            return b.buf.data();
        }
    }
    return nullptr;
}

int64_t Executor::copyExported(int32_t slot, void *dst, int64_t max_bytes)
{
    for (CpuExport &b : impl_->exports) {
        if (b.slot != slot) continue;
        const int64_t span = std::min(std::max<int64_t>(max_bytes, 0), (int64_t)b.buf.size());
        if (span > 0) memcpy(dst, b.buf.data(), (size_t)span);
        return std::min(b.rows * (int64_t)b.bytes, span);
    }
    return -1;
}

int64_t Executor::copyExportedAsync(int32_t slot, void *dst, int64_t max_bytes)
{
    for (CpuExport &b : impl_->exports) {
        if (b.slot != slot) continue;
        const int64_t span = std::min(std::max<int64_t>(max_bytes, 0), (int64_t)b.buf.size());
        if (span > 0) memcpy(dst, b.buf.data(), (size_t)span);
        return span;
    }
    return -1;
}

void Executor::copyOutExports() { packExports(*impl_); }

int32_t Executor::exportRowBytes(int32_t slot)
{
    for (CpuExport &b : impl_->exports) {
        if (b.slot == slot) return (int32_t)b.bytes;
    }
    return 0;
}

int64_t Executor::exportBufferBytes(int32_t slot)
{
    for (CpuExport &b : impl_->exports) {
        if (b.slot == slot) return (int64_t)b.buf.size();
    }
    return -1;
}

void *Executor::columnBase(int32_t archetype, int32_t column, int32_t *capacity, uint32_t *bytes)
{
    const StateView &v = impl_->mgr->hostView();
    if (archetype < 0 || archetype >= v.numArchetypes) return nullptr;
    const ArchetypeView &av = v.arch[archetype];
    if (column < 0 || column >= av.numColumns) return nullptr;
    if (capacity) *capacity = av.capacity;
    if (bytes) *bytes = av.colBytes[column];
    return av.cols[column];
}

int32_t Executor::numRows(int32_t archetype, int32_t world)
{
    return impl_->mgr->hostView().arch[archetype].numRows[world];
}

double Executor::timeNode(const char *name, int32_t num_steps)
{
    Impl &I = *impl_;
    const std::string saved = I.timedName;
    const int32_t saved_index = I.timedIndex;
    const int64_t ns0 = I.timedNs.load(), l0 = I.timedLaunches;
    I.timedName = name ? name : "";
    I.timedIndex = -1;
    for (int32_t s = 0; s < num_steps; s++) runAsync();
    const int64_t ns = I.timedNs.load() - ns0, l = I.timedLaunches - l0;
    I.timedNs = ns0;
    I.timedLaunches = l0;
    I.timedName = saved;
    I.timedIndex = saved_index;
    // per launch = one run of the node over every world (summed worker time)
    return l > 0 ? (double)ns * 1e-6 / (double)l : -1.0;
}

void Executor::setTimedNode(const char *name, int32_t every)
{
    (void)every;   // host timing costs no graph split: every step is timed
    impl_->timedName = name ? name : "";
    impl_->timedIndex = -1;
    impl_->timedNs = 0;
    impl_->timedLaunches = 0;
}

void Executor::setTimedNodeIndex(int32_t node, int32_t every)
{
    if (node < 0 || node >= impl_->graph.numNodes()) {
        throw std::runtime_error("setTimedNodeIndex: node index past the graph");
    }
    setTimedNode(impl_->graph.nodeName(node), every);
    impl_->timedIndex = node;
}

double Executor::timedNodeMs(int64_t *launches)
{
    if (launches) *launches = impl_->timedLaunches;
    return (double)impl_->timedNs.load() * 1e-6;
}

void Executor::enableTracing(int64_t)
{
    throw std::runtime_error("device tracing is a gfx950 feature (libmadrona_mw.so)");
}

int64_t Executor::readTrace(void *, int64_t, int64_t *) { return -1; }
const char *Executor::traceFuncName(int32_t) { return nullptr; }

int32_t Executor::numNodes() const { return impl_->graph.numNodes(); }
int32_t Executor::worldWalkRuns() const { return 0; }
int32_t Executor::walkRunEnd(int32_t node) const { return node + 1; }

const char *Executor::nodeName(int32_t node) const
{
    if (node < 0 || node >= impl_->graph.numNodes()) throw std::runtime_error("no such node");
    return impl_->graph.nodeName(node);
}

int32_t Executor::nodeBlocksPerCU(int32_t) const { return 0; }

void Executor::setNodeBlocksPerCU(int32_t, int32_t)
{
    throw std::runtime_error("launch configuration is a gfx950 feature (libmadrona_mw.so)");
}

bool Executor::entityLoc(int32_t world, Entity e, Loc *out)
{
    StateView &v = impl_->mgr->hostView();
    if (world < 0 || world >= v.numWorlds) return false;
    const Loc l = v.ids(world).lookup(e);
    if (!l.valid()) return false;
    *out = l;
    return true;
}

void Executor::downloadState() {}
const StateView &Executor::hostView() { return impl_->mgr->hostView(); }

int32_t Executor::errorFlags()
{
    const StateView &v = impl_->mgr->hostView();
    int32_t r = 0;
    for (int32_t w = 0; w < v.numWorlds; w++) r |= v.errorFlags[w];
    return r;
}

}
