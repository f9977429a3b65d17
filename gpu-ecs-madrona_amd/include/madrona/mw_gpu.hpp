// MI355X multi-world executor.
//
// Reference interfaces: MWCudaExecutor (include/madrona/mw_gpu.hpp:20-76,
// src/mw/cuda_exec.cpp:1692-1815) and TaskGraphExecutor (include/madrona/
// mw_cpu.hpp:53-81, mw_cpu.inl).  The reference JIT-compiles user sources
// with NVRTC at executor construction; here the environment is compiled ahead
// of time by hipcc for gfx950 and the executor is a template over the world
// type, exactly like TaskGraphExecutor<ContextT, WorldT, ConfigT, InitT>.
//
// Construction (host):  registerTypes -> finalize arena -> per-world WorldT
// ctor into the host mirror (IDs as the reference computes them) -> upload ->
// setupTasks / build -> capture the step into a hipGraph.
// run():  one hipGraphLaunch on the executor's stream (+ sync unless async).
#pragma once

#include <madrona/taskgraph.hpp>

#include <functional>
#include <memory>
#include <new>
#include <vector>

namespace madrona {

inline constexpr int32_t kDefaultTmpAllocBytes = 16 * 1024;    // Context::tmpAlloc per world
inline constexpr int32_t kDefaultDeferredPerWorld = 256;        // deferred destroys per node per world
inline constexpr int32_t kCommitMaxRows = 4096;                 // ordered-commit table limit

struct ExecConfig {
    int32_t numWorlds;
    int32_t gpuID;
    int32_t defaultCapacity;        // rows per world per archetype
    int32_t numExportedBuffers;
    int32_t useGraph;               // capture the step into a hipGraph
    int32_t tmpAllocBytesPerWorld = -1;   // -1: kDefaultTmpAllocBytes, 0: no arena
    int32_t maxDeferredPerWorld = 0;      // 0: kDefaultDeferredPerWorld
    int32_t numWorkers = 0;               // CPU back end: worker threads (0: every core
                                          // of the process's affinity mask)
    int32_t serialNodes = 0;              // 1: every ParallelForNode / CustomParallelForNode
                                          // runs world-serially (WorldSerialForNode); the
                                          // CPU back end always does
};

// Non-template core (csrc/runtime/executor.cpp).
class Executor {
public:
    explicit Executor(const ExecConfig &cfg);
    ~Executor();

    StateManager &stateManager();
    ECSRegistry registry();

    // Phase hooks used by the TaskGraphExecutor template below.
    void finalizeRegistration(uint32_t world_bytes, uint32_t world_align);
    Context makeHostContext(int32_t world);
    char *hostWorldData(int32_t world);
    void uploadState();
    void setGraph(TaskGraph &&graph);

    void run();                               // step + sync
    void runAsync();                          // step, no sync
    void sync();
    void *stream() const;

    // Packed export (reference getExported contract: rows of all worlds,
    // world-major).  Valid after run().
    void *getExported(int32_t slot, int64_t *num_rows = nullptr);
    // Stream-ordered copy of export `slot` into dst (device or host), one
    // sync; returns the bytes of packed rows copied (-1: no such slot).
    int64_t copyExported(int32_t slot, void *dst, int64_t max_bytes);
    // Same copy (device destination), enqueued without a host wait.
    int64_t copyExportedAsync(int32_t slot, void *dst, int64_t max_bytes);
    void copyOutExports();
    int32_t exportRowBytes(int32_t slot);
    int64_t exportBufferBytes(int32_t slot);  // capacity of the packed buffer

    // Raw column access (device pointer of a [world][capacity] slab).
    void *columnBase(int32_t archetype, int32_t column, int32_t *capacity, uint32_t *bytes);
    int32_t numRows(int32_t archetype, int32_t world);
    void downloadState();
    // IDMap lookup of a live entity (false: not alive).
    bool entityLoc(int32_t world, Entity e, Loc *out);
    const StateView &hostView();
    int32_t numWorlds() const;
    int32_t errorFlags();                     // OR of per-world error flags

    // Eagerly run num_steps steps with HIP events around every launch of the
    // node kind `name` (on the executor stream); mean ms per launch.
    double timeNode(const char *name, int32_t num_steps);
    // Live timing of one node kind inside the replayed step (HIP events on
    // the executor stream); setTimedNode re-captures the graph and resets.
    // every > 1: only every every-th step (the first of each run of
    // `every`) is split and timed, the others replay the unsplit graph.
    void setTimedNode(const char *name, int32_t every = 1);
    double timedNodeMs(int64_t *launches);

    // Device tracing (reference mw_gpu/tracing.hpp): records of every step
    // run after this call, up to max_records 40-byte DeviceLogs in total (0
    // disables); re-captures the step graph with the node markers.
    void enableTracing(int64_t max_records);
    // Copies the records so far (all traced steps, in log order) into dst;
    // returns their byte size (-1 when tracing is off).
    int64_t readTrace(void *dst, int64_t max_bytes, int64_t *dropped);
    const char *traceFuncName(int32_t func_id);

    // Per-node launch configuration (reference MADRONA_MWGPU_EXEC_CONFIG_*,
    // also read from the environment when the graph is set): blocks per CU
    // for the node's grid-stride / persistent kernels, 0 = full grid;
    // node -1 = the default of every node without its own value (-1 there:
    // use the default).  Setting re-captures the step graph.
    // Device-side arguments of the ordered structural commit (executor.hip).
    const void *commitArgs() const;

    int32_t numNodes() const;
    const char *nodeName(int32_t node) const;
    int32_t nodeBlocksPerCU(int32_t node) const;
    void setNodeBlocksPerCU(int32_t node, int32_t blocks_per_cu);

    struct Impl;
private:
    std::unique_ptr<Impl> impl_;
};

template <typename ContextT, typename WorldT, typename ConfigT, typename InitT>
class TaskGraphExecutor : public Executor {
public:
    TaskGraphExecutor(const ExecConfig &cfg, const ConfigT &user_cfg, const InitT *user_inits)
        : Executor(cfg)
    {
        ECSRegistry reg = registry();
        WorldT::registerTypes(reg, user_cfg);
        finalizeRegistration((uint32_t)sizeof(WorldT), (uint32_t)alignof(WorldT));

        for (int32_t w = 0; w < cfg.numWorlds; w++) {
            Context base = makeHostContext(w);
            WorldT *world = (WorldT *)hostWorldData(w);
            ContextT ctx(world, WorkerInit { &stateManager().hostView(), w, &stateManager() });
            new (world) WorldT(ctx, user_cfg, user_inits[w]);
            (void)base;
        }

        uploadState();

        WorldT *world0 = (WorldT *)hostWorldData(0);
        ContextT ctx0(world0, WorkerInit { &stateManager().hostView(), 0, &stateManager() });
        TaskGraph::Builder builder(ctx0);
        WorldT::setupTasks(builder, user_cfg);
        setGraph(builder.build());
    }
};

}
