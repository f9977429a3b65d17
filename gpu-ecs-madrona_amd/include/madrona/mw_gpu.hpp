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
#include <madrona/importer.hpp>

#include <functional>
#include <memory>
#include <new>
#include <vector>

namespace madrona {

inline constexpr int32_t kDefaultTmpAllocBytes = 16 * 1024;    // Context::tmpAlloc per world
inline constexpr int32_t kDefaultDeferredPerWorld = 256;        // deferred destroys per node per world

// Default chained tmpAlloc pool (device): twice the worlds' arenas, at least
// 16 MiB, at most 1 GiB.
inline int64_t defaultTmpPoolBytes(int32_t num_worlds, int32_t arena_bytes_per_world)
{
    const int64_t b = 2 * (int64_t)num_worlds * (arena_bytes_per_world > 0 ? arena_bytes_per_world : 0);
    return b < (16ll << 20) ? (16ll << 20) : (b > (1ll << 30) ? (1ll << 30) : b);
}

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
    int64_t tmpPoolBytes = -1;            // chained tmpAlloc pool past the per-world arenas:
                                          // -1: kDefaultTmpPoolBytes rule, 0: none
    int32_t serialNodes = 0;              // 1: every ParallelForNode / CustomParallelForNode
                                          // runs world-serially (WorldSerialForNode); the
                                          // CPU back end always does
};

namespace render {
// Reference mw_render.hpp camera modes (the batch renderer itself is out of
// scope); kept so StateConfig / ThreadPoolExecutor::Config
// aggregate-initialise exactly as the reference's drivers write them.
enum class CameraMode : uint32_t {
    Perspective,
    Lidar,
    None,
};
}

// Reference ThreadPoolExecutor::Config (include/madrona/mw_cpu.hpp:11-21),
// the first argument of the CPU TaskGraphExecutor.  Only numWorlds,
// numExportedBuffers and numWorkers drive the executor; the render fields
// are accepted and ignored (no renderer).
class ThreadPoolExecutor {
public:
    struct Config {
        uint32_t numWorlds;
        uint32_t maxViewsPerWorld;
        uint32_t maxInstancesPerWorld;
        uint32_t renderWidth;
        uint32_t renderHeight;
        uint32_t maxObjects;
        uint32_t numExportedBuffers;
        render::CameraMode cameraMode;
        int32_t renderGPUID;
        uint32_t numWorkers = 0;
    };
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
    // n steps, no sync.  gfx950: n graph replays.  CPU back end: when every
    // node is world-local, each worker steps its worlds n times in a row
    // (world-major: a world's state stays in the worker's caches), else n
    // single steps.
    void runSteps(int32_t n);
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
    // The same for one node of the graph (its index in sorted order), e.g.
    // one of several ParallelForNodes; throws on an index past the graph.
    void setTimedNodeIndex(int32_t node, int32_t every = 1);
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
    // World-walk launches per step (runs of world-local nodes walked by one
    // persistent kernel; MADRONA_MW_WORLD_WALK=1 when the graph is set).
    // 0 when off or on the CPU back end.
    int32_t worldWalkRuns() const;
    // The end of the walk run node `node` starts (one launch for nodes
    // [node, end)); node + 1 when it starts none.
    int32_t walkRunEnd(int32_t node) const;
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
    // Reference constructor (include/madrona/mw_cpu.hpp:54-63): numWorlds
    // worlds, numWorkers threads on the CPU back end (0: every core).
    TaskGraphExecutor(const ThreadPoolExecutor::Config &cfg, const ConfigT &user_cfg,
                      const InitT *user_inits)
        : TaskGraphExecutor(fromThreadPoolConfig(cfg), user_cfg, user_inits)
    {}

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

    // Reference TaskGraphExecutor::loadObjects feeds the batch renderer,
    // which is out of scope: refused with an error.
    int64_t loadObjects(Span<const imp::SourceObject> objs)
    {
        if (objs.size() == 0) return 0;
        throw std::runtime_error("loadObjects: render objects need the batch renderer, which this "
                                 "framework does not build (physics hulls: PhysicsLoader)");
    }
    uint8_t *rgbObservations() const { return nullptr; }
    float *depthObservations() const { return nullptr; }

private:
    static ExecConfig fromThreadPoolConfig(const ThreadPoolExecutor::Config &c)
    {
        ExecConfig e {};
        e.numWorlds = (int32_t)c.numWorlds;
        e.gpuID = 0;
        e.defaultCapacity = 64;
        e.numExportedBuffers = (int32_t)c.numExportedBuffers;
        e.useGraph = 1;
        e.numWorkers = (int32_t)c.numWorkers;
        return e;
    }
};

// ---------------------------------------------------------------------------
// Reference MWCudaExecutor (include/madrona/mw_gpu.hpp:20-76,
// src/mw/cuda_exec.cpp:1692-1815) on gfx950.  The reference NVRTC-compiles
// CompileConfig::userSources and finds the entry `entryName`; here worlds are
// compiled ahead of time, so entryName names a registered world (built in, or
// registered by an object built with world.mk) and every userSources entry
// that is a shared object (".so") is loaded first, as mw_load_env does.
// Other source entries and the compile flags / modes are accepted and unused.
// StateConfig: worldInitPtr holds numWorlds InitT records numWorldInitBytes
// apart, userConfigPtr the world's ConfigT (numUserConfigBytes must equal its
// size); the world data size / alignment come from the compiled WorldT.
// ---------------------------------------------------------------------------
struct StateConfig {
    void *worldInitPtr;
    uint32_t numWorldInitBytes;
    void *userConfigPtr;
    uint32_t numUserConfigBytes;
    uint32_t numWorldDataBytes;
    uint32_t worldDataAlignment;
    uint32_t numWorlds;
    uint32_t maxViewsPerWorld;
    uint32_t numExportedBuffers;
    uint32_t gpuID;
    render::CameraMode cameraMode;
    uint32_t renderWidth;
    uint32_t renderHeight;
};

struct CompileConfig {
    enum class OptMode : uint32_t {
        Optimize,
        LTO,
        Debug,
    };

    enum class Executor {
        JobSystem,
        TaskGraph,
    };

    const char *entryName;
    Span<const char *const> userSources;
    Span<const char *const> userCompileFlags;
    OptMode optMode = OptMode::LTO;
    Executor execMode = Executor::TaskGraph;
};

class MWHipExecutor {
public:
    MWHipExecutor(const StateConfig &state_cfg, const CompileConfig &compile_cfg);
    MWHipExecutor(MWHipExecutor &&o);
    ~MWHipExecutor();

    // Render objects go to the batch renderer in the reference (out of scope
    // here): an empty span returns 0, anything else throws.
    int64_t loadObjects(Span<const imp::SourceObject> objs);

    // One step of every world; returns when the step has finished (the
    // reference synchronises its stream, cuda_exec.cpp:1777-1782).
    void run();

    uint8_t *rgbObservations() const;     // no renderer: nullptr
    float *depthObservations() const;     // no renderer: nullptr

    // Device pointer of exported buffer `slot` (rows of all worlds,
    // world-major), valid after run().
    void *getExported(int64_t slot) const;

    // The framework executor behind it (C ABI, timing, tracing, ...).
    Executor &executor() const;

private:
    std::unique_ptr<Executor> exec_;
};

// The reference's class name, so a driver written against it compiles with
// only its includes changed.
using MWCudaExecutor = MWHipExecutor;

// Loads a shared object that registers worlds (mw_load_env); returns the
// number it registered, throws naming the object on failure or a name clash.
int32_t loadEnvObject(const char *so_path);

}
