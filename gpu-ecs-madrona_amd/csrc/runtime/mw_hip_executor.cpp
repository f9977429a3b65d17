// MWHipExecutor: the reference's MWCudaExecutor surface (include/madrona/
// mw_gpu.hpp:20-76, src/mw/cuda_exec.cpp:1692-1815) over the framework's
// Executor.  Construction resolves CompileConfig::entryName in the world
// registry (loading the shared objects named in userSources first) and builds
// the executor from StateConfig's init records and user config; run() steps
// and synchronises like the reference's cuGraphLaunch + cudaStreamSynchronize.
#include <madrona/mw_gpu_entry.hpp>

#include <stdexcept>
#include <string>

namespace madrona {

static bool endsWith(const std::string &s, const char *suffix)
{
    const std::string suf(suffix);
    return s.size() >= suf.size() && s.compare(s.size() - suf.size(), suf.size(), suf) == 0;
}

static Executor *buildExecutor(const StateConfig &sc, const CompileConfig &cc)
{
    if (!cc.entryName) throw std::runtime_error("MWHipExecutor: CompileConfig::entryName is null");
    for (const char *src : cc.userSources) {
        // worlds compiled ahead of time: shared objects are loaded (a world
        // already registered by an earlier executor keeps its factory)
        if (src && endsWith(src, ".so") && !findEnv(cc.entryName)) loadEnvObject(src);
    }
    EnvFactory f = findEnv(cc.entryName);
    if (!f) {
        throw std::runtime_error(std::string("MWHipExecutor: no world registered as '") + cc.entryName +
                                 "' (build it with world.mk and name its .so in userSources)");
    }
    if (sc.numWorlds == 0) throw std::runtime_error("MWHipExecutor: numWorlds must be > 0");
    ExecConfig ec {};
    ec.numWorlds = (int32_t)sc.numWorlds;
    ec.gpuID = (int32_t)sc.gpuID;
    ec.defaultCapacity = 64;
    ec.numExportedBuffers = (int32_t)sc.numExportedBuffers;
    ec.useGraph = 1;
    return f(ec, sc.userConfigPtr, sc.userConfigPtr ? sc.numUserConfigBytes : 0, sc.worldInitPtr,
             sc.numWorldInitBytes);
}

MWHipExecutor::MWHipExecutor(const StateConfig &state_cfg, const CompileConfig &compile_cfg)
    : exec_(buildExecutor(state_cfg, compile_cfg))
{}

MWHipExecutor::MWHipExecutor(MWHipExecutor &&o) = default;
MWHipExecutor::~MWHipExecutor() = default;

int64_t MWHipExecutor::loadObjects(Span<const imp::SourceObject> objs)
{
    if (objs.size() == 0) return 0;
    throw std::runtime_error("MWHipExecutor::loadObjects: render objects need the batch renderer, "
                             "which this framework does not build (physics hulls: PhysicsLoader)");
}

void MWHipExecutor::run() { exec_->run(); }

uint8_t *MWHipExecutor::rgbObservations() const { return nullptr; }
float *MWHipExecutor::depthObservations() const { return nullptr; }

void *MWHipExecutor::getExported(int64_t slot) const
{
    return exec_->getExported((int32_t)slot, nullptr);
}

Executor &MWHipExecutor::executor() const { return *exec_; }

}
