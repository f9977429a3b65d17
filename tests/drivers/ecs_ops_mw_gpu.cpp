// Host driver (TEST) shaped like the reference's examples/simple_taskgraph/
// gpu.cpp: it builds the ecs_ops world with the reference's GPU executor
// class, MWCudaExecutor(StateConfig, CompileConfig) (include/madrona/
// mw_gpu.hpp:20-76), naming the world by CompileConfig::entryName and its
// compiled object in userSources, steps NUM_TICKS ticks with run() and copies
// the exported Stats rows (getExported(0), device memory) to OUT.
//
//     ecs_ops_mw_gpu NUM_WORLDS NUM_TICKS WORLD_SO OUT
#include <madrona/mw_gpu.hpp>

#include <hip/hip_runtime.h>

#include "../ext_env/ecs_ops_init.hpp"
#include "../ext_env/ecs_ops_rules.hpp"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <exception>
#include <string>
#include <vector>

using namespace madrona;

static int run(int argc, char *argv[]);

int main(int argc, char *argv[])
{
    // the reference FATALs on a bad configuration; report it and exit
    try {
        return run(argc, argv);
    } catch (const std::exception &e) {
        fprintf(stderr, "error: %s\n", e.what());
        return EXIT_FAILURE;
    }
}

static int run(int argc, char *argv[])
{
    if (argc < 5) {
        fprintf(stderr, "Usage: %s NUM_WORLDS NUM_TICKS WORLD_SO OUT\n", argv[0]);
        return EXIT_FAILURE;
    }
    const int num_worlds = atoi(argv[1]);
    if (num_worlds < 1) {
        fprintf(stderr, "NUM_WORLDS must be >= 1");
        return EXIT_FAILURE;
    }
    const uint64_t num_ticks = std::stoul(argv[2]);

    std::vector<EcsOps::Init> env_inits(num_worlds);
    for (int i = 0; i < num_worlds; i++) env_inits[i].worldIndex = i;
    EcsOps::Config cfg { ecs_ops::kNumAgents };
    const char *world_so = argv[3];

    MWCudaExecutor train_exec({
        .worldInitPtr = env_inits.data(),
        .numWorldInitBytes = sizeof(EcsOps::Init),
        .userConfigPtr = &cfg,
        .numUserConfigBytes = sizeof(EcsOps::Config),
        .numWorldDataBytes = 0,
        .worldDataAlignment = 0,
        .numWorlds = uint32_t(num_worlds),
        .maxViewsPerWorld = 0,
        .numExportedBuffers = 1,
        .gpuID = 0,
        .cameraMode = render::CameraMode::None,
        .renderWidth = 0,
        .renderHeight = 0,
    }, {
        "EcsOps::World",
        { world_so },
        { },
        CompileConfig::OptMode::LTO,
        CompileConfig::Executor::TaskGraph,
    });

    void *stats_gpu = train_exec.getExported(0);
    printf("%p\n", stats_gpu);

    auto start = std::chrono::system_clock::now();
    for (int64_t i = 0; i < (int64_t)num_ticks; i++) train_exec.run();
    auto end = std::chrono::system_clock::now();
    std::chrono::duration<double> diff = end - start;
    printf("%f %f\n", double(num_ticks * num_worlds) / diff.count(), diff.count());

    std::vector<EcsOps::Stats> stats(num_worlds);
    if (hipMemcpy(stats.data(), stats_gpu, sizeof(EcsOps::Stats) * num_worlds,
                  hipMemcpyDeviceToHost) != hipSuccess) {
        fprintf(stderr, "hipMemcpy failed\n");
        return EXIT_FAILURE;
    }
    FILE *f = fopen(argv[4], "wb");
    if (!f || fwrite(stats.data(), sizeof(EcsOps::Stats), num_worlds, f) != (size_t)num_worlds) {
        fprintf(stderr, "cannot write %s\n", argv[4]);
        return EXIT_FAILURE;
    }
    fclose(f);
    return 0;
}
