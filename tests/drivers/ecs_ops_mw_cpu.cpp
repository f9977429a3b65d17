// Host driver (TEST) shaped like the reference's examples/*/mw_cpu.cpp: it
// builds the ecs_ops world with the reference's CPU executor class,
// TaskGraphExecutor(ThreadPoolExecutor::Config, ConfigT, InitT *)
// (include/madrona/mw_cpu.hpp:54-63), steps NUM_TICKS ticks with run() and
// writes the exported Stats rows (getExported(0)) to OUT.
//
//     ecs_ops_mw_cpu NUM_WORLDS NUM_TICKS OUT
#include <madrona/mw_cpu.hpp>

#include "../ext_env/ecs_ops.hip"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

using namespace madrona;

int main(int argc, char *argv[])
{
    if (argc < 4) {
        fprintf(stderr, "Usage: %s NUM_WORLDS NUM_TICKS OUT\n", argv[0]);
        return EXIT_FAILURE;
    }
    const int num_worlds = std::stoi(argv[1]);
    const uint64_t num_ticks = std::stoul(argv[2]);
    if (num_worlds < 1) {
        fprintf(stderr, "%s: num worlds must be > 0\n", argv[0]);
        return EXIT_FAILURE;
    }

    std::vector<EcsOps::Init> inits(num_worlds);
    for (int i = 0; i < num_worlds; i++) inits[i].worldIndex = i;
    const EcsOps::Config cfg { ecs_ops::kNumAgents };

    TaskGraphExecutor<EcsOps::Engine, EcsOps::World, EcsOps::Config, EcsOps::Init> exec({
        .numWorlds = uint32_t(num_worlds),
        .maxViewsPerWorld = 0,
        .maxInstancesPerWorld = 0,
        .renderWidth = 0,
        .renderHeight = 0,
        .maxObjects = 0,
        .numExportedBuffers = 1,
        .cameraMode = render::CameraMode::None,
        .renderGPUID = -1,
        .numWorkers = 2,
    }, cfg, inits.data());

    auto start = std::chrono::steady_clock::now();
    for (uint64_t i = 0; i < num_ticks; i++) exec.run();
    auto end = std::chrono::steady_clock::now();
    const double elapsed = std::chrono::duration<double>(end - start).count();
    printf("FPS: %f, Elapsed: %f\n", double(num_ticks) * num_worlds / elapsed, elapsed);

    const EcsOps::Stats *stats = (const EcsOps::Stats *)exec.getExported(0);
    FILE *f = fopen(argv[3], "wb");
    if (!f || fwrite(stats, sizeof(EcsOps::Stats), num_worlds, f) != (size_t)num_worlds) {
        fprintf(stderr, "%s: cannot write %s\n", argv[0], argv[3]);
        return EXIT_FAILURE;
    }
    fclose(f);
    return 0;
}
