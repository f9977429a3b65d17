// Host side of the physics module shared by the gfx950 library
// (physics.hip) and the CPU back end (physics_cpu.cpp): the per-world slabs
// of PhysArgs are allocated by the back end (device memory or host memory)
// and filled by buildArgs from the arena's column slabs.
#pragma once

#include <madrona/mw_gpu.hpp>
#include <madrona/physics.hpp>

#include "physics_impl.hpp"

#include <algorithm>
#include <stdexcept>
#include <vector>

namespace madrona::phys {

struct PhysicsModule : StateExtension {
    StateManager *mgr = nullptr;
    int32_t numWorlds = 0;
    bool initialized = false;
    int32_t maxLeaves = 0;
    int32_t maxNodes = 0;
    int32_t maxContacts = 0;
    int32_t maxJoints = 0;
    int32_t candCapacity = 0;

    std::vector<Entity> leafEntitiesHost;        // [W][maxLeaves]

    // flattened object table (host staging)
    std::vector<RigidBodyMetadata> metadata;
    std::vector<math::AABB> aabbs;
    std::vector<uint32_t> types;
    std::vector<HullDev> hulls;
    std::vector<math::Vector3> vertices;
    std::vector<geometry::Plane> planes;
    std::vector<geometry::HalfEdge> hedges;
    std::vector<uint32_t> edges;
    std::vector<uint32_t> polygons;
    std::vector<EdgeQuad> edgeQuads;

    PhysArgs args {};
    std::vector<void *> allocs;
    bool uploaded = false;

    // Solver lanes per world (SolverNode): 64 (lanes64, one world per wave)
    // or 32 (lanes32, two worlds per wave).  MADRONA_MW_SOLVER_LANES = 64 /
    // 32 fixes it; by default (auto) the GPU executor starts at 64 and, at
    // synchronisations from kSolverLanesAfterSteps steps on and at most every
    // kSolverLanesEvery steps, reads the level widths of the worlds' last
    // solve (PhysArgs::solverLevelStats): levels of at most kSolverNarrowLevel
    // items on average take 32 lanes -- half a wave's lanes would idle in
    // every level pass --, of at least kSolverWideLevel 64 (the gap keeps a
    // borderline workload from switching back and forth); a change re-captures
    // the step (poll).  Both variants give the same bits, so a switch changes
    // nothing but speed.
    static constexpr int64_t kSolverLanesAfterSteps = 24;
    static constexpr int64_t kSolverLanesEvery = 64;
    // measured (8192 worlds, settled windows): simple_taskgraph's chains
    // average 5.3-5.6 items per level and run 0.370 ms per solver launch on
    // 32 lanes against 0.398 on 64; collisions' 34-35 run 0.265 on 32
    // against 0.225 on 64 (its first 150 steps, cubes still landing, read
    // 4-15)
    static constexpr double kSolverNarrowLevel = 12.0;
    static constexpr double kSolverWideLevel = 20.0;
    int32_t solverLanes = 64;
    int32_t solverLanesMode = 0;       // 0 auto, 32 / 64 fixed
    int64_t solverLanesNextCheck = kSolverLanesAfterSteps;
    double solverItemsPerLevel = 0.0;  // what the last check read
    char *solverImages[2] = {};        // global-image slabs: [0] lanes64, [1] lanes32
    bool poll(void *stream, int64_t steps) override;

    ~PhysicsModule() override;

    // Back-end memory (zero-filled) and host -> slab copies.
    void *rawAlloc(size_t bytes, void *stream);
    void rawCopy(void *dst, const void *src, size_t bytes, void *stream);

    template <typename T>
    T *alloc(size_t count, void *stream)
    {
        return (T *)rawAlloc(std::max<size_t>(count * sizeof(T), 256), stream);
    }

    template <typename T>
    T *upload(const std::vector<T> &v, void *stream)
    {
        T *p = alloc<T>(v.size(), stream);
        if (!v.empty()) rawCopy(p, v.data(), sizeof(T) * v.size(), stream);
        return p;
    }

    // PhysArgs from the arena (StateManager::deviceViewHost) + module slabs.
    void buildArgs(void *stream);
    // Back end: buildArgs plus its own launch sizing.
    void upload(void *stream_ptr) override;
    // A growable non-body table can grow the entity ID store: the solver's
    // and the narrowphase's entity lookups follow it (the graphs that hold
    // `args` are re-captured after the growth).
    void stateResized() override
    {
        if (!uploaded || !initialized) return;
        const StateView &dv = mgr->deviceViewHost();
        args.idNodes = dv.idNodes;
        args.idsPerWorld = dv.idsPerWorld;
    }
};

PhysicsModule &physicsModule(StateManager &mgr);
StateManager &ctxManager(Context &ctx);

}
