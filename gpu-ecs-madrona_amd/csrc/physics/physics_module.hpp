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
