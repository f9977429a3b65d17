// Shared asset table of the physics environments: object 0 = unit cube hull
// (half extent 1, the 2-unit cube of examples/collisions/collisions.cpp:
// 100-109), object 1 = ground plane.  Built through the same half-edge
// construction the reference uses (src/physics/geometry.cpp:52-194).
#pragma once

#include <madrona/physics.hpp>
#include <madrona/physics_assets.hpp>
#include "../../../include/madrona_mw.h"

#include <cfloat>
#include <string>
#include <vector>

namespace madrona::envs {

// Object table: 0 = cube hull (half extent 1), 1 = ground plane.
inline phys::ObjectManager *makeCubeObjectManager(const mw_collisions_config &c)
{
    using namespace phys;
    using namespace math;
    auto *mgr = new ObjectManager {};
    mgr->numObjects = 2;
    mgr->metadata = new RigidBodyMetadata[2];
    mgr->aabbs = new AABB[2];
    mgr->primitives = new CollisionPrimitive[2];

    const Vector3 verts[8] = {
        { -1, -1, -1 }, { 1, -1, -1 }, { 1, 1, -1 }, { -1, 1, -1 },
        { -1, -1, 1 }, { 1, -1, 1 }, { 1, 1, 1 }, { -1, 1, 1 },
    };
    const uint32_t faces[6][4] = {
        { 0, 3, 2, 1 }, { 4, 5, 6, 7 }, { 0, 1, 5, 4 },
        { 3, 7, 6, 2 }, { 0, 4, 7, 3 }, { 1, 2, 6, 5 },
    };
    geometry::FastPolygonList pl {};
    pl.allocate(6 * 5);
    for (int f = 0; f < 6; f++) pl.addPolygon(Span<const uint32_t>(faces[f], 4));
    mgr->primitives[0].type = CollisionPrimitive::Type::Hull;
    mgr->primitives[0].hull.halfEdgeMesh.construct(pl, 8, verts);
    pl.free();
    mgr->metadata[0] = RigidBodyMetadata {
        { c.cube_inv_inertia, c.cube_inv_inertia, c.cube_inv_inertia }, c.cube_inv_mass,
        c.mu_s, c.mu_d };
    mgr->aabbs[0] = AABB { { -1, -1, -1 }, { 1, 1, 1 } };

    mgr->primitives[1].type = CollisionPrimitive::Type::Plane;
    mgr->metadata[1] = RigidBodyMetadata { { 0.f, 0.f, 0.f }, 0.f, c.mu_s, c.mu_d };
    mgr->aabbs[1] = AABB { { -FLT_MAX, -FLT_MAX, -FLT_MAX }, { FLT_MAX, FLT_MAX, 0.f } };
    return mgr;
}

inline std::vector<std::string> splitHullPaths(const char *paths)
{
    std::vector<std::string> out;
    if (!paths) return out;
    std::string cur;
    for (const char *p = paths;; p++) {
        if (*p == ';' || *p == '\0') {
            if (!cur.empty()) out.push_back(cur);
            cur.clear();
            if (*p == '\0') break;
        } else {
            cur.push_back(*p);
        }
    }
    return out;
}

// Object table from OBJ hulls through the asset path (PhysicsLoader, the
// reference's physics_assets.cpp flow): objects 0..n-1 = the hulls (mass
// properties from the config), object n = ground plane.  The loader (and
// with it the table) lives as long as the process, like the cube table.
inline phys::ObjectManager *makeHullObjectManager(const mw_collisions_config &c,
                                                  const std::vector<std::string> &paths)
{
    using namespace phys;
    using namespace math;
    const CountT n = (CountT)paths.size();
    auto *loader = new PhysicsLoader(PhysicsLoader::StorageType::HIP, n + 1);
    std::vector<RigidBodyMetadata> meta;
    std::vector<AABB> aabbs;
    std::vector<CollisionPrimitive> prims(n + 1);
    for (CountT i = 0; i < n; i++) {
        PhysicsLoader::LoadedHull h = loader->loadHullFromDisk(paths[i].c_str());
        prims[i].type = CollisionPrimitive::Type::Hull;
        prims[i].hull.halfEdgeMesh = h.collisionMesh;
        aabbs.push_back(h.aabb);
        meta.push_back(RigidBodyMetadata {
            { c.cube_inv_inertia, c.cube_inv_inertia, c.cube_inv_inertia }, c.cube_inv_mass,
            c.mu_s, c.mu_d });
    }
    prims[n].type = CollisionPrimitive::Type::Plane;
    meta.push_back(RigidBodyMetadata { { 0.f, 0.f, 0.f }, 0.f, c.mu_s, c.mu_d });
    aabbs.push_back(AABB { { -FLT_MAX, -FLT_MAX, -FLT_MAX }, { FLT_MAX, FLT_MAX, 0.f } });
    loader->loadObjects(meta.data(), aabbs.data(), prims.data(), n + 1);
    return &loader->getObjectManager();
}

}
