// Physics asset path (reference include/madrona/physics_assets.hpp,
// src/physics/physics_assets.cpp:18-396): OBJ file -> half-edge convex hull
// -> object table handed to RigidBodyPhysicsSystem::init.
//
// MI355X design: the table stays on the host until RigidBodyPhysicsSystem
// flattens every hull into one device slab per attribute (vertices, planes,
// half edges, edge topology) at executor upload, so StorageType only names
// where the caller means the objects to end up; both values produce the same
// host table.
#pragma once

#include <madrona/physics.hpp>

#include <memory>

namespace madrona::phys {

class PhysicsLoader {
public:
    enum class StorageType {
        CPU,
        HIP,
        CUDA = HIP,      // source compatibility with the reference enum
    };

    PhysicsLoader(StorageType storage_type, CountT max_objects);
    ~PhysicsLoader();
    PhysicsLoader(PhysicsLoader &&o);

    struct LoadedHull {
        math::AABB aabb;
        geometry::HalfEdgeMesh collisionMesh;
    };

    // First mesh of the file (the reference asserts exactly one) as a
    // half-edge mesh plus its AABB (AABB::point + expand over the vertices).
    // Throws std::runtime_error where the reference calls FATAL.
    LoadedHull loadHullFromDisk(const char *obj_path);

    // Appends objects to the table; returns the index of the first one.
    CountT loadObjects(const RigidBodyMetadata *metadatas,
                       const math::AABB *aabbs,
                       const CollisionPrimitive *primitives,
                       CountT num_objs);

    ObjectManager &getObjectManager();

private:
    struct Impl;
    std::unique_ptr<Impl> impl_;
};

}
