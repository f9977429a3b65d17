// PhysicsLoader (reference src/physics/physics_assets.cpp:18-396), host side.
#include <madrona/physics_assets.hpp>
#include <madrona/importer.hpp>

#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace madrona::phys {

using namespace math;

struct PhysicsLoader::Impl {
    StorageType storageType;
    CountT maxObjs;
    std::vector<RigidBodyMetadata> metadatas;
    std::vector<AABB> aabbs;
    std::vector<CollisionPrimitive> primitives;
    ObjectManager mgr {};
};

PhysicsLoader::PhysicsLoader(StorageType storage_type, CountT max_objects)
    : impl_(new Impl {})
{
    impl_->storageType = storage_type;
    impl_->maxObjs = max_objects;
    impl_->metadatas.reserve(max_objects);
    impl_->aabbs.reserve(max_objects);
    impl_->primitives.reserve(max_objects);
}

PhysicsLoader::~PhysicsLoader() = default;
PhysicsLoader::PhysicsLoader(PhysicsLoader &&o) = default;

PhysicsLoader::LoadedHull PhysicsLoader::loadHullFromDisk(const char *obj_path)
{                                                          // physics_assets.cpp:205-254
    std::string err;
    auto obj = imp::ImportedObject::importObject(obj_path, &err);
    if (!obj.has_value()) {
        throw std::runtime_error(std::string("Failed to load collision mesh from ") + obj_path +
                                 ": " + err);
    }
    if (obj->meshes.size() != 1) {
        throw std::runtime_error(std::string("collision mesh must hold exactly one mesh: ") +
                                 obj_path);
    }
    const imp::SourceMesh &m = obj->meshes[0];
    if (m.numVertices == 0) throw std::runtime_error("collision mesh has no vertices");

    uint32_t space = 0;
    for (uint32_t f = 0; f < m.numFaces; f++) space += m.faceCounts[f] + 1;
    geometry::FastPolygonList pl {};
    pl.allocate(space);
    uint32_t off = 0;
    for (uint32_t f = 0; f < m.numFaces; f++) {
        pl.addPolygon(Span<const uint32_t>(m.indices + off, m.faceCounts[f]));
        off += m.faceCounts[f];
    }
    LoadedHull out {};
    out.collisionMesh.construct(pl, m.numVertices, m.positions);
    pl.free();

    out.aabb = AABB { m.positions[0], m.positions[0] };      // AABB::point
    for (uint32_t v = 1; v < m.numVertices; v++) out.aabb.expand(m.positions[v]);
    return out;
}

CountT PhysicsLoader::loadObjects(const RigidBodyMetadata *metadatas, const AABB *aabbs,
                                  const CollisionPrimitive *primitives, CountT num_objs)
{                                                          // physics_assets.cpp:256-391
    Impl &I = *impl_;
    const CountT offset = (CountT)I.primitives.size();
    if (offset + num_objs > I.maxObjs) {
        throw std::runtime_error("PhysicsLoader: more objects than max_objects");
    }
    for (CountT i = 0; i < num_objs; i++) {
        I.metadatas.push_back(metadatas[i]);
        I.aabbs.push_back(aabbs[i]);
        I.primitives.push_back(primitives[i]);
    }
    I.mgr.metadata = I.metadatas.data();
    I.mgr.aabbs = I.aabbs.data();
    I.mgr.primitives = I.primitives.data();
    I.mgr.numObjects = (int32_t)I.primitives.size();
    return offset;
}

ObjectManager &PhysicsLoader::getObjectManager()
{
    return impl_->mgr;
}

}
