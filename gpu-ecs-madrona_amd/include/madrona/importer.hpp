// OBJ mesh import (reference include/madrona/importer.hpp,
// src/common/importer.cpp:35-439), host only.  Feeds the physics asset path
// (PhysicsLoader::loadHullFromDisk, include/madrona/physics_assets.hpp).
#pragma once

#include <madrona/math.hpp>

#include <cstdint>
#include <optional>
#include <string>
#include <vector>

namespace madrona::imp {

struct SourceMesh {
    const math::Vector3 *positions;
    const math::Vector3 *normals;      // nullptr when the OBJ has none
    const math::Vector4 *tangentAndSigns;
    const math::Vector2 *uvs;          // nullptr when the OBJ has none
    const uint32_t *indices;
    const uint32_t *faceCounts;        // always set (the reference passes
                                       // nullptr for all-triangle meshes)
    uint32_t numVertices;
    uint32_t numFaces;
};

// One object of meshes (reference imp::SourceObject), the argument of
// MWCudaExecutor::loadObjects / TaskGraphExecutor::loadObjects.
struct SourceObject {
    const SourceMesh *meshes;
    int64_t numMeshes;
};

struct ImportedObject {
    std::vector<std::vector<math::Vector3>> positionArrays;
    std::vector<std::vector<math::Vector3>> normalArrays;
    std::vector<std::vector<math::Vector2>> uvArrays;
    std::vector<std::vector<uint32_t>> indexArrays;
    std::vector<std::vector<uint32_t>> faceCountArrays;
    std::vector<SourceMesh> meshes;

    // Loads an .obj file; std::nullopt (and *err set) on a malformed file or
    // an unknown extension, where the reference calls FATAL.
    static std::optional<ImportedObject> importObject(const char *path,
                                                      std::string *err = nullptr);
};

}
