// OBJ import, restating the reference loader (src/common/importer.cpp:35-439):
// 'v' / 'vn' / 'vt' records, 'f' records of pos[/uv[/normal]] 1-based
// indices, 'o' starts a new mesh.  Each mesh is un-indexed and re-indexed by
// unique (position, normal, uv) tuples in order of first use -- the remap
// meshopt_generateVertexRemapMulti computes (bitwise vertex equality).
// Floats parse with strtof (correctly rounded, like fast_float).
#include <madrona/importer.hpp>

#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <tuple>

namespace madrona::imp {

using namespace math;

namespace {

struct ObjIdx {
    uint32_t pos, normal, uv;
};

bool readFloats(const char *s, const char *end, float *out, int n)
{
    for (int i = 0; i < n; i++) {
        while (s < end && *s == ' ') s++;
        char *e = nullptr;
        float v = strtof(s, &e);
        if (e == s) return false;
        out[i] = v;
        s = e;
    }
    return true;
}

const char *readU32(const char *s, const char *end, uint32_t *out)
{
    uint64_t v = 0;
    const char *p = s;
    while (p < end && *p >= '0' && *p <= '9') {
        v = v * 10 + (uint64_t)(*p - '0');
        if (v > 0xffffffffull) return s;
        p++;
    }
    *out = (uint32_t)v;
    return p;
}

// readIdxTriple (importer.cpp:131-191)
const char *readIdxTriple(const char *s, const char *end, ObjIdx *idx, bool *ok)
{
    *idx = ObjIdx { 0, 0, 0 };
    const char *p = readU32(s, end, &idx->pos);
    if (p == s) { *ok = false; return end; }
    if (p == end || *p != '/') return p;
    p++;
    if (p < end && *p == '/') {
        idx->uv = 0;
    } else {
        const char *q = readU32(p, end, &idx->uv);
        if (q == p) { *ok = false; return end; }
        p = q;
    }
    if (p == end || *p != '/') return p;
    p++;
    const char *q = readU32(p, end, &idx->normal);
    if (q == p) { *ok = false; return end; }
    return q;
}

struct VertexKey {
    uint32_t bits[8];
    bool operator<(const VertexKey &o) const { return memcmp(bits, o.bits, sizeof(bits)) < 0; }
};

}

std::optional<ImportedObject> ImportedObject::importObject(const char *path, std::string *err)
{
    auto fail = [&](const std::string &msg) -> std::optional<ImportedObject> {
        if (err) *err = msg;
        return std::nullopt;
    };
    const char *dot = strrchr(path, '.');
    if (!dot || strcmp(dot + 1, "obj") != 0) return fail("unsupported extension (only .obj)");
    std::ifstream file(path);
    if (!file) return fail(std::string("cannot open ") + path);

    ImportedObject out;
    std::vector<Vector3> positions, normals;
    std::vector<Vector2> uvs;
    std::vector<ObjIdx> indices;
    std::vector<uint32_t> face_counts;

    // commitMesh (importer.cpp:205-350)
    auto commit = [&]() -> bool {
        if (indices.empty()) return positions.empty() && normals.empty() && uvs.empty();
        const bool has_n = indices[0].normal > 0, has_uv = indices[0].uv > 0;
        std::map<VertexKey, uint32_t> remap;
        std::vector<Vector3> new_pos, new_n;
        std::vector<Vector2> new_uv;
        std::vector<uint32_t> new_idx;
        new_idx.reserve(indices.size());
        for (const ObjIdx &ix : indices) {
            if (ix.pos == 0 || ix.pos - 1 >= positions.size()) return false;
            // every vertex must agree on having a normal / uv (:219-240)
            if ((ix.normal > 0) != has_n || (ix.uv > 0) != has_uv) return false;
            if (has_n && ix.normal - 1 >= normals.size()) return false;
            if (has_uv && ix.uv - 1 >= uvs.size()) return false;
            VertexKey k {};
            Vector3 p = positions[ix.pos - 1];
            memcpy(k.bits, &p, 12);
            if (has_n) memcpy(k.bits + 3, &normals[ix.normal - 1], 12);
            if (has_uv) memcpy(k.bits + 6, &uvs[ix.uv - 1], 8);
            auto it = remap.find(k);
            if (it == remap.end()) {
                it = remap.emplace(k, (uint32_t)new_pos.size()).first;
                new_pos.push_back(p);
                if (has_n) new_n.push_back(normals[ix.normal - 1]);
                if (has_uv) new_uv.push_back(uvs[ix.uv - 1]);
            }
            new_idx.push_back(it->second);
        }
        out.positionArrays.push_back(std::move(new_pos));
        out.normalArrays.push_back(std::move(new_n));
        out.uvArrays.push_back(std::move(new_uv));
        out.indexArrays.push_back(std::move(new_idx));
        out.faceCountArrays.push_back(face_counts);
        positions.clear();
        normals.clear();
        uvs.clear();
        indices.clear();
        face_counts.clear();
        return true;
    };

    std::string line;
    while (std::getline(file, line)) {
        if (line.empty() || line[0] == '#' || line[0] == 's') continue;
        const char *s = line.data(), *end = line.data() + line.size();
        if (line[0] == 'o') {
            if (!commit()) return fail("invalid mesh before 'o'");
        } else if (line[0] == 'v' && line.size() > 1) {
            float f[3];
            if (line[1] == ' ') {
                if (!readFloats(s + 1, end, f, 3)) return fail("bad 'v' record: " + line);
                positions.push_back(Vector3 { f[0], f[1], f[2] });
            } else if (line[1] == 'n') {
                if (!readFloats(s + 2, end, f, 3)) return fail("bad 'vn' record: " + line);
                normals.push_back(Vector3 { f[0], f[1], f[2] });
            } else if (line[1] == 't') {
                if (!readFloats(s + 2, end, f, 2)) return fail("bad 'vt' record: " + line);
                uvs.push_back(Vector2 { f[0], f[1] });
            }
        } else if (line[0] == 'f') {
            const char *p = s + 1;
            uint32_t count = 0;
            bool ok = true;
            while (true) {
                while (p < end && (*p == ' ' || *p == '\r')) p++;
                if (p == end) break;
                ObjIdx ix;
                p = readIdxTriple(p, end, &ix, &ok);
                if (!ok) return fail("bad 'f' record: " + line);
                indices.push_back(ix);
                count++;
            }
            if (count == 0) return fail("empty face");
            face_counts.push_back(count);
        }
    }
    if (!commit()) return fail("invalid mesh");

    for (size_t m = 0; m < out.positionArrays.size(); m++) {
        out.meshes.push_back(SourceMesh {
            out.positionArrays[m].data(),
            out.normalArrays[m].empty() ? nullptr : out.normalArrays[m].data(),
            nullptr,
            out.uvArrays[m].empty() ? nullptr : out.uvArrays[m].data(),
            out.indexArrays[m].data(),
            out.faceCountArrays[m].data(),
            (uint32_t)out.positionArrays[m].size(),
            (uint32_t)out.faceCountArrays[m].size(),
        });
    }
    return out;
}

}
