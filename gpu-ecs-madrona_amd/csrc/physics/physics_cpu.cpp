// CPU back end of the rigid-body physics module (libmadrona_cpu.so): the
// reference's per-world physics step, run world by world on the CPU
// executor's pinned workers (reference TaskGraphExecutor + ThreadPoolExecutor,
// include/madrona/mw_cpu.hpp:53-81, src/mw/cpu_exec.cpp:162-284).
//
// Every function restates the reference CPU path it cites, serially per world
// and in the reference's iteration order (body rows in query order, candidates
// in BVH traversal order, contacts in narrowphase append order, Gauss-Seidel
// in contact order), over the same arena columns and module slabs the gfx950
// kernels use (PhysArgs with host pointers).  The float evaluation order is
// the one include/madrona/math.hpp fixes for both back ends; the library is
// built with -ffp-contract=off and no fast-math (Makefile, cpu target).
#include "physics_module.hpp"

#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <utility>

namespace madrona::phys {

using namespace math;
using namespace base;

bool PhysicsModule::poll(void *, int64_t) { return false; }   // one world per worker: no lanes

PhysicsModule::~PhysicsModule()
{
    for (void *p : allocs) free(p);
}

void *PhysicsModule::rawAlloc(size_t bytes, void *)
{
    void *p = aligned_alloc(256, (bytes + 255) & ~size_t(255));
    if (!p) throw std::runtime_error("physics: host allocation failed");
    memset(p, 0, bytes);
    allocs.push_back(p);
    return p;
}

void PhysicsModule::rawCopy(void *dst, const void *src, size_t bytes, void *)
{
    memcpy(dst, src, bytes);
}

void PhysicsModule::upload(void *stream_ptr)
{
    if (!initialized) return;
    buildArgs(stream_ptr);
    uploaded = true;
}

namespace {

// ---------------------------------------------------------------------------
// Body access (Cols ABI: Position .. LeafID are columns 1..12)
// ---------------------------------------------------------------------------
struct Body {
    const BodyArch *B;
    size_t i;                       // w * capacity + row

    template <typename T>
    T &col(CountT c) const { return ((T *)B->cols[c])[i]; }
    Entity &entity() const { return ((Entity *)B->cols[0])[i]; }
    Vector3 &pos() const { return col<Vector3>(Cols::Position); }
    Quat &rot() const { return col<Quat>(Cols::Rotation); }
    Diag3x3 &scale() const { return col<Diag3x3>(Cols::Scale); }
    Velocity &vel() const { return col<Velocity>(Cols::Velocity); }
    int32_t obj() const { return col<ObjectID>(Cols::ObjectID).idx; }
    ResponseType resp() const { return col<ResponseType>(Cols::ResponseType); }
    solver::SubstepPrevState &prev() const { return col<solver::SubstepPrevState>(Cols::SubstepPrevState); }
    solver::PreSolvePositional &psPos() const { return col<solver::PreSolvePositional>(Cols::PreSolvePositional); }
    solver::PreSolveVelocity &psVel() const { return col<solver::PreSolveVelocity>(Cols::PreSolveVelocity); }
    Vector3 &extF() const { return col<Vector3>(Cols::ExternalForce); }
    Vector3 &extT() const { return col<Vector3>(Cols::ExternalTorque); }
    int32_t leaf() const { return col<broadphase::LeafID>(Cols::LeafID).id; }
};

Body bodyAt(const PhysArgs &P, int32_t w, Loc l)
{
    for (int32_t a = 0; a < P.numBodyArchs; a++) {
        if (P.body[a].archetype == (int32_t)l.archetype) {
            return Body { &P.body[a], (size_t)w * P.body[a].capacity + l.row };
        }
    }
    throw std::runtime_error("physics: Loc outside the physics body archetypes");
}

// Rows of every body archetype in query order (archetype order, table rows).
template <typename Fn>
void forEachBody(const PhysArgs &P, int32_t w, Fn &&fn)
{
    for (int32_t a = 0; a < P.numBodyArchs; a++) {
        const BodyArch &B = P.body[a];
        const int32_t n = B.numRows[w];
        for (int32_t r = 0; r < n; r++) fn(Body { &B, (size_t)w * B.capacity + r }, r);
    }
}

Loc lookup(const PhysArgs &P, int32_t w, Entity e)
{
    if (e.id < 0 || e.id >= P.idsPerWorld) return Loc::none();
    const IDNode &n = P.idNodes[(size_t)w * P.idsPerWorld + e.id];
    return n.gen == e.gen ? n.val : Loc::none();
}

Vector3 multDiag(Vector3 d, Vector3 v) { return Vector3 { d.x * v.x, d.y * v.y, d.z * v.z }; }

// ---------------------------------------------------------------------------
// Broadphase (src/physics/broadphase.cpp)
// ---------------------------------------------------------------------------
AABB expandAABBWithMotion(AABB aabb, const Vector3 &v, float vel_exp, float acc_exp)
{                                                         // broadphase.cpp:435-459
    for (int32_t i = 0; i < 3; i++) {
        float pos_delta = vel_exp * v[i];
        float min_delta = pos_delta - acc_exp;
        float max_delta = pos_delta + acc_exp;
        if (min_delta < 0.f) aabb.pMin[i] += min_delta;
        if (max_delta > 0.f) aabb.pMax[i] += max_delta;
    }
    return aabb;
}

void updateLeafPositions(const PhysArgs &P, int32_t w)   // broadphase.cpp:858-873, 461-480
{
    const broadphase::BVH &bvh = P.bvh[w];
    forEachBody(P, w, [&](Body b, int32_t) {
        const int32_t leaf = b.leaf();
        if (leaf < 0 || leaf >= P.maxLeaves) {
            P.errorFlags[w] |= kErrIndexGuard;
            return;
        }
        AABB world_aabb = P.objs.aabbs[b.obj()].applyTRS(b.pos(), b.rot(), b.scale());
        const size_t li = (size_t)w * P.maxLeaves + leaf;
        P.leafAABBs[li] = expandAABBWithMotion(world_aabb, b.vel().linear,
                                               bvh.leafVelocityExpansion, bvh.leafAccelExpansion);
        P.sortedLeaves[li] = leaf;
    });
}

int32_t midpointSplit(const AABB *aabbs, int32_t *sorted, int32_t base, int32_t n)
{                                                         // broadphase.cpp:106-170
    auto center = [&](int32_t i) {
        const AABB &a = aabbs[sorted[base + i]];
        return (a.pMin + a.pMax) / 2.f;
    };
    Vector3 cmin { FLT_MAX, FLT_MAX, FLT_MAX };
    Vector3 cmax { -FLT_MAX, -FLT_MAX, -FLT_MAX };
    for (int32_t i = 0; i < n; i++) {
        Vector3 c = center(i);
        cmin = Vector3::min(cmin, c);
        cmax = Vector3::max(cmax, c);
    }
    Vector3 d = cmax - cmin;
    int axis;
    if (d.x > d.y && d.x > d.z) axis = 0;
    else if (d.y > d.x && d.y > d.z) axis = 1;
    else axis = 2;
    float split_val = 0.5f * (cmin[axis] + cmax[axis]);
    int32_t start = 0, end = n;
    while (start < end) {
        while (start < end && center(start)[axis] < split_val) ++start;
        while (start < end && center(end - 1)[axis] >= split_val) --end;
        if (start < end) {
            std::swap(sorted[base + start], sorted[base + end - 1]);
            ++start;
            --end;
        }
    }
    if (start > 0 && start < n) return start;
    return n / 2;
}

void rebuildBVH(const PhysArgs &P, int32_t w)             // broadphase.cpp:42-280
{
    broadphase::BVH &bvh = P.bvh[w];
    BVHNode *nodes = P.nodes + (size_t)w * P.maxNodes;
    const AABB *aabbs = P.leafAABBs + (size_t)w * P.maxLeaves;
    int32_t *sorted = P.sortedLeaves + (size_t)w * P.maxLeaves;
    uint32_t *parents = P.leafParents + (size_t)w * P.maxLeaves;

    bvh.numNodes = numInternalNodes(bvh.numLeaves);
    struct StackEntry { int32_t nodeID, parentID, offset, numObjs; };
    StackEntry stack[128];
    stack[0] = { -1, -1, 0, bvh.numLeaves };
    int32_t cur_node_offset = 0;
    int32_t stack_size = 1;
    while (stack_size > 0) {
        StackEntry &entry = stack[stack_size - 1];
        int32_t node_id;
        if (entry.numObjs <= 4) {
            node_id = cur_node_offset++;
            BVHNode &node = nodes[node_id];
            node.parentID = entry.parentID;
            for (int i = 0; i < 4; i++) {
                if (i < entry.numObjs) {
                    int32_t leaf_id = sorted[entry.offset + i];
                    const AABB &a = aabbs[leaf_id];
                    parents[leaf_id] = ((uint32_t)node_id << 2) | (uint32_t)i;
                    node.children[i] = (int32_t)(0x80000000u | (uint32_t)leaf_id);
                    node.minX[i] = a.pMin.x; node.minY[i] = a.pMin.y; node.minZ[i] = a.pMin.z;
                    node.maxX[i] = a.pMax.x; node.maxY[i] = a.pMax.y; node.maxZ[i] = a.pMax.z;
                } else {
                    node.children[i] = -1;
                    node.minX[i] = FLT_MAX; node.minY[i] = FLT_MAX; node.minZ[i] = FLT_MAX;
                    node.maxX[i] = -FLT_MAX; node.maxY[i] = -FLT_MAX; node.maxZ[i] = -FLT_MAX;
                }
            }
        } else if (entry.nodeID == -1) {
            node_id = cur_node_offset++;
            entry.nodeID = node_id;
            BVHNode &node = nodes[node_id];
            for (int i = 0; i < 4; i++) node.children[i] = -1;
            node.parentID = entry.parentID;
            int32_t second = midpointSplit(aabbs, sorted, entry.offset, entry.numObjs);
            int32_t nh1 = second;
            int32_t nh2 = entry.numObjs - second;
            int32_t first = midpointSplit(aabbs, sorted, entry.offset, nh1);
            int32_t third = midpointSplit(aabbs, sorted, entry.offset + second, nh2);
            int32_t eid = entry.nodeID, eoff = entry.offset;
            if (stack_size + 4 > 128) {
                P.errorFlags[w] |= kErrBVHStack;
                return;
            }
            stack[stack_size++] = { -1, eid, eoff + nh1 + third, nh2 - third };
            stack[stack_size++] = { -1, eid, eoff + nh1, third };
            stack[stack_size++] = { -1, eid, eoff + first, nh1 - first };
            stack[stack_size++] = { -1, eid, eoff, first };
            continue;
        } else {
            node_id = entry.nodeID;
        }
        stack_size -= 1;
        BVHNode &node = nodes[node_id];
        if (node.parentID == -1) continue;
        AABB combined = AABB::invalid();
        for (int i = 0; i < 4; i++) {
            if (node.children[i] == -1) break;
            combined = AABB::merge(combined, AABB {
                { node.minX[i], node.minY[i], node.minZ[i] },
                { node.maxX[i], node.maxY[i], node.maxZ[i] } });
        }
        BVHNode &parent = nodes[node.parentID];
        int c;
        for (c = 0; c < 4; c++) if (parent.children[c] == -1) break;
        parent.children[c] = node_id;
        parent.minX[c] = combined.pMin.x; parent.minY[c] = combined.pMin.y;
        parent.minZ[c] = combined.pMin.z; parent.maxX[c] = combined.pMax.x;
        parent.maxY[c] = combined.pMax.y; parent.maxZ[c] = combined.pMax.z;
    }
    bvh.usedNodes = cur_node_offset;
}

void updateBVH(const PhysArgs &P, int32_t w)              // BVH::updateTree, broadphase.cpp:282-293
{
    broadphase::BVH &bvh = P.bvh[w];
    if (!bvh.forceRebuild) return;
    bvh.forceRebuild = 0;
    rebuildBVH(P, w);
}

void refitLeaf(const PhysArgs &P, int32_t w, int32_t leaf_id)   // broadphase.cpp:545-642
{
    BVHNode *nodes = P.nodes + (size_t)w * P.maxNodes;
    const AABB a = P.leafAABBs[(size_t)w * P.maxLeaves + leaf_id];
    const uint32_t lp = P.leafParents[(size_t)w * P.maxLeaves + leaf_id];
    int32_t node_idx = (int32_t)(lp >> 2);
    const int sub = (int)(lp & 3);
    auto minUpd = [](float *p, float v) { float old = *p; if (v < old) *p = v; return old; };
    auto maxUpd = [](float *p, float v) { float old = *p; if (v > old) *p = v; return old; };
    auto step = [&](BVHNode &n, int c) {
        float xm = minUpd(&n.minX[c], a.pMin.x);
        float ym = minUpd(&n.minY[c], a.pMin.y);
        float zm = minUpd(&n.minZ[c], a.pMin.z);
        float xM = maxUpd(&n.maxX[c], a.pMax.x);
        float yM = maxUpd(&n.maxY[c], a.pMax.y);
        float zM = maxUpd(&n.maxZ[c], a.pMax.z);
        return a.pMin.x < xm || a.pMin.y < ym || a.pMin.z < zm ||
               a.pMax.x > xM || a.pMax.y > yM || a.pMax.z > zM;
    };
    if (node_idx < 0 || node_idx >= P.maxNodes) {
        P.errorFlags[w] |= kErrIndexGuard;
        return;
    }
    BVHNode &leaf_node = nodes[node_idx];
    if (!step(leaf_node, sub)) return;
    int32_t child_idx = node_idx;
    node_idx = leaf_node.parentID;
    while (node_idx != -1) {
        BVHNode &n = nodes[node_idx];
        int c = -1;
        for (int j = 0; j < 4; j++) {
            if (n.children[j] == child_idx) { c = j; break; }
        }
        if (c < 0) {
            P.errorFlags[w] |= kErrIndexGuard;
            return;
        }
        if (!step(n, c)) break;
        child_idx = node_idx;
        node_idx = n.parentID;
    }
}

void refit(const PhysArgs &P, int32_t w)                  // refitEntry, broadphase.cpp:891-895
{
    forEachBody(P, w, [&](Body b, int32_t) { refitLeaf(P, w, b.leaf()); });
}

void findOverlapping(const PhysArgs &P, int32_t w)        // broadphase.cpp:897-932
{
    const BVHNode *nodes = P.nodes + (size_t)w * P.maxNodes;
    const Entity *leaf_entities = P.leafEntities + (size_t)w * P.maxLeaves;
    CandidateCollision *cands = P.cands + (size_t)w * P.candCapacity;
    int32_t n = P.numCands[w];
    forEachBody(P, w, [&](Body ba, int32_t) {
        const Entity ea = ba.entity();
        const Loc a_loc = lookup(P, w, ea);
        const bool a_static = ba.resp() == ResponseType::Static;
        const AABB q = P.leafAABBs[(size_t)w * P.maxLeaves + ba.leaf()];
        int32_t stack[128];                               // physics.inl:61-100
        stack[0] = 0;
        int32_t ss = 1;
        while (ss > 0) {
            const BVHNode &node = nodes[stack[--ss]];
            for (int i = 0; i < 4; i++) {
                const int32_t child = node.children[i];
                if (child == -1) continue;
                AABB c { { node.minX[i], node.minY[i], node.minZ[i] },
                         { node.maxX[i], node.maxY[i], node.maxZ[i] } };
                if (!q.overlaps(c)) continue;
                if (child & 0x80000000) {
                    const Entity o = leaf_entities[child & ~0x80000000];
                    if (ea.id < o.id) {
                        const Loc b_loc = lookup(P, w, o);
                        if (a_static && bodyAt(P, w, b_loc).resp() == ResponseType::Static) continue;
                        if (n >= P.candCapacity) {
                            P.errorFlags[w] |= kErrCandidateOverflow;
                            continue;
                        }
                        cands[n++] = CandidateCollision { a_loc, b_loc };
                    }
                } else if (ss < 128) {
                    stack[ss++] = child;
                } else {
                    P.errorFlags[w] |= kErrBVHStack;
                }
            }
        }
    });
    P.numCands[w] = n;
    P.lastNumCands[w] = n;
}

// ---------------------------------------------------------------------------
// substepRigidBodies (src/physics/physics.cpp:79-164)
// ---------------------------------------------------------------------------
void substepRigidBodies(const PhysArgs &P, int32_t w)
{
    const SolverData &solver = P.solver[w];
    forEachBody(P, w, [&](Body b, int32_t) {
        Vector3 x = b.pos();
        Quat q = b.rot();
        auto &prev = b.prev();
        auto &ps_pos = b.psPos();
        auto &ps_vel = b.psVel();
        if (b.resp() == ResponseType::Static) {
            prev.prevPosition = x;
            prev.prevRotation = q;
            ps_pos.x = x;
            ps_pos.q = q;
            ps_vel.v = Vector3::zero();
            ps_vel.omega = Vector3::zero();
            return;
        }
        Vector3 v = b.vel().linear;
        Vector3 omega = b.vel().angular;
        prev.prevPosition = x;
        prev.prevRotation = q;
        const RigidBodyMetadata md = P.objs.metadata[b.obj()];
        const float inv_m = md.invMass;
        const Vector3 inv_I = md.invInertiaTensor;
        const float h = solver.h;
        if (b.resp() == ResponseType::Dynamic) v += h * solver.g;
        v += h * inv_m * b.extF();
        x += h * v;
        Vector3 I {
            (inv_I.x == 0) ? 0.0f : 1.0f / inv_I.x,
            (inv_I.y == 0) ? 0.0f : 1.0f / inv_I.y,
            (inv_I.z == 0) ? 0.0f : 1.0f / inv_I.z,
        };
        Quat to_local = q.inv();
        Vector3 tau_ext_local = to_local.rotateVec(b.extT());
        Vector3 omega_local = to_local.rotateVec(omega);
        Vector3 I_omega_local = multDiag(I, omega_local);
        omega_local += h * multDiag(inv_I, tau_ext_local - cross(omega_local, I_omega_local));
        omega = q.rotateVec(omega_local);
        Quat apply_omega = Quat::fromAngularVec(0.5f * h * omega);
        q += apply_omega * q;
        q = q.normalize();
        b.pos() = x;
        b.rot() = q;
        ps_pos.x = x;
        ps_pos.q = q;
        ps_vel.v = v;
        ps_vel.omega = omega;
    });
}

// ---------------------------------------------------------------------------
// Narrowphase (src/physics/narrowphase.cpp, CPU branch)
// ---------------------------------------------------------------------------
struct HullView {                 // one hull of the flattened object table
    const HullDev *h;
    const ObjDev *O;
    const Vector3 &vertex(int32_t v) const { return O->vertices[h->vertOffset + v]; }
    const geometry::Plane &plane(int32_t f) const { return O->planes[h->faceOffset + f]; }
    const geometry::HalfEdge &hedge(uint32_t e) const { return O->hedges[h->hedgeOffset + e]; }
    uint32_t edge(int32_t i) const { return O->edges[h->edgeOffset + i]; }
    uint32_t polygon(int32_t f) const { return O->polygons[h->faceOffset + f]; }
};

struct HullState {                // makeHullState's tmp buffers (narrowphase.cpp:139-212)
    std::vector<Vector3> vertices;
    std::vector<geometry::Plane> facePlanes;
    HullView hull;
    Vector3 center;
};

void makeHullState(HullState &hs, HullView hull, Vector3 t, Quat r, Diag3x3 s)
{
    Mat3x3 unscaled = Mat3x3::fromQuat(r);
    Mat3x3 vtx = unscaled * s;
    Mat3x3 nrm = unscaled * s.inv();
    hs.hull = hull;
    hs.center = t;
    hs.vertices.resize(hull.h->numVerts);
    hs.facePlanes.resize(hull.h->numFaces);
    for (int32_t i = 0; i < hull.h->numVerts; i++) hs.vertices[i] = vtx * hull.vertex(i) + t;
    for (int32_t i = 0; i < hull.h->numFaces; i++) {
        geometry::Plane op = hull.plane(i);
        Vector3 origin = vtx * (op.normal * op.d) + t;
        Vector3 n = (nrm * op.normal).normalize();
        hs.facePlanes[i] = geometry::Plane { n, dot(n, origin) };
    }
}

float distFromPlane(const geometry::Plane &p, const Vector3 &a)   // narrowphase.cpp:238-243
{
    float adotn = a.dot(p.normal);
    return adotn - p.d;
}

Vector3 planeIntersection(const geometry::Plane &p, const Vector3 &p1, const Vector3 &p2)
{                                                         // narrowphase.cpp:246-250
    float distance = distFromPlane(p, p1);
    return p1 + (p2 - p1) * (-distance / p.normal.dot(p2 - p1));
}

float hullDistFromPlane(const geometry::Plane &p, const HullState &h)   // :309-350
{
    float min_dot = FLT_MAX;
    for (const Vector3 &v : h.vertices) {
        float d = p.normal.dot(v);
        if (d < min_dot) min_dot = d;
    }
    return min_dot - p.d;
}

struct FaceQuery { float separation; int32_t faceIdx; geometry::Plane plane; };
struct EdgeQuery { float separation; Vector3 normal; int32_t edgeA, edgeB; };

FaceQuery queryFaceDirections(const HullState &a, const HullState &b)   // :352-378
{
    geometry::Plane max_plane {};
    int32_t max_face = -1;
    float max_dist = -FLT_MAX;
    for (int32_t f = 0; f < (int32_t)a.facePlanes.size(); f++) {
        geometry::Plane p = a.facePlanes[f];
        float d = hullDistFromPlane(p, b);
        if (d > max_dist) {
            max_dist = d;
            max_face = f;
            max_plane = p;
            if (max_dist > 0) break;
        }
    }
    return { max_dist, max_face, max_plane };
}

bool isMinkowskiFace(const Vector3 &a, const Vector3 &b, const Vector3 &c, const Vector3 &d)
{                                                         // :380-393
    Vector3 bxa = b.cross(a);
    Vector3 dxc = d.cross(c);
    float cba = c.dot(bxa);
    float dba = d.dot(bxa);
    float adc = a.dot(dxc);
    float bdc = b.dot(dxc);
    return cba * dba < 0.0f && adc * bdc < 0.0f && cba * bdc > 0.0f;
}

EdgeQuery queryEdgeDirections(const HullState &a, const HullState &b)   // :474-576
{
    Vector3 normal {};
    int32_t ea_max = 0, eb_max = 0;
    float max_d = -FLT_MAX;
    const HullView &ha = a.hull, &hb = b.hull;
    for (int32_t i = 0; i < ha.h->numEdges; i++) {
        const int32_t he_a = (int32_t)ha.edge(i);
        const geometry::HalfEdge &ea = ha.hedge(he_a);
        Vector3 an1 = a.facePlanes[ea.polygon].normal;
        Vector3 an2 = a.facePlanes[ha.hedge(ea.twin).polygon].normal;
        for (int32_t j = 0; j < hb.h->numEdges; j++) {
            const int32_t he_b = (int32_t)hb.edge(j);
            const geometry::HalfEdge &eb = hb.hedge(he_b);
            Vector3 bn1 = b.facePlanes[eb.polygon].normal;
            Vector3 bn2 = b.facePlanes[hb.hedge(eb.twin).polygon].normal;
            float sep = -FLT_MAX;
            Vector3 n {};
            if (isMinkowskiFace(an1, an2, -bn1, -bn2)) {  // edgeDistance :433-472
                Vector3 pa1 = a.vertices[ea.rootVertex];
                Vector3 pa2 = a.vertices[ha.hedge(ea.next).rootVertex];
                Vector3 pb1 = b.vertices[eb.rootVertex];
                Vector3 pb2 = b.vertices[hb.hedge(eb.next).rootVertex];
                Vector3 da = pa2 - pa1, db = pb2 - pb1;
                Vector3 uc = da.cross(db);
                float l2 = uc.length2();
                if (l2 != 0) {
                    float inv = 1.f / sqrtf(l2);
                    n = uc * inv;
                    if (n.dot(pa1 - a.center) < 0.0f) n = -n;
                    sep = n.dot(pb1 - pa1);
                }
            }
            if (sep > max_d) {
                max_d = sep;
                normal = n;
                ea_max = he_a;
                eb_max = he_b;
                if (max_d > 0) return { max_d, normal, ea_max, eb_max };
            }
        }
    }
    return { max_d, normal, ea_max, eb_max };
}

int32_t findIncidentFace(const HullState &h, Vector3 ref_normal)   // :578-624
{
    float min_dot = FLT_MAX;
    int32_t face = 0;
    for (int32_t f = 0; f < (int32_t)h.facePlanes.size(); f++) {
        float d = dot(h.facePlanes[f].normal, ref_normal);
        if (d < min_dot) { min_dot = d; face = f; }
    }
    return face;
}

int clipPolygon(Vector3 *dst, geometry::Plane cp, const Vector3 *in, int n)   // :626-661
{
    int out = 0;
    if (n == 0) return 0;
    Vector3 v1 = in[n - 1];
    float d1 = distFromPlane(cp, v1);
    for (int i = 0; i < n; i++) {
        Vector3 v2 = in[i];
        float d2 = distFromPlane(cp, v2);
        if (d1 <= 0.0f && d2 <= 0.0f) {
            dst[out++] = v2;
        } else if (d1 <= 0.0f && d2 > 0.0f) {
            dst[out++] = planeIntersection(cp, v1, v2);
        } else if (d2 <= 0.0f && d1 > 0.0f) {
            dst[out++] = planeIntersection(cp, v1, v2);
            dst[out++] = v2;
        }
        v1 = v2;
        d1 = d2;
    }
    return out;
}

struct Manifold { Vector3 cp[4]; float depth[4]; int32_t num; Vector3 normal; };

// buildFaceContactManifold (narrowphase.cpp:790-864).  A slot the reference
// leaves unwritten when every point lies on one side of the p0-p1 line is
// zero here, as in the gfx950 kernel (reference UB).
Manifold buildFaceContactManifold(Vector3 n, Vector3 *contacts, float *depths, int num)
{
    Manifold m {};
    if (num <= 4) {
        m.num = num;
        for (int i = 0; i < num; i++) { m.cp[i] = contacts[i]; m.depth[i] = depths[i]; }
    } else {
        m.num = 4;
        m.cp[0] = contacts[0];
        m.depth[0] = depths[0];
        Vector3 p0 = m.cp[0];
        float largest_d2 = 0.0f;
        int largest_d2_idx = 0;
        for (int i = 1; i < num; i++) {
            Vector3 c = contacts[i];
            float d2 = p0.distance2(c);
            if (d2 > largest_d2) {
                largest_d2 = d2;
                m.cp[1] = c; m.depth[1] = depths[i];
                largest_d2_idx = i;
            }
        }
        contacts[largest_d2_idx] = m.cp[0];
        Vector3 diff0 = m.cp[1] - p0;
        float largest_area = 0.0f;         // never updated in the reference
        int largest_area_idx = 0;
        for (int i = 1; i < num; i++) {
            Vector3 c = contacts[i];
            Vector3 diff1 = c - p0;
            float area = n.dot(diff0.cross(diff1));
            if (area > largest_area) {
                m.cp[2] = c; m.depth[2] = depths[i];
                largest_area_idx = i;
            }
        }
        contacts[largest_area_idx] = m.cp[0];
        for (int i = 1; i < num; i++) {
            Vector3 c = contacts[i];
            Vector3 diff1 = c - p0;
            float area = n.dot(diff0.cross(diff1));
            if (area < largest_area) { m.cp[3] = c; m.depth[3] = depths[i]; }
        }
    }
    const Quat ident { 1, 0, 0, 0 };
    for (int i = 0; i < m.num; i++) m.cp[i] = ident.rotateVec(m.cp[i]) + Vector3::zero();
    m.normal = ident.rotateVec(n);
    return m;
}

geometry::Segment shortestSegmentBetween(const geometry::Segment &s1, const geometry::Segment &s2)
{                                                         // :1020-1051
    Vector3 v1 = s1.p2 - s1.p1;
    Vector3 v2 = s2.p2 - s2.p1;
    Vector3 v21 = s2.p1 - s1.p1;
    float dotv22 = v2.dot(v2);
    float dotv11 = v1.dot(v1);
    float dotv21 = v2.dot(v1);
    float dotv211 = v21.dot(v1);
    float dotv212 = v21.dot(v2);
    float denom = dotv21 * dotv21 - dotv22 * dotv11;
    float s, t;
    if (fabsf(denom) < 0.00001f) {
        s = 0.0f;
        t = (dotv11 * s - dotv211) / dotv21;
    } else {
        s = (dotv212 * dotv21 - dotv22 * dotv211) / denom;
        t = (-dotv211 * dotv21 + dotv11 * dotv212) / denom;
    }
    s = fmaxRef(fminRef(s, 1.0f), 0.0f);
    t = fmaxRef(fminRef(t, 1.0f), 0.0f);
    return { s1.p1 + s * v1, s2.p1 + t * v2 };
}

// Per-world narrowphase state of one substep.  Each body's world AABB and
// hull state (makeHullState) are computed once, the first time a pair needs
// them, instead of once per pair as runNarrowphase does: the same function
// of the same pose, so the same bits, and no body moves during the pass.
struct NarrowScratch {
    HullState a, b;
    std::vector<Vector3> tmp1, tmp2;
    std::vector<float> depths;
    std::vector<AABB> box;            // [body slot]
    std::vector<HullState> hull;      // [body slot]
    std::vector<uint8_t> haveBox, haveHull;

    void reset(int32_t bodies)
    {
        if ((int32_t)box.size() < bodies) {
            box.resize(bodies);
            hull.resize(bodies);
        }
        haveBox.assign(bodies, 0);
        haveHull.assign(bodies, 0);
    }
};

// Slot of a body in its world: the body archetypes' rows laid end to end.
int32_t bodySlotOf(const PhysArgs &P, const Body &b, int32_t w)
{
    return b.B->slotBase + (int32_t)(b.i - (size_t)w * b.B->capacity);
}

const AABB &cachedWorldAABB(const PhysArgs &P, NarrowScratch &S, const Body &b, int32_t slot)
{
    if (!S.haveBox[slot]) {
        S.box[slot] = P.objs.aabbs[b.obj()].applyTRS(b.pos(), b.rot(), b.scale());
        S.haveBox[slot] = 1;
    }
    return S.box[slot];
}

const HullState &cachedHullState(NarrowScratch &S, HullView h, const Body &b, int32_t slot)
{
    if (!S.haveHull[slot]) {
        makeHullState(S.hull[slot], h, b.pos(), b.rot(), b.scale());
        S.haveHull[slot] = 1;
    }
    return S.hull[slot];
}

// generateContacts -> addManifoldToSolver (narrowphase.cpp:1123-1162,
// 1366-1513): the world's contacts in append order.
void addManifold(const PhysArgs &P, int32_t w, int32_t &num_contacts, const Manifold &m,
                 Loc ref, Loc other)
{
    if (num_contacts >= P.maxContacts || num_contacts >= P.candCapacity) {
        P.errorFlags[w] |= kErrContactOverflow;
        return;
    }
    Contact &c = P.candContacts[(size_t)w * P.candCapacity + num_contacts];
    P.contactOrder[(size_t)w * P.candCapacity + num_contacts] = num_contacts;
    num_contacts++;
    memset(&c, 0, sizeof(c));
    c.ref = ref;
    c.alt = other;
    for (int i = 0; i < 4; i++) c.points[i] = Vector4::fromVector3(m.cp[i], m.depth[i]);
    c.numPoints = m.num;
    c.normal = m.normal;
}

void runNarrowphasePair(const PhysArgs &P, int32_t w, NarrowScratch &S, int32_t &num_contacts,
                        Loc a_loc, Loc b_loc)     // narrowphase.cpp:1515-1728
{
    Body ba = bodyAt(P, w, a_loc), bb = bodyAt(P, w, b_loc);
    const ObjDev &O = P.objs;
    uint32_t ta = O.types[ba.obj()];
    uint32_t tb = O.types[bb.obj()];
    if (ta > tb) {
        std::swap(a_loc, b_loc);
        std::swap(ba, bb);
        std::swap(ta, tb);
    }
    const int32_t sa = bodySlotOf(P, ba, w), sb = bodySlotOf(P, bb, w);
    if (!cachedWorldAABB(P, S, ba, sa).overlaps(cachedWorldAABB(P, S, bb, sb))) return;

    const uint32_t hull_t = (uint32_t)CollisionPrimitive::Type::Hull;
    const uint32_t plane_t = (uint32_t)CollisionPrimitive::Type::Plane;
    const uint32_t test = ta | tb;
    if (test == hull_t) {                                  // HullHull
        HullView ha { &O.hulls[ba.obj()], &O }, hb { &O.hulls[bb.obj()], &O };
        const HullState &A = cachedHullState(S, ha, ba, sa);
        const HullState &B = cachedHullState(S, hb, bb, sb);
        // doSAT (narrowphase.cpp:678-758)
        FaceQuery fa = queryFaceDirections(A, B);
        if (fa.separation > 0.0f) return;
        FaceQuery fb = queryFaceDirections(B, A);
        if (fb.separation > 0.0f) return;
        EdgeQuery eq = queryEdgeDirections(A, B);
        if (eq.separation > 0.0f) return;

        const bool face_a = fa.separation > eq.separation;
        const bool face_b = fb.separation > eq.separation;
        Manifold m;
        Loc ref_loc, other_loc;
        if (face_a || face_b) {
            const bool a_is_ref = fa.separation >= fb.separation;
            const geometry::Plane ref_plane = a_is_ref ? fa.plane : fb.plane;
            const int32_t ref_face = a_is_ref ? fa.faceIdx : fb.faceIdx;
            const HullState &ref = a_is_ref ? A : B;
            const HullState &inc = a_is_ref ? B : A;
            const int32_t inc_face = findIncidentFace(inc, ref_plane.normal);
            ref_loc = a_is_ref ? a_loc : b_loc;
            other_loc = a_is_ref ? b_loc : a_loc;

            // createFaceContact (narrowphase.cpp:866-972)
            const size_t cap = (size_t)(inc.hull.h->numHedges + ref.hull.h->numHedges) * 2 + 8;
            if (S.tmp1.size() < cap) { S.tmp1.resize(cap); S.tmp2.resize(cap); S.depths.resize(cap); }
            int n_in = 0;
            {
                uint32_t hidx = inc.hull.polygon(inc_face), start = hidx;
                do {
                    const geometry::HalfEdge &he = inc.hull.hedge(hidx);
                    hidx = he.next;
                    S.tmp1[n_in++] = inc.vertices[he.rootVertex];
                } while (hidx != start);
            }
            Vector3 *cin = S.tmp1.data(), *cdst = S.tmp2.data();
            int n_clip = n_in;
            {
                uint32_t hidx = ref.hull.polygon(ref_face), start = hidx;
                const geometry::HalfEdge *che = &ref.hull.hedge(hidx);
                Vector3 cur = ref.vertices[che->rootVertex];
                do {
                    hidx = che->next;
                    che = &ref.hull.hedge(hidx);
                    Vector3 next = ref.vertices[che->rootVertex];
                    Vector3 edge = next - cur;
                    Vector3 pn = cross(edge, ref_plane.normal);
                    float d = dot(pn, cur);
                    cur = next;
                    n_clip = clipPolygon(cdst, geometry::Plane { pn, d }, cin, n_clip);
                    std::swap(cdst, cin);
                } while (hidx != start);
            }
            int n_below = 0;
            for (int i = 0; i < n_clip; i++) {
                Vector3 v = cin[i];
                float d = distFromPlane(ref_plane, v);
                if (d < 0.0f) {
                    cin[n_below] = v - d * ref_plane.normal;
                    S.depths[n_below] = -d;
                    n_below++;
                }
            }
            m = buildFaceContactManifold(ref_plane.normal, cin, S.depths.data(), n_below);
        } else {
            // createEdgeContact (narrowphase.cpp:1053-1121)
            ref_loc = a_loc;
            other_loc = b_loc;
            const geometry::HalfEdge &ea = ha.hedge(eq.edgeA);
            const geometry::HalfEdge &eb = hb.hedge(eq.edgeB);
            geometry::Segment ga { A.vertices[ea.rootVertex], A.vertices[ha.hedge(ea.next).rootVertex] };
            geometry::Segment gb { B.vertices[eb.rootVertex], B.vertices[hb.hedge(eb.next).rootVertex] };
            geometry::Segment s = shortestSegmentBetween(ga, gb);
            const Quat ident { 1, 0, 0, 0 };
            m = Manifold {};
            m.cp[0] = ident.rotateVec(s.p1) + Vector3::zero();
            m.depth[0] = -eq.separation;
            m.num = 1;
            m.normal = ident.rotateVec(eq.normal);
        }
        if (m.num > 0) addManifold(P, w, num_contacts, m, ref_loc, other_loc);
    } else if (test == (hull_t | plane_t)) {               // HullPlane
        HullView ha { &O.hulls[ba.obj()], &O };
        const HullState &A = cachedHullState(S, ha, ba, sa);
        Vector3 pn = bb.rot().rotateVec(Vector3 { 0, 0, 1 });
        geometry::Plane plane { pn, dot(pn, bb.pos()) };
        // doSATPlane (narrowphase.cpp:760-788)
        float sep = hullDistFromPlane(plane, A);
        if (sep > 0.0f) return;
        const int32_t inc_face = findIncidentFace(A, plane.normal);
        // createFacePlaneContact (narrowphase.cpp:974-1017)
        const size_t cap = (size_t)ha.h->numHedges + 8;
        if (S.tmp1.size() < cap) { S.tmp1.resize(cap); S.tmp2.resize(cap); S.depths.resize(cap); }
        int n = 0;
        uint32_t hidx = ha.polygon(inc_face), start = hidx;
        do {
            const geometry::HalfEdge &he = ha.hedge(hidx);
            hidx = he.next;
            Vector3 v = A.vertices[he.rootVertex];
            float d = distFromPlane(plane, v);
            if (d < 0.0f) {
                S.tmp1[n] = v - d * plane.normal;
                S.depths[n] = -d;
                n++;
            }
        } while (hidx != start);
        Manifold m = buildFaceContactManifold(plane.normal, S.tmp1.data(), S.depths.data(), n);
        if (m.num > 0) addManifold(P, w, num_contacts, m, b_loc, a_loc);
    }
    // Sphere and plane-plane pairs: the reference asserts (narrowphase.cpp:
    // 1197-1225, 1268-1313); no manifold, as on the gfx950 path.
}

void narrowphase(const PhysArgs &P, int32_t w)
{
    thread_local NarrowScratch S;
    S.reset(P.maxBodiesPerWorld);
    int32_t num_contacts = 0;
    const CandidateCollision *cands = P.cands + (size_t)w * P.candCapacity;
    const int32_t n = P.numCands[w];
    for (int32_t i = 0; i < n; i++) runNarrowphasePair(P, w, S, num_contacts, cands[i].a, cands[i].b);
    P.lastNumContacts[w] = num_contacts;
}

// ---------------------------------------------------------------------------
// Solver (src/physics/physics.cpp)
// ---------------------------------------------------------------------------
float computePositionalLambda(Vector3 ta1, Vector3 ta2, Vector3 ra1, Vector3 ra2,
                              float im1, float im2, float c, float alpha)
{                                                          // physics.cpp:166-183
    float w1 = im1 + dot(ta1, ra1);
    float w2 = im2 + dot(ta2, ra2);
    return -c / (w1 + w2 + alpha);
}

void applyPositionalUpdate(Vector3 &x1, Vector3 &x2, Quat &q1, Quat &q2, Vector3 ral1,
                           Vector3 ral2, float im1, float im2, Vector3 n, float dl)
{                                                          // physics.cpp:185-211
    x1 += dl * im1 * n;
    x2 -= dl * im2 * n;
    float half = 0.5f * dl;
    Vector3 q1u = q1.rotateVec(half * ral1);
    Vector3 q2u = q2.rotateVec(half * ral2);
    q1 += Quat::fromAngularVec(q1u) * q1;
    q2 -= Quat::fromAngularVec(q2u) * q2;
    q1 = q1.normalize();
    q2 = q2.normalize();
}

float applyPositionalUpdateFull(Vector3 &x1, Vector3 &x2, Quat &q1, Quat &q2, Vector3 r1,
                                Vector3 r2, float im1, float im2, Vector3 iI1, Vector3 iI2,
                                Vector3 n, float c, float alpha)
{                                                          // physics.cpp:213-245
    Vector3 nl1 = q1.inv().rotateVec(n);
    Vector3 nl2 = q2.inv().rotateVec(n);
    Vector3 ta1 = cross(r1, nl1);
    Vector3 ta2 = cross(r2, nl2);
    Vector3 ra1 = multDiag(iI1, ta1);
    Vector3 ra2 = multDiag(iI2, ta2);
    float lambda = computePositionalLambda(ta1, ta2, ra1, ra2, im1, im2, c, alpha);
    applyPositionalUpdate(x1, x2, q1, q2, ra1, ra2, im1, im2, n, lambda);
    return lambda;
}

struct SolveBody {                 // invMass / invInertia, zero for static bodies
    float im;
    Vector3 iI;
    RigidBodyMetadata md;
};

SolveBody solveBody(const PhysArgs &P, Body b)
{
    SolveBody s;
    s.md = P.objs.metadata[b.obj()];
    s.im = s.md.invMass;
    s.iI = s.md.invInertiaTensor;
    if (b.resp() == ResponseType::Static) { s.im = 0.f; s.iI = Vector3::zero(); }
    return s;
}

void handleContact(const PhysArgs &P, int32_t w, Contact &c)   // physics.cpp:387-476
{
    Body b1 = bodyAt(P, w, c.ref), b2 = bodyAt(P, w, c.alt);
    const Vector3 prev1p = b1.prev().prevPosition, prev2p = b2.prev().prevPosition;
    const Quat prev1q = b1.prev().prevRotation, prev2q = b2.prev().prevRotation;
    const Vector3 ps1x = b1.psPos().x, ps2x = b2.psPos().x;
    const Quat ps1q = b1.psPos().q, ps2q = b2.psPos().q;
    const SolveBody s1 = solveBody(P, b1), s2 = solveBody(P, b2);
    Vector3 x1 = b1.pos(), x2 = b2.pos();
    Quat q1 = b1.rot(), q2 = b2.rot();
    const float avg_mu_s = 0.5f * (s1.md.muS + s2.md.muS);

    for (int i = 0; i < 4; i++) {
        if (i >= c.numPoints) continue;
        // getLocalSpaceContacts (physics.cpp:365-382)
        const Vector3 c1 = c.points[i].xyz();
        const float depth = c.points[i].w;
        const Vector3 c2 = c1 - c.normal * depth;
        const Vector3 r1 = ps1q.inv().rotateVec(c1 - ps1x);
        const Vector3 r2 = ps2q.inv().rotateVec(c2 - ps2x);
        float lambda_n = 0.f;
        // handleContactConstraint (physics.cpp:281-363)
        Vector3 p1 = q1.rotateVec(r1) + x1;
        Vector3 p2 = q2.rotateVec(r2) + x2;
        float d = dot(p1 - p2, c.normal);
        if (d > 0) {
            lambda_n = applyPositionalUpdateFull(x1, x2, q1, q2, r1, r2, s1.im, s2.im, s1.iI,
                                                 s2.iI, c.normal, d, 0);
            Vector3 p1_hat = prev1q.rotateVec(r1) + prev1p;
            Vector3 p2_hat = prev2q.rotateVec(r2) + prev2p;
            p1 = q1.rotateVec(r1) + x1;
            p2 = q2.rotateVec(r2) + x2;
            Vector3 dp = (p1 - p1_hat) - (p2 - p2_hat);
            Vector3 dpt = dp - dot(dp, c.normal) * c.normal;
            float tmag = dpt.length();
            if (tmag > 0.f) {
                Vector3 tw = dpt / tmag;
                Vector3 tl1 = q1.inv().rotateVec(tw);
                Vector3 tl2 = q2.inv().rotateVec(tw);
                Vector3 fta1 = cross(r1, tl1);
                Vector3 fta2 = cross(r2, tl2);
                Vector3 fra1 = multDiag(s1.iI, fta1);
                Vector3 fra2 = multDiag(s2.iI, fta2);
                float lambda_t = computePositionalLambda(fta1, fta2, fra1, fra2, s1.im, s2.im,
                                                         tmag, 0);
                float thresh = lambda_n * avg_mu_s;
                if (lambda_t > thresh) {
                    applyPositionalUpdate(x1, x2, q1, q2, fra1, fra2, s1.im, s2.im, tw, lambda_t);
                }
            }
        }
        c.lambdaN[i] = lambda_n;
    }
    b1.pos() = x1; b2.pos() = x2;
    b1.rot() = q1; b2.rot() = q2;
}

void computeAngularUpdate(Quat q1, Quat q2, Vector3 iI1, Vector3 iI2, Vector3 n1, Vector3 n2,
                          float theta, float alpha, Quat &u1, Quat &u2)
{                                                          // physics.cpp:247-271
    Vector3 lra1 = multDiag(iI1, n1);
    Vector3 lra2 = multDiag(iI2, n2);
    float w1 = dot(n1, lra1);
    float w2 = dot(n2, lra2);
    float dl = -theta / (w1 + w2 + alpha);
    float half = 0.5f * dl;
    u1 = Quat::fromAngularVec(q1.rotateVec(half * lra1));
    u2 = Quat::fromAngularVec(q2.rotateVec(half * lra2));
}

void angularCorrection(Quat &q1, Quat &q2, Vector3 dq, Vector3 iI1, Vector3 iI2)
{                                                          // physics.cpp:490-504, 522-534
    float mag = dq.length();
    if (mag > 0) {
        dq /= mag;
        Vector3 l1 = q1.inv().rotateVec(dq);
        Vector3 l2 = q2.inv().rotateVec(dq);
        Quat u1, u2;
        computeAngularUpdate(q1, q2, iI1, iI2, l1, l2, mag, 0, u1, u2);
        q1 = (q1 + u1 * q1).normalize();                   // applyAngularUpdate :273-279
        q2 = (q2 - u2 * q2).normalize();
    }
}

void handleJoint(const PhysArgs &P, int32_t w, const JointConstraint &j)   // physics.cpp:537-648
{
    Body b1 = bodyAt(P, w, lookup(P, w, j.e1)), b2 = bodyAt(P, w, lookup(P, w, j.e2));
    Vector3 x1 = b1.pos(), x2 = b2.pos();
    Quat q1 = b1.rot(), q2 = b2.rot();
    const SolveBody s1 = solveBody(P, b1), s2 = solveBody(P, b2);
    Vector3 corr;
    if (j.type == JointConstraint::Type::Fixed) {          // :580-615
        const Quat a1q = j.fixed.attachRot1, a2q = j.fixed.attachRot2;
        Quat o1 = (q1 * a1q).normalize();                  // applyJointOrientationConstraint
        Quat o2 = (q2 * a2q).normalize();
        Quat diff = o1 * o2.inv();
        Vector3 dq = 2.f * Vector3 { diff.x, diff.y, diff.z };
        angularCorrection(q1, q2, dq, s1.iI, s2.iI);
        Vector3 r1w = q1.rotateVec(j.r1) + x1;
        Vector3 r2w = q2.rotateVec(j.r2) + x2;
        Vector3 dr = r2w - r1w;
        Quat axes = (q1 * a1q).normalize();
        Vector3 a1 = axes.rotateVec(fwd);
        Vector3 b1v = axes.rotateVec(right);
        Vector3 c1 = cross(a1, b1v);
        corr = Vector3::zero();
        float as = dot(dr, a1);
        corr -= (as - j.fixed.separation) * a1;
        float bs = dot(dr, b1v);
        corr -= bs * b1v;
        float cs = dot(dr, c1);
        corr -= cs * c1;
    } else {                                               // Hinge, :616-627
        Vector3 ax1 = q1.rotateVec(j.hinge.a1Local);       // applyJointAxisConstraint
        Vector3 ax2 = q2.rotateVec(j.hinge.a2Local);
        angularCorrection(q1, q2, cross(ax1, ax2), s1.iI, s2.iI);
        Vector3 r1w = q1.rotateVec(j.r1) + x1;
        Vector3 r2w = q2.rotateVec(j.r2) + x2;
        corr = r2w - r1w;
    }
    float cm = corr.length();
    if (cm > 0.f) {
        corr /= cm;
        applyPositionalUpdateFull(x1, x2, q1, q2, j.r1, j.r2, s1.im, s2.im, s1.iI, s2.iI, corr,
                                  cm, 0);
    }
    b1.pos() = x1; b2.pos() = x2;
    b1.rot() = q1; b2.rot() = q2;
}

void setVelocities(const PhysArgs &P, int32_t w)          // physics.cpp:673-714
{
    const float h = P.solver[w].h;
    forEachBody(P, w, [&](Body b, int32_t) {
        Vector3 x = b.pos();
        Quat q = b.rot();
        Vector3 xp = b.prev().prevPosition;
        Quat qp = b.prev().prevRotation;
        Quat dq;
        if (q.w != qp.w || q.x != qp.x || q.y != qp.y || q.z != qp.z) {
            dq = q * qp.inv();
        } else {
            dq = Quat { 1, 0, 0, 0 };
        }
        Vector3 new_omega = 2.f / h * Vector3 { dq.x, dq.y, dq.z };
        b.vel().linear = (x - xp) / h;
        b.vel().angular = dq.w > 0.f ? new_omega : -new_omega;
    });
}

Vector3 relVel(Vector3 v1, Vector3 v2, Vector3 o1, Vector3 o2, Vector3 d1, Vector3 d2)
{                                                          // physics.cpp:716-722
    return (v1 + cross(o1, d1)) - (v2 + cross(o2, d2));
}

void applyVelocityUpdate(Vector3 &v1, Vector3 &v2, Vector3 &o1, Vector3 &o2, Quat q1, Quat q2,
                         Vector3 ta1, Vector3 ta2, float im1, float im2, Vector3 iI1,
                         Vector3 iI2, Vector3 dv, float mag)
{                                                          // physics.cpp:724-750
    Vector3 ra1 = multDiag(iI1, ta1);
    Vector3 ra2 = multDiag(iI2, ta2);
    float w1 = im1 + dot(ta1, ra1);
    float w2 = im2 + dot(ta2, ra2);
    mag *= 1.f / (w1 + w2);
    v1 += mag * im1 * dv;
    v2 -= mag * im2 * dv;
    Vector3 o1u = mag * ra1;
    Vector3 o2u = mag * ra2;
    o1 += q1.rotateVec(o1u);
    o2 -= q2.rotateVec(o2u);
}

void solveVelocitiesForContact(const PhysArgs &P, int32_t w, const Contact &c)
{                                                          // physics.cpp:865-993
    const SolverData &solver = P.solver[w];
    Body b1 = bodyAt(P, w, c.ref), b2 = bodyAt(P, w, c.alt);
    const Quat q1 = b1.rot(), q2 = b2.rot();
    const Vector3 ps1x = b1.psPos().x, ps2x = b2.psPos().x;
    const Quat ps1q = b1.psPos().q, ps2q = b2.psPos().q;
    const Vector3 ps1v = b1.psVel().v, ps2v = b2.psVel().v;
    const Vector3 ps1o = b1.psVel().omega, ps2o = b2.psVel().omega;
    const SolveBody s1 = solveBody(P, b1), s2 = solveBody(P, b2);
    Vector3 v1 = b1.vel().linear, o1 = b1.vel().angular;
    Vector3 v2 = b2.vel().linear, o2 = b2.vel().angular;
    const float mu_d = 0.5f * (s1.md.muD + s2.md.muD);

    Vector3 r1l[4], r2l[4], r1w[4], r2w[4], rt1[4], rt2[4];
    float vn_bars[4];
    for (int i = 0; i < 4; i++) {
        if (i >= c.numPoints) continue;
        const Vector3 c1 = c.points[i].xyz();
        const float depth = c.points[i].w;
        const Vector3 c2 = c1 - c.normal * depth;
        const Vector3 r1 = ps1q.inv().rotateVec(c1 - ps1x);
        const Vector3 r2 = ps2q.inv().rotateVec(c2 - ps2x);
        const Vector3 r1p = ps1q.rotateVec(r1);
        const Vector3 r2p = ps2q.rotateVec(r2);
        const Vector3 vbar = relVel(ps1v, ps2v, ps1o, ps2o, r1p, r2p);
        vn_bars[i] = dot(c.normal, vbar);
        r1l[i] = r1;
        r2l[i] = r2;
        r1w[i] = q1.rotateVec(r1);
        r2w[i] = q2.rotateVec(r2);
        rt1[i] = cross(r1, q1.inv().rotateVec(c.normal));
        rt2[i] = cross(r2, q2.inv().rotateVec(c.normal));
    }
    for (int it = 0; it < 2; it++) {                       // restitution, :813-863
        for (int i = 0; i < 4; i++) {
            if (i >= c.numPoints) continue;
            Vector3 v = relVel(v1, v2, o1, o2, r1w[i], r2w[i]);
            float vn = dot(c.normal, v);
            float vn_bar = vn_bars[i];
            float e = 0.3f;
            if (fabsf(vn_bar) <= solver.restitutionThreshold) e = 0.f;
            float mag = fminRef(-e * vn_bar, 0) - vn;
            applyVelocityUpdate(v1, v2, o1, o2, q1, q2, rt1[i], rt2[i], s1.im, s2.im, s1.iI,
                                s2.iI, c.normal, mag);
        }
    }
    for (int i = 0; i < 4; i++) {                          // friction, :752-811
        if (i >= c.numPoints) continue;
        Vector3 v = relVel(v1, v2, o1, o2, r1w[i], r2w[i]);
        float dfm = mu_d * fabsf(c.lambdaN[i]) / solver.h;
        float vn = dot(c.normal, v);
        Vector3 vt = v - c.normal * vn;
        float vt_len = vt.length();
        if (vt_len != 0 && dfm != 0.f) {
            float corrected = -fminRef(dfm, vt_len);
            Vector3 dw = vt / vt_len;
            Vector3 d1l = q1.inv().rotateVec(dw);
            Vector3 d2l = q2.inv().rotateVec(dw);
            Vector3 fta1 = cross(r1l[i], d1l);
            Vector3 fta2 = cross(r2l[i], d2l);
            applyVelocityUpdate(v1, v2, o1, o2, q1, q2, fta1, fta2, s1.im, s2.im, s1.iI, s2.iI,
                                dw, corrected);
        }
    }
    b1.vel().linear = v1; b1.vel().angular = o1;
    b2.vel().linear = v2; b2.vel().angular = o2;
}

// solvePositions (contacts in append order, then the ConstraintData rows that
// collectConstraintsSystem gathered in row order, physics.cpp:34-40,
// 650-671), setVelocities, solveVelocities (physics.cpp:995-1008).
void solve(const PhysArgs &P, int32_t w)
{
    Contact *contacts = P.candContacts + (size_t)w * P.candCapacity;
    const int32_t k = P.lastNumContacts[w];
    for (int32_t i = 0; i < k; i++) handleContact(P, w, contacts[i]);
    int32_t nj = P.numJointRows[w];
    if (nj > P.maxJoints) {
        P.errorFlags[w] |= kErrJointOverflow;
        nj = P.maxJoints;
    }
    const JointConstraint *joints = P.joints + (size_t)w * P.jointCapacity;
    for (int32_t j = 0; j < nj; j++) handleJoint(P, w, joints[j]);
    setVelocities(P, w);
    for (int32_t i = 0; i < k; i++) solveVelocitiesForContact(P, w, contacts[i]);
}

}

// ===========================================================================
// Graph nodes (CPU): same node kinds and graph shape as physics.hip
// ===========================================================================
struct PhysNodeBase : NodeBase {
    PhysicsModule *mod;
    explicit PhysNodeBase(Context &ctx) : mod(&physicsModule(ctxManager(ctx))) {}
};

#define MW_PHYS_CPU_NODE(NAME, FN)                                                   \
    struct NAME : PhysNodeBase {                                                     \
        using PhysNodeBase::PhysNodeBase;                                            \
        static TaskGraph::NodeID addToGraph(Context &ctx, TaskGraph::Builder &b,     \
                                            Span<const TaskGraph::NodeID> deps)      \
        {                                                                            \
            return b.addDefaultNode<NAME>(deps, ctx);                                \
        }                                                                            \
        static const char *nodeName() { return #NAME; }                             \
        static constexpr bool kNoTmpAlloc = true;                                    \
        static void launch(NAME *, LaunchCtx &) {}                                   \
        static void runWorld(NAME *self, CpuRunCtx &, int32_t w) { FN(self->mod->args, w); } \
    };

static void noop(const PhysArgs &, int32_t) {}

MW_PHYS_CPU_NODE(UpdateLeafPositionsNode, updateLeafPositions)
MW_PHYS_CPU_NODE(UpdateBVHNode, updateBVH)
MW_PHYS_CPU_NODE(RefitNode, refit)
MW_PHYS_CPU_NODE(FindOverlappingNode, findOverlapping)
MW_PHYS_CPU_NODE(SubstepRigidBodiesNode, substepRigidBodies)
MW_PHYS_CPU_NODE(NarrowphaseNode, narrowphase)
MW_PHYS_CPU_NODE(SolverNode, solve)
// collectConstraintsSystem only copies the ConstraintData rows, which the
// solve reads in place in the same order.
MW_PHYS_CPU_NODE(CollectConstraintsNode, noop)

TaskGraph::NodeID RigidBodyPhysicsSystem::setupBroadphaseTasks(TaskGraph::Builder &builder,
                                                               Span<const TaskGraph::NodeID> deps)
{                                                          // broadphase.cpp:934-956
    auto update_leaves = builder.addToGraph<UpdateLeafPositionsNode>(deps);
    auto bvh_update = builder.addToGraph<UpdateBVHNode>({ update_leaves });
    return builder.addToGraph<RefitNode>({ bvh_update });
}

TaskGraph::NodeID RigidBodyPhysicsSystem::setupSubstepTasks(TaskGraph::Builder &builder,
                                                            Span<const TaskGraph::NodeID> deps,
                                                            CountT num_substeps)
{                                                          // physics.cpp:1149-1199
    auto cur = builder.addToGraph<FindOverlappingNode>(deps);
    for (CountT i = 0; i < num_substeps; i++) {
        auto collect = builder.addToGraph<CollectConstraintsNode>({ cur });
        auto integrate = builder.addToGraph<SubstepRigidBodiesNode>({ cur });
        auto narrow = builder.addToGraph<NarrowphaseNode>({ integrate });
        auto reset1 = builder.addToGraph<ResetTmpAllocNode>({ narrow });
        auto solve_node = builder.addToGraph<SolverNode>({ reset1, collect });
        cur = builder.addToGraph<ResetTmpAllocNode>({ solve_node });
    }
    auto clear = builder.addToGraph<ClearTmpNode<CandidateTemporary>>({ cur });
    auto post_leaves = builder.addToGraph<UpdateLeafPositionsNode>({ clear });
    return builder.addToGraph<RefitNode>({ post_leaves });
}

TaskGraph::NodeID RigidBodyPhysicsSystem::setupCleanupTasks(TaskGraph::Builder &builder,
                                                            Span<const TaskGraph::NodeID> deps)
{
    return builder.addToGraph<ClearTmpNode<CollisionEventTemporary>>(deps);
}

}
