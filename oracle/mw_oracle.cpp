// ORACLE (test infrastructure only; never linked into the product).
//
// Serial CPU restatement of the reference per-world physics step of
// shacklettbp/gpu-ecs-madrona (src/physics/{broadphase,narrowphase,physics,
// geometry}.cpp driven through the TaskGraph node order of
// RigidBodyPhysicsSystem::setupBroadphaseTasks / setupSubstepTasks /
// setupCleanupTasks, src/physics/physics.cpp:1142-1205).  Each function cites
// the reference lines it restates.  Pinned against oracle/_ref (the reference
// itself, compiled by oracle/Makefile.ref) and the golden fixtures in
// tests/golden/ (see tests/golden/make_golden.py).
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
// load liborc.so.

#include "orc_math.hpp"
#include "orc_idmap.hpp"

#include <algorithm>
#include <cassert>
#include <cstring>
#include <map>
#include <random>
#include <thread>
#include <utility>
#include <vector>

namespace orc {

// ---------------------------------------------------------------------------
// Geometry: half-edge hull, restates src/physics/geometry.cpp:52-194
// ---------------------------------------------------------------------------
struct HalfEdge { uint32_t next, twin, rootVertex, polygon; };
struct Plane { V3 normal; float d; };
struct Segment { V3 p1, p2; };

struct Hull {
    std::vector<uint32_t> polygons;   // mPolygons: a half edge per face
    std::vector<Plane> facePlanes;    // mFacePlanes
    std::vector<uint32_t> edges;      // mEdges: a half edge per edge
    std::vector<HalfEdge> halfEdges;  // mHalfEdges
    std::vector<V3> vertices;         // mVertices
};

static Hull constructHull(const std::vector<std::vector<uint32_t>> &polys,
                          const std::vector<V3> &verts)
{
    Hull h;
    std::map<std::pair<uint32_t, uint32_t>, uint32_t> pair_to_hedge;
    size_t total_he = 0;
    for (auto &p : polys) total_he += p.size();
    h.halfEdges.resize(total_he);

    uint32_t he_count = 0;
    for (uint32_t poly_idx = 0; poly_idx < polys.size(); poly_idx++) {
        const auto &poly = polys[poly_idx];
        uint32_t new_polygon = 0;
        HalfEdge dummy {};
        HalfEdge *prev = &dummy;
        uint32_t first = he_count;
        for (size_t v = 0; v < poly.size(); v++) {
            uint32_t a = poly[v];
            uint32_t b = poly[(v + 1) % poly.size()];
            assert(pair_to_hedge.find({ a, b }) == pair_to_hedge.end());
            uint32_t hidx = he_count++;
            HalfEdge *ne = &h.halfEdges[hidx];
            ne->rootVertex = a;
            ne->polygon = poly_idx;
            auto twin = pair_to_hedge.find({ b, a });
            if (twin != pair_to_hedge.end()) {
                ne->twin = twin->second;
                h.halfEdges[twin->second].twin = hidx;
                h.edges.push_back(twin->second);
            }
            prev->next = hidx;
            prev = ne;
            pair_to_hedge[{ a, b }] = hidx;
            new_polygon = hidx;
        }
        prev->next = first;
        h.polygons.push_back(new_polygon);

        V3 fp[3];
        const HalfEdge *he = &h.halfEdges[new_polygon];
        for (int i = 0; i < 3; i++) {
            fp[i] = verts[he->rootVertex];
            he = &h.halfEdges[he->next];
        }
        V3 a = fp[1] - fp[0];
        V3 b = fp[2] - fp[0];
        V3 n = cross(a, b).normalize();
        h.facePlanes.push_back(Plane { n, dot(n, fp[0]) });
    }
    h.vertices = verts;
    return h;
}

// ---------------------------------------------------------------------------
// World state (single-world mode semantics, one per world)
// ---------------------------------------------------------------------------
enum class Response : uint32_t { Dynamic = 0, Kinematic = 1, Static = 2 };
enum class PrimType : uint32_t { Sphere = 1, Hull = 2, Plane = 4 };

struct Metadata { V3 invInertia; float invMass, muS, muD; };

struct Objects {
    std::vector<Metadata> metadata;
    std::vector<AABB> aabbs;
    std::vector<PrimType> types;
    std::vector<Hull> hulls;          // indexed by object id (empty for plane)
};

struct Body {
    Entity e;
    V3 pos; Q rot; Diag3 scale;
    V3 vLin, vAng;
    int32_t objID;
    Response resp;
    V3 prevPos; Q prevRot;            // solver::SubstepPrevState
    V3 psX; Q psQ;                    // solver::PreSolvePositional
    V3 psV, psOmega;                  // solver::PreSolveVelocity
    V3 extF, extT;
    int32_t leafID;
};

struct BVHNode {                      // include/madrona/physics.hpp:367-381
    float minX[4], minY[4], minZ[4], maxX[4], maxY[4], maxZ[4];
    int32_t children[4];
    int32_t parentID;
    bool isLeaf(int c) const { return children[c] & 0x80000000; }
    int32_t leafIDX(int c) const { return children[c] & ~0x80000000; }
    void setLeaf(int c, int32_t idx) { children[c] = (int32_t)(0x80000000u | (uint32_t)idx); }
    void setInternal(int c, int32_t idx) { children[c] = idx; }
    bool hasChild(int c) const { return children[c] != -1; }
    void clearChild(int c) { children[c] = -1; }
};
static_assert(sizeof(BVHNode) == 116);

struct Contact {                      // include/madrona/physics.hpp:126-133
    Loc ref, alt;
    float points[4][4];
    int32_t numPoints;
    V3 normal;
    float lambdaN[4];
};
static_assert(sizeof(Contact) == 112);

struct Config {
    int32_t numCubes;
    int32_t numSubsteps;
    float deltaT;
    float gravityZ;
    int32_t maxContacts;
    float cubeInvMass;
    float cubeInvInertia;
    float muS;
    float muD;
    int32_t numJoints;      // joint pairs per world (jointSpec), 0 = none
    int32_t numHingeJoints; // the last numHingeJoints of them are hinges
};

static constexpr uint32_t kBodyArchetype = 6;   // registration order, see DESIGN.md
// simple_taskgraph (examples/simple_taskgraph/simple.cpp:37-49): Sphere is
// registered where the collisions body archetype is, Agent right after it.
static constexpr uint32_t kSphereArchetype = kBodyArchetype;
static constexpr uint32_t kAgentArchetype = kBodyArchetype + 1;

// JointConstraint (include/madrona/physics.hpp:196-238), 92 B.  The union
// holds Fixed {attachRot1, attachRot2, separation} or Hinge {a1Local,
// a2Local, b1Local, b2Local}.
struct Joint {
    Entity e1, e2;
    uint32_t type;                    // 0 Fixed, 1 Hinge
    float u[12];
    V3 r1, r2;
};
static_assert(sizeof(Joint) == 92);

// The joint workload shared with oracle/ref_harness.cpp and the collisions
// environment: joint j ties cube 2j to cube 2j + 1; fixed, or hinge for the
// last numHingeJoints (JointConstraint::setupFixed / setupHinge,
// physics.inl:151-190).
static Joint jointSpec(bool hinge, Entity e1, Entity e2)
{
    Joint jt {};
    jt.e1 = e1;
    jt.e2 = e2;
    if (!hinge) {
        jt.type = 0;
        const float rot1[4] = { 1.f, 0.f, 0.f, 0.f };
        const float rot2[4] = { 0.70710678f, 0.f, 0.f, 0.70710678f };
        memcpy(jt.u, rot1, 16);
        memcpy(jt.u + 4, rot2, 16);
        jt.u[8] = 0.5f;
        jt.r1 = V3 { 0.f, 1.5f, 0.f };
        jt.r2 = V3 { 0.f, -1.5f, 0.f };
    } else {
        jt.type = 1;
        const float axes[12] = { 1, 0, 0, 1, 0, 0, 0, 1, 0, 0, 1, 0 };
        memcpy(jt.u, axes, 48);
        jt.r1 = V3 { 0.f, 0.f, 1.5f };
        jt.r2 = V3 { 0.f, 0.f, -1.5f };
    }
    return jt;
}

static constexpr uint32_t kConstraintArchetype = 5;

struct World {
    IDMap ids;
    IDMap::Cache initCache, worldCache;
    std::vector<Body> bodies;

    // broadphase::BVH (src/physics/broadphase.cpp:11-31)
    std::vector<BVHNode> nodes;
    int32_t numNodes = 0;
    int32_t usedNodes = 0;            // nodes the last rebuild wrote
    std::vector<Entity> leafEntities;
    std::vector<AABB> leafAABBs;
    std::vector<uint32_t> leafParents;
    std::vector<int32_t> sortedLeaves;
    int32_t numLeaves = 0;
    float leafVelExp = 0, leafAccelExp = 0;
    bool forceRebuild = false;

    // SolverData (src/physics/physics.cpp:15-32)
    std::vector<Contact> contacts;
    int32_t numContacts = 0;
    std::vector<Joint> joints;        // ConstraintData rows, row order
    float h = 0, gMag = 0, restThresh = 0;
    V3 g;

    std::vector<std::pair<Loc, Loc>> candidates;

    // trace (debug visibility for the GPU parity tests)
    std::vector<std::pair<Loc, Loc>> lastCandidates;
    std::vector<Contact> lastContacts;

    // Body vector = query order: archetype by archetype, rows in table
    // order.  agentBase = index of Agent row 0 (simple mode only).
    int32_t agentBase = 0;
    // Face manifolds that left contactPoints[2] or [3] unwritten in the
    // reference (narrowphase.cpp:828-853): undefined there, zero here.
    int32_t ubManifolds = 0;
};

struct Sim {
    Config cfg;
    Objects objs;
    std::vector<World> worlds;
    bool simple = false;      // simple_taskgraph worlds: clamp node, two archetypes, no plane
    int32_t numHulls = 1;     // body i uses object i % numHulls, the plane is object numHulls
};

static inline int32_t bodyIndex(const World &w, Loc l)
{
    return l.archetype == kAgentArchetype ? w.agentBase + l.row : l.row;
}

static int32_t numInternalNodes(int32_t num_leaves)     // broadphase.cpp:33-40
{
    return std::max((num_leaves - 1 + 2) / 3, 1) + num_leaves;
}

static void initWorld(const Sim &sim, World &w, const float *pos, const float *rot)
{
    const Config &cfg = sim.cfg;
    // Singletons (BVH, SolverData, ObjectData) are created from the init
    // cache at registration (include/madrona/state.inl:171-187).
    for (int i = 0; i < 3; i++) (void)w.ids.acquireID(w.initCache);

    // RigidBodyPhysicsSystem::init (physics.cpp:1012-1036)
    int32_t max_leaves = cfg.numCubes + (sim.simple ? 2 : 1);
    w.nodes.resize(numInternalNodes(max_leaves));
    w.leafEntities.resize(max_leaves);
    w.leafAABBs.resize(max_leaves);
    w.leafParents.resize(max_leaves);
    w.sortedLeaves.resize(max_leaves);
    w.leafVelExp = 2.f * cfg.deltaT;
    w.leafAccelExp = 100.f * cfg.deltaT * cfg.deltaT;
    w.contacts.resize(cfg.maxContacts);
    w.h = cfg.deltaT / (float)cfg.numSubsteps;
    w.g = V3 { 0.f, 0.f, cfg.gravityZ };
    w.gMag = w.g.length();
    w.restThresh = 2.f * w.gMag * w.h;

    if (sim.simple) {
        w.bodies.resize(cfg.numCubes + 2);
        w.agentBase = cfg.numCubes + 1;
    }
    int32_t sphere_rows = 0;
    auto make = [&](V3 p, Q q, int32_t obj, Response rt, uint32_t arch = kBodyArchetype) {
        Entity e = w.ids.acquireID(w.worldCache);
        int32_t row = sim.simple ? (arch == kAgentArchetype ? 0 : sphere_rows++)
                                 : (int32_t)w.bodies.size();
        Body b {};
        b.e = e;
        b.pos = p; b.rot = q; b.scale = { 1.f, 1.f, 1.f };
        b.vLin = V3::zero(); b.vAng = V3::zero();
        b.objID = obj; b.resp = rt;
        b.prevPos = p; b.prevRot = q;
        b.psX = p; b.psQ = q;
        b.psV = V3::zero(); b.psOmega = V3::zero();
        b.extF = V3::zero(); b.extT = V3::zero();
        int32_t leaf = w.numLeaves++;                    // BVH::reserveLeaf
        w.leafEntities[leaf] = e;
        b.leafID = leaf;
        const Loc loc { arch, row };
        if (sim.simple) w.bodies[bodyIndex(w, loc)] = b;
        else w.bodies.push_back(b);
        w.ids.ref(e.id) = loc;
    };

    if (sim.simple) {                                    // simple.cpp:94-117
        for (int32_t i = 0; i < cfg.numCubes; i++) {
            make(V3 { pos[3 * i], pos[3 * i + 1], pos[3 * i + 2] },
                 Q { rot[4 * i], rot[4 * i + 1], rot[4 * i + 2], rot[4 * i + 3] },
                 0, Response::Dynamic, kSphereArchetype);
        }
        make(V3::zero(), Q { 1.f, 0.f, 0.f, 0.f }, 0, Response::Dynamic,
             kAgentArchetype);
        make(V3 { -10.f, 0.f, 0.f }, Q { 1.f, 0.f, 0.f, 0.f }, 0, Response::Dynamic,
             kSphereArchetype);
        w.forceRebuild = true;
        return;
    }

    for (int32_t i = 0; i < cfg.numCubes; i++) {
        make(V3 { pos[3 * i], pos[3 * i + 1], pos[3 * i + 2] },
             Q { rot[4 * i], rot[4 * i + 1], rot[4 * i + 2], rot[4 * i + 3] },
             i % sim.numHulls, Response::Dynamic);
    }
    make(V3::zero(), Q { 1.f, 0.f, 0.f, 0.f }, sim.numHulls, Response::Static);
    for (int32_t j = 0; j < cfg.numJoints; j++) {         // ConstraintData entities
        Entity e = w.ids.acquireID(w.worldCache);
        w.ids.ref(e.id) = Loc { kConstraintArchetype, j };
        const bool hinge = j >= cfg.numJoints - cfg.numHingeJoints;
        w.joints.push_back(jointSpec(hinge, w.bodies[2 * j].e, w.bodies[2 * j + 1].e));
    }
    w.forceRebuild = true;                               // rebuildOnUpdate
}

// ---------------------------------------------------------------------------
// Broadphase (src/physics/broadphase.cpp)
// ---------------------------------------------------------------------------
static AABB expandAABBWithMotion(AABB aabb, const V3 &v, float vel_exp, float acc_exp)
{                                                         // broadphase.cpp:435-459
    for (int i = 0; i < 3; i++) {
        float pos_delta = vel_exp * v[i];
        float min_delta = pos_delta - acc_exp;
        float max_delta = pos_delta + acc_exp;
        if (min_delta < 0.f) aabb.pMin[i] += min_delta;
        if (max_delta > 0.f) aabb.pMax[i] += max_delta;
    }
    return aabb;
}

static void updateLeafPositions(const Sim &sim, World &w)  // broadphase.cpp:858-873
{
    for (Body &b : w.bodies) {
        AABB obj_aabb = sim.objs.aabbs[b.objID];
        AABB world_aabb = obj_aabb.applyTRS(b.pos, b.rot, b.scale);
        w.leafAABBs[b.leafID] = expandAABBWithMotion(world_aabb, b.vLin,
                                                     w.leafVelExp, w.leafAccelExp);
        w.sortedLeaves[b.leafID] = b.leafID;
    }
}

static void rebuildBVH(World &w)                          // broadphase.cpp:42-280
{
    w.numNodes = numInternalNodes(w.numLeaves);
    struct StackEntry { int32_t nodeID, parentID, offset, numObjs; };
    StackEntry stack[128];
    stack[0] = { -1, -1, 0, w.numLeaves };
    int32_t cur_node_offset = 0;
    int stack_size = 1;

    auto center = [&](int32_t base, int32_t off) {
        const AABB &a = w.leafAABBs[w.sortedLeaves[base + off]];
        return (a.pMin + a.pMax) / 2.f;
    };

    auto midpoint_split = [&](int32_t base, int32_t n) -> int32_t {
        V3 cmin { FLT_MAX, FLT_MAX, FLT_MAX };
        V3 cmax { -FLT_MAX, -FLT_MAX, -FLT_MAX };
        for (int i = 0; i < n; i++) {
            V3 c = center(base, i);
            cmin = V3::min(cmin, c);
            cmax = V3::max(cmax, c);
        }
        auto split = [&](int axis) -> int32_t {
            float split_val = 0.5f * (cmin[axis] + cmax[axis]);
            int start = 0, end = n;
            while (start < end) {
                while (start < end && center(base, start)[axis] < split_val) ++start;
                while (start < end && center(base, end - 1)[axis] >= split_val) --end;
                if (start < end) {
                    std::swap(w.sortedLeaves[base + start], w.sortedLeaves[base + end - 1]);
                    ++start;
                    --end;
                }
            }
            if (start > 0 && start < n) return start;
            return n / 2;
        };
        V3 d = cmax - cmin;
        if (d.x > d.y && d.x > d.z) return split(0);
        if (d.y > d.x && d.y > d.z) return split(1);
        return split(2);
    };

    while (stack_size > 0) {
        StackEntry &entry = stack[stack_size - 1];
        int32_t node_id;
        if (entry.numObjs <= 4) {
            node_id = cur_node_offset++;
            BVHNode &node = w.nodes[node_id];
            node.parentID = entry.parentID;
            for (int i = 0; i < 4; i++) {
                if (i < entry.numObjs) {
                    int32_t leaf_id = w.sortedLeaves[entry.offset + i];
                    const AABB &a = w.leafAABBs[leaf_id];
                    w.leafParents[leaf_id] = ((uint32_t)node_id << 2) | (uint32_t)i;
                    node.setLeaf(i, leaf_id);
                    node.minX[i] = a.pMin.x; node.minY[i] = a.pMin.y; node.minZ[i] = a.pMin.z;
                    node.maxX[i] = a.pMax.x; node.maxY[i] = a.pMax.y; node.maxZ[i] = a.pMax.z;
                } else {
                    node.clearChild(i);
                    node.minX[i] = FLT_MAX; node.minY[i] = FLT_MAX; node.minZ[i] = FLT_MAX;
                    node.maxX[i] = -FLT_MAX; node.maxY[i] = -FLT_MAX; node.maxZ[i] = -FLT_MAX;
                }
            }
        } else if (entry.nodeID == -1) {
            node_id = cur_node_offset++;
            entry.nodeID = node_id;
            BVHNode &node = w.nodes[node_id];
            for (int i = 0; i < 4; i++) node.clearChild(i);
            node.parentID = entry.parentID;

            int32_t second = midpoint_split(entry.offset, entry.numObjs);
            int32_t nh1 = second;
            int32_t nh2 = entry.numObjs - second;
            int32_t first = midpoint_split(entry.offset, nh1);
            int32_t third = midpoint_split(entry.offset + second, nh2);

            int32_t eid = entry.nodeID, eoff = entry.offset;
            stack[stack_size++] = { -1, eid, eoff + nh1 + third, nh2 - third };
            stack[stack_size++] = { -1, eid, eoff + nh1, third };
            stack[stack_size++] = { -1, eid, eoff + first, nh1 - first };
            stack[stack_size++] = { -1, eid, eoff, first };
            continue;
        } else {
            node_id = entry.nodeID;
        }

        stack_size -= 1;
        BVHNode &node = w.nodes[node_id];
        if (node.parentID == -1) continue;

        AABB combined = AABB::invalid();
        for (int i = 0; i < 4; i++) {
            if (!node.hasChild(i)) break;
            combined = AABB::merge(combined, AABB {
                { node.minX[i], node.minY[i], node.minZ[i] },
                { node.maxX[i], node.maxY[i], node.maxZ[i] } });
        }
        BVHNode &parent = w.nodes[node.parentID];
        int c;
        for (c = 0; ; c++) if (parent.children[c] == -1) break;
        parent.setInternal(c, node_id);
        parent.minX[c] = combined.pMin.x; parent.minY[c] = combined.pMin.y;
        parent.minZ[c] = combined.pMin.z; parent.maxX[c] = combined.pMax.x;
        parent.maxY[c] = combined.pMax.y; parent.maxZ[c] = combined.pMax.z;
    }
    w.usedNodes = cur_node_offset;
}

static void refitLeaf(World &w, int32_t leaf_id)          // broadphase.cpp:545-642
{
    const AABB a = w.leafAABBs[leaf_id];
    uint32_t lp = w.leafParents[leaf_id];
    int32_t node_idx = (int32_t)(lp >> 2);
    int sub = (int)(lp & 3);

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

    BVHNode &leaf_node = w.nodes[node_idx];
    if (!step(leaf_node, sub)) return;

    int32_t child_idx = node_idx;
    node_idx = leaf_node.parentID;
    while (node_idx != -1) {
        BVHNode &n = w.nodes[node_idx];
        int c = -1;
        for (int j = 0; j < 4; j++) if (n.children[j] == child_idx) { c = j; break; }
        assert(c != -1);
        if (!step(n, c)) break;
        child_idx = node_idx;
        node_idx = n.parentID;
    }
}

static void refit(World &w)                                // refitEntry, :891-895
{
    for (Body &b : w.bodies) refitLeaf(w, b.leafID);
}

static bool isStatic(const Body &b) { return b.resp == Response::Static; }

static void findOverlapping(World &w)                     // broadphase.cpp:897-932
{
    for (int32_t row = 0; row < (int32_t)w.bodies.size(); row++) {
        const Body &ba = w.bodies[row];
        Loc a_loc = w.ids.lookup(ba.e);
        bool a_static = isStatic(ba);
        const AABB q = w.leafAABBs[ba.leafID];

        int32_t stack[128];                               // physics.inl:61-100
        stack[0] = 0;
        int ss = 1;
        while (ss > 0) {
            int32_t ni = stack[--ss];
            const BVHNode &n = w.nodes[ni];
            for (int i = 0; i < 4; i++) {
                if (!n.hasChild(i)) continue;
                AABB child { { n.minX[i], n.minY[i], n.minZ[i] },
                             { n.maxX[i], n.maxY[i], n.maxZ[i] } };
                if (!q.overlaps(child)) continue;
                if (n.isLeaf(i)) {
                    Entity o = w.leafEntities[n.leafIDX(i)];
                    if (ba.e.id < o.id) {
                        Loc b_loc = w.ids.lookup(o);
                        if (a_static && isStatic(w.bodies[bodyIndex(w, b_loc)])) continue;
                        w.candidates.push_back({ a_loc, b_loc });
                    }
                } else {
                    stack[ss++] = n.children[i];
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Narrowphase (src/physics/narrowphase.cpp, CPU branch)
// ---------------------------------------------------------------------------
struct HullState {
    std::vector<V3> vertices;
    std::vector<Plane> facePlanes;
    const Hull *hull;
    V3 center;
};

static void makeHullState(HullState &hs, const Hull &hull, V3 t, Q r, Diag3 s)
{                                                          // narrowphase.cpp:139-212
    M3 unscaled = M3::fromQuat(r);
    M3 vtx = unscaled * s;
    M3 nrm = unscaled * s.inv();
    hs.hull = &hull;
    hs.center = t;
    hs.vertices.resize(hull.vertices.size());
    hs.facePlanes.resize(hull.facePlanes.size());
    for (size_t i = 0; i < hull.vertices.size(); i++) {
        hs.vertices[i] = vtx * hull.vertices[i] + t;
    }
    for (size_t i = 0; i < hull.facePlanes.size(); i++) {
        Plane op = hull.facePlanes[i];
        V3 origin = vtx * (op.normal * op.d) + t;
        V3 n = (nrm * op.normal).normalize();
        hs.facePlanes[i] = Plane { n, dot(n, origin) };
    }
}

static float distFromPlane(const Plane &p, const V3 &a)   // narrowphase.cpp:238-243
{
    float adotn = a.dot(p.normal);
    return adotn - p.d;
}

static V3 planeIntersection(const Plane &p, const V3 &p1, const V3 &p2)
{                                                          // narrowphase.cpp:246-250
    float distance = distFromPlane(p, p1);
    return p1 + (p2 - p1) * (-distance / p.normal.dot(p2 - p1));
}

static float hullDistFromPlane(const Plane &p, const HullState &h)
{                                                          // narrowphase.cpp:309-350
    float min_dot = FLT_MAX;
    for (const V3 &v : h.vertices) {
        float d = p.normal.dot(v);
        if (d < min_dot) min_dot = d;
    }
    return min_dot - p.d;
}

struct FaceQuery { float separation; int32_t faceIdx; Plane plane; };
struct EdgeQuery { float separation; V3 normal; int32_t edgeA, edgeB; };

static FaceQuery queryFaceDirections(const HullState &a, const HullState &b)
{                                                          // narrowphase.cpp:352-378
    Plane max_plane {};
    int32_t max_face = -1;
    float max_dist = -FLT_MAX;
    for (int32_t f = 0; f < (int32_t)a.facePlanes.size(); f++) {
        Plane p = a.facePlanes[f];
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

static bool isMinkowskiFace(const V3 &a, const V3 &b, const V3 &c, const V3 &d)
{                                                          // narrowphase.cpp:380-393
    V3 bxa = b.cross(a);
    V3 dxc = d.cross(c);
    float cba = c.dot(bxa);
    float dba = d.dot(bxa);
    float adc = a.dot(dxc);
    float bdc = b.dot(dxc);
    return cba * dba < 0.0f && adc * bdc < 0.0f && cba * bdc > 0.0f;
}

static EdgeQuery queryEdgeDirections(const HullState &a, const HullState &b)
{                                                          // narrowphase.cpp:474-576
    V3 normal {};
    int32_t ea_max = 0, eb_max = 0;
    float max_d = -FLT_MAX;
    const Hull &ha = *a.hull, &hb = *b.hull;
    for (size_t i = 0; i < ha.edges.size(); i++) {
        int32_t he_a = (int32_t)ha.edges[i];
        const HalfEdge &ea = ha.halfEdges[he_a];
        V3 an1 = a.facePlanes[ea.polygon].normal;
        V3 an2 = a.facePlanes[ha.halfEdges[ea.twin].polygon].normal;
        for (size_t j = 0; j < hb.edges.size(); j++) {
            int32_t he_b = (int32_t)hb.edges[j];
            const HalfEdge &eb = hb.halfEdges[he_b];
            V3 bn1 = b.facePlanes[eb.polygon].normal;
            V3 bn2 = b.facePlanes[hb.halfEdges[eb.twin].polygon].normal;

            float sep = -FLT_MAX;
            V3 n {};
            if (isMinkowskiFace(an1, an2, -bn1, -bn2)) {  // edgeDistance :433-472
                V3 pa1 = a.vertices[ea.rootVertex];
                V3 pa2 = a.vertices[ha.halfEdges[ea.next].rootVertex];
                V3 pb1 = b.vertices[eb.rootVertex];
                V3 pb2 = b.vertices[hb.halfEdges[eb.next].rootVertex];
                V3 da = pa2 - pa1, db = pb2 - pb1;
                V3 uc = da.cross(db);
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

static int32_t findIncidentFace(const HullState &h, V3 ref_normal)
{                                                          // narrowphase.cpp:578-624
    float min_dot = FLT_MAX;
    int32_t face = -1;
    for (int32_t f = 0; f < (int32_t)h.facePlanes.size(); f++) {
        float d = dot(h.facePlanes[f].normal, ref_normal);
        if (d < min_dot) { min_dot = d; face = f; }
    }
    assert(face != -1);
    return face;
}

static int clipPolygon(V3 *dst, Plane cp, const V3 *in, int n)   // :626-661
{
    int out = 0;
    if (n == 0) return 0;
    V3 v1 = in[n - 1];
    float d1 = distFromPlane(cp, v1);
    for (int i = 0; i < n; i++) {
        V3 v2 = in[i];
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

struct Manifold { V3 cp[4]; float depth[4]; int32_t num; V3 normal; bool ub; };

static Manifold buildFaceContactManifold(V3 n, V3 *contacts, float *depths, int num)
{                                                          // narrowphase.cpp:790-864
    Manifold m {};
    if (num <= 4) {
        m.num = num;
        for (int i = 0; i < num; i++) { m.cp[i] = contacts[i]; m.depth[i] = depths[i]; }
    } else {
        m.num = 4;
        m.cp[0] = contacts[0];
        m.depth[0] = depths[0];
        V3 p0 = m.cp[0];
        float largest_d2 = 0.0f;
        int largest_d2_idx = 0;
        for (int i = 1; i < num; i++) {
            V3 c = contacts[i];
            float d2 = p0.distance2(c);
            if (d2 > largest_d2) {
                largest_d2 = d2;
                m.cp[1] = c; m.depth[1] = depths[i];
                largest_d2_idx = i;
            }
        }
        contacts[largest_d2_idx] = m.cp[0];
        V3 diff0 = m.cp[1] - p0;
        float largest_area = 0.0f;         // never updated in the reference
        int largest_area_idx = 0;
        bool wrote2 = false, wrote3 = false;
        for (int i = 1; i < num; i++) {
            V3 c = contacts[i];
            V3 diff1 = c - p0;
            float area = n.dot(diff0.cross(diff1));
            if (area > largest_area) {
                m.cp[2] = c; m.depth[2] = depths[i];
                largest_area_idx = i;
                wrote2 = true;
            }
        }
        contacts[largest_area_idx] = m.cp[0];
        for (int i = 1; i < num; i++) {
            V3 c = contacts[i];
            V3 diff1 = c - p0;
            float area = n.dot(diff0.cross(diff1));
            if (area < largest_area) { m.cp[3] = c; m.depth[3] = depths[i]; wrote3 = true; }
        }
        // All points on one side of the p0-p1 line: the reference leaves a
        // slot of its uninitialised Manifold unwritten (undefined value);
        // the oracle and the HIP kernel define it as zero.
        m.ub = !(wrote2 && wrote3);
    }
    const Q ident { 1, 0, 0, 0 };
    for (int i = 0; i < m.num; i++) m.cp[i] = ident.rotateVec(m.cp[i]) + V3::zero();
    m.normal = ident.rotateVec(n);
    return m;
}

static Segment shortestSegmentBetween(const Segment &s1, const Segment &s2)
{                                                          // narrowphase.cpp:1020-1051
    V3 v1 = s1.p2 - s1.p1;
    V3 v2 = s2.p2 - s2.p1;
    V3 v21 = s2.p1 - s1.p1;
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
    s = fmax_ref(fmin_ref(s, 1.0f), 0.0f);
    t = fmax_ref(fmin_ref(t, 1.0f), 0.0f);
    return { s1.p1 + s * v1, s2.p1 + t * v2 };
}

static void addManifold(World &w, const Manifold &m, Loc ref, Loc other)
{                                                          // narrowphase.cpp:1123-1162
    assert(w.numContacts < (int32_t)w.contacts.size());
    Contact &c = w.contacts[w.numContacts++];
    memset(&c, 0, sizeof(c));
    c.ref = ref;
    c.alt = other;
    for (int i = 0; i < 4; i++) {
        c.points[i][0] = m.cp[i].x; c.points[i][1] = m.cp[i].y;
        c.points[i][2] = m.cp[i].z; c.points[i][3] = m.depth[i];
    }
    c.numPoints = m.num;
    c.normal = m.normal;
}

static void runNarrowphase(const Sim &sim, World &w, Loc a_loc, Loc b_loc)
{                                                          // narrowphase.cpp:1515-1728
    const Body *ba = &w.bodies[bodyIndex(w, a_loc)];
    const Body *bb = &w.bodies[bodyIndex(w, b_loc)];
    uint32_t ta = (uint32_t)sim.objs.types[ba->objID];
    uint32_t tb = (uint32_t)sim.objs.types[bb->objID];
    if (ta > tb) {
        std::swap(a_loc, b_loc);
        std::swap(ba, bb);
        std::swap(ta, tb);
    }
    AABB aw = sim.objs.aabbs[ba->objID].applyTRS(ba->pos, ba->rot, ba->scale);
    AABB bw = sim.objs.aabbs[bb->objID].applyTRS(bb->pos, bb->rot, bb->scale);
    if (!aw.overlaps(bw)) return;

    uint32_t test = ta | tb;
    static thread_local HullState hsa, hsb;
    V3 tmp1[64], tmp2[64];
    float depths[64];

    if (test == (uint32_t)PrimType::Hull) {               // HullHull
        const Hull &ha = sim.objs.hulls[ba->objID];
        const Hull &hb = sim.objs.hulls[bb->objID];
        makeHullState(hsa, ha, ba->pos, ba->rot, ba->scale);
        makeHullState(hsb, hb, bb->pos, bb->rot, bb->scale);

        // doSAT (narrowphase.cpp:678-758)
        FaceQuery fa = queryFaceDirections(hsa, hsb);
        if (fa.separation > 0.0f) return;
        FaceQuery fb = queryFaceDirections(hsb, hsa);
        if (fb.separation > 0.0f) return;
        EdgeQuery eq = queryEdgeDirections(hsa, hsb);
        if (eq.separation > 0.0f) return;

        bool face_a = fa.separation > eq.separation;
        bool face_b = fb.separation > eq.separation;
        Manifold m;
        Loc ref_loc, other_loc;
        if (face_a || face_b) {
            bool a_is_ref = fa.separation >= fb.separation;
            Plane ref_plane = a_is_ref ? fa.plane : fb.plane;
            int32_t ref_face = a_is_ref ? fa.faceIdx : fb.faceIdx;
            const HullState &ref = a_is_ref ? hsa : hsb;
            const HullState &inc = a_is_ref ? hsb : hsa;
            int32_t inc_face = findIncidentFace(inc, ref_plane.normal);
            ref_loc = a_is_ref ? a_loc : b_loc;
            other_loc = a_is_ref ? b_loc : a_loc;

            // createFaceContact (narrowphase.cpp:866-972)
            const Hull &rh = *ref.hull, &oh = *inc.hull;
            int n_in = 0;
            {
                uint32_t hidx = oh.polygons[inc_face], start = hidx;
                do {
                    const HalfEdge &he = oh.halfEdges[hidx];
                    hidx = he.next;
                    tmp1[n_in++] = inc.vertices[he.rootVertex];
                } while (hidx != start);
            }
            V3 *cin = tmp1, *cdst = tmp2;
            int n_clip = n_in;
            {
                uint32_t hidx = rh.polygons[ref_face], start = hidx;
                const HalfEdge *che = &rh.halfEdges[hidx];
                V3 cur = ref.vertices[che->rootVertex];
                do {
                    hidx = che->next;
                    che = &rh.halfEdges[hidx];
                    V3 next = ref.vertices[che->rootVertex];
                    V3 edge = next - cur;
                    V3 pn = cross(edge, ref_plane.normal);
                    float d = dot(pn, cur);
                    cur = next;
                    n_clip = clipPolygon(cdst, Plane { pn, d }, cin, n_clip);
                    std::swap(cdst, cin);
                } while (hidx != start);
            }
            int n_below = 0;
            for (int i = 0; i < n_clip; i++) {
                V3 v = cin[i];
                float d = distFromPlane(ref_plane, v);
                if (d < 0.0f) {
                    cin[n_below] = v - d * ref_plane.normal;
                    depths[n_below] = -d;
                    n_below++;
                }
            }
            m = buildFaceContactManifold(ref_plane.normal, cin, depths, n_below);
            w.ubManifolds += m.ub;
        } else {
            // createEdgeContact (narrowphase.cpp:1053-1121)
            ref_loc = a_loc;
            other_loc = b_loc;
            const HalfEdge &ea = ha.halfEdges[eq.edgeA];
            const HalfEdge &eb = hb.halfEdges[eq.edgeB];
            Segment sa { hsa.vertices[ea.rootVertex], hsa.vertices[ha.halfEdges[ea.next].rootVertex] };
            Segment sb { hsb.vertices[eb.rootVertex], hsb.vertices[hb.halfEdges[eb.next].rootVertex] };
            Segment s = shortestSegmentBetween(sa, sb);
            const Q ident { 1, 0, 0, 0 };
            m = Manifold {};
            m.cp[0] = ident.rotateVec(s.p1) + V3::zero();
            m.depth[0] = -eq.separation;
            m.num = 1;
            m.normal = ident.rotateVec(eq.normal);
        }
        if (m.num > 0) addManifold(w, m, ref_loc, other_loc);
    } else if (test == ((uint32_t)PrimType::Hull | (uint32_t)PrimType::Plane)) {
        const Hull &ha = sim.objs.hulls[ba->objID];
        makeHullState(hsa, ha, ba->pos, ba->rot, ba->scale);
        V3 pn = bb->rot.rotateVec(V3 { 0, 0, 1 });
        Plane plane { pn, dot(pn, bb->pos) };

        // doSATPlane (narrowphase.cpp:760-788)
        float sep = hullDistFromPlane(plane, hsa);
        if (sep > 0.0f) return;
        int32_t inc_face = findIncidentFace(hsa, plane.normal);

        // createFacePlaneContact (narrowphase.cpp:974-1017)
        int n = 0;
        uint32_t hidx = ha.polygons[inc_face], start = hidx;
        do {
            const HalfEdge &he = ha.halfEdges[hidx];
            hidx = he.next;
            V3 v = hsa.vertices[he.rootVertex];
            float d = distFromPlane(plane, v);
            if (d < 0.0f) {
                tmp1[n] = v - d * plane.normal;
                depths[n] = -d;
                n++;
            }
        } while (hidx != start);
        Manifold m = buildFaceContactManifold(plane.normal, tmp1, depths, n);
        w.ubManifolds += m.ub;
        if (m.num > 0) addManifold(w, m, b_loc, a_loc);
    } else {
        assert(false && "sphere / plane-plane narrowphase unsupported (reference asserts)");
    }
}

// ---------------------------------------------------------------------------
// Solver (src/physics/physics.cpp)
// ---------------------------------------------------------------------------
static V3 multDiag(V3 d, V3 v) { return { d.x * v.x, d.y * v.y, d.z * v.z }; }

static void substepRigidBodies(const Sim &sim, World &w)  // physics.cpp:79-164
{
    for (Body &b : w.bodies) {
        V3 x = b.pos;
        Q q = b.rot;
        V3 v = b.vLin;
        V3 omega = b.vAng;
        if (b.resp == Response::Static) {
            b.prevPos = x; b.prevRot = q;
            b.psX = x; b.psQ = q;
            b.psV = V3::zero(); b.psOmega = V3::zero();
            continue;
        }
        b.prevPos = x; b.prevRot = q;
        const Metadata &md = sim.objs.metadata[b.objID];
        float inv_m = md.invMass;
        V3 inv_I = md.invInertia;
        float h = w.h;
        if (b.resp == Response::Dynamic) v += h * w.g;
        v += h * inv_m * b.extF;
        x += h * v;
        V3 I {
            (inv_I.x == 0) ? 0.0f : 1.0f / inv_I.x,
            (inv_I.y == 0) ? 0.0f : 1.0f / inv_I.y,
            (inv_I.z == 0) ? 0.0f : 1.0f / inv_I.z,
        };
        Q to_local = q.inv();
        V3 tau_local = to_local.rotateVec(b.extT);
        V3 omega_local = to_local.rotateVec(omega);
        V3 I_omega_local = multDiag(I, omega_local);
        omega_local += h * multDiag(inv_I, tau_local - cross(omega_local, I_omega_local));
        omega = q.rotateVec(omega_local);
        Q apply_omega = Q::fromAngularVec(0.5f * h * omega);
        q += apply_omega * q;
        q = q.normalize();
        b.pos = x; b.rot = q;
        b.psX = x; b.psQ = q;
        b.psV = v; b.psOmega = omega;
    }
}

static float computePositionalLambda(V3 ta1, V3 ta2, V3 ra1, V3 ra2,
                                     float im1, float im2, float c, float alpha)
{                                                          // physics.cpp:166-183
    float w1 = im1 + dot(ta1, ra1);
    float w2 = im2 + dot(ta2, ra2);
    return -c / (w1 + w2 + alpha);
}

static void applyPositionalUpdate(V3 &x1, V3 &x2, Q &q1, Q &q2, V3 ral1, V3 ral2,
                                  float im1, float im2, V3 n, float dl)
{                                                          // physics.cpp:185-211
    x1 += dl * im1 * n;
    x2 -= dl * im2 * n;
    float half = 0.5f * dl;
    V3 q1u = q1.rotateVec(half * ral1);
    V3 q2u = q2.rotateVec(half * ral2);
    q1 += Q::fromAngularVec(q1u) * q1;
    q2 -= Q::fromAngularVec(q2u) * q2;
    q1 = q1.normalize();
    q2 = q2.normalize();
}

static float applyPositionalUpdateFull(V3 &x1, V3 &x2, Q &q1, Q &q2, V3 r1, V3 r2,
                                       float im1, float im2, V3 iI1, V3 iI2,
                                       V3 n, float c, float alpha)
{                                                          // physics.cpp:213-245
    V3 nl1 = q1.inv().rotateVec(n);
    V3 nl2 = q2.inv().rotateVec(n);
    V3 ta1 = cross(r1, nl1);
    V3 ta2 = cross(r2, nl2);
    V3 ra1 = multDiag(iI1, ta1);
    V3 ra2 = multDiag(iI2, ta2);
    float lambda = computePositionalLambda(ta1, ta2, ra1, ra2, im1, im2, c, alpha);
    applyPositionalUpdate(x1, x2, q1, q2, ra1, ra2, im1, im2, n, lambda);
    return lambda;
}

static void handleContact(const Sim &sim, World &w, Contact &c)  // physics.cpp:387-476
{
    Body &b1 = w.bodies[bodyIndex(w, c.ref)];
    Body &b2 = w.bodies[bodyIndex(w, c.alt)];
    V3 prev1p = b1.prevPos, prev2p = b2.prevPos;
    Q prev1q = b1.prevRot, prev2q = b2.prevRot;
    V3 ps1x = b1.psX, ps2x = b2.psX;
    Q ps1q = b1.psQ, ps2q = b2.psQ;
    const Metadata md1 = sim.objs.metadata[b1.objID];
    const Metadata md2 = sim.objs.metadata[b2.objID];
    V3 x1 = b1.pos, x2 = b2.pos;
    Q q1 = b1.rot, q2 = b2.rot;
    float im1 = md1.invMass, im2 = md2.invMass;
    V3 iI1 = md1.invInertia, iI2 = md2.invInertia;
    if (b1.resp == Response::Static) { im1 = 0.f; iI1 = V3::zero(); }
    if (b2.resp == Response::Static) { im2 = 0.f; iI2 = V3::zero(); }
    float avg_mu_s = 0.5f * (md1.muS + md2.muS);

    for (int i = 0; i < 4; i++) {
        if (i >= c.numPoints) continue;
        // getLocalSpaceContacts (physics.cpp:365-382)
        V3 c1 { c.points[i][0], c.points[i][1], c.points[i][2] };
        float depth = c.points[i][3];
        V3 c2 = c1 - c.normal * depth;
        V3 r1 = ps1q.inv().rotateVec(c1 - ps1x);
        V3 r2 = ps2q.inv().rotateVec(c2 - ps2x);

        float lambda_n = 0.f;
        // handleContactConstraint (physics.cpp:281-363)
        V3 p1 = q1.rotateVec(r1) + x1;
        V3 p2 = q2.rotateVec(r2) + x2;
        float d = dot(p1 - p2, c.normal);
        if (d > 0) {
            lambda_n = applyPositionalUpdateFull(x1, x2, q1, q2, r1, r2, im1, im2,
                                                 iI1, iI2, c.normal, d, 0);
            V3 p1_hat = prev1q.rotateVec(r1) + prev1p;
            V3 p2_hat = prev2q.rotateVec(r2) + prev2p;
            p1 = q1.rotateVec(r1) + x1;
            p2 = q2.rotateVec(r2) + x2;
            V3 dp = (p1 - p1_hat) - (p2 - p2_hat);
            V3 dpt = dp - dot(dp, c.normal) * c.normal;
            float tmag = dpt.length();
            if (tmag > 0.f) {
                V3 tw = dpt / tmag;
                V3 tl1 = q1.inv().rotateVec(tw);
                V3 tl2 = q2.inv().rotateVec(tw);
                V3 fta1 = cross(r1, tl1);
                V3 fta2 = cross(r2, tl2);
                V3 fra1 = multDiag(iI1, fta1);
                V3 fra2 = multDiag(iI2, fta2);
                float lambda_t = computePositionalLambda(fta1, fta2, fra1, fra2,
                                                         im1, im2, tmag, 0);
                float thresh = lambda_n * avg_mu_s;
                if (lambda_t > thresh) {
                    applyPositionalUpdate(x1, x2, q1, q2, fra1, fra2, im1, im2, tw, lambda_t);
                }
            }
        }
        c.lambdaN[i] = lambda_n;
    }
    b1.pos = x1; b2.pos = x2;
    b1.rot = q1; b2.rot = q2;
}

static std::pair<Q, Q> computeAngularUpdate(Q q1, Q q2, V3 iI1, V3 iI2, V3 n1, V3 n2,
                                            float theta, float alpha)
{                                                          // physics.cpp:247-271
    V3 lra1 = multDiag(iI1, n1);
    V3 lra2 = multDiag(iI2, n2);
    float w1 = dot(n1, lra1);
    float w2 = dot(n2, lra2);
    float dl = -theta / (w1 + w2 + alpha);
    float half = 0.5f * dl;
    V3 u1 = half * lra1;
    V3 u2 = half * lra2;
    return { Q::fromAngularVec(q1.rotateVec(u1)), Q::fromAngularVec(q2.rotateVec(u2)) };
}

static void applyAngularUpdate(Q &q1, Q &q2, Q u1, Q u2)  // physics.cpp:273-279
{
    q1 = (q1 + u1 * q1).normalize();
    q2 = (q2 - u2 * q2).normalize();
}

static void angularCorrection(Q &q1, Q &q2, V3 dq, V3 iI1, V3 iI2)
{                                                          // physics.cpp:490-504, 522-534
    float mag = dq.length();
    if (mag > 0) {
        dq /= mag;
        V3 l1 = q1.inv().rotateVec(dq);
        V3 l2 = q2.inv().rotateVec(dq);
        auto [u1, u2] = computeAngularUpdate(q1, q2, iI1, iI2, l1, l2, mag, 0);
        applyAngularUpdate(q1, q2, u1, u2);
    }
}

static void handleJoint(const Sim &sim, World &w, const Joint &j)  // physics.cpp:537-648
{
    Loc l1 = w.ids.lookup(j.e1), l2 = w.ids.lookup(j.e2);
    Body &b1 = w.bodies[bodyIndex(w, l1)];
    Body &b2 = w.bodies[bodyIndex(w, l2)];
    V3 x1 = b1.pos, x2 = b2.pos;
    Q q1 = b1.rot, q2 = b2.rot;
    const Metadata md1 = sim.objs.metadata[b1.objID];
    const Metadata md2 = sim.objs.metadata[b2.objID];
    float im1 = md1.invMass, im2 = md2.invMass;
    V3 iI1 = md1.invInertia, iI2 = md2.invInertia;
    if (b1.resp == Response::Static) { im1 = 0.f; iI1 = V3::zero(); }
    if (b2.resp == Response::Static) { im2 = 0.f; iI2 = V3::zero(); }

    V3 corr;
    if (j.type == 0) {                                     // Fixed, :580-615
        Q a1q { j.u[0], j.u[1], j.u[2], j.u[3] };
        Q a2q { j.u[4], j.u[5], j.u[6], j.u[7] };
        float separation = j.u[8];
        Q o1 = (q1 * a1q).normalize();                     // applyJointOrientationConstraint
        Q o2 = (q2 * a2q).normalize();
        Q diff = o1 * o2.inv();
        V3 dq = 2.f * V3 { diff.x, diff.y, diff.z };
        angularCorrection(q1, q2, dq, iI1, iI2);

        V3 r1w = q1.rotateVec(j.r1) + x1;
        V3 r2w = q2.rotateVec(j.r2) + x2;
        V3 dr = r2w - r1w;
        Q axes = (q1 * a1q).normalize();
        V3 a1 = axes.rotateVec(V3 { 0, 1, 0 });            // math::fwd
        V3 b1v = axes.rotateVec(V3 { 1, 0, 0 });           // math::right
        V3 c1 = cross(a1, b1v);
        corr = V3::zero();
        float as = dot(dr, a1);
        corr -= (as - separation) * a1;
        float bs = dot(dr, b1v);
        corr -= bs * b1v;
        float cs = dot(dr, c1);
        corr -= cs * c1;
    } else {                                               // Hinge, :616-627
        V3 a1l { j.u[0], j.u[1], j.u[2] };
        V3 a2l { j.u[3], j.u[4], j.u[5] };
        V3 ax1 = q1.rotateVec(a1l);                        // applyJointAxisConstraint
        V3 ax2 = q2.rotateVec(a2l);
        angularCorrection(q1, q2, cross(ax1, ax2), iI1, iI2);
        V3 r1w = q1.rotateVec(j.r1) + x1;
        V3 r2w = q2.rotateVec(j.r2) + x2;
        corr = r2w - r1w;
    }
    float cm = corr.length();
    if (cm > 0.f) {
        corr /= cm;
        applyPositionalUpdateFull(x1, x2, q1, q2, j.r1, j.r2, im1, im2, iI1, iI2, corr, cm, 0);
    }
    b1.pos = x1; b2.pos = x2;
    b1.rot = q1; b2.rot = q2;
}

static void solvePositions(const Sim &sim, World &w)      // physics.cpp:650-671
{
    for (int32_t i = 0; i < w.numContacts; i++) handleContact(sim, w, w.contacts[i]);
    // collectConstraintsSystem (physics.cpp:34-40) gathers the ConstraintData
    // rows in row order every substep; they run after all contacts.
    for (const Joint &j : w.joints) handleJoint(sim, w, j);
}

static void setVelocities(World &w)                       // physics.cpp:673-714
{
    float h = w.h;
    for (Body &b : w.bodies) {
        V3 x = b.pos;
        Q q = b.rot;
        V3 xp = b.prevPos;
        Q qp = b.prevRot;
        Q dq;
        if (q.w != qp.w || q.x != qp.x || q.y != qp.y || q.z != qp.z) {
            dq = q * qp.inv();
        } else {
            dq = { 1, 0, 0, 0 };
        }
        V3 new_omega = 2.f / h * V3 { dq.x, dq.y, dq.z };
        b.vLin = (x - xp) / h;
        b.vAng = dq.w > 0.f ? new_omega : -new_omega;
    }
}

static V3 relVel(V3 v1, V3 v2, V3 o1, V3 o2, V3 d1, V3 d2)   // physics.cpp:716-722
{
    return (v1 + cross(o1, d1)) - (v2 + cross(o2, d2));
}

static void applyVelocityUpdate(V3 &v1, V3 &v2, V3 &o1, V3 &o2, Q q1, Q q2,
                                V3 ta1, V3 ta2, float im1, float im2,
                                V3 iI1, V3 iI2, V3 dv, float mag)
{                                                          // physics.cpp:724-750
    V3 ra1 = multDiag(iI1, ta1);
    V3 ra2 = multDiag(iI2, ta2);
    float w1 = im1 + dot(ta1, ra1);
    float w2 = im2 + dot(ta2, ra2);
    mag *= 1.f / (w1 + w2);
    v1 += mag * im1 * dv;
    v2 -= mag * im2 * dv;
    V3 o1u = mag * ra1;
    V3 o2u = mag * ra2;
    o1 += q1.rotateVec(o1u);
    o2 -= q2.rotateVec(o2u);
}

static void solveVelocitiesForContact(const Sim &sim, World &w, const Contact &c)
{                                                          // physics.cpp:865-993
    Body &b1 = w.bodies[bodyIndex(w, c.ref)];
    Body &b2 = w.bodies[bodyIndex(w, c.alt)];
    Q q1 = b1.rot, q2 = b2.rot;
    V3 ps1x = b1.psX, ps2x = b2.psX;
    Q ps1q = b1.psQ, ps2q = b2.psQ;
    V3 ps1v = b1.psV, ps2v = b2.psV, ps1o = b1.psOmega, ps2o = b2.psOmega;
    const Metadata md1 = sim.objs.metadata[b1.objID];
    const Metadata md2 = sim.objs.metadata[b2.objID];
    V3 v1 = b1.vLin, o1 = b1.vAng, v2 = b2.vLin, o2 = b2.vAng;
    float im1 = md1.invMass, im2 = md2.invMass;
    V3 iI1 = md1.invInertia, iI2 = md2.invInertia;
    if (b1.resp == Response::Static) { im1 = 0.f; iI1 = V3::zero(); }
    if (b2.resp == Response::Static) { im2 = 0.f; iI2 = V3::zero(); }
    float mu_d = 0.5f * (md1.muD + md2.muD);

    V3 r1l[4], r2l[4], r1w[4], r2w[4], rt1[4], rt2[4];
    float vn_bars[4];
    for (int i = 0; i < 4; i++) {
        if (i >= c.numPoints) continue;
        V3 c1 { c.points[i][0], c.points[i][1], c.points[i][2] };
        float depth = c.points[i][3];
        V3 c2 = c1 - c.normal * depth;
        V3 r1 = ps1q.inv().rotateVec(c1 - ps1x);
        V3 r2 = ps2q.inv().rotateVec(c2 - ps2x);
        V3 r1p = ps1q.rotateVec(r1);
        V3 r2p = ps2q.rotateVec(r2);
        V3 vbar = relVel(ps1v, ps2v, ps1o, ps2o, r1p, r2p);
        float vn_bar = dot(c.normal, vbar);
        r1l[i] = r1; r2l[i] = r2;
        r1w[i] = q1.rotateVec(r1);
        r2w[i] = q2.rotateVec(r2);
        rt1[i] = cross(r1, q1.inv().rotateVec(c.normal));
        rt2[i] = cross(r2, q2.inv().rotateVec(c.normal));
        vn_bars[i] = vn_bar;
    }

    for (int it = 0; it < 2; it++) {                       // restitution, :813-863
        for (int i = 0; i < 4; i++) {
            if (i >= c.numPoints) continue;
            V3 v = relVel(v1, v2, o1, o2, r1w[i], r2w[i]);
            float vn = dot(c.normal, v);
            float vn_bar = vn_bars[i];
            float e = 0.3f;
            if (fabsf(vn_bar) <= w.restThresh) e = 0.f;
            float mag = fmin_ref(-e * vn_bar, 0) - vn;
            applyVelocityUpdate(v1, v2, o1, o2, q1, q2, rt1[i], rt2[i], im1, im2,
                                iI1, iI2, c.normal, mag);
        }
    }

    for (int i = 0; i < 4; i++) {                          // friction, :752-811
        if (i >= c.numPoints) continue;
        V3 v = relVel(v1, v2, o1, o2, r1w[i], r2w[i]);
        float dfm = mu_d * fabsf(c.lambdaN[i]) / w.h;
        float vn = dot(c.normal, v);
        V3 vt = v - c.normal * vn;
        float vt_len = vt.length();
        if (vt_len != 0 && dfm != 0.f) {
            float corrected = -fmin_ref(dfm, vt_len);
            V3 dw = vt / vt_len;
            V3 d1l = q1.inv().rotateVec(dw);
            V3 d2l = q2.inv().rotateVec(dw);
            V3 fta1 = cross(r1l[i], d1l);
            V3 fta2 = cross(r2l[i], d2l);
            applyVelocityUpdate(v1, v2, o1, o2, q1, q2, fta1, fta2, im1, im2,
                                iI1, iI2, dw, corrected);
        }
    }

    b1.vLin = v1; b1.vAng = o1;
    b2.vLin = v2; b2.vAng = o2;
}

static void solveVelocities(const Sim &sim, World &w)     // physics.cpp:995-1008
{
    for (int32_t i = 0; i < w.numContacts; i++) {
        solveVelocitiesForContact(sim, w, w.contacts[i]);
    }
}

// ---------------------------------------------------------------------------
// One taskgraph step (node order of setupBroadphaseTasks / setupSubstepTasks /
// setupCleanupTasks; see DESIGN.md §2 for the table)
// ---------------------------------------------------------------------------
static float clampRef(float v, float lo, float hi)        // std::clamp
{
    return v < lo ? lo : (hi < v ? hi : v);
}

static void stepWorld(const Sim &sim, World &w)
{
    if (sim.simple) {                                     // 0 clampSystem (simple.cpp:22-35)
        for (Body &b : w.bodies) {
            b.pos.x = clampRef(b.pos.x, -10.f, 10.f);
            b.pos.y = clampRef(b.pos.y, -10.f, 10.f);
            b.pos.z = clampRef(b.pos.z, 0.f, 10.f);
        }
    }
    updateLeafPositions(sim, w);                          // 1 updateLeafPositionsEntry
    if (w.forceRebuild) {                                 // 2 updateBVHEntry
        w.forceRebuild = false;
        rebuildBVH(w);
    }
    refit(w);                                             // 3 refitEntry
    w.candidates.clear();
    findOverlapping(w);                                   // 4 findOverlappingEntry
    w.lastCandidates = w.candidates;

    for (int s = 0; s < sim.cfg.numSubsteps; s++) {
        substepRigidBodies(sim, w);                       // 5-6
        w.numContacts = 0;
        for (auto &cand : w.candidates) runNarrowphase(sim, w, cand.first, cand.second);  // 7
        solvePositions(sim, w);                           // 9
        setVelocities(w);                                 // 10
        w.lastContacts.assign(w.contacts.begin(), w.contacts.begin() + w.numContacts);
        solveVelocities(sim, w);                          // 11
        w.numContacts = 0;
    }
    w.candidates.clear();                                 // 13 ClearTmpNode<Candidate>
    updateLeafPositions(sim, w);                          // 14
    refit(w);                                             // 15
}

static Objects makeObjects(const Config &cfg)
{
    Objects o;
    std::vector<V3> verts = {
        { -1, -1, -1 }, { 1, -1, -1 }, { 1, 1, -1 }, { -1, 1, -1 },
        { -1, -1, 1 }, { 1, -1, 1 }, { 1, 1, 1 }, { -1, 1, 1 },
    };
    std::vector<std::vector<uint32_t>> faces = {
        { 0, 3, 2, 1 }, { 4, 5, 6, 7 }, { 0, 1, 5, 4 },
        { 3, 7, 6, 2 }, { 0, 4, 7, 3 }, { 1, 2, 6, 5 },
    };
    o.hulls.push_back(constructHull(faces, verts));
    o.hulls.push_back(Hull {});
    o.types = { PrimType::Hull, PrimType::Plane };
    o.metadata = {
        { { cfg.cubeInvInertia, cfg.cubeInvInertia, cfg.cubeInvInertia },
          cfg.cubeInvMass, cfg.muS, cfg.muD },
        { { 0, 0, 0 }, 0.f, cfg.muS, cfg.muD },
    };
    o.aabbs = {
        { { -1, -1, -1 }, { 1, 1, 1 } },
        { { -FLT_MAX, -FLT_MAX, -FLT_MAX }, { FLT_MAX, FLT_MAX, 0.f } },
    };
    return o;
}

// Object table of OBJ hulls (PhysicsLoader::loadHullFromDisk, reference
// physics_assets.cpp:205-254: half-edge construction over the imported
// polygons, AABB = point(v0) expanded by every vertex) + the ground plane.
static Objects makeHullObjects(const Config &cfg, int32_t num_hulls, const int32_t *num_verts,
                               const float *verts, const int32_t *num_faces,
                               const int32_t *face_counts, const uint32_t *indices)
{
    Objects o;
    const Metadata md { { cfg.cubeInvInertia, cfg.cubeInvInertia, cfg.cubeInvInertia },
                        cfg.cubeInvMass, cfg.muS, cfg.muD };
    for (int32_t h = 0; h < num_hulls; h++) {
        std::vector<V3> vs;
        for (int32_t v = 0; v < num_verts[h]; v++) {
            vs.push_back(V3 { verts[0], verts[1], verts[2] });
            verts += 3;
        }
        std::vector<std::vector<uint32_t>> faces;
        for (int32_t f = 0; f < num_faces[h]; f++) {
            faces.emplace_back(indices, indices + *face_counts);
            indices += *face_counts;
            face_counts++;
        }
        AABB box { vs[0], vs[0] };
        for (size_t v = 1; v < vs.size(); v++) {           // AABB::expand, else-if kept
            const V3 p = vs[v];
            for (int a = 0; a < 3; a++) {
                if (p[a] < box.pMin[a]) box.pMin[a] = p[a];
                else if (p[a] > box.pMax[a]) box.pMax[a] = p[a];
            }
        }
        o.hulls.push_back(constructHull(faces, vs));
        o.types.push_back(PrimType::Hull);
        o.metadata.push_back(md);
        o.aabbs.push_back(box);
    }
    o.hulls.push_back(Hull {});
    o.types.push_back(PrimType::Plane);
    o.metadata.push_back(Metadata { { 0, 0, 0 }, 0.f, cfg.muS, cfg.muD });
    o.aabbs.push_back(AABB { { -FLT_MAX, -FLT_MAX, -FLT_MAX }, { FLT_MAX, FLT_MAX, 0.f } });
    return o;
}

}  // namespace orc

using namespace orc;

extern "C" {

// Output record shared with oracle/ref_harness.cpp (RefBodyState).
struct OrcBodyState {
    uint32_t gen;
    int32_t id;
    float pos[3];
    float rot[4];
    float vel[6];
    float prevPos[3];
    float prevRot[4];
    float presolvePos[3];
    float presolveRot[4];
    float presolveVel[6];
    int32_t leafID;
    int32_t objID;
    uint32_t responseType;
};

__attribute__((visibility("default")))
void orc_gen_collisions_inits(int32_t num_worlds, int32_t num_cubes, uint32_t seed,
                              float *pos_out, float *rot_out)
{
    // examples/collisions/collisions.cpp:20-39,48-51,76-80: one mt19937 drawn
    // serially over worlds; per body x, y, z then the Y-axis angle.
    std::mt19937 gen(seed);
    std::uniform_real_distribution<float> xd(-10.f, 10.f), yd(-10.f, 10.f), zd(0.f, 10.f);
    std::uniform_real_distribution<float> ad(0.f, 3.14159265358979323846264338327950288f);
    for (int64_t w = 0; w < num_worlds; w++) {
        for (int64_t i = 0; i < num_cubes; i++) {
            int64_t k = w * num_cubes + i;
            float x = xd(gen), y = yd(gen), z = zd(gen);
            float angle = ad(gen);
            pos_out[3 * k] = x; pos_out[3 * k + 1] = y; pos_out[3 * k + 2] = z;
            float ch = cosf(angle / 2.f), sh = sinf(angle / 2.f);   // Quat::angleAxis
            rot_out[4 * k] = ch;
            rot_out[4 * k + 1] = 0.f * sh;
            rot_out[4 * k + 2] = 1.f * sh;
            rot_out[4 * k + 3] = 0.f * sh;
        }
    }
}

__attribute__((visibility("default")))
void *orc_phys_create(int32_t num_worlds, const Config *cfg,
                      const float *pos, const float *rot)
{
    auto *sim = new Sim {};
    sim->cfg = *cfg;
    sim->objs = makeObjects(*cfg);
    sim->worlds.resize(num_worlds);
    for (int32_t w = 0; w < num_worlds; w++) {
        initWorld(*sim, sim->worlds[w], pos + (size_t)w * cfg->numCubes * 3,
                  rot + (size_t)w * cfg->numCubes * 4);
    }
    return sim;
}

// One hull of the asset path, for pinning HalfEdgeMesh::construct and the
// AABB against the reference (ref_build_hull) and the product's loader
// (mw_load_hull): counts_out = {vertices, faces, edges, half edges}; outputs
// sized by the caller (vertices num_verts, faces num_faces, half edges and
// edges 2 * total face indices).
__attribute__((visibility("default")))
void orc_build_hull(int32_t num_verts, const float *verts, int32_t num_faces,
                    const int32_t *face_counts, const uint32_t *indices, int32_t *counts_out,
                    float *verts_out, float *planes_out, uint32_t *half_edges_out,
                    uint32_t *polys_out, uint32_t *edges_out, float *aabb_out)
{
    Config cfg {};
    Objects o = makeHullObjects(cfg, 1, &num_verts, verts, &num_faces, face_counts, indices);
    const Hull &h = o.hulls[0];
    counts_out[0] = (int32_t)h.vertices.size();
    counts_out[1] = (int32_t)h.polygons.size();
    counts_out[2] = (int32_t)h.edges.size();
    counts_out[3] = (int32_t)h.halfEdges.size();
    memcpy(verts_out, h.vertices.data(), 12 * h.vertices.size());
    memcpy(planes_out, h.facePlanes.data(), 16 * h.facePlanes.size());
    memcpy(half_edges_out, h.halfEdges.data(), 16 * h.halfEdges.size());
    memcpy(polys_out, h.polygons.data(), 4 * h.polygons.size());
    memcpy(edges_out, h.edges.data(), 4 * h.edges.size());
    memcpy(aabb_out, &o.aabbs[0], 24);
}

// Collisions worlds over OBJ hulls: body i uses hull i % num_hulls.  Hull h
// has num_verts[h] vertices (xyz, concatenated in verts) and num_faces[h]
// polygons (vertex counts in face_counts, indices concatenated).
__attribute__((visibility("default")))
void *orc_phys_create_hulls(int32_t num_worlds, const Config *cfg, const float *pos,
                            const float *rot, int32_t num_hulls, const int32_t *num_verts,
                            const float *verts, const int32_t *num_faces,
                            const int32_t *face_counts, const uint32_t *indices)
{
    auto *sim = new Sim {};
    sim->cfg = *cfg;
    sim->numHulls = num_hulls;
    sim->objs = makeHullObjects(*cfg, num_hulls, num_verts, verts, num_faces, face_counts,
                                indices);
    sim->worlds.resize(num_worlds);
    for (int32_t w = 0; w < num_worlds; w++) {
        initWorld(*sim, sim->worlds[w], pos + (size_t)w * cfg->numCubes * 3,
                  rot + (size_t)w * cfg->numCubes * 4);
    }
    return sim;
}

// Steps every world num_steps times on up to num_threads host threads
// (worlds are independent, so the split never changes a result).
__attribute__((visibility("default")))
void orc_phys_step(void *handle, int32_t num_steps, int32_t num_threads)
{
    auto *sim = (Sim *)handle;
    int32_t W = (int32_t)sim->worlds.size();
    if (num_threads <= 1) {
        for (int32_t s = 0; s < num_steps; s++)
            for (World &w : sim->worlds) stepWorld(*sim, w);
        return;
    }
    std::vector<std::thread> pool;
    for (int32_t t = 0; t < num_threads; t++) {
        pool.emplace_back([=]() {
            for (int32_t w = t; w < W; w += num_threads)
                for (int32_t s = 0; s < num_steps; s++) stepWorld(*sim, sim->worlds[w]);
        });
    }
    for (auto &th : pool) th.join();
}

__attribute__((visibility("default")))
int32_t orc_phys_read_bodies(void *handle, int32_t world, OrcBodyState *out)
{
    auto *sim = (Sim *)handle;
    World &w = sim->worlds[world];
    for (size_t i = 0; i < w.bodies.size(); i++) {
        const Body &b = w.bodies[i];
        OrcBodyState &o = out[i];
        o.gen = b.e.gen; o.id = b.e.id;
        memcpy(o.pos, &b.pos, 12); memcpy(o.rot, &b.rot, 16);
        memcpy(o.vel, &b.vLin, 12); memcpy(o.vel + 3, &b.vAng, 12);
        memcpy(o.prevPos, &b.prevPos, 12); memcpy(o.prevRot, &b.prevRot, 16);
        memcpy(o.presolvePos, &b.psX, 12); memcpy(o.presolveRot, &b.psQ, 16);
        memcpy(o.presolveVel, &b.psV, 12); memcpy(o.presolveVel + 3, &b.psOmega, 12);
        o.leafID = b.leafID; o.objID = b.objID; o.responseType = (uint32_t)b.resp;
    }
    return (int32_t)w.bodies.size();
}

__attribute__((visibility("default")))
int32_t orc_phys_read_bvh(void *handle, int32_t world, void *nodes_out,
                          float *leaf_aabbs_out, uint32_t *leaf_parents_out,
                          int32_t *sorted_leaves_out)
{
    auto *sim = (Sim *)handle;
    World &w = sim->worlds[world];
    // Nodes past usedNodes are never written by the reference build
    // (uninitialised rawAlloc memory there), so only the used prefix is
    // meaningful; the return value is that prefix length.
    if (nodes_out) memcpy(nodes_out, w.nodes.data(), sizeof(BVHNode) * w.usedNodes);
    if (leaf_aabbs_out) memcpy(leaf_aabbs_out, w.leafAABBs.data(), sizeof(AABB) * w.numLeaves);
    if (leaf_parents_out) memcpy(leaf_parents_out, w.leafParents.data(), 4 * w.numLeaves);
    if (sorted_leaves_out) memcpy(sorted_leaves_out, w.sortedLeaves.data(), 4 * w.numLeaves);
    return w.usedNodes;
}

// Candidates found by the last step's findOverlapping node: (a, b) Locs.
__attribute__((visibility("default")))
int32_t orc_phys_read_candidates(void *handle, int32_t world, int32_t *out, int32_t cap)
{
    auto *sim = (Sim *)handle;
    World &w = sim->worlds[world];
    int32_t n = (int32_t)w.lastCandidates.size();
    for (int32_t i = 0; i < n && i < cap; i++) {
        out[4 * i] = (int32_t)w.lastCandidates[i].first.archetype;
        out[4 * i + 1] = w.lastCandidates[i].first.row;
        out[4 * i + 2] = (int32_t)w.lastCandidates[i].second.archetype;
        out[4 * i + 3] = w.lastCandidates[i].second.row;
    }
    return n;
}

// Contacts of the last substep of the last step (112-B records, lambdaN
// filled by solvePositions).  Returns the count.
__attribute__((visibility("default")))
int32_t orc_phys_read_contacts(void *handle, int32_t world, void *out, int32_t cap)
{
    auto *sim = (Sim *)handle;
    World &w = sim->worlds[world];
    int32_t n = (int32_t)w.lastContacts.size();
    if (n > 0 && cap > 0) memcpy(out, w.lastContacts.data(), sizeof(Contact) * std::min(n, cap));
    return n;
}

// Cumulative count of face manifolds whose reference result is undefined
// (see buildFaceContactManifold); parity against the live reference holds
// only while this is zero.
__attribute__((visibility("default")))
int32_t orc_phys_ub_manifolds(void *handle, int32_t world)
{
    return ((Sim *)handle)->worlds[world].ubManifolds;
}

// simple_taskgraph worlds (examples/simple_taskgraph/simple.cpp): numCubes
// objects + agent (Agent archetype) + test object; clamp before physics.
__attribute__((visibility("default")))
void *orc_simple_create(int32_t num_worlds, const Config *cfg,
                        const float *pos, const float *rot)
{
    auto *sim = new Sim {};
    sim->cfg = *cfg;
    sim->simple = true;
    sim->objs = makeObjects(*cfg);
    sim->worlds.resize(num_worlds);
    for (int32_t w = 0; w < num_worlds; w++) {
        initWorld(*sim, sim->worlds[w], pos + (size_t)w * cfg->numCubes * 3,
                  rot + (size_t)w * cfg->numCubes * 4);
    }
    return sim;
}

__attribute__((visibility("default")))
void orc_phys_destroy(void *handle)
{
    delete (Sim *)handle;
}

}
