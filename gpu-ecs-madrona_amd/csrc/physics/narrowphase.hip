// Substep integration + narrowphase kernels (reference src/physics/physics.cpp:79-164,
// src/physics/narrowphase.cpp CPU branch).
#include "physics_device.hpp"

#include <cfloat>

namespace madrona::phys {

// ===========================================================================
// Substep integration (physics.cpp:79-164) fused with the world-space hull
// transform the narrowphase needs (narrowphase.cpp:139-212, CPU branch).
// ===========================================================================

__global__ void __launch_bounds__(256) integrateKernel(PhysArgs P)
{
    const BodyArch &B = P.body[blockIdx.y];
    RowIdx ri = rowIndex(P, B);
    if (!ri.valid) return;
    const int32_t w = ri.w, r = ri.r;

    Vector3 &pos = bcol<Vector3>(B, Cols::Position, w, r);
    Quat &rot = bcol<Quat>(B, Cols::Rotation, w, r);
    const Velocity vel = bcol<Velocity>(B, Cols::Velocity, w, r);
    const int32_t obj = bcol<ObjectID>(B, Cols::ObjectID, w, r).idx;
    const ResponseType rt = bcol<ResponseType>(B, Cols::ResponseType, w, r);
    auto &prev = bcol<solver::SubstepPrevState>(B, Cols::SubstepPrevState, w, r);
    auto &ps_pos = bcol<solver::PreSolvePositional>(B, Cols::PreSolvePositional, w, r);
    auto &ps_vel = bcol<solver::PreSolveVelocity>(B, Cols::PreSolveVelocity, w, r);

    Vector3 x = pos;
    Quat q = rot;
    if (rt == ResponseType::Static) {
        prev.prevPosition = x;
        prev.prevRotation = q;
        ps_pos.x = x;
        ps_pos.q = q;
        ps_vel.v = Vector3::zero();
        ps_vel.omega = Vector3::zero();
    } else {
        Vector3 v = vel.linear;
        Vector3 omega = vel.angular;
        prev.prevPosition = x;
        prev.prevRotation = q;
        const SolverData &solver = P.solver[w];
        const RigidBodyMetadata md = P.objs.metadata[obj];
        const float inv_m = md.invMass;
        const Vector3 inv_I = md.invInertiaTensor;
        const float h = solver.h;
        const Vector3 ext_force = bcol<Vector3>(B, Cols::ExternalForce, w, r);
        const Vector3 ext_torque = bcol<Vector3>(B, Cols::ExternalTorque, w, r);
        if (rt == ResponseType::Dynamic) v += h * solver.g;
        v += h * inv_m * ext_force;
        x += h * v;
        Vector3 I {
            (inv_I.x == 0) ? 0.0f : 1.0f / inv_I.x,
            (inv_I.y == 0) ? 0.0f : 1.0f / inv_I.y,
            (inv_I.z == 0) ? 0.0f : 1.0f / inv_I.z,
        };
        Quat to_local = q.inv();
        Vector3 tau_ext_local = to_local.rotateVec(ext_torque);
        Vector3 omega_local = to_local.rotateVec(omega);
        Vector3 I_omega_local = multDiag(I, omega_local);
        omega_local += h * multDiag(inv_I, tau_ext_local - cross(omega_local, I_omega_local));
        omega = q.rotateVec(omega_local);
        Quat apply_omega = Quat::fromAngularVec(0.5f * h * omega);
        q += apply_omega * q;
        q = q.normalize();
        pos = x;
        rot = q;
        ps_pos.x = x;
        ps_pos.q = q;
        ps_vel.v = v;
        ps_vel.omega = omega;
    }

    const Diag3x3 scale = bcol<Diag3x3>(B, Cols::Scale, w, r);
    const int32_t leaf = bcol<broadphase::LeafID>(B, Cols::LeafID, w, r).id;
    // World AABB the narrowphase recheck uses (narrowphase.cpp:1590-1594).
    P.bodyAABBs[(size_t)w * P.maxLeaves + leaf] = P.objs.aabbs[obj].applyTRS(x, q, scale);

    // World-space hull for this body (makeHullState with dst buffers).
    if (P.objs.types[obj] == (uint32_t)CollisionPrimitive::Type::Hull) {
        const HullDev hd = P.objs.hulls[obj];
        Mat3x3 unscaled_rot = Mat3x3::fromQuat(q);
        Mat3x3 vertex_txfm = unscaled_rot * scale;
        Mat3x3 normal_txfm = unscaled_rot * scale.inv();
        Vector3 *dv = P.hullVerts + ((size_t)w * P.maxLeaves + leaf) * P.objs.maxVerts;
        geometry::Plane *dp = P.hullPlanes + ((size_t)w * P.maxLeaves + leaf) * P.objs.maxFaces;
        for (int32_t i = 0; i < hd.numVerts; i++) {
            dv[i] = vertex_txfm * P.objs.vertices[hd.vertOffset + i] + x;
        }
        for (int32_t i = 0; i < hd.numFaces; i++) {
            geometry::Plane op = P.objs.planes[hd.faceOffset + i];
            Vector3 origin = vertex_txfm * (op.normal * op.d) + x;
            Vector3 n = (normal_txfm * op.normal).normalize();
            dp[i] = geometry::Plane { n, dot(n, origin) };
        }
    }
}

// ===========================================================================
// Narrowphase (narrowphase.cpp, CPU branch).
//
// A 16-lane group owns one candidate pair at a time: the SAT queries
// (face directions A->B and B->A, all edge pairs) are spread over the
// group's lanes and combined with (value, index) reductions whose tie-break
// reproduces the reference's serial strict-'>' scan exactly (first
// occurrence wins, NaN never wins); the clip / manifold tail runs on the
// group's leader lane with its scratch polygons in LDS.
// ===========================================================================
constexpr int32_t kGroup = 16;
constexpr int32_t kGroupsPerBlock = kNarrowBlock / kGroup;
constexpr int32_t kMaxClip = 32;

struct HullRef {
    const Vector3 *verts;          // world space
    const geometry::Plane *planes; // world space
    HullDev hd;
    Vector3 center;
};

// Per-edge SAT inputs gathered once per pair (edgeDistance's operands,
// narrowphase.cpp:433-472 via queryEdgeDirections :474-540).
struct EdgeRec {
    Vector3 n1, n2;                // normals of the two faces sharing the edge
    Vector3 p1, p2;                // root vertex, root vertex of next
};

struct GroupScratch {
    EdgeRec *edgesA;               // [maxEdges]
    EdgeRec *edgesB;               // [maxEdges]
    Vector3 *clip0;                // [kMaxClip]
    Vector3 *clip1;                // [kMaxClip]
    float *depths;                 // [kMaxClip]
};

__host__ __device__ inline size_t groupScratchBytes(int32_t max_edges)
{
    return (size_t)2 * max_edges * sizeof(EdgeRec) + 2 * kMaxClip * sizeof(Vector3) +
           kMaxClip * sizeof(float);
}

size_t narrowphaseSharedBytes(const PhysArgs &P)
{
    return kGroupsPerBlock * groupScratchBytes(P.objs.maxEdges);
}

__device__ __forceinline__ GroupScratch groupScratch(char *smem, int32_t group, int32_t max_edges)
{
    char *p = smem + (size_t)group * groupScratchBytes(max_edges);
    GroupScratch g;
    g.edgesA = (EdgeRec *)p;
    p += max_edges * sizeof(EdgeRec);
    g.edgesB = (EdgeRec *)p;
    p += max_edges * sizeof(EdgeRec);
    g.clip0 = (Vector3 *)p;
    p += kMaxClip * sizeof(Vector3);
    g.clip1 = (Vector3 *)p;
    p += kMaxClip * sizeof(Vector3);
    g.depths = (float *)p;
    return g;
}

// LDS writes of one lane are visible to the other lanes of its wave once the
// wave's LDS queue drains; this keeps the compiler from moving accesses
// across that point.
__device__ __forceinline__ void groupSync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Would (v1, k1) replace (v2, k2) in a serial `if (v > best)` scan visiting
// indices in increasing order?  NaN never wins; ties go to the lower index.
__device__ __forceinline__ bool scanWins(float v1, int32_t k1, float v2, int32_t k2)
{
    if (v1 != v1) return false;
    if (v2 != v2) return true;
    return v1 > v2 || (v1 == v2 && k1 < k2);
}

__device__ __forceinline__ void groupArgMax(float &v, int32_t &k)
{
#pragma unroll
    for (int32_t off = kGroup / 2; off > 0; off >>= 1) {
        const float ov = __shfl_xor(v, off, kGroup);
        const int32_t ok = __shfl_xor(k, off, kGroup);
        if (scanWins(ov, ok, v, k)) { v = ov; k = ok; }
    }
}

__device__ __forceinline__ float distFromPlane(const geometry::Plane &p, const Vector3 &a)
{
    float adotn = a.dot(p.normal);
    return adotn - p.d;
}

__device__ __forceinline__ Vector3 planeIntersection(const geometry::Plane &p, const Vector3 &p1,
                                                     const Vector3 &p2)
{
    float distance = distFromPlane(p, p1);
    return p1 + (p2 - p1) * (-distance / p.normal.dot(p2 - p1));
}

__device__ __forceinline__ float hullDistFromPlane(const geometry::Plane &p, const HullRef &h)
{
    float min_dot = FLT_MAX;
    for (int32_t i = 0; i < h.hd.numVerts; i++) {
        float d = p.normal.dot(h.verts[i]);
        if (d < min_dot) min_dot = d;
    }
    return min_dot - p.d;
}

struct FaceQuery {
    float separation;
    int32_t faceIdx;
    geometry::Plane plane;
};

// queryFaceDirections (narrowphase.cpp:395-431).  The reference stops at the
// first face with positive distance; any positive result rejects the pair,
// so the group evaluates every face and only the non-positive case needs the
// serial argmax, which groupArgMax reproduces.
__device__ FaceQuery groupFaceQuery(const HullRef &a, const HullRef &b, int32_t lane)
{
    float v = __builtin_nanf("");
    int32_t k = INT32_MAX;
    for (int32_t f = lane; f < a.hd.numFaces; f += kGroup) {
        const float d = hullDistFromPlane(a.planes[f], b);
        if (scanWins(d, f, v, k)) { v = d; k = f; }
    }
    groupArgMax(v, k);
    if (v > -FLT_MAX) return { v, k, a.planes[k] };
    return { -FLT_MAX, -1, geometry::Plane { { 0, 0, 0 }, 0 } };
}

__device__ __forceinline__ bool isMinkowskiFace(const Vector3 &a, const Vector3 &b,
                                                const Vector3 &c, const Vector3 &d)
{
    Vector3 bxa = b.cross(a);
    Vector3 dxc = d.cross(c);
    float cba = c.dot(bxa);
    float dba = d.dot(bxa);
    float adc = a.dot(dxc);
    float bdc = b.dot(dxc);
    return cba * dba < 0.0f && adc * bdc < 0.0f && cba * bdc > 0.0f;
}

// edgeDistance (narrowphase.cpp:433-472) for one edge pair: separation along
// the edges' cross product, or -FLT_MAX when the edges do not form a face of
// the Minkowski difference or are parallel.
__device__ __forceinline__ float edgePairSeparation(const EdgeRec &ea, const EdgeRec &eb,
                                                    const Vector3 &a_center, Vector3 *normal_out)
{
    float sep = -FLT_MAX;
    Vector3 n { 0, 0, 0 };
    if (isMinkowskiFace(ea.n1, ea.n2, -eb.n1, -eb.n2)) {
        Vector3 da = ea.p2 - ea.p1, db = eb.p2 - eb.p1;
        Vector3 uc = da.cross(db);
        float l2 = uc.length2();
        if (l2 != 0) {
            float inv = 1.f / sqrtf(l2);
            n = uc * inv;
            if (n.dot(ea.p1 - a_center) < 0.0f) n = -n;
            sep = n.dot(eb.p1 - ea.p1);
        }
    }
    if (normal_out) *normal_out = n;
    return sep;
}

__device__ __forceinline__ void stageEdges(const ObjDev &O, const HullRef &h, EdgeRec *dst,
                                           int32_t lane)
{
    const geometry::HalfEdge *he = O.hedges + h.hd.hedgeOffset;
    for (int32_t i = lane; i < h.hd.numEdges; i += kGroup) {
        const geometry::HalfEdge e = he[O.edges[h.hd.edgeOffset + i]];
        EdgeRec r;
        r.n1 = h.planes[e.polygon].normal;
        r.n2 = h.planes[he[e.twin].polygon].normal;
        r.p1 = h.verts[e.rootVertex];
        r.p2 = h.verts[he[e.next].rootVertex];
        dst[i] = r;
    }
}

struct EdgeQuery {
    float separation;
    Vector3 normal;
    int32_t edgeA;                 // half-edge indices (queryEdgeDirections' result)
    int32_t edgeB;
};

// queryEdgeDirections (narrowphase.cpp:474-540) over the staged edge records.
// Pair index k = i * nB + j is the reference's loop order.
__device__ EdgeQuery groupEdgeQuery(const ObjDev &O, const HullRef &a, const HullRef &b,
                                    const GroupScratch &g, int32_t lane)
{
    const int32_t nA = a.hd.numEdges, nB = b.hd.numEdges;
    float v = __builtin_nanf("");
    int32_t k = INT32_MAX;
    for (int32_t p = lane; p < nA * nB; p += kGroup) {
        const int32_t i = p / nB, j = p - i * nB;
        const float sep = edgePairSeparation(g.edgesA[i], g.edgesB[j], a.center, nullptr);
        if (scanWins(sep, p, v, k)) { v = sep; k = p; }
    }
    groupArgMax(v, k);
    if (!(v > -FLT_MAX)) return { -FLT_MAX, { 0, 0, 0 }, 0, 0 };
    const int32_t i = k / nB, j = k - i * nB;
    EdgeQuery q;
    q.separation = edgePairSeparation(g.edgesA[i], g.edgesB[j], a.center, &q.normal);
    q.edgeA = (int32_t)O.edges[a.hd.edgeOffset + i];
    q.edgeB = (int32_t)O.edges[b.hd.edgeOffset + j];
    return q;
}

__device__ __forceinline__ int32_t findIncidentFace(const HullRef &h, Vector3 ref_normal)
{
    float min_dot = FLT_MAX;
    int32_t face = -1;
    for (int32_t f = 0; f < h.hd.numFaces; f++) {
        float d = dot(h.planes[f].normal, ref_normal);
        if (d < min_dot) { min_dot = d; face = f; }
    }
    return face;
}

__device__ __forceinline__ int32_t clipPolygon(Vector3 *dst, geometry::Plane cp,
                                               const Vector3 *in, int32_t n)
{                                                          // narrowphase.cpp:626-661
    if (n == 0) return 0;
    int32_t out = 0;
    Vector3 v1 = in[n - 1];
    float d1 = distFromPlane(cp, v1);
    for (int32_t i = 0; i < n; i++) {
        Vector3 v2 = in[i];
        float d2 = distFromPlane(cp, v2);
        if (d1 <= 0.0f && d2 <= 0.0f) {
            if (out < kMaxClip) dst[out++] = v2;
        } else if (d1 <= 0.0f && d2 > 0.0f) {
            if (out < kMaxClip) dst[out++] = planeIntersection(cp, v1, v2);
        } else if (d2 <= 0.0f && d1 > 0.0f) {
            if (out < kMaxClip) dst[out++] = planeIntersection(cp, v1, v2);
            if (out < kMaxClip) dst[out++] = v2;
        }
        v1 = v2;
        d1 = d2;
    }
    return out;
}

// buildFaceContactManifold (narrowphase.cpp:790-864) written straight into
// the contact slot.
__device__ void storeFaceManifold(Contact &c, Vector3 n, Vector3 *contacts, const float *depths,
                                  int32_t num, Loc ref, Loc alt)
{
    Vector3 cp[4];
    float depth[4];
    for (int i = 0; i < 4; i++) { cp[i] = Vector3::zero(); depth[i] = 0.f; }
    int32_t m;
    if (num <= 4) {
        m = num;
        for (int32_t i = 0; i < num; i++) { cp[i] = contacts[i]; depth[i] = depths[i]; }
    } else {
        m = 4;
        cp[0] = contacts[0];
        depth[0] = depths[0];
        Vector3 p0 = cp[0];
        float largest_d2 = 0.0f;
        int32_t largest_d2_idx = 0;
        for (int32_t i = 1; i < num; i++) {
            Vector3 c2 = contacts[i];
            float d2 = p0.distance2(c2);
            if (d2 > largest_d2) {
                largest_d2 = d2;
                cp[1] = c2;
                depth[1] = depths[i];
                largest_d2_idx = i;
            }
        }
        contacts[largest_d2_idx] = cp[0];
        Vector3 diff0 = cp[1] - p0;
        const float largest_area = 0.0f;        // never updated in the reference
        int32_t largest_area_idx = 0;
        for (int32_t i = 1; i < num; i++) {
            Vector3 c2 = contacts[i];
            Vector3 diff1 = c2 - p0;
            float area = n.dot(diff0.cross(diff1));
            if (area > largest_area) {
                cp[2] = c2;
                depth[2] = depths[i];
                largest_area_idx = i;
            }
        }
        contacts[largest_area_idx] = cp[0];
        for (int32_t i = 1; i < num; i++) {
            Vector3 c2 = contacts[i];
            Vector3 diff1 = c2 - p0;
            float area = n.dot(diff0.cross(diff1));
            if (area < largest_area) {
                cp[3] = c2;
                depth[3] = depths[i];
            }
        }
    }
    if (m == 0) return;
    const Quat ident { 1, 0, 0, 0 };
    c.ref = ref;
    c.alt = alt;
    for (int i = 0; i < 4; i++) {
        Vector3 p = (i < m) ? ident.rotateVec(cp[i]) + Vector3::zero() : cp[i];
        c.points[i] = Vector4::fromVector3(p, depth[i]);
    }
    c.numPoints = m;
    c.normal = ident.rotateVec(n);
    for (int i = 0; i < 4; i++) c.lambdaN[i] = 0.f;
}

__device__ __forceinline__ geometry::Segment shortestSegmentBetween(const geometry::Segment &s1,
                                                                    const geometry::Segment &s2)
{                                                          // narrowphase.cpp:1020-1051
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

// Candidate order: runNarrowphase's type swap (narrowphase.cpp:1574-1580).
struct CandBodies {
    Loc a_loc, b_loc;
    const BodyArch *BA, *BB;
    int32_t a_obj, b_obj;
    uint32_t ta, tb;
};

__device__ __forceinline__ CandBodies orderCandidate(const PhysArgs &P, int32_t w,
                                                     const CandidateCollision &cand)
{
    const ObjDev &O = P.objs;
    CandBodies c;
    c.a_loc = cand.a;
    c.b_loc = cand.b;
    c.BA = &P.body[bodyArchIndex(P, c.a_loc.archetype)];
    c.BB = &P.body[bodyArchIndex(P, c.b_loc.archetype)];
    c.a_obj = bcol<ObjectID>(*c.BA, Cols::ObjectID, w, c.a_loc.row).idx;
    c.b_obj = bcol<ObjectID>(*c.BB, Cols::ObjectID, w, c.b_loc.row).idx;
    c.ta = O.types[c.a_obj];
    c.tb = O.types[c.b_obj];
    if (c.ta > c.tb) {
        Loc tl = c.a_loc; c.a_loc = c.b_loc; c.b_loc = tl;
        const BodyArch *tB = c.BA; c.BA = c.BB; c.BB = tB;
        int32_t to = c.a_obj; c.a_obj = c.b_obj; c.b_obj = to;
        uint32_t tt = c.ta; c.ta = c.tb; c.tb = tt;
    }
    return c;
}

// World-space AABB recheck (narrowphase.cpp:1589-1603) against the per-body
// AABBs the integrate kernel cached (same applyTRS, same inputs).
__device__ __forceinline__ bool candidateOverlaps(const PhysArgs &P, int32_t w,
                                                  const CandidateCollision &cand)
{
    const BodyArch &BA = P.body[bodyArchIndex(P, cand.a.archetype)];
    const BodyArch &BB = P.body[bodyArchIndex(P, cand.b.archetype)];
    const int32_t la = bcol<broadphase::LeafID>(BA, Cols::LeafID, w, cand.a.row).id;
    const int32_t lb = bcol<broadphase::LeafID>(BB, Cols::LeafID, w, cand.b.row).id;
    const AABB a = P.bodyAABBs[(size_t)w * P.maxLeaves + la];
    const AABB b = P.bodyAABBs[(size_t)w * P.maxLeaves + lb];
    return a.overlaps(b);
}

__device__ __forceinline__ HullRef hullOf(const PhysArgs &P, int32_t w, const BodyArch &B,
                                          Loc loc, int32_t obj)
{
    const int32_t leaf = bcol<broadphase::LeafID>(B, Cols::LeafID, w, loc.row).id;
    HullRef h;
    h.hd = P.objs.hulls[obj];
    h.verts = P.hullVerts + ((size_t)w * P.maxLeaves + leaf) * P.objs.maxVerts;
    h.planes = P.hullPlanes + ((size_t)w * P.maxLeaves + leaf) * P.objs.maxFaces;
    h.center = bcol<Vector3>(B, Cols::Position, w, loc.row);
    return h;
}

// Hull-hull: doSAT (narrowphase.cpp:678-758) on the group, then
// createFaceContact (:866-972) or createEdgeContact (:1053-1121) on the
// leader lane.  All group lanes must enter.
__device__ void hullHullPair(const PhysArgs &P, int32_t w, const CandBodies &cb,
                             const GroupScratch &g, int32_t lane, Contact &out)
{
    const ObjDev &O = P.objs;
    const HullRef ha = hullOf(P, w, *cb.BA, cb.a_loc, cb.a_obj);
    const HullRef hb = hullOf(P, w, *cb.BB, cb.b_loc, cb.b_obj);

    const FaceQuery fa = groupFaceQuery(ha, hb, lane);
    if (fa.separation > 0.0f) return;
    const FaceQuery fb = groupFaceQuery(hb, ha, lane);
    if (fb.separation > 0.0f) return;
    stageEdges(O, ha, g.edgesA, lane);
    stageEdges(O, hb, g.edgesB, lane);
    groupSync();
    const EdgeQuery eq = groupEdgeQuery(O, ha, hb, g, lane);
    groupSync();
    if (eq.separation > 0.0f) return;
    if (lane != 0) return;

    if (fa.separation > eq.separation || fb.separation > eq.separation) {
        const bool a_is_ref = fa.separation >= fb.separation;
        const geometry::Plane ref_plane = a_is_ref ? fa.plane : fb.plane;
        const int32_t ref_face = a_is_ref ? fa.faceIdx : fb.faceIdx;
        const HullRef &ref = a_is_ref ? ha : hb;
        const HullRef &inc = a_is_ref ? hb : ha;
        const int32_t inc_face = findIncidentFace(inc, ref_plane.normal);

        const geometry::HalfEdge *rh = O.hedges + ref.hd.hedgeOffset;
        const geometry::HalfEdge *oh = O.hedges + inc.hd.hedgeOffset;
        int32_t n_in = 0;
        {
            uint32_t hidx = O.polygons[inc.hd.faceOffset + inc_face], start = hidx;
            do {
                const geometry::HalfEdge he = oh[hidx];
                hidx = he.next;
                if (n_in < kMaxClip) g.clip0[n_in++] = inc.verts[he.rootVertex];
            } while (hidx != start);
        }
        Vector3 *cin = g.clip0, *cdst = g.clip1;
        int32_t n_clip = n_in;
        {
            uint32_t hidx = O.polygons[ref.hd.faceOffset + ref_face], start = hidx;
            geometry::HalfEdge che = rh[hidx];
            Vector3 cur = ref.verts[che.rootVertex];
            do {
                hidx = che.next;
                che = rh[hidx];
                Vector3 next = ref.verts[che.rootVertex];
                Vector3 edge = next - cur;
                Vector3 pn = cross(edge, ref_plane.normal);
                float d = dot(pn, cur);
                cur = next;
                n_clip = clipPolygon(cdst, geometry::Plane { pn, d }, cin, n_clip);
                Vector3 *t = cdst; cdst = cin; cin = t;
            } while (hidx != start);
        }
        int32_t n_below = 0;
        for (int32_t i = 0; i < n_clip; i++) {
            Vector3 v = cin[i];
            float d = distFromPlane(ref_plane, v);
            if (d < 0.0f) {
                cin[n_below] = v - d * ref_plane.normal;
                g.depths[n_below] = -d;
                n_below++;
            }
        }
        storeFaceManifold(out, ref_plane.normal, cin, g.depths, n_below,
                          a_is_ref ? cb.a_loc : cb.b_loc, a_is_ref ? cb.b_loc : cb.a_loc);
    } else {
        const geometry::HalfEdge *ha_e = O.hedges + ha.hd.hedgeOffset;
        const geometry::HalfEdge *hb_e = O.hedges + hb.hd.hedgeOffset;
        const geometry::HalfEdge ea = ha_e[eq.edgeA];
        const geometry::HalfEdge eb = hb_e[eq.edgeB];
        geometry::Segment sa { ha.verts[ea.rootVertex], ha.verts[ha_e[ea.next].rootVertex] };
        geometry::Segment sb { hb.verts[eb.rootVertex], hb.verts[hb_e[eb.next].rootVertex] };
        geometry::Segment s = shortestSegmentBetween(sa, sb);
        const Quat ident { 1, 0, 0, 0 };
        out.ref = cb.a_loc;
        out.alt = cb.b_loc;
        out.points[0] = Vector4::fromVector3(ident.rotateVec(s.p1) + Vector3::zero(),
                                             -eq.separation);
        for (int i = 1; i < 4; i++) out.points[i] = Vector4::fromVector3(Vector3::zero(), 0.f);
        out.numPoints = 1;
        out.normal = ident.rotateVec(eq.normal);
        for (int i = 0; i < 4; i++) out.lambdaN[i] = 0.f;
    }
}

// Hull-plane: doSATPlane (narrowphase.cpp:760-788) + createFacePlaneContact
// (:974-1017) on the leader lane.
__device__ void hullPlanePair(const PhysArgs &P, int32_t w, const CandBodies &cb,
                              const GroupScratch &g, Contact &out)
{
    const ObjDev &O = P.objs;
    const HullRef ha = hullOf(P, w, *cb.BA, cb.a_loc, cb.a_obj);
    const Vector3 b_pos = bcol<Vector3>(*cb.BB, Cols::Position, w, cb.b_loc.row);
    const Quat b_rot = bcol<Quat>(*cb.BB, Cols::Rotation, w, cb.b_loc.row);
    Vector3 pn = b_rot.rotateVec(Vector3 { 0, 0, 1 });
    geometry::Plane plane { pn, dot(pn, b_pos) };
    float sep = hullDistFromPlane(plane, ha);
    if (sep > 0.0f) return;
    int32_t inc_face = findIncidentFace(ha, plane.normal);
    const geometry::HalfEdge *hh = O.hedges + ha.hd.hedgeOffset;
    int32_t n = 0;
    uint32_t hidx = O.polygons[ha.hd.faceOffset + inc_face], start = hidx;
    do {
        const geometry::HalfEdge he = hh[hidx];
        hidx = he.next;
        Vector3 v = ha.verts[he.rootVertex];
        float d = distFromPlane(plane, v);
        if (d < 0.0f && n < kMaxClip) {
            g.clip0[n] = v - d * plane.normal;
            g.depths[n] = -d;
            n++;
        }
    } while (hidx != start);
    storeFaceManifold(out, plane.normal, g.clip0, g.depths, n, cb.b_loc, cb.a_loc);
}

// runNarrowphaseSystem over every candidate of a world (one block per world):
//   A. lane-per-candidate AABB recheck, block scan -> survivor list (order kept)
//   B. group-per-survivor SAT + contact generation into survivor slots
//   C. block scan of survivors with a manifold -> the solver's contact order
//      (== the reference's addManifoldToSolver append order).
__global__ void __launch_bounds__(kNarrowBlock) narrowphaseKernel(PhysArgs P)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ int32_t s_scan[kNarrowBlock / 64];
    const int32_t w = blockIdx.x;
    const int32_t num = min(P.numCands[w], P.candCapacity);
    const CandidateCollision *cands = P.cands + (size_t)w * P.candCapacity;
    int32_t *surv = P.survivors + (size_t)w * P.candCapacity;
    Contact *slots = P.candContacts + (size_t)w * P.candCapacity;

    int32_t S = 0;
    for (int32_t chunk = 0; chunk < num; chunk += kNarrowBlock) {
        const int32_t ci = chunk + threadIdx.x;
        const int32_t keep = (ci < num && candidateOverlaps(P, w, cands[ci])) ? 1 : 0;
        int32_t total;
        const int32_t off = blockExclusiveScan(keep, s_scan, &total);
        if (keep) surv[S + off] = ci;
        S += total;
    }
    __syncthreads();

    const int32_t group = threadIdx.x / kGroup;
    const int32_t lane = threadIdx.x % kGroup;
    const GroupScratch g = groupScratch(smem, group, P.objs.maxEdges);
    for (int32_t s = group; s < S; s += kGroupsPerBlock) {
        const CandBodies cb = orderCandidate(P, w, cands[surv[s]]);
        Contact &out = slots[s];
        if (lane == 0) out.numPoints = 0;
        const uint32_t test = cb.ta | cb.tb;
        if (test == (uint32_t)CollisionPrimitive::Type::Hull) {
            hullHullPair(P, w, cb, g, lane, out);
        } else if (test == ((uint32_t)CollisionPrimitive::Type::Hull |
                            (uint32_t)CollisionPrimitive::Type::Plane)) {
            if (lane == 0) hullPlanePair(P, w, cb, g, out);
        }
        // sphere / plane-plane: the reference asserts (narrowphase.cpp:1197-1313)
        groupSync();
    }
    __syncthreads();

    int32_t *order = P.contactOrder + (size_t)w * P.candCapacity;
    int32_t K = 0;
    for (int32_t chunk = 0; chunk < S; chunk += kNarrowBlock) {
        const int32_t s = chunk + threadIdx.x;
        const int32_t has = (s < S && slots[s].numPoints > 0) ? 1 : 0;
        int32_t total;
        const int32_t off = blockExclusiveScan(has, s_scan, &total);
        if (has) order[K + off] = s;
        K += total;
    }
    if (threadIdx.x == 0) {
        if (K > P.maxContacts) {
            // The reference asserts here (narrowphase.cpp:1130); flag, truncate.
            atomicOr(P.errorFlags + w, kErrContactOverflow);
            K = P.maxContacts;
        }
        P.solver[w].numContacts = K;
        P.lastNumContacts[w] = K;
    }
}

}
