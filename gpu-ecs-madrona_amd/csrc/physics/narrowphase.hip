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
// Narrowphase (narrowphase.cpp, CPU branch), one lane per candidate
// ===========================================================================
struct HullRef {
    const Vector3 *verts;          // world space
    const geometry::Plane *planes; // world space
    HullDev hd;
    Vector3 center;
};

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

__device__ FaceQuery queryFaceDirections(const HullRef &a, const HullRef &b)
{
    geometry::Plane max_plane { { 0, 0, 0 }, 0 };
    int32_t max_face = -1;
    float max_dist = -FLT_MAX;
    for (int32_t f = 0; f < a.hd.numFaces; f++) {
        geometry::Plane p = a.planes[f];
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

struct EdgeQuery {
    float separation;
    Vector3 normal;
    int32_t edgeA;
    int32_t edgeB;
};

__device__ EdgeQuery queryEdgeDirections(const ObjDev &O, const HullRef &a, const HullRef &b)
{
    Vector3 normal { 0, 0, 0 };
    int32_t ea_max = 0, eb_max = 0;
    float max_d = -FLT_MAX;
    const geometry::HalfEdge *ha = O.hedges + a.hd.hedgeOffset;
    const geometry::HalfEdge *hb = O.hedges + b.hd.hedgeOffset;
    for (int32_t i = 0; i < a.hd.numEdges; i++) {
        const int32_t he_a = (int32_t)O.edges[a.hd.edgeOffset + i];
        const geometry::HalfEdge ea = ha[he_a];
        const Vector3 an1 = a.planes[ea.polygon].normal;
        const Vector3 an2 = a.planes[ha[ea.twin].polygon].normal;
        const Vector3 pa1 = a.verts[ea.rootVertex];
        const Vector3 pa2 = a.verts[ha[ea.next].rootVertex];
        for (int32_t j = 0; j < b.hd.numEdges; j++) {
            const int32_t he_b = (int32_t)O.edges[b.hd.edgeOffset + j];
            const geometry::HalfEdge eb = hb[he_b];
            const Vector3 bn1 = b.planes[eb.polygon].normal;
            const Vector3 bn2 = b.planes[hb[eb.twin].polygon].normal;
            float sep = -FLT_MAX;
            Vector3 n { 0, 0, 0 };
            if (isMinkowskiFace(an1, an2, -bn1, -bn2)) {      // edgeDistance :433-472
                const Vector3 pb1 = b.verts[eb.rootVertex];
                const Vector3 pb2 = b.verts[hb[eb.next].rootVertex];
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

constexpr int32_t kMaxClip = 32;

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

struct Manifold {
    Vector3 cp[4];
    float depth[4];
    int32_t num;
    Vector3 normal;
};

__device__ Manifold buildFaceContactManifold(Vector3 n, Vector3 *contacts, float *depths,
                                             int32_t num)
{                                                          // narrowphase.cpp:790-864
    Manifold m;
    for (int i = 0; i < 4; i++) { m.cp[i] = Vector3::zero(); m.depth[i] = 0.f; }
    if (num <= 4) {
        m.num = num;
        for (int32_t i = 0; i < num; i++) { m.cp[i] = contacts[i]; m.depth[i] = depths[i]; }
    } else {
        m.num = 4;
        m.cp[0] = contacts[0];
        m.depth[0] = depths[0];
        Vector3 p0 = m.cp[0];
        float largest_d2 = 0.0f;
        int32_t largest_d2_idx = 0;
        for (int32_t i = 1; i < num; i++) {
            Vector3 c = contacts[i];
            float d2 = p0.distance2(c);
            if (d2 > largest_d2) {
                largest_d2 = d2;
                m.cp[1] = c;
                m.depth[1] = depths[i];
                largest_d2_idx = i;
            }
        }
        contacts[largest_d2_idx] = m.cp[0];
        Vector3 diff0 = m.cp[1] - p0;
        const float largest_area = 0.0f;        // never updated in the reference
        int32_t largest_area_idx = 0;
        for (int32_t i = 1; i < num; i++) {
            Vector3 c = contacts[i];
            Vector3 diff1 = c - p0;
            float area = n.dot(diff0.cross(diff1));
            if (area > largest_area) {
                m.cp[2] = c;
                m.depth[2] = depths[i];
                largest_area_idx = i;
            }
        }
        contacts[largest_area_idx] = m.cp[0];
        for (int32_t i = 1; i < num; i++) {
            Vector3 c = contacts[i];
            Vector3 diff1 = c - p0;
            float area = n.dot(diff0.cross(diff1));
            if (area < largest_area) {
                m.cp[3] = c;
                m.depth[3] = depths[i];
            }
        }
    }
    const Quat ident { 1, 0, 0, 0 };
    for (int32_t i = 0; i < m.num; i++) m.cp[i] = ident.rotateVec(m.cp[i]) + Vector3::zero();
    m.normal = ident.rotateVec(n);
    return m;
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

__device__ __forceinline__ void storeManifold(Contact &c, const Manifold &m, Loc ref, Loc alt)
{
    c.ref = ref;
    c.alt = alt;
    for (int i = 0; i < 4; i++) c.points[i] = Vector4::fromVector3(m.cp[i], m.depth[i]);
    c.numPoints = m.num;
    c.normal = m.normal;
    for (int i = 0; i < 4; i++) c.lambdaN[i] = 0.f;
}



// Candidate order helper shared by the filter and the SAT phase:
// runNarrowphase's type swap (narrowphase.cpp:1574-1580).
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

// SAT + contact generation for one candidate that passed the AABB recheck;
// writes out.numPoints (0 = no contact) and, on contact, the manifold.
__device__ void narrowphaseCandidate(const PhysArgs &P, int32_t w,
                                     const CandidateCollision &cand, Contact &out)
{
    const ObjDev &O = P.objs;
    out.numPoints = 0;
    do {
        const CandBodies cb = orderCandidate(P, w, cand);
        const Loc a_loc = cb.a_loc, b_loc = cb.b_loc;
        const BodyArch *BA = cb.BA, *BB = cb.BB;
        const int32_t a_obj = cb.a_obj, b_obj = cb.b_obj;
        const uint32_t ta = cb.ta, tb = cb.tb;
        const Vector3 a_pos = bcol<Vector3>(*BA, Cols::Position, w, a_loc.row);
        const Vector3 b_pos = bcol<Vector3>(*BB, Cols::Position, w, b_loc.row);
        const Quat b_rot = bcol<Quat>(*BB, Cols::Rotation, w, b_loc.row);
        const uint32_t test = ta | tb;
        const int32_t a_leaf = bcol<broadphase::LeafID>(*BA, Cols::LeafID, w, a_loc.row).id;
        HullRef ha;
        ha.hd = O.hulls[a_obj];
        ha.verts = P.hullVerts + ((size_t)w * P.maxLeaves + a_leaf) * O.maxVerts;
        ha.planes = P.hullPlanes + ((size_t)w * P.maxLeaves + a_leaf) * O.maxFaces;
        ha.center = a_pos;
        Vector3 tmp1[kMaxClip], tmp2[kMaxClip];
        float depths[kMaxClip];

        if (test == (uint32_t)CollisionPrimitive::Type::Hull) {
            const int32_t b_leaf = bcol<broadphase::LeafID>(*BB, Cols::LeafID, w, b_loc.row).id;
            HullRef hb;
            hb.hd = O.hulls[b_obj];
            hb.verts = P.hullVerts + ((size_t)w * P.maxLeaves + b_leaf) * O.maxVerts;
            hb.planes = P.hullPlanes + ((size_t)w * P.maxLeaves + b_leaf) * O.maxFaces;
            hb.center = b_pos;

            // doSAT (narrowphase.cpp:678-758)
            FaceQuery fa = queryFaceDirections(ha, hb);
            if (fa.separation > 0.0f) continue;
            FaceQuery fb = queryFaceDirections(hb, ha);
            if (fb.separation > 0.0f) continue;
            EdgeQuery eq = queryEdgeDirections(O, ha, hb);
            if (eq.separation > 0.0f) continue;

            Manifold m;
            Loc ref_loc, other_loc;
            if (fa.separation > eq.separation || fb.separation > eq.separation) {
                const bool a_is_ref = fa.separation >= fb.separation;
                const geometry::Plane ref_plane = a_is_ref ? fa.plane : fb.plane;
                const int32_t ref_face = a_is_ref ? fa.faceIdx : fb.faceIdx;
                const HullRef &ref = a_is_ref ? ha : hb;
                const HullRef &inc = a_is_ref ? hb : ha;
                const int32_t inc_face = findIncidentFace(inc, ref_plane.normal);
                ref_loc = a_is_ref ? a_loc : b_loc;
                other_loc = a_is_ref ? b_loc : a_loc;

                // createFaceContact (narrowphase.cpp:866-972)
                const geometry::HalfEdge *rh = O.hedges + ref.hd.hedgeOffset;
                const geometry::HalfEdge *oh = O.hedges + inc.hd.hedgeOffset;
                int32_t n_in = 0;
                {
                    uint32_t hidx = O.polygons[inc.hd.faceOffset + inc_face], start = hidx;
                    do {
                        const geometry::HalfEdge he = oh[hidx];
                        hidx = he.next;
                        if (n_in < kMaxClip) tmp1[n_in++] = inc.verts[he.rootVertex];
                    } while (hidx != start);
                }
                Vector3 *cin = tmp1, *cdst = tmp2;
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
                        depths[n_below] = -d;
                        n_below++;
                    }
                }
                m = buildFaceContactManifold(ref_plane.normal, cin, depths, n_below);
            } else {
                // createEdgeContact (narrowphase.cpp:1053-1121)
                ref_loc = a_loc;
                other_loc = b_loc;
                const geometry::HalfEdge *ha_e = O.hedges + ha.hd.hedgeOffset;
                const geometry::HalfEdge *hb_e = O.hedges + hb.hd.hedgeOffset;
                const geometry::HalfEdge ea = ha_e[eq.edgeA];
                const geometry::HalfEdge eb = hb_e[eq.edgeB];
                geometry::Segment sa { ha.verts[ea.rootVertex], ha.verts[ha_e[ea.next].rootVertex] };
                geometry::Segment sb { hb.verts[eb.rootVertex], hb.verts[hb_e[eb.next].rootVertex] };
                geometry::Segment s = shortestSegmentBetween(sa, sb);
                const Quat ident { 1, 0, 0, 0 };
                for (int i = 0; i < 4; i++) { m.cp[i] = Vector3::zero(); m.depth[i] = 0.f; }
                m.cp[0] = ident.rotateVec(s.p1) + Vector3::zero();
                m.depth[0] = -eq.separation;
                m.num = 1;
                m.normal = ident.rotateVec(eq.normal);
            }
            if (m.num > 0) storeManifold(out, m, ref_loc, other_loc);
        } else if (test == ((uint32_t)CollisionPrimitive::Type::Hull |
                            (uint32_t)CollisionPrimitive::Type::Plane)) {
            Vector3 pn = b_rot.rotateVec(Vector3 { 0, 0, 1 });
            geometry::Plane plane { pn, dot(pn, b_pos) };
            // doSATPlane (narrowphase.cpp:760-788)
            float sep = hullDistFromPlane(plane, ha);
            if (sep > 0.0f) continue;
            int32_t inc_face = findIncidentFace(ha, plane.normal);
            // createFacePlaneContact (narrowphase.cpp:974-1017)
            const geometry::HalfEdge *hh = O.hedges + ha.hd.hedgeOffset;
            int32_t n = 0;
            uint32_t hidx = O.polygons[ha.hd.faceOffset + inc_face], start = hidx;
            do {
                const geometry::HalfEdge he = hh[hidx];
                hidx = he.next;
                Vector3 v = ha.verts[he.rootVertex];
                float d = distFromPlane(plane, v);
                if (d < 0.0f && n < kMaxClip) {
                    tmp1[n] = v - d * plane.normal;
                    depths[n] = -d;
                    n++;
                }
            } while (hidx != start);
            Manifold m = buildFaceContactManifold(plane.normal, tmp1, depths, n);
            if (m.num > 0) storeManifold(out, m, b_loc, a_loc);
        }
        // sphere / plane-plane: the reference asserts (narrowphase.cpp:1197-1313)
    } while (0);
}

// runNarrowphaseSystem over every candidate of a world (one block per world):
//   A. lane-per-candidate AABB recheck, block scan -> survivor list (order kept)
//   B. lane-per-survivor SAT + contact generation into survivor slots
//   C. block scan of survivors with a manifold -> the solver's contact order
//      (== the reference's addManifoldToSolver append order).
__global__ void __launch_bounds__(kNarrowBlock) narrowphaseKernel(PhysArgs P)
{
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

    for (int32_t s = threadIdx.x; s < S; s += kNarrowBlock) {
        narrowphaseCandidate(P, w, cands[surv[s]], slots[s]);
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
