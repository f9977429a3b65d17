// XPBD solver kernel (reference src/physics/physics.cpp:166-1008).
// Compiled twice: as is (namespace lanes64: one world per 64-lane wave) and
// through solver32.hip (MW_SOLVER_LANES=32, namespace lanes32: two worlds per
// wave, one per half).  The physics module picks one per executor from the
// level widths the kernel reports (SolverNode, physics.hip).
#include "physics_device.hpp"

#include <cfloat>

#ifndef MW_SOLVER_NS
#define MW_SOLVER_NS lanes64
#endif
// the debug entry points of the 32-lane copy carry a suffix
#ifndef MW_SOLVER_C
#define MW_SOLVER_C(name) name
#endif

namespace madrona::phys {
namespace MW_SOLVER_NS {

// ===========================================================================
// XPBD solver: solvePositions + setVelocities + solveVelocities
// (physics.cpp:166-1008), one wave per world, body state in LDS,
// level-scheduled contacts.
// ===========================================================================
// Mutable body state kept in LDS (random access by contact); the read-only
// substep state (prev / pre-solve pose and velocity, mass properties) is
// read from its columns when a contact needs it, so a world's LDS image is
// 56 B per body and ~2.5x more worlds stay resident per CU.
struct SMut {
    Vector3 x;
    Quat q;
    Vector3 v;
    Vector3 omega;
    uint32_t meta;        // ResponseType | body arch index << 8 | ObjectID << 16
};
static_assert(sizeof(SMut) == 56);

// The pre-solve state of a body (PreSolvePositional, PreSolveVelocity),
// staged in the world's LDS image by the bodies' coalesced load: the
// contact solves read it from LDS instead of two uncoalesced column loads
// per body side and item.  PreSolvePositional is the pose the integration
// has just written to Position / Rotation as well (integrateApply), so it
// comes with the pose; PreSolveVelocity (the integrated velocity, which the
// Velocity column does not hold) is loaded with the row.
// Off by default (MW_SOLVER_PRE_LDS=1 turns it on): the 52 B per body
// cost residency -- 13 -> 9 worlds per CU on collisions, SolverNode 0.224
// -> 0.269 ms per launch; the warm-up below is the cheaper way to the same
// loads.
#ifndef MW_SOLVER_PRE_LDS
#define MW_SOLVER_PRE_LDS 0
#endif
struct SPre {
    Vector3 x;
    Quat q;
    Vector3 v;
    Vector3 omega;
};
static_assert(sizeof(SPre) == 52);
constexpr int32_t kPreBytes = MW_SOLVER_PRE_LDS ? (int32_t)sizeof(SPre) : 0;

__device__ __forceinline__ bool isStaticBody(uint32_t meta)
{
    return (meta & 0xffu) == (uint32_t)ResponseType::Static;
}

// Read-only state of the body in LDS slot `slot` (physics.cpp:281-476,
// 865-993 read these through the contact's Locs).
struct BodyRO {
    int32_t arch, row;
    uint32_t obj;
};

__device__ __forceinline__ BodyRO bodyRO(const PhysArgs &P, int32_t slot, uint32_t meta)
{
    const int32_t a = (int32_t)((meta >> 8) & 0xffu);
    return BodyRO { a, slot - P.body[a].slotBase, meta >> 16 };
}

__device__ __forceinline__ int32_t bodySlot(const PhysArgs &P, Loc l)
{
    return P.body[bodyArchIndex(P, l.archetype)].slotBase + l.row;
}

__device__ __forceinline__ float computePositionalLambda(Vector3 ta1, Vector3 ta2, Vector3 ra1,
                                                         Vector3 ra2, float im1, float im2,
                                                         float c, float alpha)
{                                                          // physics.cpp:166-183
    float w1 = im1 + dot(ta1, ra1);
    float w2 = im2 + dot(ta2, ra2);
    return -c / (w1 + w2 + alpha);
}

__device__ __forceinline__ void applyPositionalUpdate(Vector3 &x1, Vector3 &x2, Quat &q1, Quat &q2,
                                                      Vector3 ral1, Vector3 ral2, float im1,
                                                      float im2, Vector3 n, float dl)
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

struct PairConst {
    float im1, im2;
    Vector3 iI1, iI2;
    Vector3 n;
    float mu;             // avg mu_s (positions) / avg mu_d (velocities)
};

__device__ __forceinline__ PairConst pairConstOf(const RigidBodyMetadata &m1, const RigidBodyMetadata &m2,
                                                 const SMut &b1, const SMut &b2, Vector3 n, bool velocities)
{
    PairConst k;
    k.im1 = m1.invMass;
    k.im2 = m2.invMass;
    k.iI1 = m1.invInertiaTensor;
    k.iI2 = m2.invInertiaTensor;
    if (isStaticBody(b1.meta)) { k.im1 = 0.f; k.iI1 = Vector3::zero(); }
    if (isStaticBody(b2.meta)) { k.im2 = 0.f; k.iI2 = Vector3::zero(); }
    k.n = n;
    k.mu = velocities ? 0.5f * (m1.muD + m2.muD) : 0.5f * (m1.muS + m2.muS);
    return k;
}

// A contact item's global inputs besides the manifold: both bodies' substep
// columns and object metadata.  Their addresses depend only on the LDS body
// records, so the item issues them in the same round of loads as the
// manifold (loaded inside the solves, after the branch on the manifold's
// bound check, they cost a second memory round trip per item).
struct PosIn {
    solver::PreSolvePositional ps1, ps2;
    solver::SubstepPrevState pv1, pv2;
    RigidBodyMetadata m1, m2;
};

struct VelIn {
    solver::PreSolvePositional ps1, ps2;
    solver::PreSolveVelocity pv1, pv2;
    RigidBodyMetadata m1, m2;
};

// skip1 / skip2: the side's per-substep columns are not read (an invariant
// static body the solve skips); the general solve of such an item reloads
// them (loadPosIn with both false).
__device__ __forceinline__ solver::PreSolvePositional prePos(const PhysArgs &P, const SPre *pre, int32_t w,
                                                            int32_t s, const BodyRO &o)
{
#if MW_SOLVER_PRE_LDS
    (void)P; (void)w; (void)o;
    const float *f = (const float *)(pre + s);
    return solver::PreSolvePositional { Vector3 { f[0], f[1], f[2] }, Quat { f[3], f[4], f[5], f[6] } };
#else
    (void)pre; (void)s;
    return bcol<solver::PreSolvePositional>(P.body[o.arch], Cols::PreSolvePositional, w, o.row);
#endif
}

__device__ __forceinline__ solver::PreSolveVelocity preVel(const PhysArgs &P, const SPre *pre, int32_t w,
                                                         int32_t s, const BodyRO &o)
{
#if MW_SOLVER_PRE_LDS
    (void)P; (void)w; (void)o;
    const float *f = (const float *)(pre + s) + 7;
    return solver::PreSolveVelocity { Vector3 { f[0], f[1], f[2] }, Vector3 { f[3], f[4], f[5] } };
#else
    (void)pre; (void)s;
    return bcol<solver::PreSolveVelocity>(P.body[o.arch], Cols::PreSolveVelocity, w, o.row);
#endif
}

__device__ __forceinline__ PosIn loadPosIn(const PhysArgs &P, int32_t w, const SPre *pre, const SMut &b1,
                                           int32_t s1, const SMut &b2, int32_t s2, bool skip1, bool skip2)
{
    const BodyRO o1 = bodyRO(P, s1, b1.meta), o2 = bodyRO(P, s2, b2.meta);
    PosIn in;
    in.ps1 = prePos(P, pre, w, s1, o1);
    in.ps2 = prePos(P, pre, w, s2, o2);
    in.pv1 = {};
    in.pv2 = {};
    if (!skip1) in.pv1 = bcol<solver::SubstepPrevState>(P.body[o1.arch], Cols::SubstepPrevState, w, o1.row);
    if (!skip2) in.pv2 = bcol<solver::SubstepPrevState>(P.body[o2.arch], Cols::SubstepPrevState, w, o2.row);
    in.m1 = P.objs.metadata[o1.obj];
    in.m2 = P.objs.metadata[o2.obj];
    return in;
}

__device__ __forceinline__ VelIn loadVelIn(const PhysArgs &P, int32_t w, const SPre *pre, const SMut &b1,
                                           int32_t s1, const SMut &b2, int32_t s2, bool skip1, bool skip2)
{
    const BodyRO o1 = bodyRO(P, s1, b1.meta), o2 = bodyRO(P, s2, b2.meta);
    VelIn in;
    in.ps1 = {};
    in.ps2 = {};
    in.pv1 = {};
    in.pv2 = {};
    if (!skip1) {
        in.ps1 = prePos(P, pre, w, s1, o1);
        in.pv1 = preVel(P, pre, w, s1, o1);
    }
    if (!skip2) {
        in.ps2 = prePos(P, pre, w, s2, o2);
        in.pv2 = preVel(P, pre, w, s2, o2);
    }
    in.m1 = P.objs.metadata[o1.obj];
    in.m2 = P.objs.metadata[o2.obj];
    return in;
}

// ---------------------------------------------------------------------------
// Skipping an invariant static body (staticInvariant below: static, finite,
// no -0 component, normalize() idempotent, previous pose == pose, pre-solve
// velocity +0).  Every solver write to such a body is an exact no-op, and
// its terms in the other body's update are exact zeros:
//   ra_s = 0 * ta_s has the sign of ta_s, so ta_s . ra_s = +0 and
//   w_s = 0 + (+0) = +0: the lambdas  -c / ((w1 + w2) + 0)  are computed
//   with w_s the constant +0 (the same IEEE additions);
//   x_s +- (dl * 0) * n and q_s +- (+-0 quaternion) keep their bits, and
//   normalize() returns q_s itself;
//   p_s - p_s_hat = +0 (pose == previous pose, same operations);
//   v_s = omega_s = +0 after setVelocities, so v_s + cross(omega_s, r) = +0.
// This holds while the lever arms and lambdas are finite: the contact's
// input bound (boundedInput) guarantees it for ta_s, and a non-finite lambda
// / velocity magnitude abandons the skipping solve before anything of the
// bodies is written; the full solve then runs (it writes the static body,
// which the level schedule treated as untouched, so the world is flagged).
// sk1 / sk2: skip the ref / alt body.  With both false the functions are the
// reference's op sequence verbatim.  Skipping cuts ~1/3 of a point's VALU;
// the kind-sorted schedule keeps a wave's lanes on the same side.
// ---------------------------------------------------------------------------
enum : int32_t { kSolveDone = 0, kSolveNonFinite = 1 };

// A contact's solver inputs, loaded with one batch of independent 16-B
// loads when its item starts (the point loop would otherwise wait on a
// global load per point): all four point slots, normal, count, lambdas.
struct ContactIn {
    Vector4 pts[4];
    Vector3 n;
    int32_t np;
    float lam[4];
};

__device__ __forceinline__ ContactIn loadContact(const Contact &c)
{
    static_assert(offsetof(Contact, points) == 16 && offsetof(Contact, numPoints) == 80 &&
                  offsetof(Contact, normal) == 84 && offsetof(Contact, lambdaN) == 96);
    const float4 *v = (const float4 *)((const char *)&c + 16);
    const float4 a0 = v[0], a1 = v[1], a2 = v[2], a3 = v[3], a4 = v[4], a5 = v[5];
    ContactIn ci;
    ci.pts[0] = Vector4 { a0.x, a0.y, a0.z, a0.w };
    ci.pts[1] = Vector4 { a1.x, a1.y, a1.z, a1.w };
    ci.pts[2] = Vector4 { a2.x, a2.y, a2.z, a2.w };
    ci.pts[3] = Vector4 { a3.x, a3.y, a3.z, a3.w };
    ci.np = __float_as_int(a4.x);
    ci.n = Vector3 { a4.y, a4.z, a4.w };
    ci.lam[0] = a5.x; ci.lam[1] = a5.y; ci.lam[2] = a5.z; ci.lam[3] = a5.w;
    return ci;
}

__device__ __forceinline__ bool finiteF(float f) { return __builtin_isfinite(f); }

__device__ __forceinline__ bool boundedInput(const ContactIn &c)
{
    constexpr float kBound = 1e18f;
    bool ok = fabsf(c.n.x) <= kBound && fabsf(c.n.y) <= kBound &&
              fabsf(c.n.z) <= kBound;   // false for NaN
    // fully unrolled with static indices (a `break` here kept the loop, and
    // its dynamic c.pts[i] sent the whole ContactIn through scratch)
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const Vector4 p = c.pts[i];
        const bool in = fabsf(p.x) <= kBound && fabsf(p.y) <= kBound && fabsf(p.z) <= kBound &&
                        fabsf(p.w) <= kBound;
        ok = ok && (i >= c.np || in);
    }
    return ok;
}

template <int ST>
__device__ __forceinline__ int32_t solveContactPositionsT(SMut &b1, SMut &b2, const ContactIn &c,
                                                          const PosIn &in, float *lambda_out)
{                                                          // physics.cpp:281-476
    constexpr bool sk1 = ST == 1, sk2 = ST == 2;
    const solver::PreSolvePositional &ps1 = in.ps1, &ps2 = in.ps2;
    const solver::SubstepPrevState &pv1 = in.pv1, &pv2 = in.pv2;
    const PairConst k = pairConstOf(in.m1, in.m2, b1, b2, c.n, false);
    const bool sk = sk1 || sk2;
    const Vector3 n = k.n;
    Vector3 x1 = b1.x, x2 = b2.x;
    Quat q1 = b1.q, q2 = b2.q;
    const int32_t np = c.np;
    Vector4 pa = c.pts[0], pb = c.pts[1], pc = c.pts[2], pd = c.pts[3];
#pragma unroll 1
    for (int i = 0; i < np; i++) {                         // :400-474
        const Vector4 pt = pa;                             // point i (registers shift)
        pa = pb; pb = pc; pc = pd;
        Vector3 c1 = pt.xyz();
        float depth = pt.w;
        Vector3 c2 = c1 - n * depth;
        Vector3 r1 = ps1.q.inv().rotateVec(c1 - ps1.x);
        Vector3 r2 = ps2.q.inv().rotateVec(c2 - ps2.x);
        float lambda_n = 0.f;
        Vector3 p1 = q1.rotateVec(r1) + x1;
        Vector3 p2 = q2.rotateVec(r2) + x2;
        float d = dot(p1 - p2, n);
        if (d > 0) {
            Vector3 ra1 = Vector3::zero(), ra2 = Vector3::zero();
            float w1 = 0.f, w2 = 0.f;
            if (!sk1) {
                Vector3 nl1 = q1.inv().rotateVec(n);
                Vector3 ta1 = cross(r1, nl1);
                ra1 = multDiag(k.iI1, ta1);
                w1 = k.im1 + dot(ta1, ra1);
            }
            if (!sk2) {
                Vector3 nl2 = q2.inv().rotateVec(n);
                Vector3 ta2 = cross(r2, nl2);
                ra2 = multDiag(k.iI2, ta2);
                w2 = k.im2 + dot(ta2, ra2);
            }
            lambda_n = -d / (w1 + w2 + 0.f);               // computePositionalLambda
            if (sk && !finiteF(lambda_n)) return kSolveNonFinite;
            float half = 0.5f * lambda_n;                  // applyPositionalUpdate
            if (!sk1) {
                x1 += lambda_n * k.im1 * n;
                Vector3 q1u = q1.rotateVec(half * ra1);
                q1 += Quat::fromAngularVec(q1u) * q1;
                q1 = q1.normalize();
            }
            if (!sk2) {
                x2 -= lambda_n * k.im2 * n;
                Vector3 q2u = q2.rotateVec(half * ra2);
                q2 -= Quat::fromAngularVec(q2u) * q2;
                q2 = q2.normalize();
            }

            Vector3 e1 = Vector3::zero(), e2 = Vector3::zero();   // p - p_hat
            if (!sk1) {
                Vector3 p1_hat = pv1.prevRotation.rotateVec(r1) + pv1.prevPosition;
                e1 = (q1.rotateVec(r1) + x1) - p1_hat;
            }
            if (!sk2) {
                Vector3 p2_hat = pv2.prevRotation.rotateVec(r2) + pv2.prevPosition;
                e2 = (q2.rotateVec(r2) + x2) - p2_hat;
            }
            Vector3 dp = e1 - e2;
            Vector3 dpt = dp - dot(dp, n) * n;
            float tmag = dpt.length();
            if (tmag > 0.f) {
                Vector3 tw = dpt / tmag;
                Vector3 fra1 = Vector3::zero(), fra2 = Vector3::zero();
                float wt1 = 0.f, wt2 = 0.f;
                if (!sk1) {
                    Vector3 tl1 = q1.inv().rotateVec(tw);
                    Vector3 fta1 = cross(r1, tl1);
                    fra1 = multDiag(k.iI1, fta1);
                    wt1 = k.im1 + dot(fta1, fra1);
                }
                if (!sk2) {
                    Vector3 tl2 = q2.inv().rotateVec(tw);
                    Vector3 fta2 = cross(r2, tl2);
                    fra2 = multDiag(k.iI2, fta2);
                    wt2 = k.im2 + dot(fta2, fra2);
                }
                float lambda_t = -tmag / (wt1 + wt2 + 0.f);
                if (sk && !finiteF(lambda_t)) return kSolveNonFinite;
                float thresh = lambda_n * k.mu;
                if (lambda_t > thresh) {
                    float half_t = 0.5f * lambda_t;
                    if (!sk1) {
                        x1 += lambda_t * k.im1 * tw;
                        Vector3 q1u = q1.rotateVec(half_t * fra1);
                        q1 += Quat::fromAngularVec(q1u) * q1;
                        q1 = q1.normalize();
                    }
                    if (!sk2) {
                        x2 -= lambda_t * k.im2 * tw;
                        Vector3 q2u = q2.rotateVec(half_t * fra2);
                        q2 -= Quat::fromAngularVec(q2u) * q2;
                        q2 = q2.normalize();
                    }
                }
            }
        }
        lambda_out[i] = lambda_n;
    }
    if (!sk1) { b1.x = x1; b1.q = q1; }
    if (!sk2) { b2.x = x2; b2.q = q2; }
    return kSolveDone;
}

// Joint constraints (physics.cpp:247-279, 478-648), run after the contacts
// of solvePositions in ConstraintData row order.
__device__ __forceinline__ void angularCorrection(Quat &q1, Quat &q2, Vector3 dq, Vector3 iI1,
                                                  Vector3 iI2)
{                                                          // physics.cpp:490-504, 522-534
    const float mag = dq.length();
    if (mag > 0) {
        dq /= mag;
        const Vector3 n1 = q1.inv().rotateVec(dq);
        const Vector3 n2 = q2.inv().rotateVec(dq);
        // computeAngularUpdate (:247-271) + applyAngularUpdate (:273-279)
        const Vector3 lra1 = multDiag(iI1, n1);
        const Vector3 lra2 = multDiag(iI2, n2);
        const float w1 = dot(n1, lra1);
        const float w2 = dot(n2, lra2);
        const float dl = -mag / (w1 + w2 + 0.f);
        const float half = 0.5f * dl;
        const Quat u1 = Quat::fromAngularVec(q1.rotateVec(half * lra1));
        const Quat u2 = Quat::fromAngularVec(q2.rotateVec(half * lra2));
        q1 = (q1 + u1 * q1).normalize();
        q2 = (q2 - u2 * q2).normalize();
    }
}

__device__ void solveJoint(const PhysArgs &P, SMut &b1, SMut &b2, const JointConstraint &j)
{                                                          // handleJointConstraint, :537-648
    const RigidBodyMetadata m1 = P.objs.metadata[b1.meta >> 16];
    const RigidBodyMetadata m2 = P.objs.metadata[b2.meta >> 16];
    Vector3 x1 = b1.x, x2 = b2.x;
    Quat q1 = b1.q, q2 = b2.q;
    float im1 = m1.invMass, im2 = m2.invMass;
    Vector3 iI1 = m1.invInertiaTensor, iI2 = m2.invInertiaTensor;
    if (isStaticBody(b1.meta)) { im1 = 0.f; iI1 = Vector3::zero(); }
    if (isStaticBody(b2.meta)) { im2 = 0.f; iI2 = Vector3::zero(); }

    Vector3 corr;
    if (j.type == JointConstraint::Type::Fixed) {          // :580-615
        const JointConstraint::Fixed f = j.fixed;
        const Quat o1 = (q1 * f.attachRot1).normalize();  // applyJointOrientationConstraint
        const Quat o2 = (q2 * f.attachRot2).normalize();
        const Quat diff = o1 * o2.inv();
        angularCorrection(q1, q2, 2.f * Vector3 { diff.x, diff.y, diff.z }, iI1, iI2);
        const Vector3 r1w = q1.rotateVec(j.r1) + x1;
        const Vector3 r2w = q2.rotateVec(j.r2) + x2;
        const Vector3 dr = r2w - r1w;
        const Quat axes = (q1 * f.attachRot1).normalize();
        const Vector3 a1 = axes.rotateVec(math::fwd);
        const Vector3 b1v = axes.rotateVec(math::right);
        const Vector3 c1 = cross(a1, b1v);
        corr = Vector3::zero();
        const float as = dot(dr, a1);
        corr -= (as - f.separation) * a1;
        const float bs = dot(dr, b1v);
        corr -= bs * b1v;
        const float cs = dot(dr, c1);
        corr -= cs * c1;
    } else {                                               // Hinge, :616-627
        const JointConstraint::Hinge hg = j.hinge;
        // applyJointAxisConstraint (:507-535) without its debug printf
        const Vector3 ax1 = q1.rotateVec(hg.a1Local);
        const Vector3 ax2 = q2.rotateVec(hg.a2Local);
        angularCorrection(q1, q2, cross(ax1, ax2), iI1, iI2);
        const Vector3 r1w = q1.rotateVec(j.r1) + x1;
        const Vector3 r2w = q2.rotateVec(j.r2) + x2;
        corr = r2w - r1w;
    }
    const float cm = corr.length();
    if (cm > 0.f) {
        corr /= cm;
        // applyPositionalUpdate overload with lever arms (:213-245)
        const Vector3 nl1 = q1.inv().rotateVec(corr);
        const Vector3 nl2 = q2.inv().rotateVec(corr);
        const Vector3 ta1 = cross(j.r1, nl1);
        const Vector3 ta2 = cross(j.r2, nl2);
        const Vector3 ra1 = multDiag(iI1, ta1);
        const Vector3 ra2 = multDiag(iI2, ta2);
        const float dl = computePositionalLambda(ta1, ta2, ra1, ra2, im1, im2, cm, 0);
        applyPositionalUpdate(x1, x2, q1, q2, ra1, ra2, im1, im2, corr, dl);
    }
    b1.x = x1; b2.x = x2;
    b1.q = q1; b2.q = q2;
}

__device__ __forceinline__ Vector3 relVel(Vector3 v1, Vector3 v2, Vector3 o1, Vector3 o2,
                                          Vector3 d1, Vector3 d2)
{
    return (v1 + cross(o1, d1)) - (v2 + cross(o2, d2));
}

__device__ __forceinline__ void applyVelocityUpdate(Vector3 &v1, Vector3 &v2, Vector3 &o1,
                                                    Vector3 &o2, Quat q1, Quat q2, Vector3 ta1,
                                                    Vector3 ta2, float im1, float im2,
                                                    Vector3 iI1, Vector3 iI2, Vector3 dv,
                                                    float mag)
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

template <int ST>
__device__ __forceinline__ int32_t solveContactVelocitiesT(SMut &b1, SMut &b2, const ContactIn &c,
                                                           const VelIn &in, float h, float rest_thresh)
{                                                          // physics.cpp:865-993
    constexpr bool sk1 = ST == 1, sk2 = ST == 2;
    const solver::PreSolvePositional &ps1 = in.ps1, &ps2 = in.ps2;
    const solver::PreSolveVelocity &pv1 = in.pv1, &pv2 = in.pv2;
    const PairConst k = pairConstOf(in.m1, in.m2, b1, b2, c.n, true);
    const bool sk = sk1 || sk2;
    const Quat q1 = b1.q, q2 = b2.q;
    Vector3 v1 = b1.v, o1v = b1.omega, v2 = b2.v, o2v = b2.omega;
    const Vector3 n = k.n;

    // The world-space lever arms q.rotateVec(r_local): q is fixed during
    // this phase, so they are computed once per point instead of at each of
    // their three uses -- the same operations on the same inputs, so the
    // same bits -- wherever the registers are free: in the skipping solves
    // (the general solve sets the kernel's register peak), and in the general
    // solve too where LDS, not registers, bounds residency (the 32-lane
    // variant: two worlds' images per block).  Level 2 also keeps each
    // moving side's angular terms of the normal impulse, ra = I^-1 (r x n_l)
    // and w = m^-1 + ta . ra, which both iterations apply unchanged.
#ifndef MW_SOLVER_VEL_ARMS
#define MW_SOLVER_VEL_ARMS 1
#endif
#ifndef MW_SOLVER_GENERAL_CACHE
#define MW_SOLVER_GENERAL_CACHE (MW_SOLVER_LANES == 32)
#endif
    constexpr bool kCache = sk || MW_SOLVER_GENERAL_CACHE;
    constexpr bool kArms1 = MW_SOLVER_VEL_ARMS >= 1 && kCache && !sk1;
    constexpr bool kArms2 = MW_SOLVER_VEL_ARMS >= 1 && kCache && !sk2;
    constexpr bool kTerms = MW_SOLVER_VEL_ARMS >= 2 && kCache;
    Vector3 arm1[4], arm2[4], rac1[4], rac2[4];
    float wc1[4], wc2[4];
    // relVel (physics.cpp:716-722) as t1 - t2, a skipped side's term = +0
    auto rel = [&](int32_t i, Vector3 r1l, Vector3 r2l) {
        Vector3 t1 = Vector3::zero(), t2 = Vector3::zero();
        if (!sk1) t1 = v1 + cross(o1v, kArms1 ? arm1[i] : q1.rotateVec(r1l));
        if (!sk2) t2 = v2 + cross(o2v, kArms2 ? arm2[i] : q2.rotateVec(r2l));
        return t1 - t2;
    };
    // applyVelocityUpdate (physics.cpp:724-750), false on a non-finite
    // magnitude when a side is skipped (nothing is written then); applyRW
    // takes the sides' angular terms ready-made
    auto applyRW = [&](Vector3 ra1, float w1, Vector3 ra2, float w2, Vector3 dv, float mag) {
        mag *= 1.f / (w1 + w2);
        if (sk && !finiteF(mag)) return false;
        if (!sk1) {
            v1 += mag * k.im1 * dv;
            o1v += q1.rotateVec(mag * ra1);
        }
        if (!sk2) {
            v2 -= mag * k.im2 * dv;
            o2v -= q2.rotateVec(mag * ra2);
        }
        return true;
    };
    auto apply = [&](Vector3 ta1, Vector3 ta2, Vector3 dv, float mag) {
        Vector3 ra1 = Vector3::zero(), ra2 = Vector3::zero();
        float w1 = 0.f, w2 = 0.f;
        if (!sk1) { ra1 = multDiag(k.iI1, ta1); w1 = k.im1 + dot(ta1, ra1); }
        if (!sk2) { ra2 = multDiag(k.iI2, ta2); w2 = k.im2 + dot(ta2, ra2); }
        return applyRW(ra1, w1, ra2, w2, dv, mag);
    };

    // Per point only the body-local lever arms and the pre-solve normal
    // velocity stay live; the world-space arms (q fixed during this phase)
    // and the angular terms are recomputed where used -- the same operations
    // on the same inputs, so bit-identical, at a third of the registers.
    Vector3 r1l[4], r2l[4];
    float vn_bars[4];
    Vector3 nl1 = Vector3::zero(), nl2 = Vector3::zero();
    if (!sk1) nl1 = q1.inv().rotateVec(n);
    if (!sk2) nl2 = q2.inv().rotateVec(n);
#pragma unroll
    for (int i = 0; i < 4; i++) {
        if (i >= c.np) continue;
        Vector3 c1 = c.pts[i].xyz();
        float depth = c.pts[i].w;
        Vector3 c2 = c1 - n * depth;
        Vector3 t1 = Vector3::zero(), t2 = Vector3::zero();
        r1l[i] = Vector3::zero();
        r2l[i] = Vector3::zero();
        if (!sk1) {
            r1l[i] = ps1.q.inv().rotateVec(c1 - ps1.x);
            t1 = pv1.v + cross(pv1.omega, ps1.q.rotateVec(r1l[i]));
        }
        if (!sk2) {
            r2l[i] = ps2.q.inv().rotateVec(c2 - ps2.x);
            t2 = pv2.v + cross(pv2.omega, ps2.q.rotateVec(r2l[i]));
        }
        vn_bars[i] = dot(n, t1 - t2);
        if constexpr (kArms1) arm1[i] = q1.rotateVec(r1l[i]);
        if constexpr (kArms2) arm2[i] = q2.rotateVec(r2l[i]);
        if constexpr (kTerms) {
            rac1[i] = rac2[i] = Vector3::zero();
            wc1[i] = wc2[i] = 0.f;
            if (!sk1) {
                const Vector3 ta = cross(r1l[i], nl1);
                rac1[i] = multDiag(k.iI1, ta);
                wc1[i] = k.im1 + dot(ta, rac1[i]);
            }
            if (!sk2) {
                const Vector3 ta = cross(r2l[i], nl2);
                rac2[i] = multDiag(k.iI2, ta);
                wc2[i] = k.im2 + dot(ta, rac2[i]);
            }
        }
    }
    for (int it = 0; it < 2; it++) {                       // :813-863
#pragma unroll
        for (int i = 0; i < 4; i++) {
            if (i >= c.np) continue;
            float vn = dot(n, rel(i, r1l[i], r2l[i]));
            float vn_bar = vn_bars[i];
            float e = 0.3f;
            if (fabsf(vn_bar) <= rest_thresh) e = 0.f;
            float mag = fminRef(-e * vn_bar, 0) - vn;
            if constexpr (kTerms) {
                if (!applyRW(rac1[i], wc1[i], rac2[i], wc2[i], n, mag)) return kSolveNonFinite;
            } else {
                if (!apply(cross(r1l[i], nl1), cross(r2l[i], nl2), n, mag)) return kSolveNonFinite;
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {                          // :752-811
        if (i >= c.np) continue;
        Vector3 v = rel(i, r1l[i], r2l[i]);
        float dfm = k.mu * fabsf(c.lam[i]) / h;
        float vn = dot(n, v);
        Vector3 vt = v - n * vn;
        float vt_len = vt.length();
        if (vt_len != 0 && dfm != 0.f) {
            float corrected = -fminRef(dfm, vt_len);
            Vector3 dw = vt / vt_len;
            Vector3 fta1 = Vector3::zero(), fta2 = Vector3::zero();
            if (!sk1) fta1 = cross(r1l[i], q1.inv().rotateVec(dw));
            if (!sk2) fta2 = cross(r2l[i], q2.inv().rotateVec(dw));
            if (!apply(fta1, fta2, dw, corrected)) return kSolveNonFinite;
        }
    }
    if (!sk1) { b1.v = v1; b1.omega = o1v; }
    if (!sk2) { b2.v = v2; b2.omega = o2v; }
    return kSolveDone;
}

__device__ __forceinline__ bool isNegZero(float f) { return __float_as_uint(f) == 0x80000000u; }
__device__ __forceinline__ bool sameBits(float a, float b) { return __float_as_uint(a) == __float_as_uint(b); }

// A static body is never written through if every solver write to it is an
// exact no-op: x +- (+-0) and q +- (+-0) keep bits when no component is -0,
// and normalize() must be idempotent on its rotation (static velocities are
// always +0 after setVelocities).  Such bodies add no ordering edge.  The
// specialised contact solves (solveContact*Static) further use that its
// previous pose equals its pose, that its pre-solve velocity is +0 and that
// its position is finite and bounded; integrateKernel establishes all three
// for every static body, and they are checked here.
__device__ __forceinline__ bool staticInvariant(const SMut &b, Vector3 prev_x, Quat prev_q,
                                                Vector3 ps_v, Vector3 ps_om)
{
    if (!isStaticBody(b.meta)) return false;
    if (isNegZero(b.x.x) || isNegZero(b.x.y) || isNegZero(b.x.z)) return false;
    if (isNegZero(b.q.w) || isNegZero(b.q.x) || isNegZero(b.q.y) || isNegZero(b.q.z)) return false;
    constexpr float kBound = 1e18f;
    if (!(fabsf(b.x.x) <= kBound && fabsf(b.x.y) <= kBound && fabsf(b.x.z) <= kBound)) return false;
    if (!(finiteF(b.q.w) && finiteF(b.q.x) && finiteF(b.q.y) && finiteF(b.q.z))) return false;
    if (!(sameBits(prev_x.x, b.x.x) && sameBits(prev_x.y, b.x.y) && sameBits(prev_x.z, b.x.z) &&
          sameBits(prev_q.w, b.q.w) && sameBits(prev_q.x, b.q.x) && sameBits(prev_q.y, b.q.y) &&
          sameBits(prev_q.z, b.q.z))) return false;
    const uint32_t vbits = __float_as_uint(ps_v.x) | __float_as_uint(ps_v.y) |
                           __float_as_uint(ps_v.z) | __float_as_uint(ps_om.x) |
                           __float_as_uint(ps_om.y) | __float_as_uint(ps_om.z);
    if (vbits != 0) return false;
    Quat nq = b.q.normalize();
    return sameBits(nq.w, b.q.w) && sameBits(nq.x, b.q.x) && sameBits(nq.y, b.q.y) &&
           sameBits(nq.z, b.q.z);
}

// Body states in the world's LDS image (SolverLDS::state, one int16 per
// body slot): an ordinary body holds the latest item of the earlier chunks
// touching it while the levels are scheduled (-1: none); an invariant static
// body takes no ordering edges (kStateStatic); kStateStaticSkip also makes
// every per-body phase an exact no-op for it -- its Velocity column is +0
// (what setVelocities derives from an unchanged pose, and what the
// write-back stores), its pre-solve pose equals its pose (the fused
// integration's static branch rewrites pose, previous and pre-solve state
// with the same values) and its BodyBox in P.bodyBoxes is current (computed
// from the same pose and scale by the last integration: integrateKernel
// each step, then each substep's tail) -- so setVelocities, the write-back
// and the next substep's integration skip it, and the filter's LDS box image
// takes its box from P.bodyBoxes.  collisions: the ground plane, alone in
// the third row batch of every world, which then issues no work.  A
// general solve that may write such a body (a joint, or the fallback of a
// non-finite skipping solve, flagged kErrStaticSchedule) marks it
// kStateStaticWritten: still without ordering edges, but the per-body
// phases treat it as any body.
constexpr int16_t kStateStatic = -3;
constexpr int16_t kStateStaticSkip = -4;
constexpr int16_t kStateStaticWritten = -5;
__device__ __forceinline__ bool invariantState(int16_t v) { return v <= kStateStatic; }

__device__ __forceinline__ bool staticSkippable(const SMut &b, Vector3 ps_x, Quat ps_q)
{
    const uint32_t vbits = __float_as_uint(b.v.x) | __float_as_uint(b.v.y) | __float_as_uint(b.v.z) |
                           __float_as_uint(b.omega.x) | __float_as_uint(b.omega.y) |
                           __float_as_uint(b.omega.z);
    return vbits == 0 && sameBits(ps_x.x, b.x.x) && sameBits(ps_x.y, b.x.y) && sameBits(ps_x.z, b.x.z) &&
           sameBits(ps_q.w, b.q.w) && sameBits(ps_q.x, b.q.x) && sameBits(ps_q.y, b.q.y) &&
           sameBits(ps_q.z, b.q.z);
}

// Per-item solver record: body slots of ref / alt (e1 / e2 for a joint)
// and the item's level (1 + max level of earlier items sharing a
// non-invariant body).  Items are the world's contacts followed by its
// joints, the reference's solvePositions order.
struct CRec {
    int16_t s1, s2, lvl, slot;   // slot: survivor slot holding the manifold;
                                 // a joint: -1 - ConstraintData row
};
static_assert(sizeof(CRec) == 8);

// Contacts whose records stay in LDS; worlds with more contacts keep them
// in a global slab instead, so the LDS footprint (and with it the number of
// worlds resident per CU) does not scale with SolverData::maxContacts.
#ifndef MW_SOLVER_LDS_CONTACTS
#define MW_SOLVER_LDS_CONTACTS 128
#endif
constexpr int32_t kSolverLDSContacts = MW_SOLVER_LDS_CONTACTS;

// Item kinds, in schedule order within a level: contacts whose ref (1) or
// alt (2) body is an invariant static body take the specialised solves, the
// rest (and joints) the general ones.  Sorting a level by kind keeps a
// wave's lanes on one code path.
enum : int32_t { kKindStaticRef = 0, kKindStaticAlt = 1, kKindGeneral = 2, kNumKinds = 3 };

// Per-world LDS image: bodies, ordering state, contact records.
struct SolverLDS {
    SMut *bodies;         // [nb]
    SPre *pre;            // [nb] pre-solve state (MW_SOLVER_PRE_LDS)
    uint64_t *touch;      // [nb] lanes of the current 64-item chunk touching the body
    int16_t *state;       // [nb] ordinary body: latest item of the earlier chunks touching it
                          // (-1: none); invariant static body: kStateStatic* (<= -3)
    CRec *recs;           // [kSolverLDSContacts]
    int32_t *prevs;       // [kSolverLDSContacts] (prev item on s1, on s2) as 2 x int16
};

__host__ __device__ inline size_t solverA16(size_t b) { return (b + 15) & ~size_t(15); }

__host__ __device__ inline size_t solverWorldLDSBytes(int32_t nb)
{
    return solverA16(sizeof(SMut) * nb) + solverA16((size_t)kPreBytes * nb) + solverA16(sizeof(uint64_t) * nb) +
           solverA16(sizeof(int16_t) * nb) +
           (sizeof(CRec) + sizeof(int32_t)) * kSolverLDSContacts;
}

// Block-shared schedule: every (world, item) of the block sorted by (level,
// kind), so one pass over a level keeps all of the block's lanes on that
// level's items from all of its worlds.
constexpr int32_t kSolverItems = kSolverWorlds * kSolverLDSContacts;
// Dependency levels the block's bucket table holds; a deeper world (a tall
// stack: the benchmark's worlds average 1.7 levels) solves from the global
// records instead.  48, not 128: one world's LDS drops to 12.1 KB and 12
// single-world blocks fit a CU (the VGPR limit) instead of 11.
#ifndef MW_SOLVER_MAX_LEVELS
#define MW_SOLVER_MAX_LEVELS 48
#endif
constexpr int32_t kSolverBuckets = kNumKinds * (MW_SOLVER_MAX_LEVELS + 2);

// The block schedule: items (world << 16 | kind << 12 | k) and the bucket
// offsets of the counting sort, then four block scalars.
__host__ __device__ inline size_t solverScheduleBytes()
{
    return sizeof(uint32_t) * kSolverItems + sizeof(int32_t) * kSolverBuckets;
}

// With one world per block the schedule needs no LDS of its own: the world's
// touch masks (bucket offsets) and predecessor records (items) are dead once
// its levels are scheduled, and the sort comes after (touch is zeroed again
// by the next launch's body load).  That keeps a collisions world at 10.1 KB
// of LDS (16 blocks per CU) instead of 12.1 KB (13).
__host__ __device__ inline bool solverAliasSchedule(int32_t nb)
{
    return kSolverWorlds == 1 && solverA16(sizeof(uint64_t) * nb) >= sizeof(int32_t) * kSolverBuckets &&
           sizeof(int32_t) * kSolverLDSContacts >= sizeof(uint32_t) * kSolverItems;
}

__host__ __device__ inline size_t solverBlockLDSBytes(int32_t nb)
{
    return kSolverWorlds * solverWorldLDSBytes(nb) + (solverAliasSchedule(nb) ? 0 : solverScheduleBytes()) +
           sizeof(int32_t) * 4;                            // block scalars
}

struct SolverBlockLDS {
    uint32_t *items;
    int32_t *bucketOff;   // [(Lmax + 2) * kNumKinds]; after the sort bucketOff[b] = end of bucket b
    int32_t *scalars;     // [1] max items, [2] max level, [3] max level (global records)
};

__device__ __forceinline__ SolverLDS solverWorldLDS(char *smem, int32_t nb, int32_t wi)
{
    SolverLDS L;
    char *p = smem + (size_t)wi * solverWorldLDSBytes(nb);
    L.bodies = (SMut *)p;
    p += solverA16(sizeof(SMut) * nb);
    L.pre = (SPre *)p;
    p += solverA16((size_t)kPreBytes * nb);
    L.touch = (uint64_t *)p;
    p += solverA16(sizeof(uint64_t) * nb);
    L.state = (int16_t *)p;
    p += solverA16(sizeof(int16_t) * nb);
    L.recs = (CRec *)p;
    p += sizeof(CRec) * kSolverLDSContacts;
    L.prevs = (int32_t *)p;
    return L;
}

// p: the block schedule's LDS (after the world images, or all of the
// dynamic LDS when the images are global); alias: in world 0's dead arrays
// (solverAliasSchedule)
__device__ __forceinline__ SolverBlockLDS solverBlockLDS(char *p, const SolverLDS *alias)
{
    SolverBlockLDS B;
    if (alias) {
        B.items = (uint32_t *)alias->prevs;
        B.bucketOff = (int32_t *)alias->touch;
    } else {
        B.items = (uint32_t *)p;
        p += sizeof(uint32_t) * kSolverItems;
        B.bucketOff = (int32_t *)p;
        p += sizeof(int32_t) * kSolverBuckets;
    }
    B.scalars = (int32_t *)p;
    return B;
}

// One world's LDS is owned by one wave; within a wave LDS writes become
// visible after the wave's LDS queue drains.
__device__ __forceinline__ void waveSync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Column reads as plain floats (no aggregate copies through scratch).
__device__ __forceinline__ Vector3 ldV3(const void *p)
{
    const float *f = (const float *)p;
    return Vector3 { f[0], f[1], f[2] };
}
__device__ __forceinline__ Quat ldQ(const void *p)
{
    const float *f = (const float *)p;
    return Quat { f[0], f[1], f[2], f[3] };
}
__device__ __forceinline__ void stV3(void *p, Vector3 v)
{
    float *f = (float *)p;
    f[0] = v.x; f[1] = v.y; f[2] = v.z;
}
__device__ __forceinline__ void stQ(void *p, Quat q)
{
    float *f = (float *)p;
    f[0] = q.w; f[1] = q.x; f[2] = q.y; f[3] = q.z;
}

// Rows of a world a lane handles per batch in the per-body loops: every
// column load of a batch is issued before the first row's stores, so a
// world of up to 64 * kRowBatch bodies pays one memory round trip per loop
// instead of one per 64 rows (collisions: 129 bodies, 3 rounds -> 1).
constexpr int32_t kRowBatch = 3;
// The write-back's batch (it also holds each row's integration inputs for
// the next substep, so its batch costs registers the load's does not).
#ifndef MW_SOLVER_WRITE_BATCH
#define MW_SOLVER_WRITE_BATCH 3
#endif
constexpr int32_t kWriteBatch = MW_SOLVER_WRITE_BATCH;

// Cache warming (MW_SOLVER_WARM, default on).  The contacts and the
// bodies' substep columns the level passes read per item were written by
// other kernels (narrowphase, the last substep's tail), usually on another
// XCD, so their first reads miss L2; and a level pass issues its items'
// loads only when it starts, one pass after the other.  So the world's
// load touches one dword of every line those reads will need -- the
// substep columns of every body with its coalesced row loads (no extra
// round trip), every contact's two lines once the contacts are gathered --
// and the values are consumed (nothing computed) only when the level passes
// begin: the lines are in L2 by then.
#ifndef MW_SOLVER_WARM
#define MW_SOLVER_WARM 1
#endif
__device__ __forceinline__ void keepLoaded(uint32_t v) { asm volatile("" ::"v"(v)); }

// Load one world's bodies into its LDS image (wave `lane` 0..63) and reset
// its ordering state.
__device__ __forceinline__ void loadWorldBodies(const PhysArgs &P, int32_t w, SolverLDS &L,
                                                int32_t lane)
{
    for (int32_t ba = 0; ba < P.numBodyArchs; ba++) {
        const BodyArch &B = P.body[ba];
        const int32_t rows = B.numRows[w];
        for (int32_t r0 = 0; r0 < rows; r0 += kSolverBlock * kRowBatch) {
            SMut s[kRowBatch];
#if MW_SOLVER_PRE_LDS
            Vector3 pv[kRowBatch], pw[kRowBatch];
#endif
#if MW_SOLVER_WARM
            uint32_t warm[kRowBatch];
#endif
#pragma unroll
            for (int32_t j = 0; j < kRowBatch; j++) {
                const int32_t r = r0 + j * kSolverBlock + lane;
                if (r >= rows) continue;
#if MW_SOLVER_WARM
                // a row of 24-28 B starts in every 128-B line of the columns
                warm[j] = *(const uint32_t *)&bcol<solver::PreSolvePositional>(B, Cols::PreSolvePositional, w, r) ^
                          *(const uint32_t *)&bcol<solver::SubstepPrevState>(B, Cols::SubstepPrevState, w, r) ^
                          *(const uint32_t *)&bcol<solver::PreSolveVelocity>(B, Cols::PreSolveVelocity, w, r);
#endif
#if MW_SOLVER_PRE_LDS
                const auto &psv = bcol<solver::PreSolveVelocity>(B, Cols::PreSolveVelocity, w, r);
                pv[j] = ldV3(&psv.v);
                pw[j] = ldV3(&psv.omega);
#endif
                s[j].x = ldV3(&bcol<Vector3>(B, Cols::Position, w, r));
                s[j].q = ldQ(&bcol<Quat>(B, Cols::Rotation, w, r));
                const Velocity &vel = bcol<Velocity>(B, Cols::Velocity, w, r);
                s[j].v = ldV3(&vel.linear);
                s[j].omega = ldV3(&vel.angular);
                const uint32_t obj = (uint32_t)bcol<ObjectID>(B, Cols::ObjectID, w, r).idx;
                const uint32_t rt = (uint32_t)bcol<ResponseType>(B, Cols::ResponseType, w, r) & 0xffu;
                s[j].meta = rt | ((uint32_t)ba << 8) | (obj << 16);
            }
#pragma unroll
            for (int32_t j = 0; j < kRowBatch; j++) {
                const int32_t r = r0 + j * kSolverBlock + lane;
                if (r >= rows) continue;
                int16_t fl = -1;
                if ((s[j].meta & 0xffu) == (uint32_t)ResponseType::Static) {
                    const auto &pv = bcol<solver::SubstepPrevState>(B, Cols::SubstepPrevState, w, r);
                    const auto &psv = bcol<solver::PreSolveVelocity>(B, Cols::PreSolveVelocity, w, r);
                    const auto &psp = bcol<solver::PreSolvePositional>(B, Cols::PreSolvePositional, w, r);
                    if (staticInvariant(s[j], ldV3(&pv.prevPosition), ldQ(&pv.prevRotation),
                                        ldV3(&psv.v), ldV3(&psv.omega)))
                        fl = staticSkippable(s[j], ldV3(&psp.x), ldQ(&psp.q)) ? kStateStaticSkip : kStateStatic;
                }
#if MW_SOLVER_WARM
                keepLoaded(warm[j]);
#endif
                const int32_t slot = B.slotBase + r;
                SMut *d = L.bodies + slot;
                stV3(&d->x, s[j].x);
                stQ(&d->q, s[j].q);
                stV3(&d->v, s[j].v);
                stV3(&d->omega, s[j].omega);
                d->meta = s[j].meta;
#if MW_SOLVER_PRE_LDS
                {
                    SPre *e = L.pre + slot;           // PreSolvePositional = the pose
                    stV3(&e->x, s[j].x);
                    stQ(&e->q, s[j].q);
                    stV3(&e->v, pv[j]);
                    stV3(&e->omega, pw[j]);
                }
#endif
                L.state[slot] = fl;
                L.touch[slot] = 0;
            }
        }
    }
}

__device__ __forceinline__ SMut ldBody(const SMut *p)
{
    SMut s;
    s.x = ldV3(&p->x);
    s.q = ldQ(&p->q);
    s.v = ldV3(&p->v);
    s.omega = ldV3(&p->omega);
    s.meta = p->meta;
    return s;
}

// The world's contacts: survivors with a manifold in survivor order (==
// the reference's addManifoldToSolver append order, narrowphase.cpp:
// 1123-1162), capped at maxContacts like the reference's assert
// (narrowphase.cpp:1130).  One pass over the compact per-survivor records
// (4 B, coalesced, 8 chunks' loads in flight): records k < rec_cap are
// written, the count covers all of them.
constexpr int32_t kInfoUnroll = 8;

template <typename RecPtr>
__device__ __forceinline__ int32_t gatherContacts(const PhysArgs &P, int32_t w, RecPtr recs,
                                                  int32_t rec_cap, int32_t lane)
{
    const int32_t nb = P.maxBodiesPerWorld;
    const uint32_t *info = P.survInfo + (size_t)w * P.candCapacity;
    int32_t *order = P.contactOrder + (size_t)w * P.candCapacity;
    int32_t *flags = P.errorFlags + w;
    const int32_t S = P.survCount[w];
    const int32_t maxK = P.maxContacts;
    const int32_t cap = min(rec_cap, maxK);
    const uint64_t lt_mask = (1ull << lane) - 1;
    int32_t k0 = 0;
    for (int32_t chunk = 0; chunk < S; chunk += kSolverBlock * kInfoUnroll) {
        uint32_t v[kInfoUnroll];
#pragma unroll
        for (int32_t u = 0; u < kInfoUnroll; u++) {
            const int32_t s = chunk + u * kSolverBlock + lane;
            v[u] = s < S ? info[s] : kNoManifold;
        }
#pragma unroll
        for (int32_t u = 0; u < kInfoUnroll; u++) {
            const int32_t s = chunk + u * kSolverBlock + lane;
            const bool has = v[u] != kNoManifold;
            const uint64_t mask = worldBallot(has);
            const int32_t k = k0 + __popcll(mask & lt_mask);
            if (has && k < maxK) order[k] = s;
            if (has && k < cap) {
                recs[k] = CRec { (int16_t)guardIndex((int32_t)(v[u] & 0xffffu), nb, flags, kGuardSolverBody),
                                 (int16_t)guardIndex((int32_t)(v[u] >> 16), nb, flags, kGuardSolverBody),
                                 0, (int16_t)s };
            }
            k0 += __popcll(mask);
        }
    }
    if (k0 > maxK) {
        if (lane == 0) atomicOr(flags, kErrContactOverflow);
        k0 = maxK;
    }
    if (lane == 0) P.lastNumContacts[w] = k0;
    return k0;
}

// ConstraintData rows the substep solves (collectConstraintsSystem copies
// every row, physics.cpp:34-40), capped at maxJointConstraints.
__device__ __forceinline__ int32_t worldJointCount(const PhysArgs &P, int32_t w, int32_t lane)
{
    int32_t J = P.numJointRows[w];
    const int32_t cap = min(P.maxJoints, P.jointCapacity);
    if (J > cap) {
        if (lane == 0) atomicOr(P.errorFlags + w, kErrJointOverflow);
        J = cap;
    }
    return J;
}

// Body slot of a joint's entity (ctx.getLoc + getDirect, physics.cpp:540-553).
__device__ __forceinline__ int32_t jointBodySlot(const PhysArgs &P, int32_t w, Entity e)
{
    const Loc l = entityLoc(P, w, e);
    int32_t slot = -1;
    for (int i = 0; i < P.numBodyArchs; i++) {
        if ((uint32_t)P.body[i].archetype == l.archetype && l.row >= 0 &&
            l.row < P.body[i].numRows[w]) {
            slot = P.body[i].slotBase + l.row;
        }
    }
    return guardIndex(slot, P.maxBodiesPerWorld, P.errorFlags + w, kGuardSolverBody);
}

// Joint items K .. K+J-1 (the reference solves joints after contacts).
template <typename RecPtr>
__device__ __forceinline__ void appendJoints(const PhysArgs &P, int32_t w, RecPtr recs, int32_t K,
                                             int32_t J, int32_t lane)
{
    const JointConstraint *jrows = P.joints + (size_t)w * P.jointCapacity;
    for (int32_t j = lane; j < J; j += kSolverBlock) {
        const JointConstraint &jc = jrows[j];
        recs[K + j] = CRec { (int16_t)jointBodySlot(P, w, jc.e1), (int16_t)jointBodySlot(P, w, jc.e2),
                             0, (int16_t)(-1 - j) };
    }
}

// Dependency levels of the world's N items: an item waits only for the
// latest earlier item on each of its bodies (invariant static bodies
// excepted); level = 1 + max(levels of those predecessors), relaxed to its
// fixpoint.  Predecessors chunk by chunk (64 items, one per lane): each
// body's touch mask holds the chunk's lanes touching it, so an item's
// predecessor is the highest lower lane in that mask, else the body's latest
// item of the earlier chunks.  One wave per world.
template <typename RecPtr, typename PrevPtr>
__device__ __forceinline__ int32_t scheduleLevels(SolverLDS &L, int32_t N, RecPtr recs,
                                                  PrevPtr prevs, int32_t lane)
{
    const uint64_t lt_mask = (1ull << lane) - 1;
    for (int32_t base = 0; base < N; base += kSolverBlock) {
        const int32_t k = base + lane;
        const bool valid = k < N;
        const CRec r = valid ? recs[k] : CRec { 0, 0, 0, 0 };
        const bool on1 = valid && !invariantState(L.state[r.s1]);
        const bool on2 = valid && !invariantState(L.state[r.s2]) && r.s2 != r.s1;
        if (on1) atomicOr((unsigned long long *)&L.touch[r.s1], 1ull << lane);
        if (on2) atomicOr((unsigned long long *)&L.touch[r.s2], 1ull << lane);
        waveSync();
        int32_t p1 = -1, p2 = -1;
        uint64_t m1 = 0, m2 = 0;
        if (on1) {
            m1 = L.touch[r.s1];
            const uint64_t lo = m1 & lt_mask;
            p1 = lo ? base + 63 - __clzll(lo) : L.state[r.s1];
        }
        if (on2) {
            m2 = L.touch[r.s2];
            const uint64_t lo = m2 & lt_mask;
            p2 = lo ? base + 63 - __clzll(lo) : L.state[r.s2];
        }
        waveSync();
        // the chunk's last item on each body becomes the body's latest
        if (on1 && 63 - __clzll(m1) == lane) L.state[r.s1] = (int16_t)k;
        if (on2 && 63 - __clzll(m2) == lane) L.state[r.s2] = (int16_t)k;
        if (on1) L.touch[r.s1] = 0;
        if (on2) L.touch[r.s2] = 0;
        if (valid) {
            prevs[k] = (p1 & 0xffff) | (p2 << 16);
            recs[k].lvl = 1;
        }
        waveSync();
    }
    for (;;) {
        bool changed = false;
        for (int32_t k = lane; k < N; k += kSolverBlock) {
            const int32_t pv = prevs[k];
            const int32_t p1 = (int16_t)(pv & 0xffff), p2 = pv >> 16;
            const int32_t l1 = p1 >= 0 ? recs[p1].lvl : 0;
            const int32_t l2 = p2 >= 0 ? recs[p2].lvl : 0;
            const int32_t l = max(l1, l2) + 1;
            if (l != recs[k].lvl) {
                recs[k].lvl = (int16_t)l;
                changed = true;
            }
        }
        waveSync();
        if (!__any(changed)) break;
    }
    int32_t max_level = 0;
    for (int32_t k = lane; k < N; k += kSolverBlock) max_level = max(max_level, (int32_t)recs[k].lvl);
#pragma unroll
    for (int32_t off = kSolverBlock / 2; off > 0; off >>= 1)
        max_level = max(max_level, __shfl_xor(max_level, off));
    return max_level;
}

__device__ __forceinline__ int32_t itemKind(const SolverLDS &L, const CRec r)
{
    if (r.slot < 0) return kKindGeneral;
    const bool i1 = invariantState(L.state[r.s1]), i2 = invariantState(L.state[r.s2]);
    if (i1 && !i2) return kKindStaticRef;
    if (i2 && !i1) return kKindStaticAlt;
    return kKindGeneral;
}

__device__ __forceinline__ bool bodySkips(const SolverLDS &L, int32_t slot)
{
    return L.state[slot] == kStateStaticSkip;
}

// setVelocities (physics.cpp:673-714) for one world, one wave.
__device__ __forceinline__ void setWorldVelocities(const PhysArgs &P, int32_t w, SolverLDS &L,
                                                   float h, int32_t lane)
{
    for (int32_t ba = 0; ba < P.numBodyArchs; ba++) {
        const BodyArch &B = P.body[ba];
        const int32_t rows = B.numRows[w];
        for (int32_t r0 = 0; r0 < rows; r0 += kSolverBlock * kRowBatch) {
            Vector3 px[kRowBatch];
            Quat qp[kRowBatch];
            bool act[kRowBatch];
#pragma unroll
            for (int32_t j = 0; j < kRowBatch; j++) {
                const int32_t r = r0 + j * kSolverBlock + lane;
                act[j] = r < rows && !bodySkips(L, B.slotBase + r);
                if (!act[j]) continue;
                const auto &prev = bcol<solver::SubstepPrevState>(B, Cols::SubstepPrevState, w, r);
                px[j] = ldV3(&prev.prevPosition);
                qp[j] = ldQ(&prev.prevRotation);
            }
#pragma unroll
            for (int32_t j = 0; j < kRowBatch; j++) {
                const int32_t r = r0 + j * kSolverBlock + lane;
                if (!act[j]) continue;
                SMut *s = L.bodies + B.slotBase + r;
                const Vector3 x = ldV3(&s->x);
                const Quat q = ldQ(&s->q);
                Quat dq;
                if (q.w != qp[j].w || q.x != qp[j].x || q.y != qp[j].y || q.z != qp[j].z) {
                    dq = q * qp[j].inv();
                } else {
                    dq = Quat { 1, 0, 0, 0 };
                }
                Vector3 new_omega = 2.f / h * Vector3 { dq.x, dq.y, dq.z };
                stV3(&s->v, (x - px[j]) / h);
                stV3(&s->omega, dq.w > 0.f ? new_omega : -new_omega);
            }
        }
    }
}

// Write the solved bodies back; integrate_next: then run the next
// substep's substepRigidBodies on them (integrateApply writes the pose) and
// the next substep's narrowphase filter for the world (filterWorldOnWave,
// into the nextSatWork list set) from the bodies' new boxes, which are kept
// in the world's LDS image: box slot s (32 B) overwrites the SMut bytes of
// slots <= s only, and slots are processed in increasing order with every
// lane's SMut reads of a round issued before its box writes, so no SMut
// entry is overwritten before it is read.  A batch's integration inputs
// (columns, then object tables) are loaded before its first row.
__device__ __forceinline__ void writeWorldBodies(const PhysArgs &P, int32_t w, SolverLDS &L,
                                                 int32_t lane, bool integrate_next)
{
    static_assert(sizeof(BodyBox) <= sizeof(SMut), "box image aliases the body image");
    BodyBox *boxes = (BodyBox *)L.bodies;
    for (int32_t ba = 0; ba < P.numBodyArchs; ba++) {
        const BodyArch &B = P.body[ba];
        const int32_t rows = B.numRows[w];
        for (int32_t r0 = 0; r0 < rows; r0 += kSolverBlock * kWriteBatch) {
            IntegrateIn in[kWriteBatch];
            IntegrateObj od[kWriteBatch];
            bool skip[kWriteBatch];
#pragma unroll
            for (int32_t j = 0; j < kWriteBatch; j++) {
                const int32_t r = r0 + j * kSolverBlock + lane;
                skip[j] = r < rows && bodySkips(L, B.slotBase + r);
            }
            if (integrate_next) {
#pragma unroll
                for (int32_t j = 0; j < kWriteBatch; j++) {
                    const int32_t r = r0 + j * kSolverBlock + lane;
                    if (r < rows && !skip[j]) in[j] = integrateLoad(B, w, r);
                    if (skip[j]) {
                        // a skipped static body's current box rides in the
                        // row's integration records (an array of its own
                        // stayed in scratch: 112 B per lane)
                        const BodyBox bb = P.bodyBoxes[(size_t)w * P.maxBodiesPerWorld + B.slotBase + r];
                        od[j].aabb = bb.box;
                        in[j].obj = bb.obj;
                        od[j].type = bb.type;
                    }
                }
#pragma unroll
                for (int32_t j = 0; j < kWriteBatch; j++) {
                    const int32_t r = r0 + j * kSolverBlock + lane;
                    if (r < rows && !skip[j]) od[j] = integrateObj(P, in[j].obj);
                }
            }
#pragma unroll
            for (int32_t j = 0; j < kWriteBatch; j++) {
                const int32_t r = r0 + j * kSolverBlock + lane;
                const bool live = r < rows && !skip[j];
                if (skip[j]) {
                    // every write of this body would store the value it holds
                    if (integrate_next) {
                        waveSync();                       // the round's SMut reads first
                        boxes[B.slotBase + r] = BodyBox { od[j].aabb, in[j].obj, od[j].type };
                    }
                } else if (live) {
                    const SMut *s = L.bodies + B.slotBase + r;
                    const Vector3 x = ldV3(&s->x), v = ldV3(&s->v), om = ldV3(&s->omega);
                    const Quat q = ldQ(&s->q);
                    Velocity &vel = bcol<Velocity>(B, Cols::Velocity, w, r);
                    stV3(&vel.linear, v);
                    stV3(&vel.angular, om);
                    if (integrate_next) {
                        const BodyBox bb = integrateApply(P, B, w, r, in[j], od[j], x, q, v, om);
                        waveSync();                       // the round's SMut reads first
                        boxes[B.slotBase + r] = bb;
                    } else {
                        stV3(&bcol<Vector3>(B, Cols::Position, w, r), x);
                        stQ(&bcol<Quat>(B, Cols::Rotation, w, r), q);
                    }
                } else if (integrate_next) {
                    waveSync();                           // matches the live lanes' barrier
                }
            }
        }
    }
    if (lane == 0) P.solver[w].numContacts = 0;           // physics.cpp:1007
    if (integrate_next) {
        waveSync();
        filterWorldOnWave(P, w, boxes, lane, P.nextSatWork, P.nextSatWorkCount);
    }
}

#if defined(MW_SOLVER_PROFILE)
static __device__ unsigned long long g_solverPhase[16];
static __device__ unsigned long long g_solverBlockT[2 * 16384];   // start, end per block (last launch)
#endif

// One positional item: a contact (solveContactPositions) or a joint.  A
// contact against an invariant static body skips that body's side; if the
// skipping solve meets a non-finite lambda it is redone in full, which
// writes the static body the level schedule treated as untouched: the world
// is flagged.
// The solves by static side (ST: 0 = both bodies, 1 = skip the ref body --
// the ground plane of a hull-plane manifold, nearly every contact --,
// 2 = skip the alt body).
__device__ __forceinline__ int32_t solvePositionsGeneral(SMut &b1, SMut &b2, const ContactIn &c,
                                                         const PosIn &in, float *lambda_out)
{
    return solveContactPositionsT<0>(b1, b2, c, in, lambda_out);
}
__device__ __forceinline__ int32_t solvePositionsStaticAlt(SMut &b1, SMut &b2, const ContactIn &c,
                                                           const PosIn &in, float *lambda_out)
{
    return solveContactPositionsT<2>(b1, b2, c, in, lambda_out);
}
__device__ __forceinline__ int32_t solveVelocitiesGeneral(SMut &b1, SMut &b2, const ContactIn &c,
                                                          const VelIn &in, float h, float rt)
{
    return solveContactVelocitiesT<0>(b1, b2, c, in, h, rt);
}
__device__ __forceinline__ int32_t solveVelocitiesStaticAlt(SMut &b1, SMut &b2, const ContactIn &c,
                                                            const VelIn &in, float h, float rt)
{
    return solveContactVelocitiesT<2>(b1, b2, c, in, h, rt);
}

// Which solve an item takes: its kind, unless a contact's inputs are out of
// the bound the skipping solves rely on.
__device__ __forceinline__ int32_t solveKind(int32_t kind, const ContactIn &c)
{
    if (kind != kKindGeneral && !boundedInput(c)) return kKindGeneral;
    return kind;
}

#if defined(MW_SAT_CUTS)
// timing build: cut 7 = the positions phase with its loads only
static __device__ int32_t g_solverCut;
#endif

// A general solve (a joint, a contact of the general kind, or the fallback of
// a skipping solve) may write an invariant static body it touches: it then
// takes the per-body phases again (bodySkips).
__device__ __forceinline__ void markStaticWritten(SolverLDS &L, const CRec r)
{
    if (invariantState(L.state[r.s1])) L.state[r.s1] = kStateStaticWritten;
    if (invariantState(L.state[r.s2])) L.state[r.s2] = kStateStaticWritten;
}

__device__ __forceinline__ void solveItemPositions(const PhysArgs &P, int32_t w, SolverLDS &L,
                                                   const CRec r, int32_t kind)
{
    if (r.slot >= 0) {
        Contact &cr = P.candContacts[(size_t)w * P.candCapacity + r.slot];
        SMut &b1 = L.bodies[r.s1], &b2 = L.bodies[r.s2];
        // one round of loads: the manifold and the bodies' columns
        const ContactIn c = loadContact(cr);
        PosIn in = loadPosIn(P, w, L.pre, b1, r.s1, b2, r.s2, kind == kKindStaticRef, kind == kKindStaticAlt);
#if defined(MW_SAT_CUTS)
        if (g_solverCut == 7) {               // every loaded word kept alive, no solve
            float acc = (float)c.np;
            const float *fc = (const float *)&c;
            for (size_t i = 0; i < sizeof(ContactIn) / 4; i++) acc += fc[i];
            const float *fi = (const float *)&in;
            for (size_t i = 0; i < sizeof(PosIn) / 4; i++) acc += fi[i];
            if (acc == 1.2345f) b1.x.x = acc;
            return;
        }
#endif
        const int32_t k = solveKind(kind, c);
        int32_t res = kSolveNonFinite;
        if (k == kKindStaticRef) {
            res = solveContactPositionsT<1>(b1, b2, c, in, cr.lambdaN);
        } else if (k == kKindStaticAlt) {
            res = solvePositionsStaticAlt(b1, b2, c, in, cr.lambdaN);
        }
        if (res != kSolveDone) {
            if (k != kKindGeneral) atomicOr(P.errorFlags + w, kErrStaticSchedule);
            if (kind != kKindGeneral) in = loadPosIn(P, w, L.pre, b1, r.s1, b2, r.s2, false, false);
            markStaticWritten(L, r);
            solvePositionsGeneral(b1, b2, c, in, cr.lambdaN);
        }
    } else {
        const JointConstraint &j = P.joints[(size_t)w * P.jointCapacity + (-1 - r.slot)];
        markStaticWritten(L, r);
        solveJoint(P, L.bodies[r.s1], L.bodies[r.s2], j);
    }
}

__device__ __forceinline__ void solveItemVelocities(const PhysArgs &P, int32_t w, SolverLDS &L,
                                                    const CRec r, int32_t kind)
{
    if (r.slot < 0) return;                                // joints: positions only
    SMut &b1 = L.bodies[r.s1], &b2 = L.bodies[r.s2];
    const ContactIn c = loadContact(P.candContacts[(size_t)w * P.candCapacity + r.slot]);
    VelIn in = loadVelIn(P, w, L.pre, b1, r.s1, b2, r.s2, kind == kKindStaticRef, kind == kKindStaticAlt);
    const SolverData &sd = P.solver[w];
    const int32_t k = solveKind(kind, c);
    int32_t res = kSolveNonFinite;
    if (k == kKindStaticRef) {
        res = solveContactVelocitiesT<1>(b1, b2, c, in, sd.h, sd.restitutionThreshold);
    } else if (k == kKindStaticAlt) {
        res = solveVelocitiesStaticAlt(b1, b2, c, in, sd.h, sd.restitutionThreshold);
    }
    if (res != kSolveDone) {
        if (k != kKindGeneral) atomicOr(P.errorFlags + w, kErrStaticSchedule);
        if (kind != kKindGeneral) in = loadVelIn(P, w, L.pre, b1, r.s1, b2, r.s2, false, false);
        markStaticWritten(L, r);
        solveVelocitiesGeneral(b1, b2, c, in, sd.h, sd.restitutionThreshold);
    }
}

// Phase profile (experiments only, -DMW_SOLVER_PROFILE): per-phase sums of
// block time in 10 ns device-clock ticks, read by mw_debug_solver_phases.
#if defined(MW_SOLVER_PROFILE)
#define MW_SOLVER_MARK(i)                                                        \
    do {                                                                         \
        if (threadIdx.x == 0) {                                                  \
            const long long t__ = wall_clock64();                                \
            atomicAdd(&g_solverPhase[(i)], (unsigned long long)(t__ - prof_t));  \
            prof_t = t__;                                                        \
        }                                                                        \
    } while (0)
#else
#define MW_SOLVER_MARK(i) ((void)0)
#endif

// Occupancy: latency bound (dependent LDS / column reads per contact), so
// residency matters more than packed math; built without SLP vectorisation
// (Makefile) it fits 3 waves per SIMD without spills.
// Timing build only (make BUILD=build_cut EXTRA=-DMW_SAT_CUTS): the solver
// block returns after phase g_solverCut (1 load + count, 2 levels, 3 sort,
// 4 positions, 5 setVelocities, 6 velocities; 0: whole), relaunched on one
// substep's inputs by mw_debug_time_solver (physics.hip).
#if defined(MW_SAT_CUTS)
extern "C" int MW_SOLVER_C(mw_debug_set_solver_cut)(int32_t cut)
{
    return hipMemcpyToSymbol(HIP_SYMBOL(g_solverCut), &cut, sizeof(cut)) == hipSuccess ? 0 : -1;
}
#define MW_SOLVER_CUT(i) do { if (g_solverCut == (i) || ((i) == 4 && g_solverCut == 7)) return; } while (0)
#else
#define MW_SOLVER_CUT(i) ((void)0)
#endif

#ifndef MW_SOLVER_WAVES_PER_EU
#define MW_SOLVER_WAVES_PER_EU 3
#endif

// XPBD solver, kSolverWorlds worlds per block (one wave each for the
// per-world phases).  The Gauss-Seidel passes run level by level over the
// block's (level, kind)-sorted (world, item) list, so a level's items from
// all of the block's worlds share the lanes and a wave's lanes mostly share
// a code path.
// kGlobal: the worlds' body images exceed a workgroup's LDS and live in the
// block's slab of P.solverImage (solverGlobalKernel); the block schedule
// (items, buckets) stays in LDS.
template <bool kGlobal>
__device__ __forceinline__ void solverBlock(const PhysArgs &P, int32_t integrate_next)
{
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    const int32_t nb = P.maxBodiesPerWorld;
    // world images at `smem`, the block schedule after kSolverWorlds of them
    char *smem = kGlobal ? P.solverImage + (size_t)blockIdx.x * kSolverWorlds * solverWorldLDSBytes(nb)
                         : smem_raw;
    const int32_t wi = threadIdx.x / kSolverBlock;
    const int32_t lane = threadIdx.x % kSolverBlock;
    __shared__ int32_t s_worlds[kSolverWorlds];
    const int32_t wslot = blockIdx.x * kSolverWorlds + wi;
    const bool live = wslot < P.numWorlds;
    const int32_t w = live ? P.solverOrder[wslot] : 0;
    if (lane == 0) s_worlds[wi] = w;
    SolverLDS L = solverWorldLDS(smem, nb, wi);
    const bool alias = !kGlobal && solverAliasSchedule(nb);
    SolverBlockLDS BL = solverBlockLDS(kGlobal ? smem_raw : smem + kSolverWorlds * solverWorldLDSBytes(nb),
                                       alias ? &L : nullptr);

#if defined(MW_SOLVER_PROFILE)
    long long prof_t = wall_clock64();
    if (threadIdx.x == 0 && blockIdx.x < 16384) g_solverBlockT[2 * blockIdx.x] = (unsigned long long)prof_t;
#endif
    if (threadIdx.x == 0) { BL.scalars[1] = 0; BL.scalars[2] = 0; BL.scalars[3] = 0; }
    int32_t K = 0, J = 0;
#if MW_SOLVER_WARM
    constexpr int32_t kWarmContacts = (kSolverLDSContacts + kSolverBlock - 1) / kSolverBlock;
    uint32_t cwarm[2 * kWarmContacts];
#pragma unroll
    for (int32_t i = 0; i < 2 * kWarmContacts; i++) cwarm[i] = 0;
#endif
    if (live) {
        loadWorldBodies(P, w, L, lane);
        J = worldJointCount(P, w, lane);
        K = gatherContacts(P, w, L.recs, kSolverLDSContacts, lane);
#if MW_SOLVER_WARM
        // the lines of the manifold words a solve reads (bytes 16-111)
        waveSync();
        const Contact *cbase = P.candContacts + (size_t)w * P.candCapacity;
#pragma unroll
        for (int32_t i = 0; i < kWarmContacts; i++) {
            const int32_t k = lane + i * kSolverBlock;
            if (k < min(K, kSolverLDSContacts)) {
                const uint32_t *c = (const uint32_t *)(cbase + L.recs[k].slot);
                cwarm[2 * i] = c[4];
                cwarm[2 * i + 1] = c[27];
            }
        }
#endif
    }
    __syncthreads();
    if (live && lane == 0) atomicMax(&BL.scalars[1], K + J);
    __syncthreads();
    const bool fits = BL.scalars[1] <= kSolverLDSContacts;
    MW_SOLVER_MARK(0);
    MW_SOLVER_CUT(1);

    // Levels of the world's items (contacts, then joints) in LDS, unless the
    // items overflow the LDS records or the levels the bucket table holds:
    // then every world of the block takes the global records -- its items
    // gathered and levelled again in its slab, each wave solving its own
    // world level by level (same bits).  Both paths share the solve loops
    // below, so the solves are inlined once (a second inlined copy had cost
    // 20 VGPRs and 40 % of the kernel's code).
    int32_t N = K + J;
    int32_t max_level = 0;
    if (fits) {
        int32_t my_levels = 0;
        if (live) {
            appendJoints(P, w, L.recs, K, J, lane);
            waveSync();
            my_levels = scheduleLevels(L, N, L.recs, L.prevs, lane);
        }
        if (live && lane == 0) atomicMax(&BL.scalars[2], my_levels);
        if (live && lane == 0 && P.solverLevelStats) P.solverLevelStats[w] = (uint32_t)N | (uint32_t)my_levels << 16;
        __syncthreads();
        max_level = BL.scalars[2];
    }
    MW_SOLVER_MARK(1);
    MW_SOLVER_CUT(2);
    const bool global = !fits || max_level > MW_SOLVER_MAX_LEVELS;
    CRec *grecs = (CRec *)(P.solverRecs + (size_t)w * P.recStride);
    if (global) {
        int32_t my_levels = 0;
        N = 0;
        if (live) {
            if (fits) {                       // scheduled once already: afresh
                for (int32_t b = lane; b < nb; b += kSolverBlock) {
                    if (!invariantState(L.state[b])) L.state[b] = -1;
                }
                waveSync();
            }
            K = gatherContacts(P, w, grecs, INT32_MAX, lane);
            appendJoints(P, w, grecs, K, J, lane);
            waveSync();
            N = K + J;
            my_levels = scheduleLevels(L, N, grecs, P.solverPrevs + (size_t)w * P.recStride, lane);
        }
        if (live && lane == 0) atomicMax(&BL.scalars[3], my_levels);
        if (live && lane == 0 && P.solverLevelStats)
            P.solverLevelStats[w] = (uint32_t)min(N, 0xffff) | (uint32_t)min(my_levels, 0xffff) << 16;
        __syncthreads();
        max_level = BL.scalars[3];
    } else {
        // counting sort of the block's items by (level, kind), in place:
        // counts, exclusive offsets, then each item's atomicAdd on its
        // offset -- which leaves bucketOff[b] = the end of bucket b, i.e.
        // the start of b + 1
        const int32_t nbk = (max_level + 2) * kNumKinds;
        for (int32_t i = threadIdx.x; i < nbk; i += kSolverThreads) BL.bucketOff[i] = 0;
        __syncthreads();
        if (live) {
            for (int32_t k = lane; k < N; k += kSolverBlock) {
                const CRec r = L.recs[k];
                atomicAdd(&BL.bucketOff[r.lvl * kNumKinds + itemKind(L, r)], 1);
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int32_t run = 0;
            for (int32_t b = 0; b < nbk; b++) {
                const int32_t c = BL.bucketOff[b];
                BL.bucketOff[b] = run;
                run += c;
            }
        }
        __syncthreads();
        if (live) {
            for (int32_t k = lane; k < N; k += kSolverBlock) {
                const CRec r = L.recs[k];
                const int32_t kind = itemKind(L, r);
                const int32_t b = r.lvl * kNumKinds + kind;
                const int32_t pos = atomicAdd(&BL.bucketOff[b], 1);
                BL.items[pos] = ((uint32_t)wi << 16) | ((uint32_t)kind << 12) | (uint32_t)k;
            }
        }
        __syncthreads();
    }
    MW_SOLVER_MARK(2);
    MW_SOLVER_CUT(3);

    // The items of level l: the block's (level, kind)-sorted run, or
    // (global) this wave's world's records at level l.
    struct LevelItem {
        int32_t iw, kind;
        CRec r;
    };
    auto levelItem = [&](int32_t l, int32_t t, LevelItem &it) -> bool {
        if (global) {
            it.r = grecs[t];
            if (it.r.lvl != l) return false;
            it.iw = wi;
            it.kind = itemKind(L, it.r);
        } else {
            const uint32_t e = BL.items[t];
            it.iw = (int32_t)(e >> 16);
            it.kind = (int32_t)((e >> 12) & 0xfu);
            it.r = solverWorldLDS(smem, nb, it.iw).recs[e & 0xfffu];
        }
        return true;
    };
    const int32_t stride = global ? kSolverBlock : kSolverThreads;
#if MW_SOLVER_WARM
#pragma unroll
    for (int32_t i = 0; i < 2 * kWarmContacts; i++) keepLoaded(cwarm[i]);
#endif

    // solvePositions, level by level
    for (int32_t l = 1; l <= max_level; l++) {
        int32_t t = global ? lane : BL.bucketOff[l * kNumKinds - 1] + threadIdx.x;
        const int32_t end = global ? N : BL.bucketOff[(l + 1) * kNumKinds - 1];
        for (; t < end; t += stride) {
            LevelItem it;
            const bool got = levelItem(l, t, it);
#if defined(MW_SOLVER_PROFILE)
            {   // item kinds per wave pass: static-side items, general ones,
                // passes, passes mixing both (the wave runs both solves)
                const uint64_t ms = __ballot(got && it.kind != kKindGeneral);
                const uint64_t mg = __ballot(got && it.kind == kKindGeneral);
                if ((threadIdx.x & 63) == 0) {
                    atomicAdd(&g_solverPhase[9], (unsigned long long)__popcll(ms));
                    atomicAdd(&g_solverPhase[10], (unsigned long long)__popcll(mg));
                    atomicAdd(&g_solverPhase[11], 1ull);
                    if (ms && mg) atomicAdd(&g_solverPhase[12], 1ull);
                    if (__popcll(ms | mg) <= 16) atomicAdd(&g_solverPhase[13], 1ull);
                }
            }
#endif
            if (!got) continue;
            SolverLDS LW = solverWorldLDS(smem, nb, it.iw);
            solveItemPositions(P, s_worlds[it.iw], LW, it.r, it.kind);
        }
        __syncthreads();
    }

    MW_SOLVER_MARK(3);
    MW_SOLVER_CUT(4);
    if (live) setWorldVelocities(P, w, L, P.solver[w].h, lane);
    __syncthreads();
    MW_SOLVER_MARK(4);
    MW_SOLVER_CUT(5);

    // solveVelocities, same schedule (joints: positions only; in the global
    // records they sort last, k >= K)
    for (int32_t l = 1; l <= max_level; l++) {
        int32_t t = global ? lane : BL.bucketOff[l * kNumKinds - 1] + threadIdx.x;
        const int32_t end = global ? K : BL.bucketOff[(l + 1) * kNumKinds - 1];
        for (; t < end; t += stride) {
            LevelItem it;
            if (!levelItem(l, t, it)) continue;
            SolverLDS LW = solverWorldLDS(smem, nb, it.iw);
            solveItemVelocities(P, s_worlds[it.iw], LW, it.r, it.kind);
        }
        __syncthreads();
    }

    MW_SOLVER_MARK(5);
    MW_SOLVER_CUT(6);
    if (live) writeWorldBodies(P, w, L, lane, integrate_next != 0);
    __syncthreads();
    MW_SOLVER_MARK(6);
#if defined(MW_SOLVER_PROFILE)
    if (threadIdx.x == 0 && blockIdx.x < 16384) g_solverBlockT[2 * blockIdx.x + 1] = (unsigned long long)wall_clock64();
    if (threadIdx.x == 0) atomicAdd(&g_solverPhase[7], 1ull);
    if (threadIdx.x == 0) atomicAdd(&g_solverPhase[8], (unsigned long long)max_level);
#endif
}

__global__ void __launch_bounds__(kSolverThreads)
__attribute__((amdgpu_waves_per_eu(MW_SOLVER_WAVES_PER_EU, 8))) solverKernel(PhysArgs P,
                                                                            int32_t integrate_next)
{
    MW_TRACE_BLOCK(0);
    solverBlock<false>(P, integrate_next);
}

__global__ void __launch_bounds__(kSolverThreads) solverGlobalKernel(PhysArgs P, int32_t integrate_next)
{
    MW_TRACE_BLOCK(0);
    solverBlock<true>(P, integrate_next);
}

#if defined(MW_SOLVER_PROFILE)
extern "C" int MW_SOLVER_C(mw_debug_solver_block_times)(unsigned long long *out, int n)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_solverBlockT), sizeof(unsigned long long) * 2 * n) == hipSuccess ? 0 : -1;
}

extern "C" int MW_SOLVER_C(mw_debug_solver_phases)(unsigned long long *out)
{
    unsigned long long z[16] = {};
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_solverPhase), sizeof(z)) != hipSuccess) return -1;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_solverPhase), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif

size_t solverSharedBytes(const PhysArgs &P)
{
    return solverBlockLDSBytes(P.maxBodiesPerWorld);
}

size_t solverGlobalSharedBytes(const PhysArgs &P)
{
    return solverScheduleBytes() + sizeof(int32_t) * 4;
}

size_t solverImageBytes(const PhysArgs &P)
{
    return kSolverWorlds * solverWorldLDSBytes(P.maxBodiesPerWorld);
}

SolverVariant solverVariant()
{
    return SolverVariant { (const void *)&solverKernel, (const void *)&solverGlobalKernel,
                           kSolverThreads, kSolverWorlds, kSolverBlock, &solverSharedBytes,
                           &solverGlobalSharedBytes, &solverImageBytes };
}

}   // namespace MW_SOLVER_NS
}
