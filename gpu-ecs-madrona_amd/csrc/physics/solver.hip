// XPBD solver kernel (reference src/physics/physics.cpp:166-1008).
#include "physics_device.hpp"

#include <cfloat>

namespace madrona::phys {

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

__device__ void solveContactPositions(const PhysArgs &P, int32_t w, SMut &b1, int32_t s1,
                                      SMut &b2, int32_t s2, Contact &c)
{                                                          // physics.cpp:281-476
    const BodyRO o1 = bodyRO(P, s1, b1.meta), o2 = bodyRO(P, s2, b2.meta);
    const auto ps1 = bcol<solver::PreSolvePositional>(P.body[o1.arch], Cols::PreSolvePositional, w, o1.row);
    const auto ps2 = bcol<solver::PreSolvePositional>(P.body[o2.arch], Cols::PreSolvePositional, w, o2.row);
    const auto pv1 = bcol<solver::SubstepPrevState>(P.body[o1.arch], Cols::SubstepPrevState, w, o1.row);
    const auto pv2 = bcol<solver::SubstepPrevState>(P.body[o2.arch], Cols::SubstepPrevState, w, o2.row);
    const RigidBodyMetadata m1 = P.objs.metadata[o1.obj], m2 = P.objs.metadata[o2.obj];
    Vector3 x1 = b1.x, x2 = b2.x;
    Quat q1 = b1.q, q2 = b2.q;
    float im1 = m1.invMass, im2 = m2.invMass;
    Vector3 iI1 = m1.invInertiaTensor, iI2 = m2.invInertiaTensor;
    if (isStaticBody(b1.meta)) { im1 = 0.f; iI1 = Vector3::zero(); }
    if (isStaticBody(b2.meta)) { im2 = 0.f; iI2 = Vector3::zero(); }
    const float avg_mu_s = 0.5f * (m1.muS + m2.muS);
    const Vector3 n = c.normal;
    const int32_t np = c.numPoints;
#pragma unroll 1
    for (int i = 0; i < np; i++) {
        Vector3 c1 = c.points[i].xyz();
        float depth = c.points[i].w;
        Vector3 c2 = c1 - n * depth;
        Vector3 r1 = ps1.q.inv().rotateVec(c1 - ps1.x);
        Vector3 r2 = ps2.q.inv().rotateVec(c2 - ps2.x);
        float lambda_n = 0.f;
        Vector3 p1 = q1.rotateVec(r1) + x1;
        Vector3 p2 = q2.rotateVec(r2) + x2;
        float d = dot(p1 - p2, n);
        if (d > 0) {
            Vector3 nl1 = q1.inv().rotateVec(n);
            Vector3 nl2 = q2.inv().rotateVec(n);
            Vector3 ta1 = cross(r1, nl1);
            Vector3 ta2 = cross(r2, nl2);
            Vector3 ra1 = multDiag(iI1, ta1);
            Vector3 ra2 = multDiag(iI2, ta2);
            lambda_n = computePositionalLambda(ta1, ta2, ra1, ra2, im1, im2, d, 0);
            applyPositionalUpdate(x1, x2, q1, q2, ra1, ra2, im1, im2, n, lambda_n);

            Vector3 p1_hat = pv1.prevRotation.rotateVec(r1) + pv1.prevPosition;
            Vector3 p2_hat = pv2.prevRotation.rotateVec(r2) + pv2.prevPosition;
            p1 = q1.rotateVec(r1) + x1;
            p2 = q2.rotateVec(r2) + x2;
            Vector3 dp = (p1 - p1_hat) - (p2 - p2_hat);
            Vector3 dpt = dp - dot(dp, n) * n;
            float tmag = dpt.length();
            if (tmag > 0.f) {
                Vector3 tw = dpt / tmag;
                Vector3 tl1 = q1.inv().rotateVec(tw);
                Vector3 tl2 = q2.inv().rotateVec(tw);
                Vector3 fta1 = cross(r1, tl1);
                Vector3 fta2 = cross(r2, tl2);
                Vector3 fra1 = multDiag(iI1, fta1);
                Vector3 fra2 = multDiag(iI2, fta2);
                float lambda_t = computePositionalLambda(fta1, fta2, fra1, fra2, im1, im2, tmag, 0);
                float thresh = lambda_n * avg_mu_s;
                if (lambda_t > thresh) {
                    applyPositionalUpdate(x1, x2, q1, q2, fra1, fra2, im1, im2, tw, lambda_t);
                }
            }
        }
        c.lambdaN[i] = lambda_n;
    }
    b1.x = x1; b2.x = x2;
    b1.q = q1; b2.q = q2;
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

__device__ void solveContactVelocities(const PhysArgs &P, int32_t w, SMut &b1, int32_t s1,
                                       SMut &b2, int32_t s2, const Contact &c, float h,
                                       float rest_thresh)
{                                                          // physics.cpp:865-993
    const BodyRO o1 = bodyRO(P, s1, b1.meta), o2 = bodyRO(P, s2, b2.meta);
    const auto ps1 = bcol<solver::PreSolvePositional>(P.body[o1.arch], Cols::PreSolvePositional, w, o1.row);
    const auto ps2 = bcol<solver::PreSolvePositional>(P.body[o2.arch], Cols::PreSolvePositional, w, o2.row);
    const auto pv1 = bcol<solver::PreSolveVelocity>(P.body[o1.arch], Cols::PreSolveVelocity, w, o1.row);
    const auto pv2 = bcol<solver::PreSolveVelocity>(P.body[o2.arch], Cols::PreSolveVelocity, w, o2.row);
    const RigidBodyMetadata m1 = P.objs.metadata[o1.obj], m2 = P.objs.metadata[o2.obj];
    const Quat q1 = b1.q, q2 = b2.q;
    Vector3 v1 = b1.v, o1v = b1.omega, v2 = b2.v, o2v = b2.omega;
    float im1 = m1.invMass, im2 = m2.invMass;
    Vector3 iI1 = m1.invInertiaTensor, iI2 = m2.invInertiaTensor;
    if (isStaticBody(b1.meta)) { im1 = 0.f; iI1 = Vector3::zero(); }
    if (isStaticBody(b2.meta)) { im2 = 0.f; iI2 = Vector3::zero(); }
    const float mu_d = 0.5f * (m1.muD + m2.muD);
    const Vector3 n = c.normal;

    // Per point only the body-local lever arms and the pre-solve normal
    // velocity stay live; the world-space arms (q fixed during this phase)
    // and the angular terms are recomputed where used -- the same operations
    // on the same inputs, so bit-identical, at a third of the registers.
    Vector3 r1l[4], r2l[4];
    float vn_bars[4];
    const Vector3 nl1 = q1.inv().rotateVec(n);
    const Vector3 nl2 = q2.inv().rotateVec(n);
#pragma unroll
    for (int i = 0; i < 4; i++) {
        if (i >= c.numPoints) continue;
        Vector3 c1 = c.points[i].xyz();
        float depth = c.points[i].w;
        Vector3 c2 = c1 - n * depth;
        Vector3 r1 = ps1.q.inv().rotateVec(c1 - ps1.x);
        Vector3 r2 = ps2.q.inv().rotateVec(c2 - ps2.x);
        Vector3 r1p = ps1.q.rotateVec(r1);
        Vector3 r2p = ps2.q.rotateVec(r2);
        Vector3 vbar = relVel(pv1.v, pv2.v, pv1.omega, pv2.omega, r1p, r2p);
        vn_bars[i] = dot(n, vbar);
        r1l[i] = r1;
        r2l[i] = r2;
    }
    for (int it = 0; it < 2; it++) {                       // :813-863
#pragma unroll
        for (int i = 0; i < 4; i++) {
            if (i >= c.numPoints) continue;
            Vector3 v = relVel(v1, v2, o1v, o2v, q1.rotateVec(r1l[i]), q2.rotateVec(r2l[i]));
            float vn = dot(n, v);
            float vn_bar = vn_bars[i];
            float e = 0.3f;
            if (fabsf(vn_bar) <= rest_thresh) e = 0.f;
            float mag = fminRef(-e * vn_bar, 0) - vn;
            applyVelocityUpdate(v1, v2, o1v, o2v, q1, q2, cross(r1l[i], nl1), cross(r2l[i], nl2),
                                im1, im2, iI1, iI2, n, mag);
        }
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {                          // :752-811
        if (i >= c.numPoints) continue;
        Vector3 v = relVel(v1, v2, o1v, o2v, q1.rotateVec(r1l[i]), q2.rotateVec(r2l[i]));
        float dfm = mu_d * fabsf(c.lambdaN[i]) / h;
        float vn = dot(n, v);
        Vector3 vt = v - n * vn;
        float vt_len = vt.length();
        if (vt_len != 0 && dfm != 0.f) {
            float corrected = -fminRef(dfm, vt_len);
            Vector3 dw = vt / vt_len;
            Vector3 d1l = q1.inv().rotateVec(dw);
            Vector3 d2l = q2.inv().rotateVec(dw);
            Vector3 fta1 = cross(r1l[i], d1l);
            Vector3 fta2 = cross(r2l[i], d2l);
            applyVelocityUpdate(v1, v2, o1v, o2v, q1, q2, fta1, fta2, im1, im2, iI1, iI2, dw,
                                corrected);
        }
    }
    b1.v = v1; b1.omega = o1v;
    b2.v = v2; b2.omega = o2v;
}

__device__ __forceinline__ bool isNegZero(float f) { return __float_as_uint(f) == 0x80000000u; }

// A static body is never written through if every solver write to it is an
// exact no-op: x +- (+-0) and q +- (+-0) keep bits when no component is -0,
// and normalize() must be idempotent on its rotation (static velocities are
// always +0 after setVelocities).  Such bodies add no ordering edge.
__device__ __forceinline__ bool staticInvariant(const SMut &b)
{
    if (!isStaticBody(b.meta)) return false;
    if (isNegZero(b.x.x) || isNegZero(b.x.y) || isNegZero(b.x.z)) return false;
    if (isNegZero(b.q.w) || isNegZero(b.q.x) || isNegZero(b.q.y) || isNegZero(b.q.z)) return false;
    Quat nq = b.q.normalize();
    return __float_as_uint(nq.w) == __float_as_uint(b.q.w) &&
           __float_as_uint(nq.x) == __float_as_uint(b.q.x) &&
           __float_as_uint(nq.y) == __float_as_uint(b.q.y) &&
           __float_as_uint(nq.z) == __float_as_uint(b.q.z);
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

// Per-world LDS image: bodies, ordering flags, contact records.
struct SolverLDS {
    SMut *bodies;         // [nb]
    int16_t *lastLevel;   // [nb] -1: invariant static body (no ordering edges)
    CRec *recs;           // [kSolverLDSContacts]
    int32_t *prevs;       // [kSolverLDSContacts] (prev contact on s1, on s2) as 2 x int16
};

__host__ __device__ inline size_t solverA16(size_t b) { return (b + 15) & ~size_t(15); }

__host__ __device__ inline size_t solverWorldLDSBytes(int32_t nb)
{
    return solverA16(sizeof(SMut) * nb) + solverA16(sizeof(int16_t) * nb) +
           (sizeof(CRec) + sizeof(int32_t)) * kSolverLDSContacts;
}

// Block-shared level schedule: every (world, contact) of the block sorted
// by level, so one pass over a level keeps all of the block's lanes on that
// level's contacts from all of its worlds.
constexpr int32_t kSolverItems = kSolverWorlds * kSolverLDSContacts;

__host__ __device__ inline size_t solverBlockLDSBytes(int32_t nb)
{
    return kSolverWorlds * solverWorldLDSBytes(nb) +
           sizeof(uint32_t) * kSolverItems +               // items (world << 16 | k)
           sizeof(int32_t) * 2 * (kSolverItems + 2) +      // level offsets / cursors
           sizeof(int32_t) * 4;                            // block scalars
}

struct SolverBlockLDS {
    uint32_t *items;
    int32_t *levelOff;    // [Lmax + 2]
    int32_t *levelCur;    // [Lmax + 2]
    int32_t *scalars;     // [0] sum K, [1] max K, [2] max level
};

__device__ __forceinline__ SolverLDS solverWorldLDS(char *smem, int32_t nb, int32_t wi)
{
    SolverLDS L;
    char *p = smem + (size_t)wi * solverWorldLDSBytes(nb);
    L.bodies = (SMut *)p;
    p += solverA16(sizeof(SMut) * nb);
    L.lastLevel = (int16_t *)p;
    p += solverA16(sizeof(int16_t) * nb);
    L.recs = (CRec *)p;
    p += sizeof(CRec) * kSolverLDSContacts;
    L.prevs = (int32_t *)p;
    return L;
}

__device__ __forceinline__ SolverBlockLDS solverBlockLDS(char *smem, int32_t nb)
{
    SolverBlockLDS B;
    char *p = smem + kSolverWorlds * solverWorldLDSBytes(nb);
    B.items = (uint32_t *)p;
    p += sizeof(uint32_t) * kSolverItems;
    B.levelOff = (int32_t *)p;
    p += sizeof(int32_t) * (kSolverItems + 2);
    B.levelCur = (int32_t *)p;
    p += sizeof(int32_t) * (kSolverItems + 2);
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

// Load one world's bodies into its LDS image (wave `lane` 0..63).
__device__ __forceinline__ void loadWorldBodies(const PhysArgs &P, int32_t w, SolverLDS &L,
                                                int32_t lane)
{
    for (int32_t ba = 0; ba < P.numBodyArchs; ba++) {
        const BodyArch &B = P.body[ba];
        const int32_t rows = B.numRows[w];
        for (int32_t r = lane; r < rows; r += kSolverBlock) {
            SMut s;
            s.x = bcol<Vector3>(B, Cols::Position, w, r);
            s.q = bcol<Quat>(B, Cols::Rotation, w, r);
            const Velocity vel = bcol<Velocity>(B, Cols::Velocity, w, r);
            s.v = vel.linear;
            s.omega = vel.angular;
            const uint32_t obj = (uint32_t)bcol<ObjectID>(B, Cols::ObjectID, w, r).idx;
            s.meta = ((uint32_t)bcol<ResponseType>(B, Cols::ResponseType, w, r) & 0xffu) |
                     ((uint32_t)ba << 8) | (obj << 16);
            L.bodies[B.slotBase + r] = s;
            L.lastLevel[B.slotBase + r] = staticInvariant(s) ? (int16_t)-1 : (int16_t)0;
        }
    }
}

// Number of survivors with a manifold (the world's contact count), capped at
// maxContacts like the reference's assert (narrowphase.cpp:1130).  Reads the
// compact per-survivor records (4 B, coalesced) with 8 chunks' loads in
// flight, instead of the 112-B Contact records.
constexpr int32_t kInfoUnroll = 8;

__device__ __forceinline__ int32_t worldContactCount(const PhysArgs &P, int32_t w, int32_t lane)
{
    const uint32_t *info = P.survInfo + (size_t)w * P.candCapacity;
    const int32_t S = P.survCount[w];
    int32_t K = 0;
    for (int32_t chunk = 0; chunk < S; chunk += kSolverBlock * kInfoUnroll) {
        uint32_t v[kInfoUnroll];
#pragma unroll
        for (int32_t u = 0; u < kInfoUnroll; u++) {
            const int32_t s = chunk + u * kSolverBlock + lane;
            v[u] = s < S ? info[s] : kNoManifold;
        }
#pragma unroll
        for (int32_t u = 0; u < kInfoUnroll; u++) K += __popcll(__ballot(v[u] != kNoManifold));
    }
    if (K > P.maxContacts) {
        if (lane == 0) atomicOr(P.errorFlags + w, kErrContactOverflow);
        K = P.maxContacts;
    }
    return K;
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

// Contact records in survivor order (== the reference's addManifoldToSolver
// append order, narrowphase.cpp:1123-1162) and their dependency levels: a
// contact waits only for the latest earlier contact on each of its bodies
// (invariant static bodies excepted); level = 1 + max(levels of those
// predecessors), relaxed to its fixpoint.  One wave per world.
template <typename RecPtr, typename PrevPtr>
__device__ __forceinline__ int32_t orderAndLevel(const PhysArgs &P, int32_t w, SolverLDS &L,
                                                 int32_t K, int32_t J, RecPtr recs,
                                                 PrevPtr prevs, int32_t lane)
{
    const int32_t nb = P.maxBodiesPerWorld;
    const uint32_t *info = P.survInfo + (size_t)w * P.candCapacity;
    int32_t *order = P.contactOrder + (size_t)w * P.candCapacity;
    const int32_t S = P.survCount[w];
    const uint64_t lt_mask = (1ull << lane) - 1;
    int32_t *flags = P.errorFlags + w;
    int32_t k0 = 0;
    for (int32_t chunk = 0; chunk < S && k0 < K; chunk += kSolverBlock * kInfoUnroll) {
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
            const uint64_t mask = __ballot(has);
            const int32_t k = k0 + __popcll(mask & lt_mask);
            if (has && k < K) {
                recs[k] = CRec { (int16_t)guardIndex((int32_t)(v[u] & 0xffffu), nb, flags, kGuardSolverBody),
                                 (int16_t)guardIndex((int32_t)(v[u] >> 16), nb, flags, kGuardSolverBody),
                                 0, (int16_t)s };
                order[k] = s;
            }
            k0 += __popcll(mask);
        }
    }
    const JointConstraint *jrows = P.joints + (size_t)w * P.jointCapacity;
    for (int32_t j = lane; j < J; j += kSolverBlock) {
        const JointConstraint &jc = jrows[j];
        recs[K + j] = CRec { (int16_t)jointBodySlot(P, w, jc.e1), (int16_t)jointBodySlot(P, w, jc.e2),
                             0, (int16_t)(-1 - j) };
    }
    K += J;
    waveSync();
    for (int32_t k = lane; k < K; k += kSolverBlock) {
        CRec r = recs[k];
        const bool on1 = L.lastLevel[r.s1] >= 0, on2 = L.lastLevel[r.s2] >= 0;
        int32_t p1 = -1, p2 = -1;
        for (int32_t j = k - 1; j >= 0 && ((on1 && p1 < 0) || (on2 && p2 < 0)); j--) {
            const CRec q = recs[j];
            if (on1 && p1 < 0 && (q.s1 == r.s1 || q.s2 == r.s1)) p1 = j;
            if (on2 && p2 < 0 && (q.s1 == r.s2 || q.s2 == r.s2)) p2 = j;
        }
        prevs[k] = (p1 & 0xffff) | (p2 << 16);
        r.lvl = 1;
        recs[k] = r;
    }
    waveSync();
    for (;;) {
        bool changed = false;
        for (int32_t k = lane; k < K; k += kSolverBlock) {
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
    for (int32_t k = lane; k < K; k += kSolverBlock) max_level = max(max_level, (int32_t)recs[k].lvl);
#pragma unroll
    for (int32_t off = 32; off > 0; off >>= 1) max_level = max(max_level, __shfl_xor(max_level, off));
    if (lane == 0) P.lastNumContacts[w] = K - J;
    return max_level;
}

// setVelocities (physics.cpp:673-714) for one world, one wave.
__device__ __forceinline__ void setWorldVelocities(const PhysArgs &P, int32_t w, SolverLDS &L,
                                                   float h, int32_t lane)
{
    for (int32_t ba = 0; ba < P.numBodyArchs; ba++) {
        const BodyArch &B = P.body[ba];
        const int32_t rows = B.numRows[w];
        for (int32_t r = lane; r < rows; r += kSolverBlock) {
            SMut &s = L.bodies[B.slotBase + r];
            const auto prev = bcol<solver::SubstepPrevState>(B, Cols::SubstepPrevState, w, r);
            const Quat q = s.q, qp = prev.prevRotation;
            Quat dq;
            if (q.w != qp.w || q.x != qp.x || q.y != qp.y || q.z != qp.z) {
                dq = q * qp.inv();
            } else {
                dq = Quat { 1, 0, 0, 0 };
            }
            Vector3 new_omega = 2.f / h * Vector3 { dq.x, dq.y, dq.z };
            s.v = (s.x - prev.prevPosition) / h;
            s.omega = dq.w > 0.f ? new_omega : -new_omega;
        }
    }
}

__device__ __forceinline__ void writeWorldBodies(const PhysArgs &P, int32_t w, SolverLDS &L,
                                                 int32_t lane)
{
    for (int32_t ba = 0; ba < P.numBodyArchs; ba++) {
        const BodyArch &B = P.body[ba];
        const int32_t rows = B.numRows[w];
        for (int32_t r = lane; r < rows; r += kSolverBlock) {
            const SMut &s = L.bodies[B.slotBase + r];
            bcol<Vector3>(B, Cols::Position, w, r) = s.x;
            bcol<Quat>(B, Cols::Rotation, w, r) = s.q;
            bcol<Velocity>(B, Cols::Velocity, w, r) = Velocity { s.v, s.omega };
        }
    }
    if (lane == 0) P.solver[w].numContacts = 0;           // physics.cpp:1007
}

// One positional item: a contact (solveContactPositions) or a joint.
__device__ __forceinline__ void solveItemPositions(const PhysArgs &P, int32_t w, SolverLDS &L,
                                                   const CRec r)
{
    if (r.slot >= 0) {
        Contact &c = P.candContacts[(size_t)w * P.candCapacity + r.slot];
        solveContactPositions(P, w, L.bodies[r.s1], r.s1, L.bodies[r.s2], r.s2, c);
    } else {
        const JointConstraint &j = P.joints[(size_t)w * P.jointCapacity + (-1 - r.slot)];
        solveJoint(P, L.bodies[r.s1], L.bodies[r.s2], j);
    }
}

// Fallback for a world whose contacts do not fit the LDS records: the whole
// solve on its own wave, records in the global slab, level by level.
__device__ __forceinline__ void solveWorldGlobal(const PhysArgs &P, int32_t w, SolverLDS L,
                                              int32_t K, int32_t J, int32_t lane)
{
    CRec *recs = (CRec *)(P.solverRecs + (size_t)w * P.recStride);
    int32_t *prevs = P.solverPrevs + (size_t)w * P.recStride;
    const int32_t max_level = orderAndLevel(P, w, L, K, J, recs, prevs, lane);
    const SolverData &sd = P.solver[w];
    const int32_t N = K + J;
    for (int32_t l = 1; l <= max_level; l++) {
        for (int32_t k = lane; k < N; k += kSolverBlock) {
            const CRec r = recs[k];
            if (r.lvl != l) continue;
            solveItemPositions(P, w, L, r);
        }
        waveSync();
    }
    setWorldVelocities(P, w, L, sd.h, lane);
    waveSync();
    for (int32_t l = 1; l <= max_level; l++) {
        for (int32_t k = lane; k < K; k += kSolverBlock) {   // joints sort last
            const CRec r = recs[k];
            if (r.lvl != l) continue;
            const Contact &c = P.candContacts[(size_t)w * P.candCapacity + r.slot];
            solveContactVelocities(P, w, L.bodies[r.s1], r.s1, L.bodies[r.s2], r.s2, c, sd.h,
                                   sd.restitutionThreshold);
        }
        waveSync();
    }
}

// Phase profile (experiments only, -DMW_SOLVER_PROFILE): per-phase sums of
// block time in 10 ns device-clock ticks, read by mw_debug_solver_phases.
#if defined(MW_SOLVER_PROFILE)
static __device__ unsigned long long g_solverPhase[16];
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
#ifndef MW_SOLVER_WAVES_PER_EU
#define MW_SOLVER_WAVES_PER_EU 3
#endif

// XPBD solver, kSolverWorlds worlds per block (one wave each for the
// per-world phases).  The Gauss-Seidel contact passes run level by level
// over the block's level-sorted (world, contact) list, so a level's
// contacts from all of the block's worlds share the lanes: sparse deep
// levels no longer cost a full wave pass per world.
__global__ void __launch_bounds__(kSolverThreads)
__attribute__((amdgpu_waves_per_eu(MW_SOLVER_WAVES_PER_EU, 8))) solverKernel(PhysArgs P)
{
    MW_TRACE_BLOCK(0);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int32_t nb = P.maxBodiesPerWorld;
    const int32_t wi = threadIdx.x / kSolverBlock;
    const int32_t lane = threadIdx.x % kSolverBlock;
    const int32_t w = blockIdx.x * kSolverWorlds + wi;
    const bool live = w < P.numWorlds;
    SolverLDS L = solverWorldLDS(smem, nb, wi);
    SolverBlockLDS BL = solverBlockLDS(smem, nb);

#if defined(MW_SOLVER_PROFILE)
    long long prof_t = wall_clock64();
#endif
    if (threadIdx.x == 0) { BL.scalars[0] = 0; BL.scalars[1] = 0; BL.scalars[2] = 0; }
    int32_t K = 0, J = 0;
    if (live) {
        loadWorldBodies(P, w, L, lane);
        K = worldContactCount(P, w, lane);
        J = worldJointCount(P, w, lane);
    }
    __syncthreads();
    if (live && lane == 0) atomicMax(&BL.scalars[1], K + J);
    __syncthreads();
    const bool fits = BL.scalars[1] <= kSolverLDSContacts;
    MW_SOLVER_MARK(0);

    if (!fits) {
        // some world of the block overflows the LDS records: every world
        // of the block solves on its own wave with global records
        if (live) {
            solveWorldGlobal(P, w, L, K, J, lane);
            writeWorldBodies(P, w, L, lane);
        }
        return;
    }

    int32_t my_levels = 0;
    if (live) my_levels = orderAndLevel(P, w, L, K, J, L.recs, L.prevs, lane);
    if (live && lane == 0) atomicMax(&BL.scalars[2], my_levels);
    __syncthreads();
    const int32_t max_level = BL.scalars[2];
    MW_SOLVER_MARK(1);

    // counting sort of the block's contacts by level
    for (int32_t i = threadIdx.x; i <= max_level + 1; i += kSolverThreads) {
        BL.levelOff[i] = 0;
        BL.levelCur[i] = 0;
    }
    __syncthreads();
    const int32_t N = K + J;     // contacts, then joints
    if (live) {
        for (int32_t k = lane; k < N; k += kSolverBlock) atomicAdd(&BL.levelOff[L.recs[k].lvl], 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int32_t run = 0;
        for (int32_t l = 0; l <= max_level + 1; l++) {
            const int32_t c = BL.levelOff[l];
            BL.levelOff[l] = run;
            run += c;
        }
    }
    __syncthreads();
    if (live) {
        for (int32_t k = lane; k < N; k += kSolverBlock) {
            const int32_t l = L.recs[k].lvl;
            const int32_t pos = BL.levelOff[l] + atomicAdd(&BL.levelCur[l], 1);
            BL.items[pos] = ((uint32_t)wi << 16) | (uint32_t)k;
        }
    }
    __syncthreads();
    MW_SOLVER_MARK(2);

    // solvePositions, level by level over the whole block
    for (int32_t l = 1; l <= max_level; l++) {
        const int32_t beg = BL.levelOff[l], end = BL.levelOff[l + 1];
        for (int32_t t = beg + threadIdx.x; t < end; t += kSolverThreads) {
            const uint32_t it = BL.items[t];
            const int32_t iw = (int32_t)(it >> 16), k = (int32_t)(it & 0xffffu);
            const int32_t ww = blockIdx.x * kSolverWorlds + iw;
            SolverLDS LW = solverWorldLDS(smem, nb, iw);
            solveItemPositions(P, ww, LW, LW.recs[k]);
        }
        __syncthreads();
    }

    MW_SOLVER_MARK(3);
    if (live) setWorldVelocities(P, w, L, P.solver[w].h, lane);
    __syncthreads();
    MW_SOLVER_MARK(4);

    // solveVelocities, same schedule
    for (int32_t l = 1; l <= max_level; l++) {
        const int32_t beg = BL.levelOff[l], end = BL.levelOff[l + 1];
        for (int32_t t = beg + threadIdx.x; t < end; t += kSolverThreads) {
            const uint32_t it = BL.items[t];
            const int32_t iw = (int32_t)(it >> 16), k = (int32_t)(it & 0xffffu);
            const int32_t ww = blockIdx.x * kSolverWorlds + iw;
            SolverLDS LW = solverWorldLDS(smem, nb, iw);
            const CRec r = LW.recs[k];
            if (r.slot < 0) continue;                      // joints: positions only
            const Contact &c = P.candContacts[(size_t)ww * P.candCapacity + r.slot];
            const SolverData &sd = P.solver[ww];
            solveContactVelocities(P, ww, LW.bodies[r.s1], r.s1, LW.bodies[r.s2], r.s2, c,
                                   sd.h, sd.restitutionThreshold);
        }
        __syncthreads();
    }

    MW_SOLVER_MARK(5);
    if (live) writeWorldBodies(P, w, L, lane);
    __syncthreads();
    MW_SOLVER_MARK(6);
#if defined(MW_SOLVER_PROFILE)
    if (threadIdx.x == 0) atomicAdd(&g_solverPhase[7], 1ull);
    if (threadIdx.x == 0) atomicAdd(&g_solverPhase[8], (unsigned long long)max_level);
#endif
}

#if defined(MW_SOLVER_PROFILE)
extern "C" int mw_debug_solver_phases(unsigned long long *out)
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

}
