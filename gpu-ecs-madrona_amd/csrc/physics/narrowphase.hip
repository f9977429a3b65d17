// Substep integration + narrowphase kernels (reference src/physics/physics.cpp:79-164,
// src/physics/narrowphase.cpp CPU branch).
#include "physics_device.hpp"

#include <cfloat>

namespace madrona::phys {

// ===========================================================================
// Substep integration (physics.cpp:79-164) plus the world AABB of every body
// for the narrowphase's recheck.
// ===========================================================================

__global__ void __launch_bounds__(256) integrateKernel(PhysArgs P)
{
    MW_TRACE_BLOCK(0);
    // first substep: both list sets start empty (this substep's filter fills
    // satWork, the solver's fused filter nextSatWork)
    if (blockIdx.x == 0 && blockIdx.y == 0) {
        resetNarrowLists(P.satWorkCount, threadIdx.x, blockDim.x);
        resetNarrowLists(P.nextSatWorkCount, threadIdx.x, blockDim.x);
    }
    const BodyArch &B = P.body[blockIdx.y];
    RowIdx ri = rowIndex(P, B);
    if (!ri.valid) return;
    const int32_t w = ri.w, r = ri.r;
    const Velocity vel = bcol<Velocity>(B, Cols::Velocity, w, r);
    integrateBody(P, B, w, r, bcol<Vector3>(B, Cols::Position, w, r), bcol<Quat>(B, Cols::Rotation, w, r),
                  vel.linear, vel.angular);
}

// ===========================================================================
// Narrowphase (narrowphase.cpp, CPU branch), three kernels per substep:
//   1. narrowFilterKernel, block per world: AABB recheck + type ordering of
//      every candidate; a block scan numbers the survivors in candidate order
//      (survivor slot == contact slot); hull-hull survivors go to the SAT
//      work list, hull-plane survivors straight to the contact job list.
//   2. narrowSATKernel, persistent, one kGroup-lane group (8) per hull-hull pair:
//      both hulls are transformed into LDS and the SAT queries are spread
//      over the group with (value, index) reductions that reproduce the
//      reference's serial strict-'>' scans (first occurrence wins, NaN never
//      wins).  A non-separated pair becomes a contact job carrying the
//      chosen feature (reference / incident face or edge pair).
//   3. narrowContactKernel, persistent, one lane per contact job: clipping
//      and manifold reduction (all lanes busy, clip polygons in LDS).
// ===========================================================================
#ifndef MW_SAT_GROUP
#define MW_SAT_GROUP 8
#endif
constexpr int32_t kGroup = MW_SAT_GROUP;               // lanes per hull-hull pair
#if defined(MW_SAT_CUTS)
// Timing build only (make BUILD=build_cut EXTRA=-DMW_SAT_CUTS): with
// mw_debug_set_sat_exp(c), c > 0, every pair is declared separated after
// staging (1), the face queries (2), the Minkowski tables (3), the edge
// query's pass masks (5) or the whole edge query (4); the phases' times by
// difference (mw_debug_time_sat).
static __device__ int32_t g_satExp;
#endif
#ifndef MW_SAT_DPP
#define MW_SAT_DPP (MW_SAT_GROUP == 8)
#endif
constexpr int32_t kGroupsPerBlock = kNarrowBlock / kGroup;

__host__ __device__ inline size_t a16(size_t b) { return (b + 15) & ~size_t(15); }

// World transform of a body's hull (makeHullState, narrowphase.cpp:139-212:
// vertices by R * S, plane normals by R * S^-1 then renormalised).  Every
// kernel derives world-space hull data through these helpers, so the SAT
// kernel's LDS copies and the contact kernel's on-the-fly values agree bit
// for bit.
struct HullXform {
    Mat3x3 vtx;
    Mat3x3 nrm;
    Vector3 x;
};

__device__ __forceinline__ HullXform hullXform(const PhysArgs &P, int32_t w, const BodyArch &B,
                                               int32_t row)
{
    const Vector3 x = bcol<Vector3>(B, Cols::Position, w, row);
    const Quat rot = bcol<Quat>(B, Cols::Rotation, w, row);
    const Diag3x3 scale = bcol<Diag3x3>(B, Cols::Scale, w, row);
    const Mat3x3 unscaled_rot = Mat3x3::fromQuat(rot);
    return HullXform { unscaled_rot * scale, unscaled_rot * scale.inv(), x };
}

__device__ __forceinline__ Vector3 worldVertex(const ObjDev &O, const HullDev &hd,
                                               const HullXform &xf, int32_t i)
{
    return xf.vtx * O.vertices[hd.vertOffset + i] + xf.x;
}

__device__ __forceinline__ geometry::Plane worldPlane(const ObjDev &O, const HullDev &hd,
                                                      const HullXform &xf, int32_t i)
{
    const geometry::Plane op = O.planes[hd.faceOffset + i];
    const Vector3 origin = xf.vtx * (op.normal * op.d) + xf.x;
    const Vector3 n = (xf.nrm * op.normal).normalize();
    return geometry::Plane { n, dot(n, origin) };
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

// ---------------------------------------------------------------------------
// SAT kernel helpers (group of kGroup lanes, hulls staged in LDS)
// ---------------------------------------------------------------------------
struct HullRef {
    const Vector3 *verts;          // world space (LDS copy)
    const geometry::Plane *planes; // world space (LDS copy)
    const EdgeQuad *quads;         // edge topology (LDS copy)
    HullDev hd;
    Vector3 center;
};

// An edge's four 16-bit indices read as one 8-byte word (one LDS load
// instead of one per field).
#ifndef MW_SAT_QUAD64
#define MW_SAT_QUAD64 1
#endif
static_assert(sizeof(EdgeQuad) == 8 && alignof(EdgeQuad) == 2, "four 16-bit fields");
__device__ __forceinline__ EdgeQuad ldQuad(const EdgeQuad *q, int32_t i)
{
#if MW_SAT_QUAD64
    const uint64_t t = *(const uint64_t *)(q + i);
    return EdgeQuad { (uint16_t)(t & 0xffffu), (uint16_t)((t >> 16) & 0xffffu),
                      (uint16_t)((t >> 32) & 0xffffu), (uint16_t)(t >> 48) };
#else
    return q[i];
#endif
}

struct GroupLDS {
    Vector3 *vA, *vB;
    geometry::Plane *pA, *pB;
    EdgeQuad *qA, *qB;
    float *sA;                     // [maxEdges][minkStride]: edge i of a x face f of b
    float *tB;                     // [maxEdges][minkStride]: edge j of b x face f of a
};

#ifndef MW_SAT_BANK_PAD
#define MW_SAT_BANK_PAD 1
#endif

__host__ __device__ inline size_t minkTableBytes(const ObjDev &O)
{
    return a16(sizeof(float) * O.maxEdges * O.minkStride);
}

// A group's staging area, padded to 16 B past a multiple of 128 B: the
// groups of a wave read the same element of their own hulls together, and
// with areas a multiple of 128 B apart those reads all fall on one LDS bank
// (4-way conflicts in each 32-lane half); 16 B more per group puts
// consecutive groups 4 banks apart.
__host__ __device__ inline size_t groupLDSBytes(const ObjDev &O)
{
    const size_t raw = 2 * a16(sizeof(Vector3) * O.maxVerts) + 2 * a16(sizeof(geometry::Plane) * O.maxFaces) +
                       2 * a16(sizeof(EdgeQuad) * O.maxEdges) + 2 * minkTableBytes(O);
#if MW_SAT_BANK_PAD
    return raw + (16 + 128 - raw % 128) % 128;
#else
    return raw;
#endif
}

// The group staging area; block 0 first uses it for the solver's world
// sort (kOrderBuckets ints, sortWorldsForSolver below), so it is never
// smaller than that.
constexpr size_t kOrderSortBytes = 1024 * sizeof(int32_t);

size_t narrowphaseSharedBytes(const PhysArgs &P)
{
    return std::max(kGroupsPerBlock * groupLDSBytes(P.objs), kOrderSortBytes) + P.satGeoBytes;
}

__device__ __forceinline__ GroupLDS groupLDS(char *smem, int32_t group, const ObjDev &O)
{
    char *p = smem + (size_t)group * groupLDSBytes(O);
    GroupLDS g;
    g.vA = (Vector3 *)p; p += a16(sizeof(Vector3) * O.maxVerts);
    g.vB = (Vector3 *)p; p += a16(sizeof(Vector3) * O.maxVerts);
    g.pA = (geometry::Plane *)p; p += a16(sizeof(geometry::Plane) * O.maxFaces);
    g.pB = (geometry::Plane *)p; p += a16(sizeof(geometry::Plane) * O.maxFaces);
    g.qA = (EdgeQuad *)p; p += a16(sizeof(EdgeQuad) * O.maxEdges);
    g.qB = (EdgeQuad *)p; p += a16(sizeof(EdgeQuad) * O.maxEdges);
    g.sA = (float *)p; p += minkTableBytes(O);
    g.tB = (float *)p;
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

// The (value, index) maximum of the group on every lane.  scanWins is a
// total order (value, then lower index; NaN never wins), so the pairing
// order of the reduction does not change the result.  For 8-lane groups the
// exchanges are DPP moves within each 8-lane row half (mirror, then the
// quad's xor 2 and xor 1 -- every lane ends with all eight), VALU
// instructions instead of the LDS permute unit that __shfl_xor uses.
__device__ __forceinline__ int32_t dppMove(int32_t x, int32_t ctrl_sel)
{
    switch (ctrl_sel) {
    case 0: return __builtin_amdgcn_update_dpp(x, x, 0x141, 0xf, 0xf, false);   // row_half_mirror
    case 1: return __builtin_amdgcn_update_dpp(x, x, 0x4e, 0xf, 0xf, false);    // quad_perm [2,3,0,1]
    default: return __builtin_amdgcn_update_dpp(x, x, 0xb1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
    }
}

__device__ __forceinline__ void groupArgMax(float &v, int32_t &k)
{
#if MW_SAT_DPP
    static_assert(kGroup == 8, "DPP reduction over 8-lane groups");
#pragma unroll
    for (int32_t step = 0; step < 3; step++) {
        const float ov = __int_as_float(dppMove(__float_as_int(v), step));
        const int32_t ok = dppMove(k, step);
        if (scanWins(ov, ok, v, k)) { v = ov; k = ok; }
    }
#else
#pragma unroll
    for (int32_t off = kGroup / 2; off > 0; off >>= 1) {
        const float ov = __shfl_xor(v, off, kGroup);
        const int32_t ok = __shfl_xor(k, off, kGroup);
        if (scanWins(ov, ok, v, k)) { v = ov; k = ok; }
    }
#endif
}

// Body columns a SAT group stages a hull from, per body archetype: an LDS
// copy of PhysArgs::body's entries (the kernel-argument array indexed by a
// per-group value is a vector load from the argument segment at every use).
struct SatArch {
    const Vector3 *pos;
    const Quat *rot;
    const Diag3x3 *scale;
    int32_t capacity;
    int32_t archetype;
};

// A body's position, rotation and scale: what its hull's world transform
// (hullXform) is made of.
struct BodyPose {
    Vector3 x;
    Quat q;
    Diag3x3 s;
};

// The column pointers come out of LDS (SatArch), where the compiler no longer
// knows they point to global memory: the loads go through address-space-1
// pointers so that they are global loads, not flat ones (a flat load also
// counts against the LDS wait counter).
typedef const __attribute__((address_space(1))) float *GlobalF;

__device__ __forceinline__ BodyPose loadPose(const SatArch &A, int32_t w, int32_t row)
{
    const size_t i = (size_t)w * A.capacity + row;
    const GlobalF p = (GlobalF)(const void *)A.pos + 3 * i;
    const GlobalF r = (GlobalF)(const void *)A.rot + 4 * i;
    const GlobalF s = (GlobalF)(const void *)A.scale + 3 * i;
    return BodyPose { Vector3 { p[0], p[1], p[2] }, Quat { r[0], r[1], r[2], r[3] },
                      Diag3x3 { s[0], s[1], s[2] } };
}

// Transform one body's hull into the group's LDS and copy its edge topology
// (hullXform / worldVertex / worldPlane, the same operations).
// `first` / `step`: the lanes of the group that stage this hull.
__device__ __forceinline__ void stageHull(const ObjDev &O, const HullDev &hd, const BodyPose &p,
                                          Vector3 *v, geometry::Plane *pl, EdgeQuad *q,
                                          int32_t first, int32_t step)
{
    const Mat3x3 unscaled_rot = Mat3x3::fromQuat(p.q);
    const HullXform xf { unscaled_rot * p.s, unscaled_rot * p.s.inv(), p.x };
    for (int32_t i = first; i < hd.numVerts; i += step)
        v[i] = xf.vtx * O.vertices[hd.vertOffset + i] + xf.x;
    for (int32_t i = first; i < hd.numFaces; i += step) {
        const geometry::Plane op = O.planes[hd.faceOffset + i];
        const Vector3 origin = xf.vtx * (op.normal * op.d) + xf.x;
        const Vector3 n = (xf.nrm * op.normal).normalize();
        pl[i] = geometry::Plane { n, dot(n, origin) };
    }
    for (int32_t i = first; i < hd.numEdges; i += step)
        *(uint64_t *)(q + i) = *(const uint64_t *)(O.edgeQuads + hd.edgeOffset + i);
}

// Both hulls of a pair staged at once: the group's first half transforms
// hull a, the second half hull b, so each lane builds one hull transform
// instead of two (the inputs are picked per lane field by field; selecting
// whole aggregates would go through scratch).
__device__ __forceinline__ void stagePair(const ObjDev &O, const HullRef &ha, const HullRef &hb,
                                          const BodyPose &pa, const BodyPose &pb, const GroupLDS &g,
                                          int32_t lane)
{
    constexpr int32_t kHalf = kGroup / 2;
    const bool second = lane >= kHalf;
    HullDev hd;
    hd.vertOffset = second ? hb.hd.vertOffset : ha.hd.vertOffset;
    hd.numVerts = second ? hb.hd.numVerts : ha.hd.numVerts;
    hd.faceOffset = second ? hb.hd.faceOffset : ha.hd.faceOffset;
    hd.numFaces = second ? hb.hd.numFaces : ha.hd.numFaces;
    hd.edgeOffset = second ? hb.hd.edgeOffset : ha.hd.edgeOffset;
    hd.numEdges = second ? hb.hd.numEdges : ha.hd.numEdges;
    BodyPose p;
    p.x = Vector3 { second ? pb.x.x : pa.x.x, second ? pb.x.y : pa.x.y, second ? pb.x.z : pa.x.z };
    p.q = Quat { second ? pb.q.w : pa.q.w, second ? pb.q.x : pa.q.x, second ? pb.q.y : pa.q.y,
                 second ? pb.q.z : pa.q.z };
    p.s = Diag3x3 { second ? pb.s.d0 : pa.s.d0, second ? pb.s.d1 : pa.s.d1, second ? pb.s.d2 : pa.s.d2 };
    stageHull(O, hd, p, second ? g.vB : g.vA, second ? g.pB : g.pA, second ? g.qB : g.qA,
              second ? lane - kHalf : lane, kHalf);
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

// A face query's result: the deepest face's separation and index (-1 when
// no face scored above -FLT_MAX); its plane is re-read from the staged hull
// when a contact job needs it.
struct FaceQuery {
    float separation;
    int32_t faceIdx;
};

// queryFaceDirections (narrowphase.cpp:395-431).  The reference stops at the
// first face with positive distance; any positive result rejects the pair,
// so the group evaluates every face and only the non-positive case needs the
// serial argmax, which groupArgMax reproduces.
__device__ __forceinline__ FaceQuery groupFaceQuery(const HullRef &a, const HullRef &b, int32_t lane)
{
    float v = __builtin_nanf("");
    int32_t k = INT32_MAX;
    for (int32_t f = lane; f < a.hd.numFaces; f += kGroup) {
        const float d = hullDistFromPlane(a.planes[f], b);
        if (scanWins(d, f, v, k)) { v = d; k = f; }
    }
    groupArgMax(v, k);
    if (v > -FLT_MAX) return { v, k };
    return { -FLT_MAX, -1 };
}

__device__ __forceinline__ geometry::Plane facePlane(const geometry::Plane *planes, int32_t f)
{
    return f >= 0 ? planes[f] : geometry::Plane { { 0, 0, 0 }, 0 };
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

// edgeDistance (narrowphase.cpp:433-472) for edge i of a against edge j of
// b: separation along the edges' cross product, or -FLT_MAX when the edges
// do not form a face of the Minkowski difference or are parallel.
__device__ __forceinline__ float edgePairSeparation(const HullRef &a, const HullRef &b,
                                                    int32_t i, int32_t j, Vector3 *normal_out)
{
    const EdgeQuad ea = ldQuad(a.quads, i), eb = ldQuad(b.quads, j);
    float sep = -FLT_MAX;
    Vector3 n { 0, 0, 0 };
    if (isMinkowskiFace(a.planes[ea.face1].normal, a.planes[ea.face2].normal,
                        -b.planes[eb.face1].normal, -b.planes[eb.face2].normal)) {
        const Vector3 pa1 = a.verts[ea.v1], pb1 = b.verts[eb.v1];
        Vector3 da = a.verts[ea.v2] - pa1, db = b.verts[eb.v2] - pb1;
        Vector3 uc = da.cross(db);
        float l2 = uc.length2();
        if (l2 != 0) {
            float inv = 1.f / sqrtf(l2);
            n = uc * inv;
            if (n.dot(pa1 - a.center) < 0.0f) n = -n;
            sep = n.dot(pb1 - pa1);
        }
    }
    if (normal_out) *normal_out = n;
    return sep;
}

// An edge query's result: the best pair index p = i * nB + j and its
// separation (-FLT_MAX, p = 0 when no pair scored); the contact normal is
// recomputed from the pair when an edge job needs it.
struct EdgeQuery {
    float separation;
    int32_t pair;
};

// queryEdgeDirections (narrowphase.cpp:474-540).  Pair index p = i * nB + j
// is the reference's loop order; the early return on a positive separation
// only ever rejects the pair.  A lane walks its pairs (i, j) incrementally
// and keeps edge i of a (its face normals and their cross product, the
// Minkowski test's a-side) while only j changes: the same operations as
// edgePairSeparation, fewer LDS reads and no division per pair.
__device__ EdgeQuery groupEdgeQuery(const HullRef &a, const HullRef &b, int32_t lane)
{
    const int32_t nA = a.hd.numEdges, nB = b.hd.numEdges;
    float v = __builtin_nanf("");
    int32_t k = INT32_MAX;
    if (nB > 0) {
        int32_t i = lane / nB, j = lane - (lane / nB) * nB;
        int32_t cur = -1;
        EdgeQuad ea {};
        Vector3 an1 {}, an2 {}, bxa {};
        for (int32_t p = lane; p < nA * nB; p += kGroup) {
            if (i != cur) {
                cur = i;
                ea = ldQuad(a.quads, i);
                an1 = a.planes[ea.face1].normal;
                an2 = a.planes[ea.face2].normal;
                bxa = an2.cross(an1);
            }
            const EdgeQuad eb = ldQuad(b.quads, j);
            const Vector3 c = -b.planes[eb.face1].normal, d = -b.planes[eb.face2].normal;
            // isMinkowskiFace(an1, an2, c, d)
            const Vector3 dxc = d.cross(c);
            const float cba = c.dot(bxa), dba = d.dot(bxa);
            const float adc = an1.dot(dxc), bdc = an2.dot(dxc);
            float sep = -FLT_MAX;
            if (cba * dba < 0.0f && adc * bdc < 0.0f && cba * bdc > 0.0f) {
                const Vector3 pa1 = a.verts[ea.v1], pb1 = b.verts[eb.v1];
                Vector3 da = a.verts[ea.v2] - pa1, db = b.verts[eb.v2] - pb1;
                Vector3 uc = da.cross(db);
                float l2 = uc.length2();
                if (l2 != 0) {
                    float inv = 1.f / sqrtf(l2);
                    Vector3 n = uc * inv;
                    if (n.dot(pa1 - a.center) < 0.0f) n = -n;
                    sep = n.dot(pb1 - pa1);
                }
            }
            if (scanWins(sep, p, v, k)) { v = sep; k = p; }
            j += kGroup;
            while (j >= nB) { j -= nB; i++; }
        }
    }
    groupArgMax(v, k);
    if (!(v > -FLT_MAX)) return { -FLT_MAX, 0 };
    return { v, k };
}

// The Minkowski-face test of edge pair (i, j) (isMinkowskiFace(a1, a2, -b1,
// -b2) with a1 / a2 the faces of edge i of a, b1 / b2 those of edge j of b)
// reads four dot products, each a function of one edge and one face:
//   cba = -b1 . (a2 x a1),  dba = -b2 . (a2 x a1)   row i of sA, columns b1 / b2
//   adc = a1 . ((-b2) x (-b1)),  bdc = a2 . ((-b2) x (-b1))   row j of tB
// so the group evaluates them once per (edge, face), not four times per
// edge pair; each entry is the same expression as in edgePairSeparation, so
// the test's verdicts are the same bits.
__device__ __forceinline__ void buildMinkTables(const HullRef &a, const HullRef &b, float *sA, float *tB,
                                                int32_t stride, int32_t lane)
{
    for (int32_t i = lane; i < a.hd.numEdges; i += kGroup) {
        const EdgeQuad ea = ldQuad(a.quads, i);
        const Vector3 bxa = a.planes[ea.face2].normal.cross(a.planes[ea.face1].normal);
        for (int32_t f = 0; f < b.hd.numFaces; f++) sA[i * stride + f] = (-b.planes[f].normal).dot(bxa);
    }
    for (int32_t j = lane; j < b.hd.numEdges; j += kGroup) {
        const EdgeQuad eb = ldQuad(b.quads, j);
        const Vector3 c = -b.planes[eb.face1].normal, d = -b.planes[eb.face2].normal;
        const Vector3 dxc = d.cross(c);
        for (int32_t f = 0; f < a.hd.numFaces; f++) tB[j * stride + f] = a.planes[f].normal.dot(dxc);
    }
}

// groupEdgeQuery with the tables: the lanes first test their edge pairs
// (four LDS reads each, in chunks of 32 pairs per lane, a bit per pair),
// then compute the separation of the pairs that passed.  In the per-pair
// form nearly every step of a wave runs the separation branch for the few
// lanes whose pair passed; here a lane runs it only for its own passes.
// The (separation, p) scan sees the same values in the same order, the
// failed pairs' -FLT_MAX included.
// The lane's (separation, p) scan over one chunk of its pairs p = base +
// kGroup t, t < count, given which passed the Minkowski-face test: failed
// pairs score -FLT_MAX (the scan keeps the first of them), passed ones
// edgePairSeparation's value.
__device__ __forceinline__ void scanPasses(const HullRef &a, const HullRef &b, uint32_t pass, int32_t count,
                                           int32_t base, float &v, int32_t &k)
{
    const int32_t nB = b.hd.numEdges;
    const uint32_t all = count == 32 ? ~0u : (1u << count) - 1u;
    if (pass != all) {
        const int32_t p0 = base + kGroup * __builtin_ctz(~pass);
        if (scanWins(-FLT_MAX, p0, v, k)) { v = -FLT_MAX; k = p0; }
    }
    while (pass) {
        const int32_t bit = __builtin_ctz(pass);
        pass &= pass - 1;
        const int32_t p = base + kGroup * bit;
        const int32_t pi = p / nB, pj = p - pi * nB;
        const EdgeQuad ea = ldQuad(a.quads, pi), eb = ldQuad(b.quads, pj);
        float sep = -FLT_MAX;
        const Vector3 pa1 = a.verts[ea.v1], pb1 = b.verts[eb.v1];
        Vector3 da = a.verts[ea.v2] - pa1, db = b.verts[eb.v2] - pb1;
        Vector3 uc = da.cross(db);
        float l2 = uc.length2();
        if (l2 != 0) {
            float inv = 1.f / sqrtf(l2);
            Vector3 nrm = uc * inv;
            if (nrm.dot(pa1 - a.center) < 0.0f) nrm = -nrm;
            sep = nrm.dot(pb1 - pa1);
        }
        if (scanWins(sep, p, v, k)) { v = sep; k = p; }
    }
}

__device__ __forceinline__ EdgeQuery groupEdgeQueryTables(const HullRef &a, const HullRef &b, const float *sA,
                                          const float *tB, int32_t stride, int32_t lane)
{
    const int32_t nA = a.hd.numEdges, nB = b.hd.numEdges, n = nA * nB;
    float v = __builtin_nanf("");
    int32_t k = INT32_MAX;
    if (nB > 0) {
        // (i, j) of p = lane, lane + kGroup, ...: each step adds (di, dj)
        // with a carry; the table rows follow incrementally
        const int32_t di = kGroup / nB, dj = kGroup - di * nB;
        int32_t i = lane / nB, j = lane - (lane / nB) * nB;
        int32_t irow = i * stride, jrow = j * stride;
        for (int32_t base = lane; base < n; base += 32 * kGroup) {
            uint32_t pass = 0;
            int32_t t = 0;
            for (int32_t p = base; p < n && t < 32; p += kGroup, t++) {
                const EdgeQuad ea = ldQuad(a.quads, i), eb = ldQuad(b.quads, j);
                const float cba = sA[irow + eb.face1], dba = sA[irow + eb.face2];
                const float adc = tB[jrow + ea.face1], bdc = tB[jrow + ea.face2];
                // all three products, no short circuit: the same verdict
                const bool m = (cba * dba < 0.0f) & (adc * bdc < 0.0f) & (cba * bdc > 0.0f);
                pass |= (uint32_t)m << t;
                i += di;
                j += dj;
                irow += di * stride;
                jrow += dj * stride;
                if (j >= nB) {
                    j -= nB;
                    jrow -= nB * stride;
                    i++;
                    irow += stride;
                }
            }
#if defined(MW_SAT_CUTS)
            if (g_satExp == 5) {                 // masks only (kept alive)
                if (pass == 0x7fffffffu) v = 0.0f;
                continue;
            }
#endif
            scanPasses(a, b, pass, t, base, v, k);
        }
    }
    groupArgMax(v, k);
    if (!(v > -FLT_MAX)) return { -FLT_MAX, 0 };
    return { v, k };
}

// The edge query on sign bits (MW_SAT_BITS; hulls of at most 16 edges and
// 32 faces, which covers every box pair).  The Minkowski-face test of pair
// (i, j) only asks for the signs of four table entries, and a product of two
// floats whose magnitudes are at least 2^-62 is never zero, so its sign is
// the xor of theirs: the three products' verdicts are bit operations on
// sign masks once every entry is either exactly zero (its test fails, as the
// product would be zero) or at least 2^-62 in magnitude.  Per row i of a
// (one lane, registers) the bits of sA's row (over faces of b); per face f
// of a the column of tB's signs and zeros over the edges j of b, and per
// face f of b which edges j of b have f as their first / second face -- both
// built with LDS ors in the table space the float tables would use.  Then
// row i's 16 pairs are tested by a handful of word operations:
//   G1 / G2 = edges j whose first / second face has a negative sA[i] entry,
//   pass_i = (G1 ^ G2) & (CB[a1] ^ CB[a2]) & ~(G1 ^ CB[a2]) & ~zeros,
// with a1 / a2 edge i's faces, CB[f] the negative tB[., f] entries.  An
// entry between 0 and 2^-62 (or not finite) sends the pair to the float
// tables (returns false).
#ifndef MW_SAT_BITS
#define MW_SAT_BITS 1
#endif
constexpr int32_t kBitsMaxEdges = 16;
constexpr int32_t kBitsMaxFaces = 32;
constexpr int32_t kBitsRows = (kBitsMaxEdges + kGroup - 1) / kGroup;

__device__ __forceinline__ bool bitsEligible(const HullRef &a, const HullRef &b)
{
    return a.hd.numEdges <= kBitsMaxEdges && b.hd.numEdges <= kBitsMaxEdges &&
           a.hd.numFaces <= kBitsMaxFaces && b.hd.numFaces <= kBitsMaxFaces;
}

// Classifies a table entry: bit 0 negative, bit 1 exactly zero, bit 2 too
// small (or not finite) for the sign rule.
__device__ __forceinline__ uint32_t entryClass(float x)
{
    const float m = fabsf(x);
    return (x < 0.0f ? 1u : 0u) | (x == 0.0f ? 2u : 0u) |
           ((x != 0.0f && !(m >= 0x1p-62f && m <= FLT_MAX)) ? 4u : 0u);
}

__device__ __forceinline__ EdgeQuery groupEdgeQueryBits(const HullRef &a, const HullRef &b, float *sA_space,
                                                        float *tB_space, int32_t lane, bool &ok)
{
    const int32_t nA = a.hd.numEdges, nB = b.hd.numEdges;
    const int32_t fA = a.hd.numFaces, fB = b.hd.numFaces;
    uint32_t *CB = (uint32_t *)sA_space;     // [fA]: negative tB[j][f] (bits 0-15), zero (16-31)
    uint32_t *FB = (uint32_t *)tB_space;     // [fB]: edges with face1 == f (0-15), face2 == f (16-31)
    for (int32_t f = lane; f < fA; f += kGroup) CB[f] = 0;
    for (int32_t f = lane; f < fB; f += kGroup) FB[f] = 0;
    groupSync();
    uint32_t bad = 0;
    // b's rows: the same expressions as buildMinkTables' tB
    for (int32_t j = lane; j < nB; j += kGroup) {
        const EdgeQuad eb = ldQuad(b.quads, j);
        const Vector3 c = -b.planes[eb.face1].normal, d = -b.planes[eb.face2].normal;
        const Vector3 dxc = d.cross(c);
        for (int32_t f = 0; f < fA; f++) {
            const uint32_t cls = entryClass(a.planes[f].normal.dot(dxc));
            bad |= cls;
            const uint32_t bits = ((cls & 1u) << j) | (((cls >> 1) & 1u) << (16 + j));
            if (bits) atomicOr(&CB[f], bits);
        }
        atomicOr(&FB[eb.face1], 1u << j);
        atomicOr(&FB[eb.face2], 1u << (16 + j));
    }
    // a's rows, kept by their lane: negative and zero entries over b's faces
    uint32_t neg[kBitsRows], zero[kBitsRows];
    EdgeQuad qa[kBitsRows];
#pragma unroll
    for (int32_t r = 0; r < kBitsRows; r++) {
        const int32_t i = lane + r * kGroup;
        neg[r] = zero[r] = 0;
        if (i < nA) {
            qa[r] = ldQuad(a.quads, i);
            const Vector3 bxa = a.planes[qa[r].face2].normal.cross(a.planes[qa[r].face1].normal);
            for (int32_t f = 0; f < fB; f++) {
                const uint32_t cls = entryClass((-b.planes[f].normal).dot(bxa));
                bad |= cls;
                neg[r] |= (cls & 1u) << f;
                zero[r] |= ((cls >> 1) & 1u) << f;
            }
        }
    }
    // any entry too small for the sign rule: the whole group falls back
    const uint64_t any_bad = __ballot((bad & 4u) != 0);
    const int32_t gbase = (int32_t)(threadIdx.x & 63) & ~(kGroup - 1);
    ok = ((any_bad >> gbase) & ((1ull << kGroup) - 1)) == 0;
    groupSync();
#if defined(MW_SAT_CUTS)
    if (g_satExp == 3) {                      // masks built (kept alive): separated
        ok = true;
        return { 1.0f + 0.0f * (float)(neg[0] ^ zero[kBitsRows - 1] ^ FB[0] ^ CB[0]), 0 };
    }
#endif
    float v = __builtin_nanf("");
    int32_t k = INT32_MAX;
    if (ok) {
        const uint32_t row_mask = (1u << nB) - 1u;
#pragma unroll
        for (int32_t r = 0; r < kBitsRows; r++) {
            const int32_t i = lane + r * kGroup;
            if (i >= nA) continue;
            uint32_t g1 = 0, g2 = 0, z = 0;
            for (int32_t f = 0; f < fB; f++) {
                const uint32_t w = FB[f];
                const uint32_t e = (w & 0xffffu) | (w >> 16);      // edges touching face f
                if ((neg[r] >> f) & 1u) { g1 |= w & 0xffffu; g2 |= w >> 16; }
                if ((zero[r] >> f) & 1u) z |= e;
            }
            const uint32_t c1 = CB[qa[r].face1], c2 = CB[qa[r].face2];
            z |= (c1 | c2) >> 16;
            const uint32_t pass = (g1 ^ g2) & (c1 ^ c2) & ~(g1 ^ c2) & ~z & row_mask;
            const uint32_t fail = ~pass & row_mask;
#if defined(MW_SAT_CUTS)
            if (g_satExp == 5) {                  // pass masks only (kept alive)
                if (pass == 0x7fffffffu) v = 0.0f;
                continue;
            }
#endif
            if (fail) {
                const int32_t p0 = i * nB + __builtin_ctz(fail);
                if (scanWins(-FLT_MAX, p0, v, k)) { v = -FLT_MAX; k = p0; }
            }
            uint32_t m = pass;
            while (m) {
                const int32_t j = __builtin_ctz(m);
                m &= m - 1;
                const EdgeQuad eb = ldQuad(b.quads, j);
                float sep = -FLT_MAX;
                const Vector3 pa1 = a.verts[qa[r].v1], pb1 = b.verts[eb.v1];
                Vector3 da = a.verts[qa[r].v2] - pa1, db = b.verts[eb.v2] - pb1;
                Vector3 uc = da.cross(db);
                float l2 = uc.length2();
                if (l2 != 0) {
                    float inv = 1.f / sqrtf(l2);
                    Vector3 nrm = uc * inv;
                    if (nrm.dot(pa1 - a.center) < 0.0f) nrm = -nrm;
                    sep = nrm.dot(pb1 - pa1);
                }
                const int32_t p = i * nB + j;
                if (scanWins(sep, p, v, k)) { v = sep; k = p; }
            }
        }
    }
    groupArgMax(v, k);
    if (!(v > -FLT_MAX)) return { -FLT_MAX, 0 };
    return { v, k };
}

__device__ __forceinline__ int32_t findIncidentFace(const geometry::Plane *planes, int32_t num_faces,
                                                    Vector3 ref_normal)
{
    float min_dot = FLT_MAX;
    int32_t face = -1;
    for (int32_t f = 0; f < num_faces; f++) {
        float d = dot(planes[f].normal, ref_normal);
        if (d < min_dot) { min_dot = d; face = f; }
    }
    return face;
}

// ---------------------------------------------------------------------------
// Contact generation helpers (one lane per job)
// ---------------------------------------------------------------------------
__device__ __forceinline__ int32_t clipPolygon(Vector3 *dst, geometry::Plane cp,
                                               const Vector3 *in, int32_t n,
                                               int32_t cap)
{                                                          // narrowphase.cpp:626-661
    if (n == 0) return 0;
    int32_t out = 0;
    Vector3 v1 = in[n - 1];
    float d1 = distFromPlane(cp, v1);
    for (int32_t i = 0; i < n; i++) {
        Vector3 v2 = in[i];
        float d2 = distFromPlane(cp, v2);
        if (d1 <= 0.0f && d2 <= 0.0f) {
            if (out < cap) dst[out++] = v2;
        } else if (d1 <= 0.0f && d2 > 0.0f) {
            if (out < cap) dst[out++] = planeIntersection(cp, v1, v2);
        } else if (d2 <= 0.0f && d1 > 0.0f) {
            if (out < cap) dst[out++] = planeIntersection(cp, v1, v2);
            if (out < cap) dst[out++] = v2;
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
#pragma unroll
        for (int32_t i = 0; i < 4; i++) {          // static indices: cp stays in registers
            if (i < num) { cp[i] = contacts[i]; depth[i] = depths[i]; }
        }
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

// buildFaceContactManifold (narrowphase.cpp:790-864) written straight into
// the contact slot from up to four chosen points (storeFaceManifold's tail).
__device__ __forceinline__ void writeFaceManifold(Contact &c, Vector3 n, const Vector3 *cp,
                                                  const float *depth, int32_t m, Loc ref, Loc alt)
{
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

// Hull a against the plane of body b: doSATPlane (narrowphase.cpp:760-788)
// + createFacePlaneContact (:974-1017) + buildFaceContactManifold (:790-864)
// with O(1) state: the incident face's loop is walked once to count the
// points below the plane and keep the first four, and -- only for a face
// with more than four such points -- again for each of the reference's
// point choices (farthest from p0, then the last positive and the last
// negative area against the p0-p1 line, each over the point list with the
// earlier choices replaced by p0).  Every walk recomputes the same vertices
// with the same operations, so the chosen points are the reference's bits.
// Returns true if a manifold was written.
// The body columns a hull-plane pair reads: the hull's position, rotation
// and scale, the plane body's position and rotation.
struct PlaneIn {
    Vector3 aPos;
    Quat aRot;
    Diag3x3 aScale;
    Vector3 bPos;
    Quat bRot;
};

__device__ __forceinline__ PlaneIn loadPlaneIn(const PhysArgs &P, const SatWork &wk)
{
    const BodyArch &BA = P.body[wk.aArch], &BB = P.body[wk.bArch];
    const int32_t w = wk.world;
    return PlaneIn { bcol<Vector3>(BA, Cols::Position, w, wk.a.row),
                     bcol<Quat>(BA, Cols::Rotation, w, wk.a.row),
                     bcol<Diag3x3>(BA, Cols::Scale, w, wk.a.row),
                     bcol<Vector3>(BB, Cols::Position, w, wk.b.row),
                     bcol<Quat>(BB, Cols::Rotation, w, wk.b.row) };
}

// An object-space vertex of the hull tables; kPad: the LDS copy holds them
// padded to 16 bytes (the plane kernel's staged table), so each is one
// aligned ds_read_b128 instead of a 12-byte read at a 4-byte-aligned address
// (SQ_LDS_UNALIGNED_STALL: 71 % of the kernel's LDS-active cycles before).
template <bool kPad>
__device__ __forceinline__ Vector3 objVertex(const ObjDev &O, int32_t i)
{
    if constexpr (kPad) {
        const float4 v = ((const float4 *)O.vertices)[i];
        return Vector3 { v.x, v.y, v.z };
    } else {
        return O.vertices[i];
    }
}

template <bool kPad>
__device__ __forceinline__ bool planeContact(const PhysArgs &P, const ObjDev &O, int32_t w,
                                             const SatWork &wk, const PlaneIn &in)
{
    // worldVertex with the table's layout (the same operations)
    auto vertex = [&](const HullDev &hd, const HullXform &xf, int32_t i) {
        return xf.vtx * objVertex<kPad>(O, hd.vertOffset + i) + xf.x;
    };
    int32_t *flags = P.errorFlags + w;
    const HullDev ha = O.hulls[wk.aObj];
    const Mat3x3 unscaled_rot = Mat3x3::fromQuat(in.aRot);
    const HullXform xa { unscaled_rot * in.aScale, unscaled_rot * in.aScale.inv(), in.aPos };
    const Vector3 b_pos = in.bPos;
    const Quat b_rot = in.bRot;
    const Vector3 pn = b_rot.rotateVec(Vector3 { 0, 0, 1 });
    const geometry::Plane plane { pn, dot(pn, b_pos) };
    float min_dot = FLT_MAX;
    for (int32_t v = 0; v < ha.numVerts; v++) {
        const float d = plane.normal.dot(vertex(ha, xa, v));
        if (d < min_dot) min_dot = d;
    }
    if (min_dot - plane.d > 0.0f) return false;
    float min_fd = FLT_MAX;
    int32_t inc_face = -1;
    for (int32_t f = 0; f < ha.numFaces; f++) {
        const float d = dot(worldPlane(O, ha, xa, f).normal, plane.normal);
        if (d < min_fd) { min_fd = d; inc_face = f; }
    }
    inc_face = guardIndex(inc_face, ha.numFaces, flags, kGuardPlaneFace);
    const geometry::HalfEdge *hh = O.hedges + ha.hedgeOffset;
    const uint32_t start = O.polygons[ha.faceOffset + inc_face];
    const int32_t cap = P.clipCap;
    // The face's below-plane points in walk order (the reference's contacts /
    // depths arrays), capped at cap like the clip buffer.
    auto walk = [&](auto &&fn) {
        int32_t n = 0, steps = 0;
        uint32_t hidx = start;
        do {
            hidx = guardIndex(hidx, ha.numHedges, flags, kGuardPlaneWalk);
            const geometry::HalfEdge he = hh[hidx];
            hidx = he.next;
            const Vector3 v = vertex(ha, xa, guardIndex(he.rootVertex, ha.numVerts, flags, kGuardVertex));
            const float d = distFromPlane(plane, v);
            if (d < 0.0f && n < cap) {
                fn(n, v - d * plane.normal, -d);
                n++;
            }
        } while (hidx != start && ++steps <= ha.numHedges);
        return n;
    };
    Vector3 cp[4];
    float depth[4];
    for (int i = 0; i < 4; i++) { cp[i] = Vector3::zero(); depth[i] = 0.f; }
    // static indices only (a dynamic cp[i] store sends both arrays to scratch)
    const int32_t num = walk([&](int32_t i, Vector3 c, float dd) {
#pragma unroll
        for (int32_t j = 0; j < 4; j++) {
            if (i == j) {
                cp[j] = c;
                depth[j] = dd;
            }
        }
    });
    int32_t m = num;
    if (num > 4) {
        m = 4;
        const Vector3 p0 = cp[0];
        Vector3 c1 = Vector3::zero(), c2 = Vector3::zero(), c3 = Vector3::zero();
        float d1 = 0.f, d2 = 0.f, d3 = 0.f;
        float largest_d2 = 0.0f;
        int32_t i1 = 0;
        walk([&](int32_t i, Vector3 c, float dd) {
            if (i == 0) return;
            const float dist2 = p0.distance2(c);
            if (dist2 > largest_d2) { largest_d2 = dist2; c1 = c; d1 = dd; i1 = i; }
        });
        const Vector3 diff0 = c1 - p0;
        int32_t i2 = 0;                                    // largest_area_idx
        walk([&](int32_t i, Vector3 c, float dd) {
            if (i == 0) return;
            if (i == i1) c = p0;                           // contacts[largest_d2_idx] = cp[0]
            const float area = plane.normal.dot(diff0.cross(c - p0));
            if (area > 0.0f) { c2 = c; d2 = dd; i2 = i; }
        });
        walk([&](int32_t i, Vector3 c, float dd) {
            if (i == 0) return;
            if (i == i1 || i == i2) c = p0;                // contacts[largest_area_idx] = cp[0]
            const float area = plane.normal.dot(diff0.cross(c - p0));
            if (area < 0.0f) { c3 = c; d3 = dd; }
        });
        cp[1] = c1; cp[2] = c2; cp[3] = c3;
        depth[1] = d1; depth[2] = d2; depth[3] = d3;
    }
    if (m == 0) return false;
    writeFaceManifold(P.candContacts[(size_t)w * P.candCapacity + wk.slot], plane.normal, cp, depth,
                      m, wk.b, wk.a);
    return true;
}

// Body slot (the solver's per-world body index) of a pair member.
__device__ __forceinline__ int32_t slotOf(const PhysArgs &P, int32_t arch_idx, Loc l)
{
    return P.body[arch_idx].slotBase + l.row;
}

// The survivor's compact solver record: ref / alt body slots.
__device__ __forceinline__ void recordManifold(const PhysArgs &P, int32_t w, int32_t slot,
                                               int32_t ref_slot, int32_t alt_slot)
{
    P.survInfo[(size_t)w * P.candCapacity + slot] =
        (uint32_t)(ref_slot & 0xffff) | ((uint32_t)(alt_slot & 0xffff) << 16);
}

// Narrowphase stage 1, block per world: AABB recheck + type ordering of
// every candidate, kFilterPer consecutive candidates per thread (their loads
// in flight together).  One block scan numbers the survivors in candidate
// order (survivor slot == contact slot, the reference's append order) and,
// packed in the same scan, the hull-hull and hull-plane survivors; the block
// then reserves its entries in its bin (world % kNarrowBins) with one atomic
// per list: hull-hull from the bin's front (for the SAT kernel), hull-plane
// from its back (for the plane-contact kernel).  The lists' order does not
// matter: every entry writes only its own slot.
constexpr int32_t kFilterPer = 3;
static_assert(kNarrowBlock * kFilterPer < 1024, "10-bit packed scan fields");

__global__ void __launch_bounds__(kNarrowBlock) narrowFilterKernel(PhysArgs P)
{
    MW_TRACE_BLOCK(0);
    __shared__ int32_t s_scan[kNarrowBlock / 64];
    __shared__ int32_t s_base[3];
    const int32_t w = blockIdx.x;
    const int32_t cap = P.candCapacity;
    const int32_t num = min(P.numCands[w], cap);
    const CandidateCollision *cands = P.cands + (size_t)w * cap;
    const uint64_t *slots = P.candSlots + (size_t)w * cap;
    const BodyBox *boxes = P.bodyBoxes + (size_t)w * P.maxBodiesPerWorld;
    uint32_t *info = P.survInfo + (size_t)w * cap;
    const int32_t bin = w % kNarrowBins;
    PackedSatWork *list = P.satWork + (size_t)bin * P.binCap;
    PackedSatWork *list_back = list + P.binCap - 1;        // plane entries grow down
    constexpr uint32_t kHull = (uint32_t)CollisionPrimitive::Type::Hull;
    constexpr uint32_t kHullPlane = kHull | (uint32_t)CollisionPrimitive::Type::Plane;

    int32_t S = 0;
    for (int32_t base = 0; base < num; base += kNarrowBlock * kFilterPer) {
        SatWork wk[kFilterPer];
        bool keep[kFilterPer];
        int32_t packed = 0;
        const int32_t first = base + (int32_t)threadIdx.x * kFilterPer;
#pragma unroll
        for (int32_t j = 0; j < kFilterPer; j++) {
            const int32_t ci = first + j;
            BodyBox A, B;
            const uint64_t cs = ci < num ? slots[ci] : 0;
            keep[j] = ci < num && candOverlaps(P, w, cs, boxes, A, B);
            if (keep[j]) wk[j] = candWork(cands[ci], cs, A, B, w);
            packed += keep[j] ? 1 : 0;
            packed += keep[j] && wk[j].test == kHull ? 1 << 10 : 0;
            packed += keep[j] && wk[j].test == kHullPlane ? 1 << 20 : 0;
        }
        int32_t total;
        const int32_t off = blockExclusiveScan(packed, s_scan, &total);
        if (threadIdx.x == 0) {
            const int32_t thh = (total >> 10) & 1023, tpl = total >> 20;
            // one reservation in both lists; an overrun of the bin is
            // refused and flagged (reserveBin, filterWorldOnWave)
            s_base[2] = !reserveBin(binCounter(P, bin, 0), thh, tpl, P.binCap, s_base[0], s_base[1]);
            if (s_base[2]) atomicOr(P.errorFlags + w, kErrIndexGuard | (kGuardList << 8));
        }
        __syncthreads();
        if (s_base[2]) {
            S = 0;
            break;
        }
        int32_t hpos = s_base[0] + ((off >> 10) & 1023);
        int32_t ppos = s_base[1] + (off >> 20);
        int32_t slot = S + (off & 1023);
#pragma unroll
        for (int32_t j = 0; j < kFilterPer; j++) {
            if (!keep[j]) continue;
            wk[j].slot = slot;
            info[slot] = kNoManifold;
            if (wk[j].test == kHull) {
                list[hpos++] = packWork(wk[j]);
            } else if (wk[j].test == kHullPlane) {
                *(list_back - ppos++) = packWork(wk[j]);
            }
            // sphere / plane-plane survivors get a slot but no manifold:
            // the reference asserts on them (narrowphase.cpp:1197-1313)
            slot++;
        }
        S += total & 1023;
    }
    if (threadIdx.x == 0) P.survCount[w] = S;
}

// The same filter with one wave per world (the solver tail's
// filterWorldOnWave on substep 0's list set, its boxes read from the
// integration's BodyBox slab): no block barriers, and four worlds per
// 256-lane block in flight independently -- narrowFilterKernel's world waits
// for its whole block at the scan.  Same survivors, slots and list entries
// (their order within a bin differs, which no reader depends on).
__global__ void __launch_bounds__(kNarrowBlock) narrowFilterWaveKernel(PhysArgs P)
{
    MW_TRACE_BLOCK(0);
    const int32_t w = blockIdx.x * (kNarrowBlock / 64) + (int32_t)(threadIdx.x >> 6);
    if (w >= P.numWorlds) return;
    filterWorldOnWave(P, w, P.bodyBoxes + (size_t)w * P.maxBodiesPerWorld, (int32_t)(threadIdx.x & 63),
                      P.satWork, P.satWorkCount);
}

// The plane kernel's LDS copy of the hull tables it walks (hulls, vertices,
// face planes, half-edges, face polygons): each pair's vertex / face scans
// and incident-face walk are chains of dependent reads over a few hundred
// bytes shared by every pair.

__host__ __device__ inline size_t planeGeoBytesFor(const ObjDev &O)
{
    return a16(sizeof(HullDev) * O.numObjects) + a16(sizeof(float4) * O.numVertsTotal) +
           a16(sizeof(geometry::Plane) * O.numPlanesTotal) +
           a16(sizeof(geometry::HalfEdge) * O.numHedgesTotal) +
           a16(sizeof(uint32_t) * O.numPolygonsTotal);
}

size_t planeSharedBytes(const PhysArgs &P)
{
    const size_t b = planeGeoBytesFor(P.objs);
    return b <= 16 * 1024 ? b : 0;
}

__device__ __forceinline__ void *stageTable(char *&dst, const void *src, size_t bytes)
{
    uint32_t *d = (uint32_t *)dst;
    const uint32_t *s = (const uint32_t *)src;
    for (size_t i = threadIdx.x; i < bytes / 4; i += blockDim.x) d[i] = s[i];
    void *out = dst;
    dst += a16(bytes);
    return out;
}

// A plane work entry's indices are inside the tables its loads index.
__device__ __forceinline__ bool planeWorkOk(const PhysArgs &P, const SatWork &wk)
{
    return (uint32_t)wk.world < (uint32_t)P.numWorlds &&
           (uint32_t)wk.slot < (uint32_t)P.candCapacity &&
           (uint32_t)wk.aObj < (uint32_t)P.objs.numObjects &&
           (uint32_t)wk.aArch < (uint32_t)P.numBodyArchs &&
           (uint32_t)wk.bArch < (uint32_t)P.numBodyArchs &&
           (uint32_t)wk.a.row < (uint32_t)P.body[wk.aArch].capacity &&
           (uint32_t)wk.b.row < (uint32_t)P.body[wk.bArch].capacity;
}

// Hull-plane contacts, one lane per pair of the bins' back parts.
// kGeo: the hull tables are staged into LDS (P.planeGeoBytes > 0) -- a
// template parameter so that their reads compile to LDS loads; behind a
// run-time test the table pointers are generic and every vertex, face and
// half-edge read is a flat load.
template <bool kGeo>
__device__ __forceinline__ void narrowPlaneBlock(const PhysArgs &P)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    ObjDev O = P.objs;
    if constexpr (kGeo) {
        static_assert(sizeof(HullDev) % 4 == 0 && sizeof(geometry::HalfEdge) % 4 == 0, "dword copies");
        char *dst = smem;
        O.hulls = (HullDev *)stageTable(dst, P.objs.hulls, sizeof(HullDev) * O.numObjects);
        {   // vertices padded to 16 B (objVertex<true>)
            float4 *d = (float4 *)dst;
            const float *src = (const float *)P.objs.vertices;
            for (int32_t i = threadIdx.x; i < O.numVertsTotal; i += blockDim.x)
                d[i] = float4 { src[3 * i], src[3 * i + 1], src[3 * i + 2], 0.f };
            O.vertices = (Vector3 *)dst;
            dst += a16(sizeof(float4) * O.numVertsTotal);
        }
        O.planes = (geometry::Plane *)stageTable(dst, P.objs.planes,
                                                 sizeof(geometry::Plane) * O.numPlanesTotal);
        O.hedges = (geometry::HalfEdge *)stageTable(dst, P.objs.hedges,
                                                    sizeof(geometry::HalfEdge) * O.numHedgesTotal);
        O.polygons = (uint32_t *)stageTable(dst, P.objs.polygons, sizeof(uint32_t) * O.numPolygonsTotal);
    }
    __shared__ int32_t s_pre[kNarrowBins + 1];
    loadBinPrefix(P, 1, s_pre);
    const int32_t total = s_pre[kNarrowBins];
    // Two-deep software pipeline over the lane's pairs: while pair i is
    // solved, the body columns of pair i + stride and the work entry of pair
    // i + 2 stride are in flight (the contact stores would otherwise order
    // every next load behind them).
    const int32_t stride = gridDim.x * kContactBlock;
    int32_t i = blockIdx.x * kContactBlock + threadIdx.x;
    SatWork wk1;
    PackedSatWork wk2;
    bool ok1 = false;
    PlaneIn in1;
    if (i < total) {
        wk1 = unpackWork(P, P.satWork[binEntry(P, s_pre, i, 1)]);
        ok1 = planeWorkOk(P, wk1);
        if (ok1) in1 = loadPlaneIn(P, wk1);
    }
    if (i + stride < total) wk2 = P.satWork[binEntry(P, s_pre, i + stride, 1)];
    for (; i < total; i += stride) {
        const SatWork wk = wk1;
        const bool ok = ok1;
        const PlaneIn in = in1;
        if (i + stride < total) {
            wk1 = unpackWork(P, wk2);
            ok1 = planeWorkOk(P, wk1);
            if (ok1) in1 = loadPlaneIn(P, wk1);
            if (i + 2 * stride < total) wk2 = P.satWork[binEntry(P, s_pre, i + 2 * stride, 1)];
        }
        if (!ok) {
            atomicOr(P.errorFlags, kErrIndexGuard | (kGuardWork << 8));
            continue;
        }
        if (planeContact<kGeo>(P, O, wk.world, wk, in))
            recordManifold(P, wk.world, wk.slot, slotOf(P, wk.bArch, wk.b), slotOf(P, wk.aArch, wk.a));
    }
}

__global__ void __launch_bounds__(kContactBlock) narrowPlaneKernel(PhysArgs P)
{
    MW_TRACE_BLOCK(0);
    narrowPlaneBlock<true>(P);
}

__global__ void __launch_bounds__(kContactBlock) narrowPlaneNoGeoKernel(PhysArgs P)
{
    MW_TRACE_BLOCK(0);
    narrowPlaneBlock<false>(P);
}

#if defined(MW_SAT_PROFILE)
// Profiling build only (make BUILD=build_prof EXTRA=-DMW_SAT_PROFILE): per
// hull-hull pair, where the SAT ended ([0] pairs, [1] separated by a face of
// a, [2] of b, [3] by an edge pair, [4] face contact, [5] edge contact) and
// the group leader's clock in each phase ([8] staging, [9] faces of a,
// [10] faces of b, [11] edge pairs, [12] contact job).
static __device__ unsigned long long g_satStage[16];

#define MW_SAT_COUNT(i) do { if (lane == 0) atomicAdd(&g_satStage[i], 1ull); } while (0)
#define MW_SAT_TICK(i) do { if (lane == 0) { const long long t__ = wall_clock64(); \
    atomicAdd(&g_satStage[i], (unsigned long long)(t__ - prof_t)); prof_t = t__; } } while (0)
#else
#define MW_SAT_COUNT(i) do {} while (0)
#define MW_SAT_TICK(i) do {} while (0)
#endif
#if defined(MW_SAT_CUTS)
#define MW_SAT_CUT(i) do { if (g_satExp == (i)) return kSatFaceSeparated; } while (0)
#else
#define MW_SAT_CUT(i) do {} while (0)
#endif

#ifndef MW_SAT_SPLIT_STAGE
#define MW_SAT_SPLIT_STAGE 0
#endif

// How a pair's SAT ended.
enum : int32_t { kSatFaceSeparated = 0, kSatEdgeSeparated = 1, kSatContact = 2 };

// The SAT of one pair after its hulls are known (doSAT, narrowphase.cpp:
// 678-758): staging, face queries, edge query, contact job.  `stride` is the
// Minkowski tables' row stride (0: the per-pair edge query).
template <bool kBits>
__device__ __forceinline__ int32_t satPair(const ObjDev &O, const HullRef &ha, const HullRef &hb,
                                        const BodyPose &pa, const BodyPose &pb, const GroupLDS &g,
                                        int32_t stride, int32_t lane, ContactJob &job)
{
#if defined(MW_SAT_PROFILE)
    long long prof_t = wall_clock64();
#endif
#if MW_SAT_SPLIT_STAGE
    stagePair(O, ha, hb, pa, pb, g, lane);
#else
    stageHull(O, ha.hd, pa, g.vA, g.pA, g.qA, lane, kGroup);
    stageHull(O, hb.hd, pb, g.vB, g.pB, g.qB, lane, kGroup);
#endif
    groupSync();
    MW_SAT_TICK(8);
    MW_SAT_CUT(1);

    const FaceQuery fa = groupFaceQuery(ha, hb, lane);
    MW_SAT_TICK(9);
    if (fa.separation > 0.0f) { MW_SAT_COUNT(1); return kSatFaceSeparated; }
    const FaceQuery fb = groupFaceQuery(hb, ha, lane);
    MW_SAT_TICK(10);
    if (fb.separation > 0.0f) { MW_SAT_COUNT(2); return kSatFaceSeparated; }
    MW_SAT_CUT(2);
    EdgeQuery eq;
    bool bits_done = false;
    if (kBits && stride > 0 && bitsEligible(ha, hb)) eq = groupEdgeQueryBits(ha, hb, g.sA, g.tB, lane, bits_done);
    if (bits_done) {
    } else if (stride > 0) {
        buildMinkTables(ha, hb, g.sA, g.tB, stride, lane);
        groupSync();
        MW_SAT_CUT(3);
        eq = groupEdgeQueryTables(ha, hb, g.sA, g.tB, stride, lane);
    } else {
        eq = groupEdgeQuery(ha, hb, lane);
    }
    MW_SAT_TICK(11);
    if (eq.separation > 0.0f) { MW_SAT_COUNT(3); return kSatEdgeSeparated; }
    MW_SAT_CUT(4);

    if (fa.separation > eq.separation || fb.separation > eq.separation) {
        const bool a_is_ref = fa.separation >= fb.separation;
        job.kind = kJobFace;
        job.refIsA = a_is_ref ? 1 : 0;
        const int32_t ref_face = a_is_ref ? fa.faceIdx : fb.faceIdx;
        job.plane = facePlane(a_is_ref ? ha.planes : hb.planes, ref_face);
        job.feature0 = ref_face;
        job.feature1 = findIncidentFace(a_is_ref ? hb.planes : ha.planes,
                                        a_is_ref ? hb.hd.numFaces : ha.hd.numFaces, job.plane.normal);
        MW_SAT_COUNT(4);
    } else {
        job.kind = kJobEdge;
        job.refIsA = 1;
        const int32_t nB = hb.hd.numEdges;
        job.feature0 = nB > 0 ? eq.pair / nB : 0;
        job.feature1 = eq.pair - job.feature0 * nB;
        if (eq.separation > -FLT_MAX) {
            Vector3 n;
            const float sep = edgePairSeparation(ha, hb, job.feature0, job.feature1, &n);
            job.plane = geometry::Plane { n, sep };
        } else {
            job.plane = geometry::Plane { { 0, 0, 0 }, -FLT_MAX };
        }
        MW_SAT_COUNT(5);
    }
    MW_SAT_TICK(12);
    return kSatContact;
}


#ifndef MW_SAT_BOX
#define MW_SAT_BOX 1
#endif

__device__ __forceinline__ bool isBoxHull(const HullDev &h)
{
    return h.numVerts == 8 && h.numFaces == 6 && h.numEdges == 12;
}

// Hull-hull SAT (doSAT, narrowphase.cpp:678-758) for one pair on one
// group.  Returns how it ended (on every lane of the group); for
// kSatContact the leader's `job` holds createFaceContact's /
// createEdgeContact's inputs.  A pair of box hulls
// (8 vertices, 6 faces, 12 edges: every pair of the benchmarks) runs a copy
// of satPair with those counts as constants -- its loops unrolled, the same
// operations in the same order.
__device__ __forceinline__ int32_t hullHullSAT(const ObjDev &O, int32_t a_obj, int32_t b_obj,
                                            const BodyPose &pa, const BodyPose &pb,
                                            const GroupLDS &g, int32_t lane, ContactJob &job)
{
    MW_SAT_COUNT(0);
    HullRef ha, hb;
    ha.hd = O.hulls[a_obj];
    hb.hd = O.hulls[b_obj];
    ha.verts = g.vA; ha.planes = g.pA; ha.quads = g.qA;
    hb.verts = g.vB; hb.planes = g.pB; hb.quads = g.qB;
    ha.center = pa.x;
    hb.center = pb.x;
#if MW_SAT_BOX
    if (O.minkStride >= 6 && isBoxHull(ha.hd) && isBoxHull(hb.hd)) {
        ha.hd.numVerts = hb.hd.numVerts = 8;
        ha.hd.numFaces = hb.hd.numFaces = 6;
        ha.hd.numEdges = hb.hd.numEdges = 12;
        return satPair<MW_SAT_BITS != 0>(O, ha, hb, pa, pb, g, 6, lane, job);
    }
#endif
    return satPair<false>(O, ha, hb, pa, pb, g, O.minkStride, lane, job);
}

#if defined(MW_SAT_PROFILE)
extern "C" int mw_debug_sat_stages(unsigned long long *out)
{
    unsigned long long z[16] = {};
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_satStage), sizeof(z)) != hipSuccess) return -1;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_satStage), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
#if defined(MW_SAT_CUTS)
extern "C" int mw_debug_set_sat_exp(int32_t cut)
{
    return hipMemcpyToSymbol(HIP_SYMBOL(g_satExp), &cut, sizeof(cut)) == hipSuccess ? 0 : -1;
}
#endif

// Solver world order.  Block durations follow the worlds' contact counts
// (p50 / p99 ~ 1 : 3), so with the grid in world-index order the heavy
// blocks that happen to be dispatched last set the launch's tail.  Block 0
// of the SAT kernel (before its pairs; the persistent grid's other blocks
// take them meanwhile) counting-sorts the worlds by descending survivor
// count (this substep's filter wrote survCount) into solverOrder; the solver
// grid takes its worlds in that order (longest first), and a block's two
// worlds have similar work.  Which block or partner solves a world does not
// change its bits: a world's items only touch its own bodies.
constexpr int32_t kOrderBuckets = 1024;
static_assert(kOrderBuckets % kNarrowBlock == 0, "buckets per thread");

__device__ __forceinline__ int32_t orderBucket(const PhysArgs &P, int32_t w)
{
    const int32_t n = P.survCount[w];
    return kOrderBuckets - 1 - min(max(n, 0), kOrderBuckets - 1);
}

// s_off: kOrderBuckets ints of LDS, s_scan: blockDim.x / 64 ints.
__device__ __forceinline__ void sortWorldsForSolver(const PhysArgs &P, int32_t *s_off, int32_t *s_scan)
{
    const int32_t t = threadIdx.x, nt = blockDim.x, W = P.numWorlds;
    const int32_t per = kOrderBuckets / nt;
    for (int32_t b = t; b < kOrderBuckets; b += nt) s_off[b] = 0;
    __syncthreads();
    for (int32_t w = t; w < W; w += nt) atomicAdd(&s_off[orderBucket(P, w)], 1);
    __syncthreads();
    int32_t sum = 0;
    for (int32_t j = 0; j < per; j++) sum += s_off[t * per + j];
    int32_t total;
    int32_t run = blockExclusiveScan(sum, s_scan, &total);
    for (int32_t j = 0; j < per; j++) {
        const int32_t c = s_off[t * per + j];
        s_off[t * per + j] = run;
        run += c;
    }
    __syncthreads();
    for (int32_t w = t; w < W; w += nt)
        P.solverOrder[atomicAdd(&s_off[orderBucket(P, w)], 1)] = w;
    __syncthreads();
}

// The SAT kernel's LDS copy of the hull tables it stages from (hulls,
// vertices, face planes, edge quads): every pair reads a few hundred bytes
// of them, shared by all pairs.  It follows the group staging area (or, in
// the global-image variant, the world sort's scratch).
__host__ __device__ inline size_t satGeoBytesFor(const ObjDev &O)
{
    return a16(sizeof(HullDev) * O.numObjects) + a16(sizeof(Vector3) * O.numVertsTotal) +
           a16(sizeof(geometry::Plane) * O.numPlanesTotal) + a16(sizeof(EdgeQuad) * O.numEdgesTotal);
}

size_t satGeoSharedBytes(const PhysArgs &P)
{
    const size_t b = satGeoBytesFor(P.objs);
    return b <= 16 * 1024 ? b : 0;
}

__host__ __device__ inline size_t satStageBytes(const ObjDev &O)
{
    return kOrderSortBytes > kGroupsPerBlock * groupLDSBytes(O) ? kOrderSortBytes
                                                                 : kGroupsPerBlock * groupLDSBytes(O);
}

// A work entry's indices are inside the tables the SAT indexes.
__device__ __forceinline__ bool satWorkOk(const PhysArgs &P, const SatArch *arch,
                                          const PackedSatWork &p)
{
    const uint32_t a_arch = (p.slotTest >> 19) & 63u, b_arch = (p.slotTest >> 25) & 63u;
    return (uint32_t)p.world < (uint32_t)P.numWorlds &&
           (p.slotTest & 0xffffu) < (uint32_t)P.candCapacity &&
           (p.objs & 0xffffu) < (uint32_t)P.objs.numObjects &&
           (p.objs >> 16) < (uint32_t)P.objs.numObjects &&
           a_arch < (uint32_t)P.numBodyArchs && b_arch < (uint32_t)P.numBodyArchs &&
           (p.rows & 0xffffu) < (uint32_t)arch[a_arch].capacity &&
           (p.rows >> 16) < (uint32_t)arch[b_arch].capacity;
}

// unpackWork with the archetypes from the LDS table.
__device__ __forceinline__ SatWork unpackSat(const PhysArgs &P, const SatArch *arch,
                                             const PackedSatWork &p)
{
    SatWork w;
    w.world = p.world;
    w.slot = (int32_t)(p.slotTest & 0xffffu);
    w.test = (p.slotTest >> 16) & 7u;
    w.aArch = (int32_t)((p.slotTest >> 19) & 63u);
    w.bArch = (int32_t)((p.slotTest >> 25) & 63u);
    w.pad = 0;
    const int32_t na = P.numBodyArchs;
    w.a = Loc { (uint32_t)(w.aArch < na ? arch[w.aArch].archetype : -1), (int32_t)(p.rows & 0xffffu) };
    w.b = Loc { (uint32_t)(w.bArch < na ? arch[w.bArch].archetype : -1), (int32_t)(p.rows >> 16) };
    w.aObj = (int32_t)(p.objs & 0xffffu);
    w.bObj = (int32_t)(p.objs >> 16);
    return w;
}

// Stage 4, persistent: each group takes hull-hull pairs off the flat list
// and leaves its verdict in the job at the same index (kind kJobNone when
// separated: only the kind is written).  The grid is what is resident at
// once; every group reaches the end of the list and exits.
#ifndef MW_SAT_MIN_BLOCKS
#define MW_SAT_MIN_BLOCKS 4
#endif
#ifndef MW_SAT_PIPE
#define MW_SAT_PIPE 0        // software pipeline depth: 0 (loads at use) or 2
#endif
#ifndef MW_SAT_SORT_ALONE
#define MW_SAT_SORT_ALONE 1  // block 0 sorts the worlds and takes no pairs
#endif
// kGlobal: the groups' hull staging exceeds a workgroup's LDS and lives in
// the block's slab of P.satImage (narrowSATGlobalKernel); the world sort
// still uses kOrderSortBytes of LDS.
// kGeo: the hull tables are staged into LDS (P.satGeoBytes > 0) -- a
// template parameter so that their reads are LDS loads, not generic ones.
template <bool kGlobal, bool kGeo>
__device__ __forceinline__ void narrowSATBlock(const PhysArgs &P)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int32_t group = threadIdx.x / kGroup;
    const int32_t lane = threadIdx.x % kGroup;
    char *stage = kGlobal ? P.satImage + (size_t)blockIdx.x * kGroupsPerBlock * groupLDSBytes(P.objs) : smem;
    const GroupLDS g = groupLDS(stage, group, P.objs);
    // the set the solver of this substep will fill (read last by the
    // previous substep's kernels); null when integrateKernel reset it
    if (blockIdx.x == 0 && P.nextSatWorkCount)
        resetNarrowLists(P.nextSatWorkCount, threadIdx.x, blockDim.x);
    if (blockIdx.x == 0) {
        // the group staging area is free until the first pair (and at
        // least kOrderSortBytes: narrowphaseSharedBytes)
        static_assert(kOrderBuckets * sizeof(int32_t) == kOrderSortBytes, "sort scratch");
        __shared__ int32_t s_sort_scan[kNarrowBlock / 64];
        sortWorldsForSolver(P, (int32_t *)smem, s_sort_scan);
    }
    // With the sort on block 0 the pairs go to the other blocks, so the sort
    // is not added to one block's share of them (whole block: no barrier is
    // left behind).
    const bool sortAlone = MW_SAT_SORT_ALONE && gridDim.x > 1;
    if (sortAlone && blockIdx.x == 0) return;
    const int32_t pairBlock = sortAlone ? blockIdx.x - 1 : blockIdx.x;
    const int32_t pairBlocks = sortAlone ? gridDim.x - 1 : gridDim.x;
    ObjDev O = P.objs;
    if constexpr (kGeo) {
        char *dst = smem + (kGlobal ? kOrderSortBytes : satStageBytes(P.objs));
        O.hulls = (HullDev *)stageTable(dst, P.objs.hulls, sizeof(HullDev) * O.numObjects);
        O.vertices = (Vector3 *)stageTable(dst, P.objs.vertices, sizeof(Vector3) * O.numVertsTotal);
        O.planes = (geometry::Plane *)stageTable(dst, P.objs.planes,
                                                 sizeof(geometry::Plane) * O.numPlanesTotal);
        O.edgeQuads = (EdgeQuad *)stageTable(dst, P.objs.edgeQuads, sizeof(EdgeQuad) * O.numEdgesTotal);
    }
    __shared__ SatArch s_arch[kMaxBodyArchetypes];
    if (threadIdx.x < kMaxBodyArchetypes) {
        const BodyArch &B = P.body[threadIdx.x];
        s_arch[threadIdx.x] = SatArch { (const Vector3 *)B.cols[Cols::Position],
                                        (const Quat *)B.cols[Cols::Rotation],
                                        (const Diag3x3 *)B.cols[Cols::Scale], B.capacity,
                                        B.archetype };
    }
    __shared__ int32_t s_pre[kNarrowBins + 1];
    loadBinPrefix(P, 0, s_pre);            // (its barrier publishes the tables)
    // the SAT verdicts (hhJobs) are indexed by list position: never past them
    const int32_t total = min(s_pre[kNarrowBins], P.numWorlds * P.candCapacity);
    const int32_t stride = pairBlocks * kGroupsPerBlock;
    // Two-deep software pipeline over the group's pairs (as the plane
    // kernel's): while pair idx is tested, the body poses of pair
    // idx + stride and the work entry of pair idx + 2 stride are in flight.
    int32_t idx = pairBlock * kGroupsPerBlock + group;
    PackedSatWork w1 {}, w2 {};
    BodyPose pa1 {}, pb1 {};
    bool ok1 = false;
    if (MW_SAT_PIPE != 0 && idx < total) {
        w1 = P.satWork[binEntry(P, s_pre, idx, 0)];
        ok1 = satWorkOk(P, s_arch, w1);
        if (ok1) {
            pa1 = loadPose(s_arch[(w1.slotTest >> 19) & 63u], w1.world, (int32_t)(w1.rows & 0xffffu));
            pb1 = loadPose(s_arch[(w1.slotTest >> 25) & 63u], w1.world, (int32_t)(w1.rows >> 16));
        }
    }
    if (MW_SAT_PIPE != 0 && idx + stride < total) w2 = P.satWork[binEntry(P, s_pre, idx + stride, 0)];
    for (; idx < total; idx += stride) {
#if MW_SAT_PIPE == 0
        w1 = P.satWork[binEntry(P, s_pre, idx, 0)];
        ok1 = satWorkOk(P, s_arch, w1);
        if (ok1) {
            pa1 = loadPose(s_arch[(w1.slotTest >> 19) & 63u], w1.world, (int32_t)(w1.rows & 0xffffu));
            pb1 = loadPose(s_arch[(w1.slotTest >> 25) & 63u], w1.world, (int32_t)(w1.rows >> 16));
        }
#endif
        const PackedSatWork pw = w1;
        const bool ok = ok1;
        const BodyPose pa = pa1, pb = pb1;
        if (MW_SAT_PIPE != 0 && idx + stride < total) {
            w1 = w2;
            ok1 = satWorkOk(P, s_arch, w1);
            if (ok1) {
                pa1 = loadPose(s_arch[(w1.slotTest >> 19) & 63u], w1.world, (int32_t)(w1.rows & 0xffffu));
                pb1 = loadPose(s_arch[(w1.slotTest >> 25) & 63u], w1.world, (int32_t)(w1.rows >> 16));
            }
            if (idx + 2 * stride < total) w2 = P.satWork[binEntry(P, s_pre, idx + 2 * stride, 0)];
        }
        ContactJob job;
        job.kind = kJobNone;
        if (ok) {
            hullHullSAT(O, (int32_t)(pw.objs & 0xffffu), (int32_t)(pw.objs >> 16), pa, pb, g, lane, job);
        } else if (lane == 0) {
            atomicOr(P.errorFlags, kErrIndexGuard | (kGuardWork << 8));
        }
        if (lane == 0 && P.hhJobs) {
            // the kind byte always, the 80-byte job only for a contact (a
            // separated pair's record is never read)
            P.hhKinds[idx] = (int8_t)job.kind;
            if (job.kind != kJobNone) {
                job.pair = unpackSat(P, s_arch, pw);
                P.hhJobs[idx] = job;
            }
        }
        groupSync();
    }
}

__global__ void __launch_bounds__(kNarrowBlock, MW_SAT_MIN_BLOCKS) narrowSATKernel(PhysArgs P)
{
    MW_TRACE_BLOCK(0);
    narrowSATBlock<false, true>(P);
}

__global__ void __launch_bounds__(kNarrowBlock, MW_SAT_MIN_BLOCKS) narrowSATNoGeoKernel(PhysArgs P)
{
    MW_TRACE_BLOCK(0);
    narrowSATBlock<false, false>(P);
}

__global__ void __launch_bounds__(kNarrowBlock) narrowSATGlobalKernel(PhysArgs P)
{
    MW_TRACE_BLOCK(0);
    narrowSATBlock<true, false>(P);
}

size_t narrowphaseImageBytes(const PhysArgs &P)
{
    return kGroupsPerBlock * groupLDSBytes(P.objs);
}

size_t narrowphaseGlobalSharedBytes(const PhysArgs &)
{
    return kOrderSortBytes;
}

#ifndef MW_CONTACT_CHUNK
#define MW_CONTACT_CHUNK 4
#endif
constexpr int32_t kContactChunk = MW_CONTACT_CHUNK;     // SAT entries per lane per gather

// One lane's clip buffers (two polygons and the depths), padded to an odd
// number of dwords: lanes touch the same element of their own buffers
// together, and with an even dword stride those accesses share LDS banks
// (a 56-dword stride -- 8-point polygons -- put every fourth lane of a
// 32-lane half on one bank).
#ifndef MW_CONTACT_BANK_PAD
#define MW_CONTACT_BANK_PAD 1
#endif
__host__ __device__ inline size_t contactLaneBytes(int32_t clip_cap)
{
    const size_t b = 2 * a16(sizeof(Vector3) * clip_cap) + a16(4 * clip_cap);
#if MW_CONTACT_BANK_PAD
    return (b / 4) % 2 == 0 ? b + 4 : b;
#else
    return b;
#endif
}

__host__ __device__ inline size_t contactLDSBytes(int32_t clip_cap)
{
    return a16((size_t)kContactBlock * contactLaneBytes(clip_cap));
}

size_t contactSharedBytes(const PhysArgs &P)
{
    return contactLDSBytes(P.clipCap);
}

size_t contactImageBytes(const PhysArgs &P)
{
    return contactLDSBytes(P.clipCap);
}


// createFaceContact / createFacePlaneContact / createEdgeContact
// (narrowphase.cpp:866-1121) for one job per lane.
// kGlobal: the lanes' clip buffers exceed a workgroup's LDS and live in the
// block's slab of P.clipImage (narrowContactGlobalKernel).
// (Staging the hull tables into LDS beside the clip buffers measured no
// faster: collisions 0.1093 against 0.1085 ms per narrowphase launch, and
// slower together with the even shares below.)
template <bool kGlobal>
__device__ __forceinline__ void narrowContactBlock(const PhysArgs &P)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const ObjDev &O = P.objs;
    const int32_t cap = P.clipCap;
    char *base = kGlobal ? P.clipImage + (size_t)blockIdx.x * contactLDSBytes(cap) : smem;
    char *mine = base + (size_t)threadIdx.x * contactLaneBytes(cap);
    Vector3 *clip0 = (Vector3 *)mine;
    Vector3 *clip1 = (Vector3 *)(mine + a16(sizeof(Vector3) * cap));
    float *depths = (float *)(mine + 2 * a16(sizeof(Vector3) * cap));
    const Quat ident { 1, 0, 0, 0 };

    __shared__ int32_t s_pre[kNarrowBins + 1];
    loadBinPrefix(P, 0, s_pre);
    const int32_t total = min(s_pre[kNarrowBins], P.numWorlds * P.candCapacity);
    // Chunks of kContactChunk entries per lane: the block first gathers the
    // chunk's jobs (most entries are separated pairs: kJobNone) into LDS,
    // then its lanes take the jobs densely -- otherwise a wave's lanes wait
    // on the few that drew a job.  Which lane solves a job does not matter:
    // each writes its own survivor slot.  Each block takes an equal
    // contiguous share of the entries (whole chunks dealt round-robin left
    // most blocks idle on a short list -- collisions: ≈65 k entries, 128
    // chunks for a 1,280-block grid; measured: simple_taskgraph 0.4645 ->
    // 0.4562 ms per narrowphase launch, collisions unchanged).
    __shared__ int32_t s_jobs[kContactBlock * kContactChunk];
    __shared__ int32_t s_njobs;
    const int32_t chunk = kContactBlock * kContactChunk;
    const int32_t share = (total + gridDim.x - 1) / gridDim.x;
    const int32_t lo = min(total, (int32_t)blockIdx.x * share), hi = min(total, lo + share);
    for (int32_t c0 = lo; c0 < hi; c0 += chunk) {
    if (threadIdx.x == 0) s_njobs = 0;
    __syncthreads();
#pragma unroll
    for (int32_t q = 0; q < kContactChunk; q++) {
        const int32_t i = c0 + q * kContactBlock + threadIdx.x;
        const bool has = i < hi && P.hhKinds[i] != (int8_t)kJobNone;
        const uint64_t m = __ballot(has);
        int32_t wb = 0;
        if ((threadIdx.x & 63) == 0 && m) wb = atomicAdd(&s_njobs, (int32_t)__popcll(m));
        wb = __shfl(wb, 0, 64);
        if (has) s_jobs[wb + __popcll(m & __lanemask_lt())] = i;
    }
    __syncthreads();
    const int32_t njobs = s_njobs;
    for (int32_t k = threadIdx.x; k < njobs; k += kContactBlock) {
        const ContactJob job = P.hhJobs[s_jobs[k]];
        const SatWork &wk = job.pair;
        if ((uint32_t)wk.world >= (uint32_t)P.numWorlds || (uint32_t)wk.slot >= (uint32_t)P.candCapacity ||
            (uint32_t)wk.aObj >= (uint32_t)P.objs.numObjects || (uint32_t)wk.bObj >= (uint32_t)P.objs.numObjects) {
            atomicOr(P.errorFlags, kErrIndexGuard | (kGuardWork << 8));
            continue;
        }
        const int32_t w = wk.world;
        int32_t *flags = P.errorFlags + w;
        Contact &out = P.candContacts[(size_t)w * P.candCapacity + wk.slot];
        const HullDev ha = O.hulls[wk.aObj];

        if (job.kind == kJobFace) {
            const bool a_is_ref = job.refIsA != 0;
            const HullDev hb = O.hulls[wk.bObj];
            const HullDev ref = a_is_ref ? ha : hb;
            const HullDev inc = a_is_ref ? hb : ha;
            const HullXform xref = a_is_ref ? hullXform(P, w, P.body[wk.aArch], wk.a.row)
                                            : hullXform(P, w, P.body[wk.bArch], wk.b.row);
            const HullXform xinc = a_is_ref ? hullXform(P, w, P.body[wk.bArch], wk.b.row)
                                            : hullXform(P, w, P.body[wk.aArch], wk.a.row);
            const geometry::Plane ref_plane = job.plane;
            const int32_t ref_face = guardIndex(job.feature0, ref.numFaces, flags, kGuardRefFace);
            const int32_t inc_face = guardIndex(job.feature1, inc.numFaces, flags, kGuardIncFace);
            const geometry::HalfEdge *rh = O.hedges + ref.hedgeOffset;
            const geometry::HalfEdge *oh = O.hedges + inc.hedgeOffset;
            int32_t n_in = 0;
            {
                uint32_t hidx = O.polygons[inc.faceOffset + inc_face], start = hidx;
                int32_t steps = 0;
                do {
                    hidx = guardIndex(hidx, inc.numHedges, flags, kGuardIncWalk);
                    const geometry::HalfEdge he = oh[hidx];
                    hidx = he.next;
                    if (n_in < cap)
                        clip0[n_in++] = worldVertex(O, inc, xinc,
                                                    guardIndex(he.rootVertex, inc.numVerts, flags,
                                                               kGuardVertex));
                } while (hidx != start && ++steps <= inc.numHedges);
            }
            Vector3 *cin = clip0, *cdst = clip1;
            int32_t n_clip = n_in;
            {
                uint32_t hidx = guardIndex(O.polygons[ref.faceOffset + ref_face], ref.numHedges,
                                           flags, kGuardRefWalk);
                const uint32_t start = hidx;
                geometry::HalfEdge che = rh[hidx];
                Vector3 cur = worldVertex(O, ref, xref,
                                          guardIndex(che.rootVertex, ref.numVerts, flags,
                                                     kGuardVertex));
                int32_t steps = 0;
                do {
                    hidx = guardIndex(che.next, ref.numHedges, flags, kGuardRefWalk);
                    che = rh[hidx];
                    const Vector3 next = worldVertex(O, ref, xref,
                                                     guardIndex(che.rootVertex, ref.numVerts,
                                                                flags, kGuardVertex));
                    const Vector3 edge = next - cur;
                    const Vector3 pn = cross(edge, ref_plane.normal);
                    const float d = dot(pn, cur);
                    cur = next;
                    n_clip = clipPolygon(cdst, geometry::Plane { pn, d }, cin, n_clip, cap);
                    Vector3 *t = cdst; cdst = cin; cin = t;
                } while (hidx != start && ++steps <= ref.numHedges);
            }
            int32_t n_below = 0;
            for (int32_t k = 0; k < n_clip; k++) {
                const Vector3 v = cin[k];
                const float d = distFromPlane(ref_plane, v);
                if (d < 0.0f) {
                    cin[n_below] = v - d * ref_plane.normal;
                    depths[n_below] = -d;
                    n_below++;
                }
            }
            storeFaceManifold(out, ref_plane.normal, cin, depths, n_below,
                              a_is_ref ? wk.a : wk.b, a_is_ref ? wk.b : wk.a);
            if (n_below > 0) {
                const int32_t sa = slotOf(P, wk.aArch, wk.a), sb = slotOf(P, wk.bArch, wk.b);
                recordManifold(P, w, wk.slot, a_is_ref ? sa : sb, a_is_ref ? sb : sa);
            }
        } else {
            const HullDev hb = O.hulls[wk.bObj];
            const HullXform xa = hullXform(P, w, P.body[wk.aArch], wk.a.row);
            const HullXform xb = hullXform(P, w, P.body[wk.bArch], wk.b.row);
            const EdgeQuad ea = O.edgeQuads[ha.edgeOffset +
                                            guardIndex(job.feature0, ha.numEdges, flags, kGuardVertex)];
            const EdgeQuad eb = O.edgeQuads[hb.edgeOffset +
                                            guardIndex(job.feature1, hb.numEdges, flags, kGuardVertex)];
            const geometry::Segment sa { worldVertex(O, ha, xa, ea.v1), worldVertex(O, ha, xa, ea.v2) };
            const geometry::Segment sb { worldVertex(O, hb, xb, eb.v1), worldVertex(O, hb, xb, eb.v2) };
            const geometry::Segment sg = shortestSegmentBetween(sa, sb);
            out.ref = wk.a;
            out.alt = wk.b;
            out.points[0] = Vector4::fromVector3(ident.rotateVec(sg.p1) + Vector3::zero(),
                                                 -job.plane.d);
            for (int k = 1; k < 4; k++) out.points[k] = Vector4::fromVector3(Vector3::zero(), 0.f);
            out.numPoints = 1;
            out.normal = ident.rotateVec(job.plane.normal);
            for (int k = 0; k < 4; k++) out.lambdaN[k] = 0.f;
            recordManifold(P, w, wk.slot, slotOf(P, wk.aArch, wk.a), slotOf(P, wk.bArch, wk.b));
        }
    }
    __syncthreads();
    }

}

__global__ void __launch_bounds__(kContactBlock) narrowContactKernel(PhysArgs P)
{
    MW_TRACE_BLOCK(0);
    narrowContactBlock<false>(P);
}

__global__ void __launch_bounds__(kContactBlock) narrowContactGlobalKernel(PhysArgs P)
{
    MW_TRACE_BLOCK(0);
    narrowContactBlock<true>(P);
}

}
