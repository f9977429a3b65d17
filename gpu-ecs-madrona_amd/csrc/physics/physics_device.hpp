// Device-side helpers shared by the physics kernels (broadphase.hip,
// narrowphase.hip, solver.hip) and the kernel entry points the host module
// (physics.hip) launches.
#pragma once

#include <madrona/physics.hpp>

#include "physics_impl.hpp"
#include <madrona/tracing.hpp>

#include <hip/hip_runtime.h>

namespace madrona::phys {

using namespace math;
using namespace base;


template <typename T>
__device__ __forceinline__ T &bcol(const BodyArch &B, int col, int32_t w, int32_t r)
{
    return ((T *)B.cols[col])[(size_t)w * B.capacity + r];
}

__device__ __forceinline__ int bodyArchIndex(const PhysArgs &P, uint32_t archetype)
{
    for (int i = 0; i < P.numBodyArchs; i++) {
        if ((uint32_t)P.body[i].archetype == archetype) return i;
    }
    return 0;
}

// Clamp a data-derived index into [0, n): a miss raises kErrIndexGuard (with
// the site in bits 8..15) on the world instead of faulting the device.
enum GuardSite : int32_t {
    kGuardRefFace = 1, kGuardIncFace, kGuardIncWalk, kGuardRefWalk, kGuardVertex,
    kGuardPlaneFace, kGuardPlaneWalk, kGuardSolverBody, kGuardSolverSlot, kGuardEntity,
    kGuardLeaf, kGuardNode, kGuardWork, kGuardList,
};

__device__ __forceinline__ int32_t guardIndex(int32_t i, int32_t n, int32_t *flags,
                                              int32_t site)
{
    if ((uint32_t)i < (uint32_t)n) return i;
    atomicOr(flags, kErrIndexGuard | (site << 8));
    return 0;
}

__device__ __forceinline__ Loc entityLoc(const PhysArgs &P, int32_t w, Entity e)
{
    const int32_t id = guardIndex(e.id, P.idsPerWorld, P.errorFlags + w, kGuardEntity);
    const IDNode &n = P.idNodes[(size_t)w * P.idsPerWorld + id];
    if (n.gen != e.gen) return Loc::none();
    return n.val;
}

// Float min/max updates with the reference's "v < old" rule; CAS loop so
// concurrent leaves of one world compose like the reference's atomicMinF
// (broadphase.cpp:494-543).  Values only shrink (min) / grow (max), so a
// stale first read is safe.
__device__ __forceinline__ float atomicMinRef(float *addr, float v)
{
    uint32_t *p = (uint32_t *)addr;
    uint32_t old = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (true) {
        float of = __uint_as_float(old);
        if (!(v < of)) return of;
        uint32_t prev = atomicCAS(p, old, __float_as_uint(v));
        if (prev == old) return of;
        old = prev;
    }
}

__device__ __forceinline__ float atomicMaxRef(float *addr, float v)
{
    uint32_t *p = (uint32_t *)addr;
    uint32_t old = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (true) {
        float of = __uint_as_float(old);
        if (!(v > of)) return of;
        uint32_t prev = atomicCAS(p, old, __float_as_uint(v));
        if (prev == old) return of;
        old = prev;
    }
}

// Grid helper: lanes over (world, row) of body archetype blockIdx.y.
struct RowIdx {
    int32_t w, r;
    bool valid;
};

__device__ __forceinline__ RowIdx rowIndex(const PhysArgs &P, const BodyArch &B)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    RowIdx ri;
    ri.w = (int32_t)(t / B.capacity);
    ri.r = (int32_t)(t - (int64_t)ri.w * B.capacity);
    ri.valid = ri.w < P.numWorlds && ri.r < B.numRows[ri.w];
    return ri;
}

__device__ __forceinline__ int32_t blockExclusiveScan(int32_t v, int32_t *scratch, int32_t *total)
{
    // Wave-level inclusive scan with DPP-friendly shuffles, then across waves.
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    int32_t x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        int32_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    if (lane == 63) scratch[wave] = x;
    __syncthreads();
    const int nwaves = blockDim.x >> 6;
    int32_t wave_base = 0, sum = 0;
    for (int i = 0; i < nwaves; i++) {
        int32_t s = scratch[i];
        if (i < wave) wave_base += s;
        sum += s;
    }
    __syncthreads();
    *total = sum;
    return wave_base + x - v;
}

__device__ __forceinline__ Vector3 multDiag(Vector3 d, Vector3 v)
{
    return Vector3 { d.x * v.x, d.y * v.y, d.z * v.z };
}

// Kernel entry points (one launch processes every world).
__global__ void leafUpdateKernel(PhysArgs P);
__global__ void bvhRebuildKernel(PhysArgs P);
__global__ void bvhRebuildWaveKernel(PhysArgs P);
constexpr int32_t kRebuildStack = 128;            // broadphase.cpp:58 stack[128]
size_t rebuildSharedBytes(const PhysArgs &P);
__global__ void refitKernel(PhysArgs P);
__global__ void findOverlapsKernel(PhysArgs P);
__global__ void integrateKernel(PhysArgs P);
__global__ void narrowFilterKernel(PhysArgs P);
__global__ void narrowFilterWaveKernel(PhysArgs P);
__global__ void narrowSATKernel(PhysArgs P);         // hull tables in LDS (satGeoBytes > 0)
__global__ void narrowSATNoGeoKernel(PhysArgs P);    // hull tables read from HBM
__global__ void narrowPlaneKernel(PhysArgs P);        // hull tables staged into LDS
__global__ void narrowPlaneNoGeoKernel(PhysArgs P);   // hull tables read from HBM
__global__ void narrowContactKernel(PhysArgs P);
// The solver kernels, per variant (solver.hip: lanes64; solver32.hip: lanes32).
struct SolverVariant {
    const void *kernel;          // solverKernel (world images in LDS)
    const void *globalKernel;    // solverGlobalKernel (world images in PhysArgs::solverImage)
    int32_t threads, worldsPerBlock, lanesPerWorld;
    size_t (*sharedBytes)(const PhysArgs &);
    size_t (*globalSharedBytes)(const PhysArgs &);
    size_t (*imageBytes)(const PhysArgs &);
};
namespace lanes64 {
__global__ void solverKernel(PhysArgs P, int32_t integrate_next);
__global__ void solverGlobalKernel(PhysArgs P, int32_t integrate_next);
size_t solverSharedBytes(const PhysArgs &P);
size_t solverGlobalSharedBytes(const PhysArgs &P);
size_t solverImageBytes(const PhysArgs &P);
SolverVariant solverVariant();
}
namespace lanes32 {
__global__ void solverKernel(PhysArgs P, int32_t integrate_next);
__global__ void solverGlobalKernel(PhysArgs P, int32_t integrate_next);
SolverVariant solverVariant();
}
// The same kernels with their per-world / per-group / per-lane LDS image in
// a global slab (PhysArgs::*Image), for worlds and hulls whose image does not
// fit a workgroup's LDS: same code, same order of operations, same bits.
__global__ void refitGlobalKernel(PhysArgs P);
__global__ void findOverlapsGlobalKernel(PhysArgs P);
__global__ void dfsStageKernel(PhysArgs P);
__global__ void dfsCountKernel(PhysArgs P);
__global__ void dfsWriteKernel(PhysArgs P);
__global__ void findOverlapsSmallKernel(PhysArgs P);
__global__ void narrowSATGlobalKernel(PhysArgs P);
__global__ void narrowContactGlobalKernel(PhysArgs P);

// substepRigidBodies (physics.cpp:79-164) for one body row, from its
// current pose and velocity (the integrate kernel reads them from the
// columns; the solver's fused tail passes the values it is about to write
// back -- the same inputs, so the same bits), plus the world AABB the
// narrowphase recheck uses (narrowphase.cpp:1590-1594), indexed by body slot.
// Split in two so a caller walking several rows per lane can issue every
// row's loads before the first row's arithmetic (integrateLoad, then
// integrateApply): the column and object-table reads are one memory round
// trip per batch instead of per row.
struct IntegrateIn {
    int32_t obj;
    ResponseType rt;
    Vector3 extForce, extTorque;
    Diag3x3 scale;
};

struct IntegrateObj {
    float invMass;
    Vector3 invInertia;
    AABB aabb;
    uint32_t type;
};

__device__ __forceinline__ IntegrateIn integrateLoad(const BodyArch &B, int32_t w, int32_t r)
{
    IntegrateIn in;
    in.obj = bcol<ObjectID>(B, Cols::ObjectID, w, r).idx;
    in.rt = bcol<ResponseType>(B, Cols::ResponseType, w, r);
    in.extForce = bcol<Vector3>(B, Cols::ExternalForce, w, r);
    in.extTorque = bcol<Vector3>(B, Cols::ExternalTorque, w, r);
    in.scale = bcol<Diag3x3>(B, Cols::Scale, w, r);
    return in;
}

__device__ __forceinline__ IntegrateObj integrateObj(const PhysArgs &P, int32_t obj)
{
    const RigidBodyMetadata md = P.objs.metadata[obj];
    return IntegrateObj { md.invMass, md.invInertiaTensor, P.objs.aabbs[obj], P.objs.types[obj] };
}

__device__ __forceinline__ BodyBox integrateApply(const PhysArgs &P, const BodyArch &B, int32_t w,
                                               int32_t r, const IntegrateIn &in,
                                               const IntegrateObj &od, Vector3 x, Quat q,
                                               Vector3 v_in, Vector3 omega_in)
{
    Vector3 &pos = bcol<Vector3>(B, Cols::Position, w, r);
    Quat &rot = bcol<Quat>(B, Cols::Rotation, w, r);
    auto &prev = bcol<solver::SubstepPrevState>(B, Cols::SubstepPrevState, w, r);
    auto &ps_pos = bcol<solver::PreSolvePositional>(B, Cols::PreSolvePositional, w, r);
    auto &ps_vel = bcol<solver::PreSolveVelocity>(B, Cols::PreSolveVelocity, w, r);

    if (in.rt == ResponseType::Static) {
        prev.prevPosition = x;
        prev.prevRotation = q;
        ps_pos.x = x;
        ps_pos.q = q;
        ps_vel.v = Vector3::zero();
        ps_vel.omega = Vector3::zero();
        pos = x;
        rot = q;
    } else {
        Vector3 v = v_in;
        Vector3 omega = omega_in;
        prev.prevPosition = x;
        prev.prevRotation = q;
        const SolverData &solver = P.solver[w];
        const float inv_m = od.invMass;
        const Vector3 inv_I = od.invInertia;
        const float h = solver.h;
        const Vector3 ext_force = in.extForce;
        const Vector3 ext_torque = in.extTorque;
        if (in.rt == ResponseType::Dynamic) v += h * solver.g;
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
    const BodyBox bb { od.aabb.applyTRS(x, q, in.scale), in.obj, od.type };
    P.bodyBoxes[(size_t)w * P.maxBodiesPerWorld + B.slotBase + r] = bb;
    return bb;
}

__device__ __forceinline__ BodyBox integrateBody(const PhysArgs &P, const BodyArch &B, int32_t w,
                                              int32_t r, Vector3 x, Quat q, Vector3 v_in,
                                              Vector3 omega_in)
{
    const IntegrateIn in = integrateLoad(B, w, r);
    return integrateApply(P, B, w, r, in, integrateObj(P, in.obj), x, q, v_in, omega_in);
}

// The narrowphase work lists are split into kNarrowBins bins (world w in
// bin w % kNarrowBins), each with its own counters on their own cache lines:
// a device-wide list with one counter serialised every filter block's
// reservation at that address (measured 86 -> 480 us per filter launch).
// kNarrowBins / kBinStride: physics_impl.hpp

__device__ __forceinline__ int32_t *binCounter(const PhysArgs &P, int32_t bin, int32_t which)
{
    return P.satWorkCount + bin * kBinStride + which;
}

// One reservation in both lists of a bin: the two counts are the halves of
// one 64-bit counter (hull-hull low, hull-plane high), so a single atomic
// returns both bases at one point of the bin's reservation order.  The
// hull-hull list grows up from the bin's front and the hull-plane list down
// from its back; every reservation sees all earlier ones of both lists, so
// refusing any whose two ends would cross (b_hh + n_hh + b_hp + n_hp >
// binCap) keeps the two lists from ever overwriting each other.  A refused
// reservation stays counted (undoing it would race with the reservations
// made meanwhile), so the bin's counts no longer describe written entries:
// the refusal poisons the bin (counts[2]) and its readers treat it as empty
// and flag every world of it (loadBinPrefix) -- never stale entries.
__device__ __forceinline__ bool reserveBin(int32_t *counts, int32_t n_hh, int32_t n_hp,
                                           int32_t bin_cap, int32_t &b_hh, int32_t &b_hp)
{
    const unsigned long long add = ((unsigned long long)(uint32_t)n_hp << 32) | (uint32_t)n_hh;
    const unsigned long long old = add ? atomicAdd((unsigned long long *)counts, add) : 0ull;
    b_hh = (int32_t)(uint32_t)old;
    b_hp = (int32_t)(uint32_t)(old >> 32);
    const bool fits = (int64_t)b_hh + n_hh + b_hp + n_hp <= (int64_t)bin_cap;
    if (!fits) atomicOr(counts + 2, 1);
    return fits;
}

// Reset the counters of a list set (`counts`: satWorkCount or
// nextSatWorkCount) before a filter appends to it; its readers, an earlier
// substep's SAT / plane / contact kernels, have finished.
__device__ __forceinline__ void resetNarrowLists(int32_t *counts, int32_t tid, int32_t nthreads)
{
    for (int32_t i = tid; i < 3 * kNarrowBins; i += nthreads)
        counts[(i / 3) * kBinStride + i % 3] = 0;
}

// Exclusive prefix of the bins' counts of list `which` into s_pre[0..64]
// (s_pre[kNarrowBins] = total); every thread of the block calls it.
__device__ __forceinline__ void loadBinPrefix(const PhysArgs &P, int32_t which, int32_t *s_pre)
{
    static_assert(kNarrowBins == 64, "one wave scans the bins");
    if (threadIdx.x < 64) {
        // a poisoned bin (a filter's reservation overran it, reserveBin) is
        // read as empty and its worlds are flagged; the clamp keeps any other
        // count that is ever wrong inside the bin
        const bool poisoned = *(volatile int32_t *)binCounter(P, threadIdx.x, 2) != 0;
        const int32_t v = poisoned ? 0 : min(*(volatile int32_t *)binCounter(P, threadIdx.x, which), P.binCap);
        if (poisoned && blockIdx.x == 0) {
            for (int32_t w = threadIdx.x; w < P.numWorlds; w += kNarrowBins)
                atomicOr(P.errorFlags + w, kErrIndexGuard | (kGuardList << 8));
        }
        int32_t x = v;
#pragma unroll
        for (int32_t o = 1; o < 64; o <<= 1) {
            const int32_t y = __shfl_up(x, o, 64);
            if ((int32_t)threadIdx.x >= o) x += y;
        }
        s_pre[threadIdx.x] = x - v;
        if (threadIdx.x == 63) s_pre[64] = x;
    }
    __syncthreads();
}

// satWork index of entry i (0 <= i < s_pre[64]) of list `which`.
__device__ __forceinline__ size_t binEntry(const PhysArgs &P, const int32_t *s_pre, int32_t i,
                                           int32_t which)
{
    int32_t lo = 0;
#pragma unroll
    for (int32_t step = 32; step > 0; step >>= 1)
        if (s_pre[lo + step] <= i) lo += step;
    const size_t k = (size_t)(i - s_pre[lo]);
    const size_t base = (size_t)lo * P.binCap;
    return which == 0 ? base + k : base + P.binCap - 1 - k;
}

// Narrowphase pair resolution and the per-wave world filter (shared by
// narrowphase.hip and the solver kernel's fused tail).
//
// The AABB recheck (narrowphase.cpp:1589-1603) of a candidate from its packed body slots (candSlots,
// written by findOverlaps beside the candidate): both members' records
// (AABB, object, type: BodyBox, written by this substep's integration), one
// 32-byte load each.  A candidate whose row failed findOverlaps' guard is
// dropped and flags the world.
template <typename BoxPtr>
__device__ __forceinline__ bool candOverlaps(const PhysArgs &P, int32_t w, uint64_t cs, BoxPtr boxes,
                                             BodyBox &A, BodyBox &B)
{
    A = boxes[(uint32_t)cs & 0xffffu];
    B = boxes[(uint32_t)(cs >> 32) & 0xffffu];
    if ((cs & (1ull << 24 | 1ull << 56)) != 0) {
        atomicOr(P.errorFlags + w, kErrIndexGuard | (kGuardWork << 8));
        return false;
    }
    return A.box.overlaps(B.box);
}

// SatWork <-> the lists' 16-byte entries (PackedSatWork).
__device__ __forceinline__ PackedSatWork packWork(const SatWork &w)
{
    return PackedSatWork { w.world,
                           ((uint32_t)w.slot & 0xffffu) | (w.test & 7u) << 16 |
                               ((uint32_t)w.aArch & 63u) << 19 | ((uint32_t)w.bArch & 63u) << 25,
                           ((uint32_t)w.a.row & 0xffffu) | ((uint32_t)w.b.row & 0xffffu) << 16,
                           ((uint32_t)w.aObj & 0xffffu) | ((uint32_t)w.bObj & 0xffffu) << 16 };
}

__device__ __forceinline__ SatWork unpackWork(const PhysArgs &P, const PackedSatWork &p)
{
    SatWork w;
    w.world = p.world;
    w.slot = (int32_t)(p.slotTest & 0xffffu);
    w.test = (p.slotTest >> 16) & 7u;
    w.aArch = (int32_t)((p.slotTest >> 19) & 63u);
    w.bArch = (int32_t)((p.slotTest >> 25) & 63u);
    w.pad = 0;
    const int32_t na = P.numBodyArchs;
    w.a = Loc { (uint32_t)(w.aArch < na ? P.body[w.aArch].archetype : -1), (int32_t)(p.rows & 0xffffu) };
    w.b = Loc { (uint32_t)(w.bArch < na ? P.body[w.bArch].archetype : -1), (int32_t)(p.rows >> 16) };
    w.aObj = (int32_t)(p.objs & 0xffffu);
    w.bObj = (int32_t)(p.objs >> 16);
    return w;
}

// A surviving candidate's work entry, in runNarrowphase's type order
// (narrowphase.cpp:1574-1580).
__device__ __forceinline__ SatWork candWork(const CandidateCollision &cand, uint64_t cs,
                                            const BodyBox &A, const BodyBox &B, int32_t w)
{
    const int32_t ia = (int32_t)((cs >> 16) & 0xffu), ib = (int32_t)((cs >> 48) & 0xffu);
    SatWork out;
    out.world = w;
    out.test = A.type | B.type;
    out.pad = 0;
    if (A.type > B.type) {
        out.a = cand.b; out.b = cand.a;
        out.aArch = ib; out.bArch = ia;
        out.aObj = B.obj; out.bObj = A.obj;
    } else {
        out.a = cand.a; out.b = cand.b;
        out.aArch = ia; out.bArch = ib;
        out.aObj = A.obj; out.bObj = B.obj;
    }
    return out;
}

// Solver blocks: kSolverWorlds worlds per block, kSolverBlock lanes per
// world.  MW_SOLVER_LANES = 32 puts two worlds on one wave (each on a half):
// a dependency level of a collisions world holds ~33 contacts, so a wave of
// its own leaves half its lanes idle in every level pass.
#ifndef MW_SOLVER_LANES
#define MW_SOLVER_LANES 64
#endif
constexpr int32_t kSolverBlock = MW_SOLVER_LANES;        // lanes per world
#ifndef MW_SOLVER_WORLDS
#define MW_SOLVER_WORLDS (64 / MW_SOLVER_LANES)
#endif
constexpr int32_t kSolverWorlds = MW_SOLVER_WORLDS;       // worlds per solver block
constexpr int32_t kSolverThreads = kSolverBlock * kSolverWorlds;
static_assert(kSolverBlock == 64 || kSolverBlock == 32, "a world's lanes: a wave or half of one");

// This world's lanes (kSolverBlock of them, aligned in the wave): a ballot
// over them (bit i = the world's lane i) and a value from one of them.
__device__ __forceinline__ uint64_t worldBallot(bool p)
{
    const uint64_t m = __ballot(p);
    if constexpr (kSolverBlock == 64) return m;
    return (m >> (threadIdx.x & 32)) & 0xffffffffull;
}
template <typename T>
__device__ __forceinline__ T worldBroadcast(T x, int32_t src)
{
    return __shfl(x, (int32_t)(threadIdx.x & (64 - kSolverBlock)) + src, 64);
}

// The filter for one world on one wave (the solver kernel's tail, after it
// integrated the world's next substep into its LDS box image): the same
// survivors, slots and list entries as narrowFilterKernel, into the
// nextSatWork set.  One pass over the candidates in batches of kFilterBatch
// 64-candidate chunks whose global loads are all issued before any is used
// (the wave otherwise waits one memory round trip per chunk): each batch's
// survivors are counted by ballot, the batch reserves its entries in both
// lists with one atomic (as narrowFilterKernel's blocks do per chunk; the
// lists' order does not matter, every entry writes only its own slot), then
// loads its survivors' Locs in one round and writes them.  (Until round 6 a
// counting pass over all candidates came first, so the world reserved once
// but read every slot and box twice: collisions 4.671 -> 4.685 M
// env-steps/s without it.)
constexpr int32_t kFilterBatch = 8;

// `sets`, `set_counts`: the list set it appends to (the solver tail: the
// next substep's, nextSatWork; narrowFilterWaveKernel: substep 0's).
__device__ __forceinline__ void filterWorldOnWave(const PhysArgs &P, int32_t w, const BodyBox *boxes,
                                                  int32_t lane, PackedSatWork *sets, int32_t *set_counts)
{
    const int32_t cap = P.candCapacity;
    const int32_t num = min(P.numCands[w], cap);
    const CandidateCollision *cands = P.cands + (size_t)w * cap;
    const uint64_t *slots = P.candSlots + (size_t)w * cap;
    uint32_t *info = P.survInfo + (size_t)w * cap;
    const int32_t bin = w % kNarrowBins;
    PackedSatWork *list = sets + (size_t)bin * P.binCap;
    PackedSatWork *list_back = list + P.binCap - 1;        // plane entries grow down
    int32_t *counts = set_counts + bin * kBinStride;
    constexpr uint32_t kHull = (uint32_t)CollisionPrimitive::Type::Hull;
    constexpr uint32_t kHullPlane = kHull | (uint32_t)CollisionPrimitive::Type::Plane;
    constexpr int32_t kBatch = kSolverBlock * kFilterBatch;
    const uint64_t lt = (1ull << lane) - 1;
    // The two lists stay inside their bin whatever the counter says (the
    // reservations fit by construction -- binCap = worlds per bin x
    // candCapacity -- while the counters were reset before this filter):
    // an overrun is refused and flagged, never written.
    auto reserve = [&](int32_t n_hh, int32_t n_hp, int32_t &b_hh, int32_t &b_hp) {
        int32_t fits = 1;
        if (lane == 0) fits = reserveBin(counts, n_hh, n_hp, P.binCap, b_hh, b_hp);
        b_hh = worldBroadcast(b_hh, 0);
        b_hp = worldBroadcast(b_hp, 0);
        fits = worldBroadcast(fits, 0);
        if (!fits && lane == 0) {
            atomicOr(P.errorFlags + w, kErrIndexGuard | (kGuardList << 8));
            P.survCount[w] = 0;
        }
        return fits != 0;
    };
    int32_t S = 0;
    for (int32_t b0 = 0; b0 < num; b0 += kBatch) {
        uint64_t s[kFilterBatch];
#pragma unroll
        for (int32_t j = 0; j < kFilterBatch; j++) {
            const int32_t i = b0 + kSolverBlock * j + lane;
            s[j] = i < num ? slots[i] : 0;
        }
        // survivors of the batch and their lists' counts first, then their
        // candidates' Locs in one round of loads
        uint32_t keep_bits = 0, hh_bits = 0, hp_bits = 0;
        int32_t n_hh = 0, n_hp = 0;
#pragma unroll
        for (int32_t j = 0; j < kFilterBatch; j++) {
            const int32_t i = b0 + kSolverBlock * j + lane;
            if (b0 + kSolverBlock * j >= num) continue;
            BodyBox A, B;
            const bool keep = i < num && candOverlaps(P, w, s[j], boxes, A, B);
            if (keep) keep_bits |= 1u << j;
            const uint32_t t = keep ? (A.type | B.type) : 0u;
            const bool hh = keep && t == kHull, hp = keep && t == kHullPlane;
            hh_bits |= (uint32_t)hh << j;
            hp_bits |= (uint32_t)hp << j;
            n_hh += __popcll(worldBallot(hh));
            n_hp += __popcll(worldBallot(hp));
        }
        int32_t b_hh = 0, b_hp = 0;
        if (!reserve(n_hh, n_hp, b_hh, b_hp)) return;
        CandidateCollision c[kFilterBatch];
#pragma unroll
        for (int32_t j = 0; j < kFilterBatch; j++) {
            if (keep_bits & (1u << j)) c[j] = cands[b0 + kSolverBlock * j + lane];
        }
#pragma unroll
        for (int32_t j = 0; j < kFilterBatch; j++) {
            if (b0 + kSolverBlock * j >= num) continue;
            const bool keep = (keep_bits >> j) & 1u;
            const BodyBox A = boxes[(uint32_t)s[j] & 0xffffu];
            const BodyBox B = boxes[(uint32_t)(s[j] >> 32) & 0xffffu];
            const bool hh = (hh_bits >> j) & 1u, hp = (hp_bits >> j) & 1u;
            const uint64_t mk = worldBallot(keep), mh = worldBallot(hh), mp = worldBallot(hp);
            if (keep) {
                SatWork wk = candWork(c[j], s[j], A, B, w);
                wk.slot = S + __popcll(mk & lt);
                info[wk.slot] = kNoManifold;
                if (hh) list[b_hh + __popcll(mh & lt)] = packWork(wk);
                if (hp) *(list_back - (b_hp + __popcll(mp & lt))) = packWork(wk);
            }
            S += __popcll(mk);
            b_hh += __popcll(mh);
            b_hp += __popcll(mp);
        }
    }
    if (lane == 0) P.survCount[w] = S;
}

size_t findOverlapsSharedBytes(const PhysArgs &P);
size_t findOverlapsGlobalSharedBytes(const PhysArgs &P);
size_t refitSharedBytes(const PhysArgs &P);
size_t narrowphaseSharedBytes(const PhysArgs &P);
size_t satGeoSharedBytes(const PhysArgs &P);
size_t contactSharedBytes(const PhysArgs &P);
size_t planeSharedBytes(const PhysArgs &P);
// Global-image variants: dynamic LDS they still use, and image bytes per
// world (findOverlaps, solver), per SAT block and per contact block.
size_t findOverlapsImageBytes(const PhysArgs &P);
size_t narrowphaseGlobalSharedBytes(const PhysArgs &P);
size_t narrowphaseImageBytes(const PhysArgs &P);
size_t contactImageBytes(const PhysArgs &P);

#ifndef MW_OVERLAP_BLOCK
#define MW_OVERLAP_BLOCK 192
#endif
constexpr int32_t kOverlapBlock = MW_OVERLAP_BLOCK;
constexpr int32_t kOverlapSmallLeaves = 256;   // findOverlapsSmallKernel: the bitmask path only
constexpr int32_t kDfsBlock = 256;             // dfs*Kernel: body rows per block
constexpr size_t kOrderedLeafBytes = 48;       // broadphase.hip OrderedLeaf
constexpr int32_t kOverlapBufRanks = 12;       // broadphase.hip kOverlapBuf
constexpr int32_t kNarrowBlock = 256;
#ifndef MW_CONTACT_BLOCK
#define MW_CONTACT_BLOCK 128
#endif
constexpr int32_t kContactBlock = MW_CONTACT_BLOCK;   // plane / contact kernels
#ifndef MW_REFIT_BLOCK
#define MW_REFIT_BLOCK 128
#endif
constexpr int32_t kRefitBlock = MW_REFIT_BLOCK;

}
