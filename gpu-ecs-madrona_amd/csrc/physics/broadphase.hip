// Broadphase kernels (reference src/physics/broadphase.cpp, physics.inl).
#include "physics_device.hpp"

#include <cfloat>

namespace madrona::phys {

// ===========================================================================
// Broadphase kernels (src/physics/broadphase.cpp)
// ===========================================================================
__device__ __forceinline__ AABB expandAABBWithMotion(AABB aabb, const Vector3 &v,
                                                     float vel_exp, float acc_exp)
{                                                          // broadphase.cpp:435-459
#pragma unroll
    for (int32_t i = 0; i < 3; i++) {
        float pos_delta = vel_exp * v[i];
        float min_delta = pos_delta - acc_exp;
        float max_delta = pos_delta + acc_exp;
        if (min_delta < 0.f) aabb.pMin[i] += min_delta;
        if (max_delta > 0.f) aabb.pMax[i] += max_delta;
    }
    return aabb;
}

// updateLeafPositionsEntry (broadphase.cpp:858-873, 461-480)
__global__ void __launch_bounds__(256) leafUpdateKernel(PhysArgs P)
{
    MW_TRACE_BLOCK(0);
    const BodyArch &B = P.body[blockIdx.y];
    RowIdx ri = rowIndex(P, B);
    if (!ri.valid) return;
    const int32_t w = ri.w, r = ri.r;
    const int32_t leaf = guardIndex(bcol<broadphase::LeafID>(B, Cols::LeafID, w, r).id,
                                    P.maxLeaves, P.errorFlags + w, kGuardLeaf);
    const Vector3 pos = bcol<Vector3>(B, Cols::Position, w, r);
    const Quat rot = bcol<Quat>(B, Cols::Rotation, w, r);
    const Diag3x3 scale = bcol<Diag3x3>(B, Cols::Scale, w, r);
    const int32_t obj = bcol<ObjectID>(B, Cols::ObjectID, w, r).idx;
    const Vector3 lin = bcol<Velocity>(B, Cols::Velocity, w, r).linear;
    const broadphase::BVH &bvh = P.bvh[w];
    AABB world_aabb = P.objs.aabbs[obj].applyTRS(pos, rot, scale);
    const size_t li = (size_t)w * P.maxLeaves + leaf;
    P.leafAABBs[li] = expandAABBWithMotion(world_aabb, lin, bvh.leafVelocityExpansion,
                                           bvh.leafAccelExpansion);
    P.sortedLeaves[li] = leaf;
}

// BVH::rebuild (broadphase.cpp:42-280): top-down midpoint 4-way split, one
// lane per world, only for worlds with force_rebuild_ set (first step).
__device__ __forceinline__ Vector3 leafCenter(const AABB *aabbs, const int32_t *sorted, int32_t i)
{
    AABB a = aabbs[sorted[i]];
    return (a.pMin + a.pMax) / 2.f;
}

__device__ int32_t midpointSplit(const AABB *aabbs, int32_t *sorted, int32_t base, int32_t n)
{
    Vector3 cmin { FLT_MAX, FLT_MAX, FLT_MAX };
    Vector3 cmax { -FLT_MAX, -FLT_MAX, -FLT_MAX };
    for (int32_t i = 0; i < n; i++) {
        Vector3 c = leafCenter(aabbs, sorted, base + i);
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
        while (start < end && leafCenter(aabbs, sorted, base + start)[axis] < split_val) ++start;
        while (start < end && leafCenter(aabbs, sorted, base + end - 1)[axis] >= split_val) --end;
        if (start < end) {
            int32_t tmp = sorted[base + start];
            sorted[base + start] = sorted[base + end - 1];
            sorted[base + end - 1] = tmp;
            ++start;
            --end;
        }
    }
    if (start > 0 && start < n) return start;
    return n / 2;
}

__global__ void __launch_bounds__(64) bvhRebuildKernel(PhysArgs P)
{
    MW_TRACE_BLOCK(0);
    const int32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= P.numWorlds) return;
    broadphase::BVH &bvh = P.bvh[w];
    if (!bvh.forceRebuild) return;                       // BVH::updateTree
    bvh.forceRebuild = 0;

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
                    const AABB a = aabbs[leaf_id];
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
            if (stack_size + 4 > 128) { atomicOr(P.errorFlags + w, kErrBVHStack); return; }
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

    // Leaf emission order of BVH::findOverlaps (physics.inl:61-100) with no
    // pruning: pop a node, emit its leaf children in slot order, push its
    // inner children.  Pruning a subtree only deletes its leaves from this
    // sequence, so every query's candidates come out in this order.
    int32_t *order = P.leafOrder + (size_t)w * P.maxLeaves;
    int32_t ostack[128];
    int32_t os = 0, emitted = 0;
    if (bvh.numLeaves > 0) ostack[os++] = 0;
    while (os > 0) {
        const BVHNode &n = nodes[ostack[--os]];
        for (int i = 0; i < 4; i++) {
            const int32_t child = n.children[i];
            if (child == -1) continue;
            if (child & 0x80000000) {
                if (emitted < P.maxLeaves) order[emitted++] = child & ~0x80000000;
            } else if (os < 128) {
                ostack[os++] = child;
            } else {
                atomicOr(P.errorFlags + w, kErrBVHStack);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// BVH::rebuild (broadphase.cpp:42-280) with one wave per world.  The serial
// kernel above walks the explicit stack on one lane; here the same stack walk
// runs wave-uniformly (entries in LDS, fields read through readfirstlane, so
// the control flow is scalar) and every midpoint split runs across the wave:
//  * centroid bounds: lane-strided fminRef / fmaxRef, then a shuffle
//    reduction.  fminRef ignores NaN on either side, so the result is the
//    serial scan's up to the sign of a zero, which neither the axis choice
//    (strict >) nor `c < split_val` can observe;
//  * the in-place two-pointer partition: it swaps the i-th element >= split
//    left of k (= #elements < split) with the i-th element < split right of
//    k counted from the end, so the misplaced positions are ranked by
//    ballots and swapped pairwise -- the serial loop's exact permutation.
// Node ids are handed out in the stack walk's order, so nodes, slots and
// parents are byte-identical.  No node is read back: a node's combined
// bounds are the in-order merge of its slots, accumulated in its stack entry
// as its children complete (every child of an inner node is a node, even an
// empty one, so slot c is always the c-th child to complete).  The leaf
// emission order of findOverlaps (inner children pushed in slot order, leaf
// children emitted in slot order) lists the leaf nodes' sorted segments in
// reverse, each segment forwards: a leaf node over [off, off + n) emits at
// numLeaves - off - n.
// ---------------------------------------------------------------------------
struct RebuildEntry {
    int32_t nodeID, parentID, offset, numObjs;
    int32_t parentIdx;          // stack index of the parent's entry
    int32_t nextSlot;           // inner node: children completed so far
    AABB acc;                   // inner node: merge of its completed slots
};

__device__ __forceinline__ void rebuildWaveSync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float uniformF(float v)
{
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

__device__ __forceinline__ int32_t uniformI(int32_t v)
{
    return __builtin_amdgcn_readfirstlane(v);
}

// Wave-wide fminRef / fmaxRef: DPP within each row of 16 (swap pairs, swap
// pairs of pairs, half-row mirror, row mirror), then the four row results
// combined in row order from readlanes, so every lane ends with one value.
template <int Ctrl>
__device__ __forceinline__ float dppF(float v)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), Ctrl, 0xf, 0xf, false));
}

__device__ __forceinline__ float readlaneF(float v, int lane)
{
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

__device__ __forceinline__ float waveMinRef(float v)
{
    v = fminRef(v, dppF<0xB1>(v));      // quad_perm [1,0,3,2]
    v = fminRef(v, dppF<0x4E>(v));      // quad_perm [2,3,0,1]
    v = fminRef(v, dppF<0x141>(v));     // row_half_mirror
    v = fminRef(v, dppF<0x140>(v));     // row_mirror
    return fminRef(fminRef(fminRef(readlaneF(v, 0), readlaneF(v, 16)), readlaneF(v, 32)),
                   readlaneF(v, 48));
}

__device__ __forceinline__ float waveMaxRef(float v)
{
    v = fmaxRef(v, dppF<0xB1>(v));
    v = fmaxRef(v, dppF<0x4E>(v));
    v = fmaxRef(v, dppF<0x141>(v));
    v = fmaxRef(v, dppF<0x140>(v));
    return fmaxRef(fmaxRef(fmaxRef(readlaneF(v, 0), readlaneF(v, 16)), readlaneF(v, 32)),
                   readlaneF(v, 48));
}

size_t rebuildSharedBytes(const PhysArgs &P)
{
    const size_t L = (size_t)P.maxLeaves;
    return L * (3 * sizeof(float) + sizeof(AABB) + 2 * sizeof(int32_t)) +
           kRebuildStack * sizeof(RebuildEntry) + 16;
}

// Up to kSplitRegChunks x 64 elements the segment's leaf ids and centroids
// stay in registers across the bounds / count / rank passes; longer segments
// (worlds over 192 leaves) re-read them from LDS per pass.
constexpr int32_t kSplitRegChunks = 3;

__device__ __forceinline__ int32_t pickAxis(Vector3 d)
{
    if (d.x > d.y && d.x > d.z) return 0;
    if (d.y > d.x && d.y > d.z) return 1;
    return 2;
}

__device__ __forceinline__ float comp(Vector3 v, int32_t axis)
{
    return axis == 0 ? v.x : (axis == 1 ? v.y : v.z);
}

__device__ __forceinline__ int32_t waveMidpointSplit(const float *cx, const float *cy, const float *cz,
                                     int32_t *sorted, int32_t *misL, int32_t *misR,
                                     int32_t base, int32_t n, int32_t lane)
{
    const uint64_t lt_mask = (1ull << lane) - 1ull;
    Vector3 cmin { FLT_MAX, FLT_MAX, FLT_MAX };
    Vector3 cmax { -FLT_MAX, -FLT_MAX, -FLT_MAX };
    int32_t k = 0, nl = 0, nr = 0;
    if (n <= 64 * kSplitRegChunks) {
        Vector3 c[kSplitRegChunks];
#pragma unroll
        for (int32_t j = 0; j < kSplitRegChunks; j++) {
            const int32_t i = j * 64 + lane;
            c[j] = Vector3 { FLT_MAX, FLT_MAX, FLT_MAX };
            if (i < n) {
                const int32_t l = sorted[base + i];
                c[j] = Vector3 { cx[l], cy[l], cz[l] };
                cmin = Vector3::min(cmin, c[j]);
                cmax = Vector3::max(cmax, c[j]);
            }
        }
        cmin = Vector3 { waveMinRef(cmin.x), waveMinRef(cmin.y), waveMinRef(cmin.z) };
        cmax = Vector3 { waveMaxRef(cmax.x), waveMaxRef(cmax.y), waveMaxRef(cmax.z) };
        const int32_t axis = pickAxis(cmax - cmin);
        const float split_val = 0.5f * (comp(cmin, axis) + comp(cmax, axis));
        bool lt[kSplitRegChunks];
#pragma unroll
        for (int32_t j = 0; j < kSplitRegChunks; j++) {
            lt[j] = j * 64 + lane < n && comp(c[j], axis) < split_val;
            k += __popcll(__ballot(lt[j]));
        }
#pragma unroll
        for (int32_t j = 0; j < kSplitRegChunks; j++) {
            const int32_t i = j * 64 + lane;
            const bool valid = i < n;
            const bool ml = valid && i < k && !lt[j];
            const bool mr = valid && i >= k && lt[j];
            const uint64_t bl = __ballot(ml), br = __ballot(mr);
            if (ml) misL[nl + __popcll(bl & lt_mask)] = i;
            if (mr) misR[nr + __popcll(br & lt_mask)] = i;
            nl += __popcll(bl);
            nr += __popcll(br);
        }
    } else {
        for (int32_t i = lane; i < n; i += 64) {
            const int32_t l = sorted[base + i];
            const Vector3 c { cx[l], cy[l], cz[l] };
            cmin = Vector3::min(cmin, c);
            cmax = Vector3::max(cmax, c);
        }
        cmin = Vector3 { waveMinRef(cmin.x), waveMinRef(cmin.y), waveMinRef(cmin.z) };
        cmax = Vector3 { waveMaxRef(cmax.x), waveMaxRef(cmax.y), waveMaxRef(cmax.z) };
        const int32_t axis = pickAxis(cmax - cmin);
        const float split_val = 0.5f * (comp(cmin, axis) + comp(cmax, axis));
        const float *ca = axis == 0 ? cx : (axis == 1 ? cy : cz);
        for (int32_t j = 0; j < n; j += 64) {
            const int32_t i = j + lane;
            const bool lt = i < n && ca[sorted[base + i]] < split_val;
            k += __popcll(__ballot(lt));
        }
        for (int32_t j = 0; j < n; j += 64) {
            const int32_t i = j + lane;
            const bool valid = i < n;
            const bool lt = valid && ca[sorted[base + i]] < split_val;
            const bool ml = valid && i < k && !lt;
            const bool mr = valid && i >= k && lt;
            const uint64_t bl = __ballot(ml), br = __ballot(mr);
            if (ml) misL[nl + __popcll(bl & lt_mask)] = i;
            if (mr) misR[nr + __popcll(br & lt_mask)] = i;
            nl += __popcll(bl);
            nr += __popcll(br);
        }
    }
    if (nl == 0) return (k > 0 && k < n) ? k : n / 2;      // already partitioned
    rebuildWaveSync();
    for (int32_t t = lane; t < nl; t += 64) {     // nl == nr
        const int32_t p = base + misL[t], q = base + misR[nl - 1 - t];
        const int32_t a = sorted[p], b = sorted[q];
        sorted[p] = b;
        sorted[q] = a;
    }
    rebuildWaveSync();
    return (k > 0 && k < n) ? k : n / 2;
}

__global__ void __launch_bounds__(64) bvhRebuildWaveKernel(PhysArgs P)
{
    MW_TRACE_BLOCK(0);
    const int32_t w = blockIdx.x;
    const int32_t lane = threadIdx.x;
    broadphase::BVH &bvh = P.bvh[w];
    if (!uniformI(bvh.forceRebuild)) return;              // BVH::updateTree
    const int32_t L = uniformI(bvh.numLeaves);
    if (lane == 0) {
        bvh.forceRebuild = 0;
        bvh.numNodes = numInternalNodes(L);
    }

    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int32_t ML = P.maxLeaves;
    AABB *s_aabb = (AABB *)smem;
    RebuildEntry *stack = (RebuildEntry *)(s_aabb + ML);
    float *cx = (float *)(stack + kRebuildStack);
    float *cy = cx + ML, *cz = cy + ML;
    int32_t *sorted = (int32_t *)(cz + ML);
    int32_t *scratch = sorted + ML;              // misplaced positions, ML/2 + 1 each side
    int32_t *misL = scratch, *misR = scratch + ML / 2 + 1;

    BVHNode *nodes = P.nodes + (size_t)w * P.maxNodes;
    const AABB *aabbs = P.leafAABBs + (size_t)w * ML;
    const int32_t *g_sorted = P.sortedLeaves + (size_t)w * ML;
    uint32_t *parents = P.leafParents + (size_t)w * ML;
    int32_t *order = P.leafOrder + (size_t)w * ML;

    for (int32_t i = lane; i < L; i += 64) {
        const AABB a = aabbs[i];
        s_aabb[i] = a;
        const Vector3 c = (a.pMin + a.pMax) / 2.f;
        cx[i] = c.x; cy[i] = c.y; cz[i] = c.z;
        sorted[i] = g_sorted[i];
    }
    if (lane == 0) stack[0] = { -1, -1, 0, L, -1, 0, AABB::invalid() };
    rebuildWaveSync();

    int32_t sp = 1, cur = 0;
    while (sp > 0) {
        const int32_t top = sp - 1;
        const int32_t e_node = uniformI(stack[top].nodeID);
        const int32_t e_parent = uniformI(stack[top].parentID);
        const int32_t e_off = uniformI(stack[top].offset);
        const int32_t e_n = uniformI(stack[top].numObjs);
        const int32_t e_pidx = uniformI(stack[top].parentIdx);
        int32_t node_id;
        AABB combined = AABB::invalid();
        if (e_n <= 4) {
            node_id = cur++;
            BVHNode &node = nodes[node_id];
            if (lane == 0) node.parentID = e_parent;
            if (lane < 4) {
                if (lane < e_n) {
                    const int32_t leaf_id = sorted[e_off + lane];
                    const AABB a = s_aabb[leaf_id];
                    parents[leaf_id] = ((uint32_t)node_id << 2) | (uint32_t)lane;
                    node.children[lane] = (int32_t)(0x80000000u | (uint32_t)leaf_id);
                    node.minX[lane] = a.pMin.x; node.minY[lane] = a.pMin.y; node.minZ[lane] = a.pMin.z;
                    node.maxX[lane] = a.pMax.x; node.maxY[lane] = a.pMax.y; node.maxZ[lane] = a.pMax.z;
                    order[L - e_off - e_n + lane] = leaf_id;
                } else {
                    node.children[lane] = -1;
                    node.minX[lane] = FLT_MAX; node.minY[lane] = FLT_MAX; node.minZ[lane] = FLT_MAX;
                    node.maxX[lane] = -FLT_MAX; node.maxY[lane] = -FLT_MAX; node.maxZ[lane] = -FLT_MAX;
                }
            }
            for (int32_t i = 0; i < e_n; i++) combined = AABB::merge(combined, s_aabb[sorted[e_off + i]]);
        } else if (e_node == -1) {
            node_id = cur++;
            if (lane == 0) nodes[node_id].parentID = e_parent;
            // second = split(all), first = split(lower half), third =
            // split(upper half): one inlined split body run three times
            int32_t split[3];
#pragma unroll 1
            for (int32_t q = 0; q < 3; q++) {
                const int32_t sb = q == 2 ? e_off + split[0] : e_off;
                const int32_t sn = q == 0 ? e_n : (q == 1 ? split[0] : e_n - split[0]);
                split[q] = waveMidpointSplit(cx, cy, cz, sorted, misL, misR, sb, sn, lane);
            }
            const int32_t second = split[0], first = split[1], third = split[2];
            const int32_t nh1 = second;
            const int32_t nh2 = e_n - second;
            if (sp + 4 > kRebuildStack) {
                if (lane == 0) atomicOr(P.errorFlags + w, kErrBVHStack);
                return;
            }
            if (lane == 0) {
                stack[top].nodeID = node_id;
                stack[sp + 0] = { -1, node_id, e_off + nh1 + third, nh2 - third, top, 0, AABB::invalid() };
                stack[sp + 1] = { -1, node_id, e_off + nh1, third, top, 0, AABB::invalid() };
                stack[sp + 2] = { -1, node_id, e_off + first, nh1 - first, top, 0, AABB::invalid() };
                stack[sp + 3] = { -1, node_id, e_off, first, top, 0, AABB::invalid() };
            }
            sp += 4;
            rebuildWaveSync();
            continue;
        } else {
            node_id = e_node;
            combined = stack[top].acc;
        }
        sp -= 1;
        if (e_parent == -1) continue;
        const int32_t c = uniformI(stack[e_pidx].nextSlot);
        BVHNode &parent = nodes[e_parent];
        if (lane == 0) {
            parent.children[c] = node_id;
            parent.minX[c] = combined.pMin.x; parent.minY[c] = combined.pMin.y;
            parent.minZ[c] = combined.pMin.z; parent.maxX[c] = combined.pMax.x;
            parent.maxY[c] = combined.pMax.y; parent.maxZ[c] = combined.pMax.z;
            stack[e_pidx].acc = AABB::merge(stack[e_pidx].acc, combined);
            stack[e_pidx].nextSlot = c + 1;
        }
        rebuildWaveSync();
    }
    if (lane == 0) bvh.usedNodes = cur;
}

// refitEntry -> BVH::refitLeaf (broadphase.cpp:545-642, 891-895), one block
// per world with the world's used BVH nodes staged in LDS: every leaf's slot
// read-modify-write and its expansion walk to the root run on LDS (atomic
// float min / max where walks meet), then the used node prefix goes back to
// HBM in one coalesced pass.  The result is order-independent: a slot ends
// as the union of its previous bounds and every descendant leaf that
// expanded it (ancestors contain their children's slots -- rebuild merges,
// refit only grows and propagates growth), which is what the reference's
// serial row-order walk produces.
__device__ __forceinline__ float ldsAtomicMinRef(float *addr, float v)
{
    uint32_t *p = (uint32_t *)addr;
    uint32_t old = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (true) {
        float of = __uint_as_float(old);
        if (!(v < of)) return of;
        uint32_t prev = old;
        if (__hip_atomic_compare_exchange_strong(p, &prev, __float_as_uint(v), __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
            return of;
        old = prev;
    }
}

__device__ __forceinline__ float ldsAtomicMaxRef(float *addr, float v)
{
    uint32_t *p = (uint32_t *)addr;
    uint32_t old = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (true) {
        float of = __uint_as_float(old);
        if (!(v > of)) return of;
        uint32_t prev = old;
        if (__hip_atomic_compare_exchange_strong(p, &prev, __float_as_uint(v), __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
            return of;
        old = prev;
    }
}

size_t refitSharedBytes(const PhysArgs &P)
{
    return sizeof(BVHNode) * (size_t)P.refitLDSNodes;
}

// kGlobal: the world's nodes exceed a workgroup's LDS; the same walk runs on
// the node slab in place (refitGlobalKernel).
template <bool kGlobal>
__device__ __forceinline__ void refitWorld(const PhysArgs &P)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int32_t w = blockIdx.x;
    const int32_t used = min(P.bvh[w].usedNodes, P.maxNodes);
    if (used <= 0) return;
    BVHNode *gnodes = P.nodes + (size_t)w * P.maxNodes;
    BVHNode *lnodes = kGlobal ? gnodes : (BVHNode *)smem;
    if (!kGlobal) {
        const uint32_t *src = (const uint32_t *)gnodes;
        uint32_t *dst = (uint32_t *)lnodes;
        const int32_t words = used * (int32_t)(sizeof(BVHNode) / 4);
        for (int32_t i = threadIdx.x; i < words; i += kRefitBlock) dst[i] = src[i];
    }
    __syncthreads();

    int32_t *flags = P.errorFlags + w;
    for (int32_t ba = 0; ba < P.numBodyArchs; ba++) {
        const BodyArch &B = P.body[ba];
        const int32_t rows = B.numRows[w];
        for (int32_t r = threadIdx.x; r < rows; r += kRefitBlock) {
            const int32_t leaf = guardIndex(bcol<broadphase::LeafID>(B, Cols::LeafID, w, r).id,
                                            P.maxLeaves, flags, kGuardLeaf);
            const size_t li = (size_t)w * P.maxLeaves + leaf;
            const AABB a = P.leafAABBs[li];
            const uint32_t lp = P.leafParents[li];
            int32_t node_idx = guardIndex((int32_t)(lp >> 2), used, flags, kGuardNode);
            const int sub = (int)(lp & 3);
            {   // leaf slot: owned by this leaf alone -> plain read-modify-write
                BVHNode &n = lnodes[node_idx];
                float xm = n.minX[sub], ym = n.minY[sub], zm = n.minZ[sub];
                float xM = n.maxX[sub], yM = n.maxY[sub], zM = n.maxZ[sub];
                if (a.pMin.x < xm) n.minX[sub] = a.pMin.x;
                if (a.pMin.y < ym) n.minY[sub] = a.pMin.y;
                if (a.pMin.z < zm) n.minZ[sub] = a.pMin.z;
                if (a.pMax.x > xM) n.maxX[sub] = a.pMax.x;
                if (a.pMax.y > yM) n.maxY[sub] = a.pMax.y;
                if (a.pMax.z > zM) n.maxZ[sub] = a.pMax.z;
                bool expanded = a.pMin.x < xm || a.pMin.y < ym || a.pMin.z < zm ||
                                a.pMax.x > xM || a.pMax.y > yM || a.pMax.z > zM;
                if (!expanded) continue;
            }
            int32_t child_idx = node_idx;
            node_idx = lnodes[node_idx].parentID;
            int32_t hops = 0;
            while (node_idx != -1) {
                if ((uint32_t)node_idx >= (uint32_t)used || ++hops > used) {
                    atomicOr(flags, kErrIndexGuard | (kGuardNode << 8));
                    break;
                }
                BVHNode &n = lnodes[node_idx];
                int c = -1;
                for (int j = 0; j < 4; j++) {
                    if (n.children[j] == child_idx) { c = j; break; }
                }
                if (c < 0) break;
                float xm = ldsAtomicMinRef(&n.minX[c], a.pMin.x);
                float ym = ldsAtomicMinRef(&n.minY[c], a.pMin.y);
                float zm = ldsAtomicMinRef(&n.minZ[c], a.pMin.z);
                float xM = ldsAtomicMaxRef(&n.maxX[c], a.pMax.x);
                float yM = ldsAtomicMaxRef(&n.maxY[c], a.pMax.y);
                float zM = ldsAtomicMaxRef(&n.maxZ[c], a.pMax.z);
                bool expanded = a.pMin.x < xm || a.pMin.y < ym || a.pMin.z < zm ||
                                a.pMax.x > xM || a.pMax.y > yM || a.pMax.z > zM;
                if (!expanded) break;
                child_idx = node_idx;
                node_idx = n.parentID;
            }
        }
    }
    __syncthreads();
    if (!kGlobal) {
        // whole nodes, one contiguous run: children / parents are unchanged
        // by a refit, but writing only each 116-byte node's 96 bytes of
        // bounds left a gap in every cache line, and partial-line writes
        // cost HBM read-modify-writes (counters: 2.5x the algorithmic bytes)
        const uint32_t *src = (const uint32_t *)lnodes;
        uint32_t *dst = (uint32_t *)gnodes;
        const int32_t words = used * (int32_t)(sizeof(BVHNode) / 4);
        for (int32_t i = threadIdx.x; i < words; i += kRefitBlock) dst[i] = src[i];
    }
}

__global__ void __launch_bounds__(kRefitBlock) refitKernel(PhysArgs P)
{
    MW_TRACE_BLOCK(0);
    // a world whose used nodes exceed the LDS capacity refits in place
    if (min(P.bvh[blockIdx.x].usedNodes, P.maxNodes) <= P.refitLDSNodes)
        refitWorld<false>(P);
    else
        refitWorld<true>(P);
}

__global__ void __launch_bounds__(kRefitBlock) refitGlobalKernel(PhysArgs P)
{
    MW_TRACE_BLOCK(0);
    refitWorld<true>(P);
}

// findOverlappingEntry + BVH::findOverlaps (broadphase.cpp:897-932,
// physics.inl:61-100).  One block per world; lanes own rows.  Pass 1 counts
// each row's candidates, a block scan gives the reference's append order,
// pass 2 writes them.

constexpr int32_t kOverlapBuf = kOverlapBufRanks;  // candidates kept per body before a second sweep
constexpr int32_t kOverlapMaskWords = 4; // worlds up to 256 leaves: hits as a register bitmask
static_assert(64 * kOverlapMaskWords == kOverlapSmallLeaves);

// findOverlappingEntry + BVH::findOverlaps (broadphase.cpp:897-932,
// physics.inl:61-100) without a per-lane tree walk.  Every ancestor slot of
// a leaf contains the leaf's slot AABB (rebuild merges children, refit only
// grows slots and propagates growth upward), so a query overlaps a leaf slot
// exactly when the walk would reach and emit it; and the walk emits leaves in
// a fixed order (BVH leafOrder, computed at rebuild) with pruned subtrees
// simply missing.  So each body sweeps the world's leaves in that order and
// tests the leaf slots: same candidates, same order, no divergent stacks.
struct alignas(16) OrderedLeaf {
    float minX, minY, minZ;
    float maxX, maxY, maxZ;
    int32_t id;                   // entity id (the e.id < other.id rule)
    int32_t isStatic;
    Loc loc;
    uint32_t slot;                // body slot | arch index << 16 | bad-row flag << 24
};
static_assert(sizeof(OrderedLeaf) == 48);

// AABB::overlaps (math.hpp) of the query against a leaf slot.
// e.id < other.id, not both static, and the slot overlaps the query
// (AABB::overlaps, strict): all terms evaluated, combined with bitwise ands.
__device__ __forceinline__ bool leafHit(const OrderedLeaf *leaves, int32_t k, const AABB &q,
                                        int32_t e_id, bool a_static)
{
    const float4 *l4 = (const float4 *)leaves + 3 * k;
    const float4 lo = l4[0];                  // minX minY minZ maxX
    const float4 hi = l4[1];                  // maxY maxZ id isStatic
    const int32_t id = __float_as_int(hi.z);
    const bool st = __float_as_int(hi.w) != 0;
    return (e_id < id) & !(a_static & st) &
           (q.pMin.x < lo.w) & (lo.x < q.pMax.x) &
           (q.pMin.y < hi.x) & (lo.y < q.pMax.y) &
           (q.pMin.z < hi.y) & (lo.z < q.pMax.z);
}

__device__ __forceinline__ bool slotOverlaps(const AABB &q, const OrderedLeaf &o)
{
    return q.pMin.x < o.maxX && o.minX < q.pMax.x &&
           q.pMin.y < o.maxY && o.minY < q.pMax.y &&
           q.pMin.z < o.maxZ && o.minZ < q.pMax.z;
}

__host__ __device__ inline size_t a16b(size_t b) { return (b + 15) & ~size_t(15); }

__host__ __device__ inline size_t overlapLDSBytes(int32_t max_leaves)
{
    return a16b(sizeof(OrderedLeaf) * max_leaves) + a16b(4 * max_leaves) +
           a16b(2 * kOverlapBlock * kOverlapBuf);
}

// The bitmask path stages its (self rank, other rank) pairs in the per-lane
// buffers' space, so the block writes the candidate run coalesced.
constexpr int32_t kOverlapStage = kOverlapBlock * kOverlapBuf / 2;

// Traversal stack depth (int16 node indices, lane-interleaved in LDS) of
// the traversal kernels (dfsCountKernel).
constexpr int32_t kOverlapStack = 64;

__host__ __device__ inline bool overlapUsesDFS(const PhysArgs &P)
{
    return P.overlapDFSLeaves >= 0 && P.maxLeaves > P.overlapDFSLeaves;
}

// A world past P.overlapDFSLeaves leaves walks the BVH (dfs*Kernel) and
// the one-block sweep kernels skip it.
__host__ __device__ inline bool overlapTraverses(const PhysArgs &P, int32_t nleaves)
{
    return overlapUsesDFS(P) && nleaves > P.overlapDFSLeaves;
}

size_t findOverlapsSharedBytes(const PhysArgs &P)
{
    return overlapLDSBytes(P.maxLeaves);
}

size_t findOverlapsGlobalSharedBytes(const PhysArgs &)
{
    return 0;
}

// Phase profile (experiments only, -DMW_SOLVER_PROFILE, the solver's
// profiling build): per-phase sums of block time in device-clock ticks,
// read (and reset) by mw_debug_overlap_phases.
#if defined(MW_SOLVER_PROFILE)
static __device__ unsigned long long g_overlapPhase[8];
#define MW_OVERLAP_MARK(i)                                                       \
    do {                                                                         \
        if (threadIdx.x == 0) {                                                  \
            const long long t__ = wall_clock64();                                \
            atomicAdd(&g_overlapPhase[(i)], (unsigned long long)(t__ - prof_t)); \
            prof_t = t__;                                                        \
        }                                                                        \
    } while (0)
extern "C" int mw_debug_overlap_phases(unsigned long long *out)
{
    unsigned long long z[8] = {};
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_overlapPhase), sizeof(z)) != hipSuccess) return -1;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_overlapPhase), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#else
#define MW_OVERLAP_MARK(i) ((void)0)
#endif
// Event counts in the same profile: [4] BVH nodes popped, [5] DFS queries,
// [6] wide queries (the wave sweeps for them).
#if defined(MW_SOLVER_PROFILE)
#define MW_OVERLAP_COUNT(i, v) atomicAdd(&g_overlapPhase[(i)], (unsigned long long)(v))
#else
#define MW_OVERLAP_COUNT(i, v) ((void)0)
#endif

// One query's hits (leafHit) over the leaves in emission order, the wave
// testing 64 leaves per step: the count, and with kWrite the candidates at
// slot0.. in that order.  q, e_id, a_static and self are the query lane's
// (wave-uniform).
template <bool kWrite>
__device__ __forceinline__ int32_t waveSweep(const OrderedLeaf *leaves, int32_t nleaves,
                                             const AABB &q, int32_t e_id, bool a_static,
                                             int32_t self, int32_t slot0,
                                             CandidateCollision *out, uint64_t *out_slots,
                                             int32_t cap)
{
    const int32_t lane = threadIdx.x & 63;
    int32_t n = 0;
    for (int32_t k0 = 0; k0 < nleaves; k0 += 64) {
        const int32_t k = k0 + lane;
        const bool hit = k < nleaves && leafHit(leaves, k, q, e_id, a_static);
        const uint64_t b = __ballot(hit);
        if (kWrite && hit) {
            const int32_t slot = slot0 + n + __popcll(b & ((1ull << lane) - 1));
            if (slot < cap) {
                out[slot] = CandidateCollision { leaves[self].loc, leaves[k].loc };
                out_slots[slot] = (uint64_t)leaves[self].slot | (uint64_t)leaves[k].slot << 32;
            }
        }
        n += __popcll(b);
    }
    return n;
}

// BVH::findOverlaps (physics.inl:61-100) for one query: pop a node, visit
// its children in slot order -- a leaf child whose slot overlaps the query
// (and passes the id / static filter) is emitted, an overlapping inner
// child is pushed.  Returns false when the stack would pass
// kOverlapStack entries (the reference's own stack holds 128), when the walk
// would pop more than `budget` nodes, or when emit() declines a leaf; the
// caller then sweeps the leaves, which emits the same sequence.  (A query
// that reaches most of the tree -- a ground plane's, say, whose hits the id
// rule drops -- is a serial chain of dependent node loads; the wave sweeps
// its leaves 64 at a time instead.)  A leaf child's filter and emission rank
// come from one 8-byte load of its DfsKey.
typedef int32_t NodeWords4 __attribute__((ext_vector_type(4), aligned(4)));
static_assert(offsetof(BVHNode, minY) == 16 && offsetof(BVHNode, children) == 96);

struct DfsKey {
    int32_t id;                   // entity id (the e.id < other.id rule)
    int32_t rankStatic;           // emission rank << 1 | isStatic
};

template <int32_t kStride, typename Emit>
__device__ __forceinline__ bool dfsQuery(const BVHNode *__restrict__ nodes, int32_t max_nodes,
                                         int32_t max_leaves, const AABB &q, int32_t e_id,
                                         bool a_static, const DfsKey *__restrict__ keys,
                                         int16_t *stk, int32_t *flags, int32_t budget, Emit &&emit)
{
    int32_t ss = 0;
    int32_t cur = 0;
    int32_t visits = 0;
#if defined(MW_SOLVER_PROFILE)
    struct Tally {
        int32_t &v;
        __device__ ~Tally() { MW_OVERLAP_COUNT(4, v); }
    } tally { visits };
#endif
    for (;;) {
        if (++visits > budget) return false;
        // The node's bounds and children into registers first, as seven
        // 16-byte loads (nodes are 116 bytes, so only 4-byte aligned; global
        // loads need no more): the stack pushes below are stores the
        // compiler cannot prove disjoint from the node, so loads left in the
        // child loop would wait behind them one slot at a time.
        int32_t nw[28];
        const NodeWords4 *src = (const NodeWords4 *)(nodes + cur);
#pragma unroll
        for (int j = 0; j < 7; j++) {
            const NodeWords4 v = src[j];
            nw[4 * j] = v.x; nw[4 * j + 1] = v.y; nw[4 * j + 2] = v.z; nw[4 * j + 3] = v.w;
        }
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int32_t child = nw[24 + i];
            const bool hit = (child != -1) &
                             (q.pMin.x < __int_as_float(nw[12 + i])) & (__int_as_float(nw[i]) < q.pMax.x) &
                             (q.pMin.y < __int_as_float(nw[16 + i])) & (__int_as_float(nw[4 + i]) < q.pMax.y) &
                             (q.pMin.z < __int_as_float(nw[20 + i])) & (__int_as_float(nw[8 + i]) < q.pMax.z);
            if (!hit) continue;
            if (child & 0x80000000) {
                // the slot test above is the leaf's (the image holds the same
                // bytes); then e.id < other.id and not both static
                const DfsKey key = keys[guardIndex(child & 0x7fffffff, max_leaves, flags, kGuardLeaf)];
                const bool keep = (e_id < key.id) & !(a_static & ((key.rankStatic & 1) != 0));
                if (keep && !emit(key.rankStatic >> 1)) return false;
            } else {
                if (ss == kOverlapStack) return false;
                stk[ss++ * kStride] = (int16_t)guardIndex(child, max_nodes, flags, kGuardNode);
            }
        }
        if (ss == 0) return true;
        cur = stk[--ss * kStride];
    }
}

size_t findOverlapsImageBytes(const PhysArgs &P)
{
    return overlapLDSBytes(P.maxLeaves);
}


// The leaf of emission rank k (leafOrder) as the sweeps and the traversal
// read it: its slot AABB from the refit tree, identity, static flag,
// location and packed body slot.  Returns the leaf id.
__device__ __forceinline__ int32_t stageLeaf(const PhysArgs &P, int32_t w, int32_t k,
                                             int32_t *flags, OrderedLeaf &ol)
{
    const BVHNode *nodes = P.nodes + (size_t)w * P.maxNodes;
    const int32_t leaf = guardIndex(P.leafOrder[(size_t)w * P.maxLeaves + k], P.maxLeaves, flags,
                                    kGuardLeaf);
    const uint32_t lp = P.leafParents[(size_t)w * P.maxLeaves + leaf];
    const BVHNode &n = nodes[guardIndex((int32_t)(lp >> 2), P.maxNodes, flags, kGuardNode)];
    const int sub = (int)(lp & 3);
    const Entity e = P.leafEntities[(size_t)w * P.maxLeaves + leaf];
    const Loc loc = entityLoc(P, w, e);
    const int32_t oa = bodyArchIndex(P, loc.archetype);
    const BodyArch &OB = P.body[oa];
    const int32_t row = guardIndex(loc.row, OB.capacity, flags, kGuardLeaf);
    ol.minX = n.minX[sub]; ol.minY = n.minY[sub]; ol.minZ = n.minZ[sub];
    ol.maxX = n.maxX[sub]; ol.maxY = n.maxY[sub]; ol.maxZ = n.maxZ[sub];
    ol.id = e.id;
    ol.isStatic = bcol<ResponseType>(OB, Cols::ResponseType, w, row) == ResponseType::Static ? 1 : 0;
    ol.loc = loc;
    ol.slot = (uint32_t)(OB.slotBase + row) | (uint32_t)oa << 16 |
              ((uint32_t)loc.row < (uint32_t)OB.capacity ? 0u : 1u << 24);
    return leaf;
}

// Runs fn(lane, its query, e_id, static, rank) with the wave, for each lane
// in m (wave-uniform).
template <typename Fn>
__device__ __forceinline__ void forWideLanes(uint64_t m, const AABB &q, int32_t e_id, bool a_static,
                                             int32_t self, Fn &&fn)
{
    for (; m; m &= m - 1) {
        const int32_t h = __ffsll((unsigned long long)m) - 1;
        AABB qh;
        qh.pMin.x = __shfl(q.pMin.x, h, 64); qh.pMin.y = __shfl(q.pMin.y, h, 64);
        qh.pMin.z = __shfl(q.pMin.z, h, 64); qh.pMax.x = __shfl(q.pMax.x, h, 64);
        qh.pMax.y = __shfl(q.pMax.y, h, 64); qh.pMax.z = __shfl(q.pMax.z, h, 64);
        fn(h, qh, __shfl(e_id, h, 64), __shfl((int32_t)a_static, h, 64) != 0, __shfl(self, h, 64));
    }
}

// The sweep worlds, one block per world (worlds that traverse return at
// once: dfsStageKernel / dfsCountKernel / dfsWriteKernel below).
// kGlobal: the world's leaf image exceeds a workgroup's LDS; it is staged in
// the world's slab of P.overlapImage instead (findOverlapsGlobalKernel).
// kSmall: every world fits the register bitmask (maxLeaves <= 256) and none
// traverses -- the general sweep is compiled out, which keeps this kernel's
// registers (and so its occupancy) to the bitmask path's own.
template <bool kGlobal, bool kSmall = false>
__device__ __forceinline__ void findOverlapsWorld(const PhysArgs &P)
{
#if defined(MW_SOLVER_PROFILE)
    long long prof_t = wall_clock64();
#endif
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ int32_t scan_scratch[kOverlapBlock / 64];
    const int32_t w = blockIdx.x;
    char *img = kGlobal ? P.overlapImage + (size_t)w * overlapLDSBytes(P.maxLeaves) : smem;
    OrderedLeaf *leaves = (OrderedLeaf *)img;
    int32_t *rank_of = (int32_t *)(img + a16b(sizeof(OrderedLeaf) * P.maxLeaves));
    uint16_t *bufs = (uint16_t *)((char *)rank_of + a16b(4 * P.maxLeaves));

    // Stage leaf slots (from the refit tree) + identity in emission order.
    const broadphase::BVH &bvh = P.bvh[w];
    const int32_t nleaves = min(bvh.numLeaves, P.maxLeaves);
    int32_t *flags = P.errorFlags + w;
    if (!kSmall && overlapTraverses(P, nleaves)) return;
    for (int32_t k = threadIdx.x; k < nleaves; k += kOverlapBlock) {
        OrderedLeaf ol;
        const int32_t leaf = stageLeaf(P, w, k, flags, ol);
        leaves[k] = ol;
        rank_of[leaf] = k;
    }
    __syncthreads();
    MW_OVERLAP_MARK(0);                                   // staging

    uint16_t *buf = bufs + threadIdx.x * kOverlapBuf;
    int32_t base = 0;
    for (int32_t ba = 0; ba < P.numBodyArchs; ba++) {
        const BodyArch &B = P.body[ba];
        const int32_t rows = B.numRows[w];
        for (int32_t chunk = 0; chunk < rows; chunk += kOverlapBlock) {
            const int32_t row = chunk + threadIdx.x;
            int32_t cnt = 0;
            AABB q = AABB::invalid();
            int32_t self = 0;
            if (row < rows) {
                const int32_t leaf = guardIndex(bcol<broadphase::LeafID>(B, Cols::LeafID, w, row).id,
                                                P.maxLeaves, flags, kGuardLeaf);
                q = P.leafAABBs[(size_t)w * P.maxLeaves + leaf];
                self = rank_of[leaf];
            }
            const OrderedLeaf &me = leaves[self];
            const int32_t e_id = me.id;
            const bool a_static = me.isStatic != 0;
            const bool active = row < rows;
            CandidateCollision *out = P.cands + (size_t)w * P.candCapacity;
            uint64_t *out_slots = P.candSlots + (size_t)w * P.candCapacity;
            int32_t total;
            if (kSmall || nleaves <= 64 * kOverlapMaskWords) {
                // The hits as a leaf-rank bitmask in registers: the sweep
                // stores nothing to LDS, so the broadcast leaf reads of
                // successive iterations are not ordered behind a possibly
                // aliasing store and stay in flight together; the writes walk
                // the set bits in rank order (the reference's emission order).
                uint64_t mask[kOverlapMaskWords];
#pragma unroll
                for (int32_t c = 0; c < kOverlapMaskWords; c++) {
                    uint64_t bits = 0;
                    const int32_t k0 = 64 * c, k1 = min(nleaves, k0 + 64);
#pragma unroll 8
                    for (int32_t k = k0; k < k1; k++) {
                        bits |= (uint64_t)leafHit(leaves, k, q, e_id, a_static) << (k - k0);
                    }
                    mask[c] = active ? bits : 0;
                    cnt += __popcll(mask[c]);
                }
                MW_OVERLAP_MARK(1);                       // sweep (thread 0's wave)
                const int32_t off = blockExclusiveScan(cnt, scan_scratch, &total);
                MW_OVERLAP_MARK(2);                       // scan (waits for every wave)
                if (total <= kOverlapStage) {
                    // Pairs of ranks into LDS at their run positions, then
                    // the block writes the run in order: each wave store
                    // covers 64 consecutive candidates instead of one lane's
                    // run per lane.  (The scan's barriers order this against
                    // the previous chunk's reads of the stage.)
                    uint32_t *stage = (uint32_t *)bufs;
                    int32_t i = off;
#pragma unroll
                    for (int32_t c = 0; c < kOverlapMaskWords; c++) {
                        uint64_t bits = mask[c];
                        while (bits) {
                            const int32_t k = 64 * c + __ffsll((unsigned long long)bits) - 1;
                            bits &= bits - 1;
                            stage[i++] = (uint32_t)self | (uint32_t)k << 16;
                        }
                    }
                    __syncthreads();
                    const int32_t lim = min(total, P.candCapacity - base);
                    for (int32_t t = threadIdx.x; t < lim; t += kOverlapBlock) {
                        const uint32_t pr = stage[t];
                        const OrderedLeaf &a = leaves[pr & 0xffff];
                        const OrderedLeaf &o = leaves[pr >> 16];
                        out[base + t] = CandidateCollision { a.loc, o.loc };
                        out_slots[base + t] = (uint64_t)a.slot | (uint64_t)o.slot << 32;
                    }
                } else if (cnt > 0) {
                    const Loc a_loc = me.loc;
                    const uint64_t a_slot = me.slot;
                    int32_t slot = base + off;
#pragma unroll
                    for (int32_t c = 0; c < kOverlapMaskWords; c++) {
                        uint64_t bits = mask[c];
                        while (bits) {
                            const int32_t k = 64 * c + __ffsll((unsigned long long)bits) - 1;
                            bits &= bits - 1;
                            const OrderedLeaf &o = leaves[k];
                            if (slot < P.candCapacity) {
                                out[slot] = CandidateCollision { a_loc, o.loc };
                                out_slots[slot] = a_slot | (uint64_t)o.slot << 32;
                            }
                            slot++;
                        }
                    }
                }
                base += total;
                MW_OVERLAP_MARK(3);                       // candidate writes (thread 0's)
                continue;
            }
            // Worlds with more leaves: the sweep counts hits and keeps the
            // first kOverlapBuf ranks in LDS; the wave re-sweeps for a body
            // with more.  The hit test is evaluated branch-free on one
            // 32-byte broadcast read per leaf.
#pragma unroll 4
            for (int32_t k = 0; k < nleaves; k++) {
                const bool hit = active & leafHit(leaves, k, q, e_id, a_static);
                if (hit) {
                    if (cnt < kOverlapBuf) buf[cnt] = (uint16_t)k;
                    cnt++;
                }
            }
            MW_OVERLAP_MARK(1);                           // sweep (thread 0's wave)
            const int32_t off = blockExclusiveScan(cnt, scan_scratch, &total);
            MW_OVERLAP_MARK(2);                           // scan (waits for every wave)
            if (cnt > 0 && cnt <= kOverlapBuf) {
                const Loc a_loc = me.loc;
                const uint64_t a_slot = me.slot;
                for (int32_t i = 0; i < cnt; i++) {
                    const int32_t slot = base + off + i;
                    const OrderedLeaf &o = leaves[buf[i]];
                    if (slot < P.candCapacity) {
                        out[slot] = CandidateCollision { a_loc, o.loc };
                        out_slots[slot] = a_slot | (uint64_t)o.slot << 32;
                    }
                }
            }
            const int32_t first = base + off;
            forWideLanes(__ballot(cnt > kOverlapBuf), q, e_id, a_static, self,
                    [&](int32_t h, const AABB &qh, int32_t eh, bool sh, int32_t selfh) {
                        waveSweep<true>(leaves, nleaves, qh, eh, sh, selfh, __shfl(first, h, 64),
                                        out, out_slots, P.candCapacity);
                    });
            base += total;
            MW_OVERLAP_MARK(3);                           // candidate writes (thread 0's)
        }
    }
    if (threadIdx.x == 0) {
        if (base > P.candCapacity) {
            atomicOr(P.errorFlags + w, kErrCandidateOverflow);
            base = P.candCapacity;
        }
        P.numCands[w] = base;
        P.lastNumCands[w] = base;
    }
#if defined(MW_SOLVER_PROFILE)
    if (threadIdx.x == 0) atomicAdd(&g_overlapPhase[7], 1ull);
#endif
}

__global__ void __launch_bounds__(kOverlapBlock) findOverlapsKernel(PhysArgs P)
{
    MW_TRACE_BLOCK(0);
    findOverlapsWorld<false>(P);
}

// Occupancy of the bitmask-path kernel: at its free register count (124
// VGPRs, 4 waves / SIMD) a world's dependent staging loads and its sweep's
// broadcast reads leave the CU idle; pinned to 8 waves / SIMD it compiles to
// 63 VGPRs without spills and runs 0.165 -> 0.116 ms per collisions launch
// (interleaved A/B; 5 and 6 waves: 0.130 / 0.129).
#ifndef MW_OVERLAP_WAVES
#define MW_OVERLAP_WAVES 8
#endif
#define MW_OVERLAP_SMALL_ATTR __attribute__((amdgpu_waves_per_eu(MW_OVERLAP_WAVES)))
__global__ void __launch_bounds__(kOverlapBlock) MW_OVERLAP_SMALL_ATTR findOverlapsSmallKernel(PhysArgs P)
{
    MW_TRACE_BLOCK(0);
    findOverlapsWorld<false, true>(P);
}

__global__ void __launch_bounds__(kOverlapBlock) findOverlapsGlobalKernel(PhysArgs P)
{
    MW_TRACE_BLOCK(0);
    findOverlapsWorld<true>(P);
}

// ---- Traversal worlds (more than P.overlapDFSLeaves leaves) ----
// BVH::findOverlaps per body (physics.inl:61-100), its cost following the
// body's overlaps rather than the world's size.  One block per world made a
// 3,200-body world the latency chain of one CU (2.31 ms per launch); the
// work now spreads over (world, chunk of kDfsBlock body rows) blocks in three
// launches:
//   dfsStageKernel  the emission-order leaf image (OrderedLeaf, what the
//                   candidate writes and the wave sweeps read) and, per leaf
//                   id, its DfsKey (entity id, static flag, emission rank);
//   dfsCountKernel  each lane walks its body's query into its first
//                   kOverlapBuf hit ranks; a wide query (more hits, a deeper
//                   stack, or a walk past 32 + leaves/32 nodes -- about what
//                   sweeping costs the wave) is counted by its wave sweeping
//                   the leaves, 64 per step, in the same order; each block
//                   records its chunk's total;
//   dfsWriteKernel  each block's first slot is the earlier chunks' totals
//                   plus a block scan; the candidates go out in row order
//                   (a wide query swept again by its wave).
// Rows are numbered across the body archetypes in order, as the sweep
// kernels visit them, so the candidate sequence is the one-block path's.
static_assert(sizeof(DfsKey) == 8 && kOrderedLeafBytes == sizeof(OrderedLeaf));
constexpr int32_t kDfsWide = 1 << 30;                 // dfsRows[].x: the wave sweeps this row

__device__ __forceinline__ bool dfsWorld(const PhysArgs &P, int32_t w, int32_t &nleaves)
{
    nleaves = min(P.bvh[w].numLeaves, P.maxLeaves);
    return overlapTraverses(P, nleaves);
}

// Row r of world w counted across the body archetypes (false past the last).
__device__ __forceinline__ bool dfsRow(const PhysArgs &P, int32_t w, int32_t r, int32_t &ba,
                                       int32_t &row)
{
    for (ba = 0; ba < P.numBodyArchs; ba++) {
        const int32_t rows = P.body[ba].numRows[w];
        if (r < rows) {
            row = r;
            return true;
        }
        r -= rows;
    }
    return false;
}

__global__ void __launch_bounds__(kDfsBlock) dfsStageKernel(PhysArgs P)
{
    MW_TRACE_BLOCK(0);
    const int32_t w = blockIdx.x;
    int32_t nleaves;
    if (!dfsWorld(P, w, nleaves)) return;
    const int32_t k = blockIdx.y * kDfsBlock + threadIdx.x;
    if (k >= nleaves) return;
    const size_t wl = (size_t)w * P.maxLeaves;
    OrderedLeaf ol;
    const int32_t leaf = stageLeaf(P, w, k, P.errorFlags + w, ol);
    ((OrderedLeaf *)P.dfsImage)[wl + k] = ol;
    ((DfsKey *)P.dfsKeys)[wl + leaf] = DfsKey { ol.id, k << 1 | ol.isStatic };
}

__global__ void __launch_bounds__(kDfsBlock) dfsCountKernel(PhysArgs P)
{
    MW_TRACE_BLOCK(0);
    const int32_t w = blockIdx.x;
    int32_t nleaves;
    if (!dfsWorld(P, w, nleaves)) return;
    __shared__ int16_t stacks[kOverlapStack * kDfsBlock];
    __shared__ int32_t scan_scratch[kDfsBlock / 64];
    int32_t *flags = P.errorFlags + w;
    const size_t wl = (size_t)w * P.maxLeaves;
    const OrderedLeaf *leaves = (const OrderedLeaf *)P.dfsImage + wl;
    const DfsKey *keys = (const DfsKey *)P.dfsKeys + wl;
    const int32_t r = blockIdx.y * kDfsBlock + threadIdx.x;
    const size_t wr = (size_t)w * P.dfsRowCap + r;

    int32_t ba = 0, row = 0, leaf = 0;
    const bool active = dfsRow(P, w, r, ba, row);
    AABB q = AABB::invalid();
    DfsKey me { 0, 0 };
    if (active) {
        const BodyArch &B = P.body[ba];
        leaf = guardIndex(bcol<broadphase::LeafID>(B, Cols::LeafID, w, row).id, P.maxLeaves, flags,
                          kGuardLeaf);
        q = P.leafAABBs[wl + leaf];
        me = keys[leaf];
    }
    const int32_t e_id = me.id;
    const bool a_static = (me.rankStatic & 1) != 0;
    const int32_t self = me.rankStatic >> 1;

    uint16_t *hits = P.dfsHits + wr * kOverlapBuf;
    int32_t cnt = 0;
    bool wide = false;
    if (active) {
        MW_OVERLAP_COUNT(5, 1);
        wide = !dfsQuery<kDfsBlock>(P.nodes + (size_t)w * P.maxNodes, P.maxNodes, P.maxLeaves, q, e_id,
                                    a_static, keys, stacks + threadIdx.x, flags, 32 + nleaves / 32,
                                    [&](int32_t k) {
                                        if (cnt == kOverlapBuf) return false;
                                        hits[cnt++] = (uint16_t)k;
                                        return true;
                                    });
    }
    if (wide) MW_OVERLAP_COUNT(6, 1);
    forWideLanes(__ballot(wide), q, e_id, a_static, self,
                 [&](int32_t h, const AABB &qh, int32_t eh, bool sh, int32_t selfh) {
                     const int32_t n = waveSweep<false>(leaves, nleaves, qh, eh, sh, selfh, 0,
                                                        nullptr, nullptr, 0);
                     if ((int32_t)(threadIdx.x & 63) == h) cnt = n;
                 });
    ((int2 *)P.dfsRows)[wr] = make_int2(wide ? (cnt | kDfsWide) : cnt, leaf);
    int32_t total;
    (void)blockExclusiveScan(cnt, scan_scratch, &total);
    if (threadIdx.x == 0) P.dfsChunkTotals[(size_t)w * P.dfsChunks + blockIdx.y] = total;
}

__global__ void __launch_bounds__(kDfsBlock) dfsWriteKernel(PhysArgs P)
{
    MW_TRACE_BLOCK(0);
    const int32_t w = blockIdx.x;
    int32_t nleaves;
    if (!dfsWorld(P, w, nleaves)) return;
    __shared__ int32_t scan_scratch[kDfsBlock / 64];
    const size_t wl = (size_t)w * P.maxLeaves;
    const OrderedLeaf *leaves = (const OrderedLeaf *)P.dfsImage + wl;
    const DfsKey *keys = (const DfsKey *)P.dfsKeys + wl;
    const int32_t *totals = P.dfsChunkTotals + (size_t)w * P.dfsChunks;
    const int32_t r = blockIdx.y * kDfsBlock + threadIdx.x;
    const size_t wr = (size_t)w * P.dfsRowCap + r;

    int32_t first = 0;
    for (int32_t c = 0; c < (int32_t)blockIdx.y; c++) first += totals[c];
    const int2 rec = ((const int2 *)P.dfsRows)[wr];
    const bool wide = (rec.x & kDfsWide) != 0;
    const int32_t cnt = rec.x & ~kDfsWide;
    int32_t total;
    const int32_t base = first + blockExclusiveScan(cnt, scan_scratch, &total);

    const int32_t cap = P.candCapacity;
    CandidateCollision *out = P.cands + (size_t)w * cap;
    uint64_t *out_slots = P.candSlots + (size_t)w * cap;
    DfsKey me { 0, 0 };
    AABB q = AABB::invalid();
    if (cnt > 0 || wide) me = keys[rec.y];           // a wide query's sweep filters by it
    if (wide) q = P.leafAABBs[wl + rec.y];
    const int32_t self = me.rankStatic >> 1;
    if (!wide && cnt > 0) {
        const uint16_t *hits = P.dfsHits + wr * kOverlapBuf;
        const OrderedLeaf &a = leaves[self];
        const Loc a_loc = a.loc;
        const uint64_t a_slot = a.slot;
        for (int32_t i = 0; i < cnt; i++) {
            const int32_t slot = base + i;
            const OrderedLeaf &o = leaves[hits[i]];
            if (slot < cap) {
                out[slot] = CandidateCollision { a_loc, o.loc };
                out_slots[slot] = a_slot | (uint64_t)o.slot << 32;
            }
        }
    }
    forWideLanes(__ballot(wide), q, me.id, (me.rankStatic & 1) != 0, self,
                 [&](int32_t h, const AABB &qh, int32_t eh, bool sh, int32_t selfh) {
                     waveSweep<true>(leaves, nleaves, qh, eh, sh, selfh, __shfl(base, h, 64), out,
                                     out_slots, cap);
                 });

    if (blockIdx.y == 0 && threadIdx.x == 0) {
        int32_t all = 0, rows = 0;
        for (int32_t c = 0; c < P.dfsChunks; c++) all += totals[c];
        for (int32_t ba = 0; ba < P.numBodyArchs; ba++) rows += P.body[ba].numRows[w];
        if (rows > P.dfsRowCap) atomicOr(P.errorFlags + w, kErrIndexGuard | (kGuardLeaf << 8));
        if (all > cap) {
            atomicOr(P.errorFlags + w, kErrCandidateOverflow);
            all = cap;
        }
        P.numCands[w] = all;
        P.lastNumCands[w] = all;
#if defined(MW_SOLVER_PROFILE)
        atomicAdd(&g_overlapPhase[7], 1ull);
#endif
    }
}

}
