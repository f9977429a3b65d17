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
}

// refitEntry -> BVH::refitLeaf (broadphase.cpp:545-642, 891-895)
__global__ void __launch_bounds__(256) refitKernel(PhysArgs P)
{
    const BodyArch &B = P.body[blockIdx.y];
    RowIdx ri = rowIndex(P, B);
    if (!ri.valid) return;
    const int32_t w = ri.w;
    const int32_t leaf = guardIndex(bcol<broadphase::LeafID>(B, Cols::LeafID, w, ri.r).id,
                                    P.maxLeaves, P.errorFlags + w, kGuardLeaf);
    const size_t li = (size_t)w * P.maxLeaves + leaf;
    const AABB a = P.leafAABBs[li];
    const uint32_t lp = P.leafParents[li];
    BVHNode *nodes = P.nodes + (size_t)w * P.maxNodes;
    int32_t node_idx = guardIndex((int32_t)(lp >> 2), P.maxNodes, P.errorFlags + w, kGuardNode);
    const int sub = (int)(lp & 3);

    {   // leaf slot: owned by this leaf alone -> plain read-modify-write
        BVHNode &n = nodes[node_idx];
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
        if (!expanded) return;
    }
    int32_t child_idx = node_idx;
    node_idx = nodes[node_idx].parentID;
    while (node_idx != -1) {
        if ((uint32_t)node_idx >= (uint32_t)P.maxNodes) {
            atomicOr(P.errorFlags + w, kErrIndexGuard | (kGuardNode << 8));
            return;
        }
        BVHNode &n = nodes[node_idx];
        int c = -1;
        for (int j = 0; j < 4; j++) {
            if (n.children[j] == child_idx) { c = j; break; }
        }
        if (c < 0) return;
        float xm = atomicMinRef(&n.minX[c], a.pMin.x);
        float ym = atomicMinRef(&n.minY[c], a.pMin.y);
        float zm = atomicMinRef(&n.minZ[c], a.pMin.z);
        float xM = atomicMaxRef(&n.maxX[c], a.pMax.x);
        float yM = atomicMaxRef(&n.maxY[c], a.pMax.y);
        float zM = atomicMaxRef(&n.maxZ[c], a.pMax.z);
        bool expanded = a.pMin.x < xm || a.pMin.y < ym || a.pMin.z < zm ||
                        a.pMax.x > xM || a.pMax.y > yM || a.pMax.z > zM;
        if (!expanded) break;
        child_idx = node_idx;
        node_idx = n.parentID;
    }
}

// findOverlappingEntry + BVH::findOverlaps (broadphase.cpp:897-932,
// physics.inl:61-100).  One block per world; lanes own rows.  Pass 1 counts
// each row's candidates, a block scan gives the reference's append order,
// pass 2 writes them.

constexpr int32_t kOverlapStack = 24;   // int16 entries; 4-wide tree depth <= 7 at 4096 leaves
constexpr int32_t kOverlapBuf = 12;     // candidates kept per body before a re-walk

// LDS image of one world's BVH (nodes padded to 128 B so a node is eight
// 16-byte LDS reads) plus per-leaf (entity id, Loc, static flag), per-lane
// traversal stacks and per-lane candidate buffers.
struct alignas(16) LNode {
    float minX[4], minY[4], minZ[4];
    float maxX[4], maxY[4], maxZ[4];
    int32_t children[4];
    int32_t pad[4];
};
static_assert(sizeof(LNode) == 128);

struct OverlapLDS {
    LNode *nodes;
    int32_t *leafId;
    Loc *leafLoc;
    int8_t *leafStatic;
    int16_t *stacks;
    uint16_t *bufs;
};

__host__ __device__ inline size_t a16b(size_t b) { return (b + 15) & ~size_t(15); }

__host__ __device__ inline size_t overlapLDSBytes(int32_t max_nodes, int32_t max_leaves)
{
    return a16b(sizeof(LNode) * max_nodes) + a16b(4 * max_leaves) + a16b(8 * max_leaves) +
           a16b(max_leaves) + a16b(2 * kOverlapBlock * kOverlapStack) +
           a16b(2 * kOverlapBlock * kOverlapBuf);
}

__device__ __forceinline__ OverlapLDS overlapLDS(char *smem, int32_t max_nodes, int32_t max_leaves)
{
    OverlapLDS L;
    char *p = smem;
    L.nodes = (LNode *)p;
    p += a16b(sizeof(LNode) * max_nodes);
    L.leafId = (int32_t *)p;
    p += a16b(4 * max_leaves);
    L.leafLoc = (Loc *)p;
    p += a16b(8 * max_leaves);
    L.leafStatic = (int8_t *)p;
    p += a16b(max_leaves);
    L.stacks = (int16_t *)p;
    p += a16b(2 * kOverlapBlock * kOverlapStack);
    L.bufs = (uint16_t *)p;
    return L;
}

size_t findOverlapsSharedBytes(const PhysArgs &P)
{
    return overlapLDSBytes(P.maxNodes, P.maxLeaves);
}

// BVH::findOverlaps for one body (physics.inl:61-100): DFS with the
// reference's push order; a hit is a leaf whose entity id is larger than the
// body's and that is not static-static.  kWrite = false: count hits and keep
// the first kOverlapBuf other-leaf indices; kWrite = true: write every hit.
template <bool kWrite>
__device__ __forceinline__ int32_t traverseOverlaps(const PhysArgs &P, const OverlapLDS &L,
                                                    int32_t w, int32_t leaf, int16_t *stack,
                                                    uint16_t *buf, int32_t out_base)
{
    const int32_t e_id = L.leafId[leaf];
    const Loc a_loc = L.leafLoc[leaf];
    const bool a_static = L.leafStatic[leaf] != 0;
    const AABB q = P.leafAABBs[(size_t)w * P.maxLeaves + leaf];

    int32_t count = 0;
    stack[0] = 0;
    int32_t ss = 1;
    while (ss > 0) {
        const LNode &n = L.nodes[stack[--ss]];
        for (int i = 0; i < 4; i++) {
            const int32_t child = n.children[i];
            if (child == -1) continue;
            AABB c { { n.minX[i], n.minY[i], n.minZ[i] }, { n.maxX[i], n.maxY[i], n.maxZ[i] } };
            if (!q.overlaps(c)) continue;
            if (child & 0x80000000) {
                const int32_t ol = child & ~0x80000000;
                if (e_id < L.leafId[ol]) {
                    if (a_static && L.leafStatic[ol]) continue;
                    if (kWrite) {
                        const int32_t slot = out_base + count;
                        if (slot < P.candCapacity) {
                            P.cands[(size_t)w * P.candCapacity + slot] =
                                CandidateCollision { a_loc, L.leafLoc[ol] };
                        }
                    } else if (count < kOverlapBuf) {
                        buf[count] = (uint16_t)ol;
                    }
                    count++;
                }
            } else {
                if (ss < kOverlapStack) {
                    stack[ss++] = (int16_t)child;
                } else {
                    atomicOr(P.errorFlags + w, kErrBVHStack);
                }
            }
        }
    }
    return count;
}

// findOverlappingEntry (broadphase.cpp:897-932): one block per world, lanes
// own body rows.  One walk per body fills a small LDS buffer; a block scan of
// the counts gives the reference's append order (row order, DFS order within
// a row); bodies with more hits than the buffer holds walk again to write.
__global__ void __launch_bounds__(kOverlapBlock) findOverlapsKernel(PhysArgs P)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ int32_t scan_scratch[kOverlapBlock / 64];
    const int32_t w = blockIdx.x;
    OverlapLDS L = overlapLDS(smem, P.maxNodes, P.maxLeaves);

    // stage nodes (29 dwords each -> 32-dword LDS slots) and leaf info
    const broadphase::BVH &bvh = P.bvh[w];
    const int32_t used = min(bvh.usedNodes, P.maxNodes);
    const uint32_t *gnodes = (const uint32_t *)(P.nodes + (size_t)w * P.maxNodes);
    uint32_t *lnodes = (uint32_t *)L.nodes;
    for (int32_t i = threadIdx.x; i < used * 32; i += kOverlapBlock) {
        const int32_t node = i >> 5, d = i & 31;
        lnodes[i] = d < 29 ? gnodes[node * 29 + d] : 0u;
    }
    const int32_t nleaves = bvh.numLeaves;
    for (int32_t l = threadIdx.x; l < nleaves; l += kOverlapBlock) {
        const Entity e = P.leafEntities[(size_t)w * P.maxLeaves + l];
        const Loc loc = entityLoc(P, w, e);
        L.leafId[l] = e.id;
        L.leafLoc[l] = loc;
        const BodyArch &OB = P.body[bodyArchIndex(P, loc.archetype)];
        const int32_t row = guardIndex(loc.row, OB.capacity, P.errorFlags + w, kGuardLeaf);
        L.leafStatic[l] =
            bcol<ResponseType>(OB, Cols::ResponseType, w, row) == ResponseType::Static ? 1 : 0;
    }
    __syncthreads();

    int16_t *stack = L.stacks + threadIdx.x * kOverlapStack;
    uint16_t *buf = L.bufs + threadIdx.x * kOverlapBuf;
    int32_t base = 0;
    for (int32_t ba = 0; ba < P.numBodyArchs; ba++) {
        const BodyArch &B = P.body[ba];
        const int32_t rows = B.numRows[w];
        for (int32_t chunk = 0; chunk < rows; chunk += kOverlapBlock) {
            const int32_t row = chunk + threadIdx.x;
            int32_t cnt = 0, leaf = 0;
            if (row < rows) {
                leaf = guardIndex(bcol<broadphase::LeafID>(B, Cols::LeafID, w, row).id,
                                  P.maxLeaves, P.errorFlags + w, kGuardLeaf);
                cnt = traverseOverlaps<false>(P, L, w, leaf, stack, buf, 0);
            }
            int32_t total;
            const int32_t off = blockExclusiveScan(cnt, scan_scratch, &total);
            if (cnt > kOverlapBuf) {
                traverseOverlaps<true>(P, L, w, leaf, stack, buf, base + off);
            } else if (cnt > 0) {
                const Loc a_loc = L.leafLoc[leaf];
                CandidateCollision *out = P.cands + (size_t)w * P.candCapacity;
                for (int32_t i = 0; i < cnt; i++) {
                    const int32_t slot = base + off + i;
                    if (slot < P.candCapacity) out[slot] = CandidateCollision { a_loc, L.leafLoc[buf[i]] };
                }
            }
            base += total;
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
}

}
