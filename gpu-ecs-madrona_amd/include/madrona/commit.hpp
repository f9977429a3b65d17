// Ordered structural commit of one world after a row-parallel node (Context,
// row-parallel mode), run by ONE wave:
//   1. the world's deferred destroys are sorted by append key (bitonic sort
//      in the working set) and their targets looked up (before anything
//      moves);
//   2. per touched archetype: the rows appended past the (unchanged) row
//      count are sorted by key; one lane replays appends and swap-removes in
//      key order on row INDICES only (slot[final position] = source row,
//      where[source row] = position: O(1) per event), which is the
//      reference's serial order (state.inl:398-472, src/core/state.cpp:
//      181-202); then the lanes move the rows that changed position -- few
//      rows through the working set's stage in one gather and one scatter
//      for all columns, more column by column through `scratch` --, remap
//      moved entities and clear the keys;
//   3. one lane releases the destroyed IDs in key order (IDMap::releaseID).
// Called by the executor's commit kernel (one-wave blocks, working set in
// LDS).  (Committing inside a one-wave-per-world row kernel, right after the
// world's rows, saved the commit launch but raised every row kernel to ~100
// VGPRs: fantasy_vs 109 -> 100 M env-steps/s; measured and dropped.)
#pragma once

#include <madrona/state.hpp>

namespace madrona::detail {

inline constexpr int32_t kCommitStageWords = 1024;
inline constexpr uint64_t kAppliedOp = 0xFFFF'FFFE'FFFF'FFFFull;

// Working-set layout: slot / where per row, the append keys and the destroy
// keys (each padded to a power of two for the bitonic sort), the moved rows'
// stage, the resolved destroy targets, then the scalars.
struct CommitShape {
    int32_t capMax;         // rows per world the index arrays hold
    int32_t sortA;          // pow2 >= capMax
    int32_t sortO;          // pow2 >= deferCap
};

MW_HD inline size_t commitWorkingBytes(const CommitShape &S)
{
    return (size_t)S.capMax * 8 + (size_t)(S.sortA + 2 * S.sortO) * 8 + (size_t)kCommitStageWords * 4 +
           16 + sizeof(int32_t) * (kMaxColumns + 1);
}

#if defined(__HIPCC__)
// One wave owns the working set: a wave-level barrier orders its lanes'
// accesses (LDS or global).
__device__ inline void commitSync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ inline void commitSortKeys(uint64_t *keys, int32_t n, int32_t lane)
{
    for (int32_t k = 2; k <= n; k <<= 1) {
        for (int32_t j = k >> 1; j > 0; j >>= 1) {
            for (int32_t i = lane; i < n; i += 64) {
                const int32_t ixj = i ^ j;
                if (ixj > i) {
                    const uint64_t a = keys[i], b = keys[ixj];
                    const bool up = (i & k) == 0;
                    if ((a > b) == up) {
                        keys[i] = b;
                        keys[ixj] = a;
                    }
                }
            }
            commitSync();
        }
    }
}

// Values other lanes updated with atomics (performed past the CU's L1):
// read the same way.
template <typename T>
__device__ inline T commitLoad(const T *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ inline int32_t commitPow2Ceil(int32_t n)
{
    int32_t p = 1;
    while (p < n) p <<= 1;
    return p;
}

// `ws`: commitWorkingBytes(S) bytes; `scratch`: S.capMax x the largest column
// bytes (moves too large for the stage).  Every lane of the wave calls it.
__device__ inline void commitWorld(StateView &st, const CommitShape &S, char *ws, char *scratch, int32_t w)
{
    const int32_t lane = (int32_t)(threadIdx.x & 63);
    int32_t *slot = (int32_t *)ws;
    int32_t *where = slot + S.capMax;
    uint64_t *akeys = (uint64_t *)(where + S.capMax);
    uint64_t *okeys = akeys + S.sortA;
    uint32_t *stage = (uint32_t *)(okeys + S.sortO);
    uint64_t *dloc = (uint64_t *)(stage + kCommitStageWords);     // resolved destroy targets
    unsigned long long *arch_mask = (unsigned long long *)(dloc + S.sortO);
    int32_t *n_final = (int32_t *)(arch_mask + 1);
    int32_t *n_moved = n_final + 1;
    int32_t *col_words = n_moved + 1;                                // [kMaxColumns + 1]

    const uint64_t dirty = commitLoad(st.appendDirty + w);
    int32_t nops = commitLoad(st.deferCount + w);
    nops = min(nops, st.deferCap);
    DeferredDestroy *log = st.deferLog + (size_t)w * st.deferCap;
    IDMapView ids = st.ids(w);

    // 1. deferred destroys: sort by key, resolve targets
    const int32_t so = commitPow2Ceil(max(nops, 1));
    for (int32_t i = lane; i < so; i += 64) {
        okeys[i] = i < nops ? ((log[i].key & ~0xFFFFull) | (uint64_t)i) : ~0ull;
    }
    if (lane == 0) *arch_mask = dirty;
    commitSync();
    commitSortKeys(okeys, so, lane);
    for (int32_t i = lane; i < nops; i += 64) {
        const Loc l = ids.lookup(log[i].e);
        dloc[i] = l.valid() ? (((uint64_t)l.archetype << 32) | (uint32_t)l.row) : ~0ull;
        if (l.valid()) atomicOr(arch_mask, 1ull << l.archetype);
    }
    commitSync();
    const uint64_t mask = commitLoad(arch_mask);

    // 2. per archetype, in index order
    for (int32_t a = 0; a < st.numArchetypes; a++) {
        if (!(mask & (1ull << a))) continue;
        ArchetypeView &av = st.arch[a];
        const int32_t cap = av.capacity;
        if (cap > S.capMax) {
            if (lane == 0) atomicOr(st.errorFlags + w, kErrFlagCommitLimit);
            commitSync();
            continue;
        }
        uint64_t *keys = av.appendKeys ? av.appendKeys + (size_t)w * cap : nullptr;
        // rows appended by the node: [numRows, numRows + pending), the ones
        // past the capacity were refused (kErrTableFull)
        const int32_t n0 = min(av.numRows[w], cap);
        const int32_t m = keys ? min(commitLoad(av.pendingRows + w), cap - n0) : 0;
        const int32_t n_end = n0 + m;
        const int32_t sa = commitPow2Ceil(max(m, 1));
        for (int32_t j = lane; j < sa; j += 64) {
            akeys[j] = j < m ? ((keys[n0 + j] & ~0xFFFFull) | (uint64_t)j) : ~0ull;
        }
        for (int32_t p = lane; p < n_end; p += 64) {
            slot[p] = p < n0 ? p : -1;
            where[p] = p < n0 ? p : -1;
        }
        commitSync();
        commitSortKeys(akeys, sa, lane);

        const bool temporary = (av.flags & kArchTemporary) != 0;
        const Entity *ecol = (const Entity *)(av.cols[0] + (size_t)w * cap * sizeof(Entity));
        if (lane == 0) {
            int32_t n = n0, ia = 0, io = 0;
            for (;;) {
                while (io < so && okeys[io] != ~0ull &&
                       (dloc[okeys[io] & 0xFFFF] == ~0ull || (int32_t)(dloc[okeys[io] & 0xFFFF] >> 32) != a)) {
                    io++;
                }
                const uint64_t ka = ia < m ? akeys[ia] : ~0ull;
                const uint64_t ko = io < so ? okeys[io] : ~0ull;
                if (ka == ~0ull && ko == ~0ull) break;
                if (ka < ko) {
                    const int32_t r = n0 + (int32_t)(ka & 0xFFFF);
                    ia++;
                    if (!temporary && ecol[r].id < 0) continue;   // ID store was full
                    slot[n] = r;
                    where[r] = n;
                    n++;
                } else {
                    const int32_t i = (int32_t)(ko & 0xFFFF);
                    const int32_t r = (int32_t)(uint32_t)dloc[i];
                    io++;
                    if (r < 0 || r >= n_end || where[r] < 0) continue;
                    const int32_t p = where[r];
                    const int32_t q = slot[n - 1];
                    slot[p] = q;
                    where[q] = p;
                    where[r] = -1;
                    n--;
                    dloc[i] = kAppliedOp;
                }
            }
            *n_final = n;
            // the moved rows' per-column word offsets
            *n_moved = 0;
            int32_t words = 0;
            bool dwords = true;
            for (int32_t c = 0; c < av.numColumns; c++) {
                col_words[c] = words;
                words += (int32_t)(av.colBytes[c] / 4);
                dwords = dwords && av.colBytes[c] % 4 == 0;
            }
            col_words[av.numColumns] = dwords ? words : -1;
        }
        commitSync();
        const int32_t nf = *n_final;

        // Rows that changed position.  Few rows move per commit (a destroy
        // moves the last row into the hole), so their words go through the
        // stage in one gather and one scatter for all columns; a move too
        // large for the stage goes column by column through `scratch`.
        int32_t *moved = (int32_t *)akeys;           // the append keys are replayed
        for (int32_t p = lane; p < nf; p += 64) {
            if (slot[p] != p) moved[atomicAdd(n_moved, 1)] = p;
        }
        commitSync();
        const int32_t nm = commitLoad(n_moved);
        const int32_t row_words = col_words[av.numColumns];
        const bool staged = row_words > 0 && (int64_t)nm * row_words <= kCommitStageWords;
        if (staged) {
            const int32_t total = nm * row_words;
            for (int32_t t = lane; t < total; t += 64) {
                const int32_t mi = t / row_words, k = t - mi * row_words;
                int32_t c = 0;
                while (col_words[c + 1] <= k) c++;
                const uint32_t nw = av.colBytes[c] / 4;
                const uint32_t *base = (const uint32_t *)(av.cols[c] + (size_t)w * cap * av.colBytes[c]);
                stage[t] = base[(size_t)slot[moved[mi]] * nw + (k - col_words[c])];
            }
            commitSync();
            for (int32_t t = lane; t < total; t += 64) {
                const int32_t mi = t / row_words, k = t - mi * row_words;
                int32_t c = 0;
                while (col_words[c + 1] <= k) c++;
                const uint32_t nw = av.colBytes[c] / 4;
                uint32_t *base = (uint32_t *)(av.cols[c] + (size_t)w * cap * av.colBytes[c]);
                base[(size_t)moved[mi] * nw + (k - col_words[c])] = stage[t];
            }
            commitSync();
        }
        for (int32_t c = 0; c < av.numColumns && !staged; c++) {
            const uint32_t nb = av.colBytes[c];
            char *base = av.cols[c] + (size_t)w * cap * nb;
            if (nb % 4 == 0) {
                const uint32_t words = nb / 4;
                const int64_t total = (int64_t)nf * words;
                for (int64_t t = lane; t < total; t += 64) {
                    const int32_t p = (int32_t)(t / words), k = (int32_t)(t - (int64_t)p * words);
                    const int32_t src = slot[p];
                    if (src != p) ((uint32_t *)scratch)[t] = ((const uint32_t *)(base + (size_t)src * nb))[k];
                }
                commitSync();
                for (int64_t t = lane; t < total; t += 64) {
                    const int32_t p = (int32_t)(t / words), k = (int32_t)(t - (int64_t)p * words);
                    if (slot[p] != p) ((uint32_t *)(base + (size_t)p * nb))[k] = ((const uint32_t *)scratch)[t];
                }
            } else {
                const int64_t total = (int64_t)nf * nb;
                for (int64_t t = lane; t < total; t += 64) {
                    const int32_t p = (int32_t)(t / nb), k = (int32_t)(t - (int64_t)p * nb);
                    const int32_t src = slot[p];
                    if (src != p) scratch[t] = base[(size_t)src * nb + k];
                }
                commitSync();
                for (int64_t t = lane; t < total; t += 64) {
                    const int32_t p = (int32_t)(t / nb), k = (int32_t)(t - (int64_t)p * nb);
                    if (slot[p] != p) base[(size_t)p * nb + k] = scratch[t];
                }
            }
            commitSync();
        }
        // remap moved / appended entities, settle the keys and the count
        if (!temporary) {
            for (int32_t p = lane; p < nf; p += 64) {
                if (slot[p] != p || p >= n0) {
                    const Entity e = ecol[p];
                    ids.nodes[e.id].val = Loc { (uint32_t)a, p };
                }
            }
        }
        if (keys) {
            for (int32_t r = n0 + lane; r < n_end; r += 64) keys[r] = kNoAppendKey;
        }
        if (lane == 0) {
            av.numRows[w] = nf;
            if (av.pendingRows) av.pendingRows[w] = 0;
        }
        commitSync();
    }

    // 3. ID releases of the applied destroys, in key order
    if (lane == 0) {
        for (int32_t s = 0; s < nops; s++) {
            const int32_t i = (int32_t)(okeys[s] & 0xFFFF);
            if (dloc[i] == kAppliedOp) ids.release(ids.st->worldCache, log[i].e.id);
        }
        st.appendDirty[w] = 0;
        st.deferCount[w] = 0;
    }
    commitSync();
}
#endif

}
