// Host-side ECS registry and arena for the MI355X framework.
//
// Restates the reference's registration semantics (src/core/state.cpp:363-435:
// IDs by registration order, Entity column first, user columns from 1;
// state.inl:171-187: one singleton entity per world from the init cache) and
// lays every archetype out as [world][capacity] column slabs (state.hpp).
#include <madrona/state.hpp>

#if !defined(MW_CPU_BACKEND)
#include <hip/hip_runtime.h>
#endif

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace madrona {

#if !defined(MW_CPU_BACKEND)
#define MW_HIP_CHECK(expr)                                                          \
    do {                                                                            \
        hipError_t err__ = (expr);                                                  \
        if (err__ != hipSuccess) {                                                  \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(err__),    \
                    __FILE__, __LINE__);                                            \
            throw std::runtime_error(hipGetErrorString(err__));                     \
        }                                                                           \
    } while (0)
#endif

struct ArchetypeInfo {
    uint64_t key;
    std::string name;
    std::vector<TypeDesc> cols;     // col 0 = Entity
    int32_t capacity;
    bool temporary;
    bool moduleRows = false;
    bool growable = false;          // registerArchetype without a size (Table::addRow grows it)
    bool pinned = false;            // a module keeps pointers into its slabs
};

struct StateManager::Impl {
    Config cfg;
    std::vector<TypeDesc> components;
    std::vector<ArchetypeInfo> archetypes;
    std::vector<uint64_t> singletons;      // archetype keys, registration order
    std::map<uint64_t, int32_t> capacityHints;
    std::vector<ExportDesc> exports;
    std::vector<std::pair<std::string, std::unique_ptr<StateExtension>>> extensions;

    bool finalized = false;
    StateView host {};
    StateView devHostCopy {};
    StateView *devView = nullptr;

    // host mirror allocations
    std::vector<char *> hostAllocs;
    // device allocations
    std::vector<void *> devAllocs;
    size_t arenaBytes = 0;

    struct ColAlloc { char *host; char *dev; size_t bytes; bool temporary; };
    std::vector<ColAlloc> colAllocs;

    // chained tmpAlloc blocks of the host view, per world
    struct HostTmpOverflow {
        std::vector<std::vector<void *>> blocks;
    };
    std::unique_ptr<HostTmpOverflow> hostOverflow;

    ~Impl()
    {
        if (hostOverflow) {
            for (auto &v : hostOverflow->blocks) {
                for (void *p : v) free(p);
            }
        }
        for (char *p : hostAllocs) free(p);
#if !defined(MW_CPU_BACKEND)
        for (void *p : devAllocs) (void)hipFree(p);
        if (devView) (void)hipFree(devView);
#endif
    }
};

static char *hostAlloc(StateManager::Impl &impl, size_t bytes)
{
    bytes = std::max<size_t>(bytes, 64);
    char *p = (char *)aligned_alloc(256, (bytes + 255) & ~size_t(255));
    if (!p) throw std::runtime_error("host allocation failed");
    memset(p, 0, bytes);
    impl.hostAllocs.push_back(p);
    return p;
}

void *hostTmpOverflowAlloc(StateView &v, int32_t world, uint64_t bytes)
{
    auto *o = (StateManager::Impl::HostTmpOverflow *)v.hostTmpOverflow;
    if (!o || world < 0 || world >= (int32_t)o->blocks.size()) return nullptr;
    void *p = aligned_alloc(256, (bytes + 255) & ~uint64_t(255));
    if (p) o->blocks[world].push_back(p);
    return p;
}

void hostTmpOverflowReset(StateView &v, int32_t world)
{
    auto *o = (StateManager::Impl::HostTmpOverflow *)v.hostTmpOverflow;
    if (!o || world < 0 || world >= (int32_t)o->blocks.size()) return;
    for (void *p : o->blocks[world]) free(p);
    o->blocks[world].clear();
}

ECSRegistry::ECSRegistry(StateManager *state_mgr, void **export_ptrs)
    : state_mgr_(state_mgr), export_ptrs_(export_ptrs)
{}

StateManager::StateManager(const Config &cfg)
    : impl_(new Impl)
{
    impl_->cfg = cfg;
    registerComponent<Entity>();                   // state.cpp:149-156
}

StateManager::~StateManager() { delete impl_; }

uint32_t StateManager::registerComponentDesc(const TypeDesc &desc)
{
    for (size_t i = 0; i < impl_->components.size(); i++) {
        if (impl_->components[i].key == desc.key) return (uint32_t)i;
    }
    impl_->components.push_back(desc);
    return (uint32_t)impl_->components.size() - 1;
}

void StateManager::setCapacityHint(uint64_t key, int32_t capacity)
{
    impl_->capacityHints[key] = capacity;
}

int32_t StateManager::capacityHint(uint64_t key) const
{
    auto it = impl_->capacityHints.find(key);
    return it == impl_->capacityHints.end() ? 0 : it->second;
}

void StateManager::setTemporary(uint64_t key)
{
    for (auto &a : impl_->archetypes) {
        if (a.key == key) a.temporary = true;
    }
}

void StateManager::setModuleRows(uint64_t key)
{
    for (auto &a : impl_->archetypes) {
        if (a.key == key) a.moduleRows = true;
    }
}

void StateManager::pinCapacity(int32_t archetype)
{
    if (archetype >= 0 && archetype < (int32_t)impl_->archetypes.size()) {
        impl_->archetypes[archetype].pinned = true;
    }
}

bool StateManager::growable(int32_t archetype) const
{
    if (archetype < 0 || archetype >= (int32_t)impl_->archetypes.size()) return false;
    const ArchetypeInfo &ai = impl_->archetypes[archetype];
    const bool singleton = std::find(impl_->singletons.begin(), impl_->singletons.end(), ai.key) !=
                           impl_->singletons.end();
    return ai.growable && !ai.pinned && !ai.moduleRows && !singleton;
}

// Entity IDs per world for the current capacities: generous slack because
// per-cache free lists can strand up to 2 x 64 IDs per cache
// (id_map_impl.inl:184-226).
static int32_t idsPerWorldFor(const StateManager::Impl &I)
{
    int64_t needed = 64;
    for (const ArchetypeInfo &ai : I.archetypes) {
        if (!ai.temporary) needed += ai.capacity;
    }
    return (int32_t)(((needed * 2 + 4 * kIDsPerCache) + kIDsPerCache - 1) / kIDsPerCache * kIDsPerCache);
}

// The ordered commit's shape (madrona/commit.hpp): the largest table that
// takes entity rows or row-parallel appends (at most kCommitMaxRows rows per
// world; larger tables raise kErrFlagCommitLimit if a row-parallel node
// mutates them), the key sorts' sizes and the widest column.
static void setCommitShape(StateView &d)
{
    int32_t cap_max = 0;
    uint32_t col_max = 4;
    for (int32_t a = 0; a < d.numArchetypes; a++) {
        const ArchetypeView &av = d.arch[a];
        if (av.flags & kArchModuleRows) continue;
        if (av.capacity > kCommitMaxRows) continue;
        cap_max = std::max(cap_max, av.capacity);
        for (int32_t c = 0; c < av.numColumns; c++) col_max = std::max(col_max, av.colBytes[c]);
    }
    d.commitCapMax = (cap_max + 63) / 64 * 64;
    d.commitSortA = 1;
    while (d.commitSortA < d.commitCapMax) d.commitSortA <<= 1;
    d.commitSortO = 1;
    while (d.commitSortO < d.deferCap) d.commitSortO <<= 1;
    d.commitColMax = col_max;
}

// [W][old_pitch] -> [W][new_pitch] bytes (new_pitch >= old_pitch; the tail
// of each world's new span keeps the destination's fill).
static void restrideHost(char *dst, const char *src, int32_t W, size_t old_pitch, size_t new_pitch)
{
    if (!src) return;
    for (int32_t w = 0; w < W; w++) memcpy(dst + (size_t)w * new_pitch, src + (size_t)w * old_pitch, old_pitch);
}

static void releaseHostAlloc(StateManager::Impl &I, char *p)
{
    auto it = std::find(I.hostAllocs.begin(), I.hostAllocs.end(), p);
    if (it != I.hostAllocs.end()) {
        I.hostAllocs.erase(it);
        free(p);
    }
}

uint32_t StateManager::registerArchetypeDesc(uint64_t key, const char *name,
                                             const TypeDesc *comps, int32_t num_comps,
                                             int32_t capacity, bool temporary)
{
    if (impl_->finalized) throw std::runtime_error("registerArchetype after finalize");
    for (size_t i = 0; i < impl_->archetypes.size(); i++) {
        if (impl_->archetypes[i].key == key) return (uint32_t)i;
    }
    if ((int32_t)impl_->archetypes.size() >= kMaxArchetypes) {
        throw std::runtime_error("too many archetypes");
    }
    if (num_comps + 1 > kMaxColumns) throw std::runtime_error("too many columns");
    ArchetypeInfo a;
    a.key = key;
    a.name = name;
    a.cols.push_back(impl_->components[0]);        // Entity column
    for (int32_t i = 0; i < num_comps; i++) {
        registerComponentDesc(comps[i]);
        a.cols.push_back(comps[i]);
    }
    if (capacity <= 0) capacity = capacityHint(key);
    a.growable = capacity <= 0;
    if (capacity <= 0) capacity = impl_->cfg.defaultCapacity;
    a.capacity = capacity;
    a.temporary = temporary;
    impl_->archetypes.push_back(std::move(a));
    return (uint32_t)impl_->archetypes.size() - 1;
}

void StateManager::registerSingletonDesc(uint64_t archetype_key)
{
    impl_->singletons.push_back(archetype_key);
}

int32_t StateManager::archetypeIndex(uint64_t key) const
{
    for (size_t i = 0; i < impl_->archetypes.size(); i++) {
        if (impl_->archetypes[i].key == key) return (int32_t)i;
    }
    return -1;
}

int32_t StateManager::numArchetypes() const { return (int32_t)impl_->archetypes.size(); }
int32_t StateManager::numWorlds() const { return impl_->cfg.numWorlds; }

void StateManager::registerExport(int32_t slot, uint64_t archetype_key, uint64_t component_key)
{
    int32_t a = archetypeIndex(archetype_key);
    if (a < 0) throw std::runtime_error("exportColumn: archetype not registered");
    const ArchetypeInfo &ai = impl_->archetypes[a];
    int32_t col = -1;
    for (size_t c = 0; c < ai.cols.size(); c++) {
        if (ai.cols[c].key == component_key) { col = (int32_t)c; break; }
    }
    if (col < 0) throw std::runtime_error("exportColumn: component not in archetype");
    impl_->exports.push_back(ExportDesc { slot, a, col, ai.cols[col].numBytes });
}

const StateManager::ExportDesc *StateManager::exports(int32_t *num) const
{
    *num = (int32_t)impl_->exports.size();
    return impl_->exports.data();
}

bool StateManager::finalized() const { return impl_->finalized; }
StateView &StateManager::hostView() { return impl_->host; }
const StateView &StateManager::hostViewConst() const { return impl_->host; }
StateView *StateManager::deviceView() const { return impl_->devView; }
const StateView &StateManager::deviceViewHost() const { return impl_->devHostCopy; }

void StateManager::finalizeLayout(uint32_t world_data_bytes, uint32_t world_data_align)
{
    Impl &I = *impl_;
    if (I.finalized) return;
    const int32_t W = I.cfg.numWorlds;
    StateView &v = I.host;
    memset(&v, 0, sizeof(v));
    v.numWorlds = W;
    v.numArchetypes = (int32_t)I.archetypes.size();

    int64_t ids_needed = 64;
    for (int32_t a = 0; a < v.numArchetypes; a++) {
        const ArchetypeInfo &ai = I.archetypes[a];
        ArchetypeView &av = v.arch[a];
        v.archKeys[a] = ai.key;
        av.numColumns = (int32_t)ai.cols.size();
        av.capacity = ai.capacity;
        av.flags = (ai.temporary ? kArchTemporary : 0u) | (ai.moduleRows ? kArchModuleRows : 0u) |
                   (ai.growable && !ai.moduleRows ? kArchGrowable : 0u);
        if (std::find(I.singletons.begin(), I.singletons.end(), ai.key) != I.singletons.end()) {
            av.flags |= kArchSingleton;
        }
        av.numRows = (int32_t *)hostAlloc(I, sizeof(int32_t) * W);
        for (int32_t c = 0; c < av.numColumns; c++) {
            size_t bytes = (size_t)W * ai.capacity * ai.cols[c].numBytes;
            av.colBytes[c] = ai.cols[c].numBytes;
            av.colKeys[c] = ai.cols[c].key;
            // Temporaries start empty: no host mirror, the device slab is
            // zero-filled at upload.
            av.cols[c] = ai.temporary ? nullptr : hostAlloc(I, bytes);
            I.colAllocs.push_back(Impl::ColAlloc { av.cols[c], nullptr, bytes, ai.temporary });
        }
        if (!ai.temporary) ids_needed += ai.capacity;
    }

    // Entity IDs per world (idsPerWorldFor)
    (void)ids_needed;
    const int64_t ids = idsPerWorldFor(I);
    v.idsPerWorld = (int32_t)ids;
    v.idNodes = (IDNode *)hostAlloc(I, sizeof(IDNode) * (size_t)W * ids);
    v.idState = (IDMapState *)hostAlloc(I, sizeof(IDMapState) * W);
    for (int32_t w = 0; w < W; w++) {
        v.idState[w].globalHead = -1;
        v.idState[w].numIDs = 0;
        v.idState[w].worldCache = IDCache { -1, 0, -1, 0 };
        v.idState[w].initCache = IDCache { -1, 0, -1, 0 };
    }
    uint32_t align = std::max<uint32_t>(world_data_align, 16);
    v.worldDataStride = (std::max<uint32_t>(world_data_bytes, 16) + align - 1) / align * align;
    v.worldData = hostAlloc(I, (size_t)v.worldDataStride * W);
    v.errorFlags = (int32_t *)hostAlloc(I, sizeof(int32_t) * W);
    // Per-world tmpAlloc arena (also used by world constructors on the host).
    v.tmpBytesPerWorld = (uint32_t)std::max(0, I.cfg.tmpAllocBytesPerWorld) / 256 * 256;
    if (v.tmpBytesPerWorld > 0) {
        v.tmpArena = hostAlloc(I, (size_t)v.tmpBytesPerWorld * W);
        v.tmpOffset = (uint32_t *)hostAlloc(I, sizeof(uint32_t) * W);
    }
    if (I.cfg.tmpPoolBytes > 0) {
        I.hostOverflow.reset(new Impl::HostTmpOverflow);
        I.hostOverflow->blocks.resize(W);
        v.hostTmpOverflow = I.hostOverflow.get();
    }
    v.deferCap = std::max(1, I.cfg.deferCap);

    // Singleton entities, per world in registration order, from the init
    // cache (state.inl:171-187).  Single-world semantics: each world's IDs
    // start at 0.
    for (uint64_t skey : I.singletons) {
        int32_t a = archetypeIndex(skey);
        for (int32_t w = 0; w < W; w++) {
            IDMapView idv = v.ids(w);
            Entity e = idv.acquire(idv.st->initCache);
            int32_t row = v.addRow(a, w);
            v.column<Entity>(a, 0, w)[row] = e;
            idv.nodes[e.id].val = Loc { (uint32_t)a, row };
        }
    }
    I.finalized = true;
}

#if defined(MW_CPU_BACKEND)
// CPU back end: the host mirror IS the arena.  Temporaries get their
// (zero-filled) slabs now, the "device" view is the host view, and the
// module extensions build their slabs in host memory.
void StateManager::uploadToDevice(void *stream_ptr)
{
    Impl &I = *impl_;
    StateView &h = I.host;
    size_t ci = 0;
    for (int32_t a = 0; a < h.numArchetypes; a++) {
        for (int32_t c = 0; c < h.arch[a].numColumns; c++, ci++) {
            Impl::ColAlloc &ca = I.colAllocs[ci];
            if (!ca.host) {
                ca.host = hostAlloc(I, ca.bytes);
                h.arch[a].cols[c] = ca.host;
            }
        }
    }
    I.devView = &I.host;
    I.devHostCopy = I.host;
    for (auto &ext : I.extensions) ext.second->upload(stream_ptr);
}

void StateManager::downloadFromDevice(void *) {}
#else
void StateManager::uploadToDevice(void *stream_ptr)
{
    Impl &I = *impl_;
    hipStream_t stream = (hipStream_t)stream_ptr;
    const int32_t W = I.cfg.numWorlds;
    StateView d = I.host;

    auto devAlloc = [&](size_t bytes) -> char * {
        void *p = nullptr;
        MW_HIP_CHECK(hipMalloc(&p, std::max<size_t>(bytes, 256)));
        I.devAllocs.push_back(p);
        I.arenaBytes += bytes;
        return (char *)p;
    };
    auto copy = [&](void *dst, const void *src, size_t bytes) {
        MW_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, stream));
    };

    size_t ci = 0;
    for (int32_t a = 0; a < d.numArchetypes; a++) {
        ArchetypeView &av = d.arch[a];
        av.numRows = (int32_t *)devAlloc(sizeof(int32_t) * W);
        copy(av.numRows, I.host.arch[a].numRows, sizeof(int32_t) * W);
        for (int32_t c = 0; c < av.numColumns; c++, ci++) {
            Impl::ColAlloc &ca = I.colAllocs[ci];
            ca.dev = devAlloc(ca.bytes);
            if (ca.temporary) {
                MW_HIP_CHECK(hipMemsetAsync(ca.dev, 0, ca.bytes, stream));
            } else {
                copy(ca.dev, ca.host, ca.bytes);
            }
            av.cols[c] = ca.dev;
        }
    }
    d.idNodes = (IDNode *)devAlloc(sizeof(IDNode) * (size_t)W * d.idsPerWorld);
    copy(d.idNodes, I.host.idNodes, sizeof(IDNode) * (size_t)W * d.idsPerWorld);
    d.idState = (IDMapState *)devAlloc(sizeof(IDMapState) * W);
    copy(d.idState, I.host.idState, sizeof(IDMapState) * W);
    d.worldData = devAlloc((size_t)d.worldDataStride * W);
    copy(d.worldData, I.host.worldData, (size_t)d.worldDataStride * W);
    d.errorFlags = (int32_t *)devAlloc(sizeof(int32_t) * W);
    copy(d.errorFlags, I.host.errorFlags, sizeof(int32_t) * W);

    // Row-parallel structural mutation (Context): append keys for every
    // table a lane may append to (not singletons, not module-written rows,
    // at most 4096 rows: the ordered commit's LDS index arrays), all keys
    // settled (kNoAppendKey = all ones); the deferred destroy log.
    for (int32_t a = 0; a < d.numArchetypes; a++) {
        ArchetypeView &av = d.arch[a];
        av.appendKeys = nullptr;
        av.pendingRows = nullptr;
        const bool singleton = std::find(I.singletons.begin(), I.singletons.end(),
                                         I.archetypes[a].key) != I.singletons.end();
        if (singleton || (av.flags & kArchModuleRows) || av.capacity > 4096) continue;
        const size_t bytes = sizeof(uint64_t) * (size_t)W * av.capacity;
        av.appendKeys = (uint64_t *)devAlloc(bytes);
        MW_HIP_CHECK(hipMemsetAsync(av.appendKeys, 0xFF, bytes, stream));
        av.pendingRows = (int32_t *)devAlloc(sizeof(int32_t) * W);
        MW_HIP_CHECK(hipMemsetAsync(av.pendingRows, 0, sizeof(int32_t) * W, stream));
    }
    d.appendDirty = (uint64_t *)devAlloc(sizeof(uint64_t) * W);
    MW_HIP_CHECK(hipMemsetAsync(d.appendDirty, 0, sizeof(uint64_t) * W, stream));
    d.deferCount = (int32_t *)devAlloc(sizeof(int32_t) * W);
    MW_HIP_CHECK(hipMemsetAsync(d.deferCount, 0, sizeof(int32_t) * W, stream));
    d.deferLog = (DeferredDestroy *)devAlloc(sizeof(DeferredDestroy) * (size_t)W * d.deferCap);
    const size_t turn_bytes = sizeof(int32_t) * kMakeTurnSlots * kMakeTurnWaves * W;
    d.makeTurn = (int32_t *)devAlloc(turn_bytes);
    MW_HIP_CHECK(hipMemsetAsync(d.makeTurn, 0, turn_bytes, stream));
    d.makeEpoch = (int32_t *)devAlloc(sizeof(int32_t));
    setCommitShape(d);
    {
        const int32_t first_epoch = 1;
        copy(d.makeEpoch, &first_epoch, sizeof(int32_t));
    }
    if (d.tmpBytesPerWorld > 0) {
        d.tmpArena = devAlloc((size_t)d.tmpBytesPerWorld * W);
        copy(d.tmpArena, I.host.tmpArena, (size_t)d.tmpBytesPerWorld * W);
        d.tmpOffset = (uint32_t *)devAlloc(sizeof(uint32_t) * W);
        copy(d.tmpOffset, I.host.tmpOffset, sizeof(uint32_t) * W);
    }
    d.hostTmpOverflow = nullptr;
    d.tmpPool = nullptr;
    d.tmpPoolOffset = nullptr;
    d.tmpPoolBytes = 0;
    if (I.cfg.tmpPoolBytes > 0) {
        d.tmpPoolBytes = (uint64_t)I.cfg.tmpPoolBytes / 256 * 256;
        d.tmpPool = devAlloc(d.tmpPoolBytes);
        d.tmpPoolOffset = (unsigned long long *)devAlloc(sizeof(unsigned long long));
        MW_HIP_CHECK(hipMemsetAsync(d.tmpPoolOffset, 0, sizeof(unsigned long long), stream));
    }

    MW_HIP_CHECK(hipMalloc(&I.devView, sizeof(StateView)));
    copy(I.devView, &d, sizeof(StateView));
    I.devHostCopy = d;

    for (auto &ext : I.extensions) ext.second->upload(stream_ptr);
    MW_HIP_CHECK(hipStreamSynchronize(stream));
}

void StateManager::downloadFromDevice(void *stream_ptr)
{
    Impl &I = *impl_;
    hipStream_t stream = (hipStream_t)stream_ptr;
    const int32_t W = I.cfg.numWorlds;
    const StateView &d = I.devHostCopy;
    StateView &h = I.host;
    size_t ci = 0;
    for (int32_t a = 0; a < d.numArchetypes; a++) {
        MW_HIP_CHECK(hipMemcpyAsync(h.arch[a].numRows, d.arch[a].numRows, sizeof(int32_t) * W,
                                    hipMemcpyDeviceToHost, stream));
        for (int32_t c = 0; c < d.arch[a].numColumns; c++, ci++) {
            Impl::ColAlloc &ca = I.colAllocs[ci];
            if (!ca.host) {
                ca.host = hostAlloc(I, ca.bytes);
                h.arch[a].cols[c] = ca.host;
            }
            MW_HIP_CHECK(hipMemcpyAsync(ca.host, ca.dev, ca.bytes, hipMemcpyDeviceToHost, stream));
        }
    }
    MW_HIP_CHECK(hipMemcpyAsync(h.idNodes, d.idNodes, sizeof(IDNode) * (size_t)W * d.idsPerWorld,
                                hipMemcpyDeviceToHost, stream));
    MW_HIP_CHECK(hipMemcpyAsync(h.idState, d.idState, sizeof(IDMapState) * W,
                                hipMemcpyDeviceToHost, stream));
    MW_HIP_CHECK(hipMemcpyAsync(h.errorFlags, d.errorFlags, sizeof(int32_t) * W,
                                hipMemcpyDeviceToHost, stream));
    MW_HIP_CHECK(hipMemcpyAsync(h.worldData, d.worldData, (size_t)d.worldDataStride * W,
                                hipMemcpyDeviceToHost, stream));
    MW_HIP_CHECK(hipStreamSynchronize(stream));
}
#endif

// Table growth (see state.hpp).  Row i of world w moves from w * cap + i to
// w * new_cap + i in every column; rows past a world's count keep no
// meaning (zero-filled), appended-row keys past it stay settled.
void StateManager::growArchetype(int32_t a, int32_t new_cap, void *stream_ptr)
{
    Impl &I = *impl_;
    if (!growable(a)) throw std::runtime_error("growArchetype: archetype " + std::to_string(a) + " is not growable");
    ArchetypeInfo &ai = I.archetypes[a];
    const int32_t cap = ai.capacity;
    if (new_cap <= cap) return;
    const int32_t W = I.cfg.numWorlds;
    StateView &h = I.host;
    size_t ci = 0;
    for (int32_t b = 0; b < a; b++) ci += I.archetypes[b].cols.size();
    const int32_t old_ids = h.idsPerWorld;
    ai.capacity = new_cap;
    const int32_t new_ids = std::max(old_ids, idsPerWorldFor(I));

    // host mirror (the arena itself on the CPU back end)
    for (size_t c = 0; c < ai.cols.size(); c++) {
        Impl::ColAlloc &ca = I.colAllocs[ci + c];
        const size_t nb = ai.cols[c].numBytes, bytes = (size_t)W * new_cap * nb;
        if (ca.host) {
            char *nh = hostAlloc(I, bytes);
            restrideHost(nh, ca.host, W, (size_t)cap * nb, (size_t)new_cap * nb);
            releaseHostAlloc(I, ca.host);
            ca.host = nh;
            h.arch[a].cols[c] = nh;
        }
    }
    h.arch[a].capacity = new_cap;
    if (new_ids > old_ids) {
        char *nh = hostAlloc(I, sizeof(IDNode) * (size_t)W * new_ids);
        restrideHost(nh, (const char *)h.idNodes, W, sizeof(IDNode) * old_ids, sizeof(IDNode) * new_ids);
        releaseHostAlloc(I, (char *)h.idNodes);
        h.idNodes = (IDNode *)nh;
        h.idsPerWorld = new_ids;
    }

#if defined(MW_CPU_BACKEND)
    (void)stream_ptr;
    for (size_t c = 0; c < ai.cols.size(); c++) I.colAllocs[ci + c].bytes = (size_t)W * new_cap * ai.cols[c].numBytes;
    I.devHostCopy = I.host;
    for (auto &ext : I.extensions) ext.second->stateResized();
#else
    hipStream_t stream = (hipStream_t)stream_ptr;
    StateView &d = I.devHostCopy;
    std::vector<void *> retired;
    // a fresh device slab filled with `fill`, registered for release
    auto devSlab = [&](size_t bytes, int fill) -> char * {
        void *p = nullptr;
        MW_HIP_CHECK(hipMalloc(&p, std::max<size_t>(bytes, 256)));
        MW_HIP_CHECK(hipMemsetAsync(p, fill, std::max<size_t>(bytes, 256), stream));
        I.devAllocs.push_back(p);
        I.arenaBytes += bytes;
        return (char *)p;
    };
    auto retire = [&](void *old) {
        auto it = std::find(I.devAllocs.begin(), I.devAllocs.end(), old);
        if (it != I.devAllocs.end()) I.devAllocs.erase(it);
        retired.push_back(old);
    };
    auto restride = [&](char *dst, const void *src, size_t old_pitch, size_t new_pitch) {
        MW_HIP_CHECK(hipMemcpy2DAsync(dst, new_pitch, src, old_pitch, old_pitch, (size_t)W,
                                      hipMemcpyDeviceToDevice, stream));
    };
    for (size_t c = 0; c < ai.cols.size(); c++) {
        Impl::ColAlloc &ca = I.colAllocs[ci + c];
        const size_t nb = ai.cols[c].numBytes, bytes = (size_t)W * new_cap * nb;
        char *nd = devSlab(bytes, 0);
        restride(nd, ca.dev, (size_t)cap * nb, (size_t)new_cap * nb);
        retire(ca.dev);
        ca.dev = nd;
        ca.bytes = bytes;
        d.arch[a].cols[c] = nd;
    }
    d.arch[a].capacity = new_cap;
    if (d.arch[a].appendKeys) {
        uint64_t *old = d.arch[a].appendKeys;
        // the same limit as at upload: the ordered commit's index arrays
        if (new_cap <= kCommitMaxRows) {
            char *nk = devSlab(sizeof(uint64_t) * (size_t)W * new_cap, 0xFF);
            restride(nk, old, sizeof(uint64_t) * cap, sizeof(uint64_t) * new_cap);
            d.arch[a].appendKeys = (uint64_t *)nk;
        } else {
            d.arch[a].appendKeys = nullptr;     // row-parallel appends now flag (kErrFlagRowParallelOp)
        }
        retire(old);
    }
    if (new_ids > old_ids) {
        char *ni = devSlab(sizeof(IDNode) * (size_t)W * new_ids, 0);
        restride(ni, d.idNodes, sizeof(IDNode) * old_ids, sizeof(IDNode) * new_ids);
        retire(d.idNodes);
        d.idNodes = (IDNode *)ni;
        d.idsPerWorld = new_ids;
    }
    setCommitShape(d);
    h.commitCapMax = d.commitCapMax;
    h.commitSortA = d.commitSortA;
    h.commitSortO = d.commitSortO;
    h.commitColMax = d.commitColMax;
    MW_HIP_CHECK(hipMemcpyAsync(I.devView, &d, sizeof(StateView), hipMemcpyHostToDevice, stream));
    MW_HIP_CHECK(hipStreamSynchronize(stream));
    for (void *p : retired) MW_HIP_CHECK(hipFree(p));
    for (auto &ext : I.extensions) ext.second->stateResized();
#endif
}

int32_t StateManager::resolveQuery(const uint64_t *keys, int32_t num_keys,
                                   int32_t *out_archetypes, int32_t *out_cols,
                                   int32_t max_out) const
{                                       // src/core/state.cpp:270-361
    const uint64_t entity_key = typeKey<Entity>();
    int32_t n = 0;
    for (size_t a = 0; a < impl_->archetypes.size(); a++) {
        const ArchetypeInfo &ai = impl_->archetypes[a];
        int32_t cols[32];
        bool ok = true;
        for (int32_t k = 0; k < num_keys && ok; k++) {
            if (keys[k] == entity_key) { cols[k] = 0; continue; }
            int32_t found = -1;
            for (size_t c = 1; c < ai.cols.size(); c++) {
                if (ai.cols[c].key == keys[k]) { found = (int32_t)c; break; }
            }
            if (found < 0) ok = false;
            cols[k] = found;
        }
        if (!ok) continue;
        if (n >= max_out) throw std::runtime_error("query matches too many archetypes");
        out_archetypes[n] = (int32_t)a;
        for (int32_t k = 0; k < num_keys; k++) out_cols[n * 12 + k] = cols[k];
        n++;
    }
    return n;
}

void StateManager::setExtension(const char *name, StateExtension *ext)
{
    for (auto &e : impl_->extensions) {
        if (e.first == name) {
            e.second.reset(ext);
            return;
        }
    }
    impl_->extensions.emplace_back(name, std::unique_ptr<StateExtension>(ext));
}

bool StateManager::pollExtensions(void *stream, int64_t steps)
{
    bool recapture = false;
    for (auto &e : impl_->extensions) recapture |= e.second->poll(stream, steps);
    return recapture;
}

StateExtension *StateManager::getExtension(const char *name) const
{
    for (auto &e : impl_->extensions) {
        if (e.first == name) return e.second.get();
    }
    return nullptr;
}

}
