// C ABI (include/madrona_mw.h) over the MI355X executor.  The same source
// builds the CPU back end's ABI (libmadrona_cpu.so, MW_CPU_BACKEND): the
// arena is host memory there, and the RCCL / stream entry points report
// that they are gfx950 features.
#include "../../../include/madrona_mw.h"

#include "env_registry.hpp"
#include "../physics/physics_impl.hpp"
#include "../physics/physics_module.hpp"

#include <madrona/mw_gpu.hpp>
#include <madrona/launch_config.hpp>
#include <madrona/physics_assets.hpp>

#if !defined(MW_CPU_BACKEND)
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#endif

#include <dlfcn.h>

#include <algorithm>
#include <cstring>
#include <exception>
#include <map>
#include <string>
#include <vector>

#if !defined(MW_CPU_BACKEND)
// RCCL is resolved at first use (dlopen of librccl.so.1) rather than linked:
// a process that already holds an RCCL (PyTorch's bundled one) shares it and
// its HIP runtime instead of mapping a second copy next to it.
struct RcclApi {
    ncclResult_t (*getUniqueId)(ncclUniqueId *);
    ncclResult_t (*commInitRank)(ncclComm_t *, int, ncclUniqueId, int);
    ncclResult_t (*allGather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t,
                              hipStream_t);
    ncclResult_t (*commDestroy)(ncclComm_t);
    const char *(*getErrorString)(ncclResult_t);
};

static const RcclApi &rccl()
{
    static RcclApi api = []() {
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) throw std::runtime_error(std::string("RCCL unavailable: ") + dlerror());
        auto sym = [h](const char *name) {
            void *f = dlsym(h, name);
            if (!f) throw std::runtime_error(std::string("RCCL symbol missing: ") + name);
            return f;
        };
        RcclApi a;
        a.getUniqueId = (decltype(a.getUniqueId))sym("ncclGetUniqueId");
        a.commInitRank = (decltype(a.commInitRank))sym("ncclCommInitRank");
        a.allGather = (decltype(a.allGather))sym("ncclAllGather");
        a.commDestroy = (decltype(a.commDestroy))sym("ncclCommDestroy");
        a.getErrorString = (decltype(a.getErrorString))sym("ncclGetErrorString");
        return a;
    }();
    return api;
}

#endif

namespace madrona {
namespace phys { PhysArgs *physicsArgs(StateManager &mgr); }

static std::map<std::string, EnvFactory> &envTable()
{
    static std::map<std::string, EnvFactory> t;
    return t;
}

// Names an object tried to register that were already taken (mw_load_env
// reports them).
static std::vector<std::string> &envClashes()
{
    static std::vector<std::string> v;
    return v;
}

EnvRegistration::EnvRegistration(const char *name, EnvFactory factory)
{
    // A name registered twice (two loaded objects defining one world) keeps
    // the first factory; mw_load_env reports the clash.
    if (!envTable().emplace(name, factory).second) envClashes().push_back(name);
}

static std::vector<std::string> envNames()
{
    std::vector<std::string> v;
    for (auto &e : envTable()) v.push_back(e.first);
    return v;
}

EnvFactory findEnv(const char *name)
{
    auto it = envTable().find(name);
    return it == envTable().end() ? nullptr : it->second;
}

int32_t loadEnvObject(const char *so_path)
{
    if (!so_path) throw std::runtime_error("mw_load_env: null path");
    const size_t before = envTable().size();
    envClashes().clear();
    // RTLD_NOW: unresolved symbols fail here, not at the first step.
    // The object's DT_NEEDED libmadrona_mw.so resolves to this loaded
    // library by its soname, so the world registers into this table.
    void *h = dlopen(so_path, RTLD_NOW | RTLD_LOCAL);
    if (!h) throw std::runtime_error(std::string("mw_load_env: ") + dlerror());
    if (!envClashes().empty()) {
        std::string names;
        for (const std::string &n : envClashes()) names += (names.empty() ? "'" : ", '") + n + "'";
        envClashes().clear();
        throw std::runtime_error(std::string("mw_load_env: ") + so_path + " registers " + names +
                                 ", already registered by another object (the first one stays)");
    }
    return (int32_t)(envTable().size() - before);
}

}

using namespace madrona;

struct mw_exec {
    Executor *exec;
#if !defined(MW_CPU_BACKEND)
    int32_t gpu = 0;              // HIP device of the executor (mw_config.gpu_id)
    ncclComm_t comm = nullptr;    // RCCL communicator for the world-shard hand-off
    hipEvent_t stepDone = nullptr; // mw_stream_wait: recorded behind the enqueued steps
#endif
};

static thread_local std::string g_last_error;

static void setError(const char *what) { g_last_error = what ? what : "unknown error"; }

#define MW_TRY(body, fail)                                 \
    try {                                                  \
        body                                               \
    } catch (const std::exception &e) {                    \
        setError(e.what());                                \
        return fail;                                       \
    } catch (...) {                                        \
        setError("unknown exception");                     \
        return fail;                                       \
    }

#if !defined(MW_CPU_BACKEND)
#define MW_HIP_OK(expr)                                                  \
    do {                                                                 \
        hipError_t e__ = (expr);                                         \
        if (e__ != hipSuccess) throw std::runtime_error(hipGetErrorString(e__)); \
    } while (0)

// Arena (device) -> caller (host) read-back.
static void copyOut(void *dst, const void *src, size_t bytes)
{
    MW_HIP_OK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
}
static void zeroArena(void *dst, size_t bytes)
{
    MW_HIP_OK(hipMemset(dst, 0, bytes));
}
#else
static void copyOut(void *dst, const void *src, size_t bytes) { memcpy(dst, src, bytes); }
static void zeroArena(void *dst, size_t bytes) { memset(dst, 0, bytes); }

[[noreturn]] static void gfx950Only(const char *what)
{
    throw std::runtime_error(std::string(what) + " is a gfx950 feature (libmadrona_mw.so); "
                             "the CPU back end steps synchronously in host memory");
}
#endif

extern "C" {

mw_exec *mw_create(const char *env, const mw_config *cfg, const void *user_cfg,
                   size_t user_cfg_bytes, const void *inits, size_t init_stride)
{
    MW_TRY({
        if (!env || !cfg) throw std::runtime_error("mw_create: null argument");
        // ABI check: a caller built against another include/madrona_mw.h
        // (or one that left the header fields unset) is refused before any
        // other field is read
        if (cfg->struct_size != sizeof(mw_config) || cfg->abi_version != MW_ABI_VERSION) {
            throw std::runtime_error(
                "mw_create: mw_config.struct_size " + std::to_string(cfg->struct_size) +
                " / abi_version " + std::to_string(cfg->abi_version) + " not supported (this "
                "library: struct_size " + std::to_string(sizeof(mw_config)) + ", abi_version " +
                std::to_string(MW_ABI_VERSION) + "); initialise with MW_CONFIG_INIT");
        }
        EnvFactory f = findEnv(env);
        if (!f) throw std::runtime_error(std::string("mw_create: unknown environment '") + env + "'");
        if (cfg->num_worlds <= 0) throw std::runtime_error("mw_create: num_worlds must be > 0");
#if !defined(MW_CPU_BACKEND)
        int ndev = 0;
        MW_HIP_OK(hipGetDeviceCount(&ndev));
        if (cfg->gpu_id < 0 || cfg->gpu_id >= ndev) {
            throw std::runtime_error("mw_create: no HIP device " + std::to_string(cfg->gpu_id));
        }
#endif
        if (cfg->num_workers < 0) throw std::runtime_error("mw_create: num_workers must be >= 0");
        ExecConfig ec;
        ec.numWorlds = cfg->num_worlds;
        ec.gpuID = cfg->gpu_id;
        ec.defaultCapacity = cfg->default_capacity > 0 ? cfg->default_capacity : 64;
        ec.numExportedBuffers = 0;
        ec.useGraph = cfg->use_graph;
        // C ABI: 0 = default, -1 = none (a zero-initialised mw_config gets
        // the default arena); ExecConfig: -1 = default, 0 = none
        ec.tmpAllocBytesPerWorld = cfg->tmp_alloc_bytes == 0    ? -1
                                   : cfg->tmp_alloc_bytes == -1 ? 0
                                                                : cfg->tmp_alloc_bytes;
        ec.maxDeferredPerWorld = cfg->max_deferred_destroys;
        ec.numWorkers = cfg->num_workers;
        ec.serialNodes = cfg->serial_nodes != 0;
        if (cfg->tmp_pool_bytes < -1) throw std::runtime_error("mw_create: tmp_pool_bytes >= -1");
        ec.tmpPoolBytes = cfg->tmp_pool_bytes == 0 ? -1 : cfg->tmp_pool_bytes == -1 ? 0 : cfg->tmp_pool_bytes;
        if (cfg->tmp_alloc_bytes < -1 || cfg->max_deferred_destroys < 0 ||
            cfg->max_deferred_destroys > 65536) {
            throw std::runtime_error("mw_create: tmp_alloc_bytes >= -1 and 0 <= max_deferred_destroys <= 65536");
        }
        Executor *e = f(ec, user_cfg, user_cfg_bytes, inits, init_stride);
        mw_exec *x = new mw_exec { e };
#if !defined(MW_CPU_BACKEND)
        x->gpu = cfg->gpu_id;
#endif
        return x;
    }, nullptr)
}

int32_t mw_load_env(const char *so_path)
{
    MW_TRY({ return loadEnvObject(so_path); }, -1)
}

int32_t mw_num_envs(void) { return (int32_t)envTable().size(); }

const char *mw_env_name(int32_t i)
{
    static thread_local std::string name;
    const std::vector<std::string> v = envNames();
    if (i < 0 || i >= (int32_t)v.size()) return nullptr;
    name = v[i];
    return name.c_str();
}

int mw_step(mw_exec *exec, int32_t num_steps)
{
    MW_TRY({
        exec->exec->runSteps(num_steps);
        exec->exec->sync();
        return 0;
    }, -1)
}

int mw_step_async(mw_exec *exec, int32_t num_steps)
{
    MW_TRY({
        exec->exec->runSteps(num_steps);
        return 0;
    }, -1)
}

int mw_sync(mw_exec *exec)
{
    MW_TRY({ exec->exec->sync(); return 0; }, -1)
}

void *mw_get_exported(mw_exec *exec, int32_t slot, int64_t *num_rows)
{
    MW_TRY({ return exec->exec->getExported(slot, num_rows); }, nullptr)
}

int64_t mw_copy_exported(mw_exec *exec, int32_t slot, void *dst, int64_t max_bytes)
{
    MW_TRY({
        // dst may be device or host memory (unified addressing)
        const int64_t n = exec->exec->copyExported(slot, dst, max_bytes);
        if (n < 0) throw std::runtime_error("mw_copy_exported: no such export slot");
        return n;
    }, (int64_t)-1)
}

int64_t mw_copy_exported_async(mw_exec *exec, int32_t slot, void *dst, int64_t max_bytes)
{
    MW_TRY({
        const int64_t n = exec->exec->copyExportedAsync(slot, dst, max_bytes);
        if (n < 0) throw std::runtime_error("mw_copy_exported_async: no such export slot");
        return n;
    }, (int64_t)-1)
}

void *mw_stream(mw_exec *exec) { return exec ? exec->exec->stream() : nullptr; }

int mw_stream_wait(mw_exec *exec, void *stream)
{
    MW_TRY({
#if defined(MW_CPU_BACKEND)
        (void)exec; (void)stream;          // steps complete before mw_step returns
#else
        if (!exec->stepDone) {
            MW_HIP_OK(hipEventCreateWithFlags(&exec->stepDone, hipEventDisableTiming));
        }
        MW_HIP_OK(hipEventRecord(exec->stepDone, (hipStream_t)exec->exec->stream()));
        MW_HIP_OK(hipStreamWaitEvent((hipStream_t)stream, exec->stepDone, 0));
#endif
        return 0;
    }, -1)
}

int mw_destroy(mw_exec *exec)
{
    MW_TRY({
        if (exec) {
#if !defined(MW_CPU_BACKEND)
            if (exec->comm) (void)rccl().commDestroy(exec->comm);
            if (exec->stepDone) (void)hipEventDestroy(exec->stepDone);
#endif
            delete exec->exec;
            delete exec;
        }
        return 0;
    }, -1)
}

const char *mw_last_error(void) { return g_last_error.c_str(); }

int mw_load_hull(const char *obj_path, int32_t *counts_out, float *aabb_out, float *verts_out,
                 int32_t vert_cap, float *planes_out, int32_t face_cap, uint32_t *half_edges_out,
                 int32_t half_edge_cap)
{
    MW_TRY({
        if (!obj_path || !counts_out || !aabb_out) throw std::runtime_error("mw_load_hull: null argument");
        madrona::phys::PhysicsLoader loader(madrona::phys::PhysicsLoader::StorageType::CPU, 1);
        madrona::phys::PhysicsLoader::LoadedHull h = loader.loadHullFromDisk(obj_path);
        const madrona::phys::geometry::HalfEdgeMesh &m = h.collisionMesh;
        counts_out[0] = (int32_t)m.mVertexCount;
        counts_out[1] = (int32_t)m.mPolygonCount;
        counts_out[2] = (int32_t)m.mEdgeCount;
        counts_out[3] = (int32_t)m.mHalfEdgeCount;
        memcpy(aabb_out, &h.aabb.pMin, 12);
        memcpy(aabb_out + 3, &h.aabb.pMax, 12);
        if ((int64_t)m.mVertexCount > vert_cap || (int64_t)m.mPolygonCount > face_cap ||
            (int64_t)m.mHalfEdgeCount > half_edge_cap) {
            return -2;
        }
        if (verts_out) memcpy(verts_out, m.mVertices, 12 * (size_t)m.mVertexCount);
        if (planes_out) memcpy(planes_out, m.mFacePlanes, 16 * (size_t)m.mPolygonCount);
        if (half_edges_out) memcpy(half_edges_out, m.mHalfEdges, 16 * (size_t)m.mHalfEdgeCount);
        return 0;
    }, -1)
}

// ---------------------------------------------------------------------------
// Training hand-off across world shards: RCCL over xGMI, issued on the
// executor's stream right behind the step that produced the export.
// ---------------------------------------------------------------------------
#if !defined(MW_CPU_BACKEND)
#define MW_NCCL_OK(expr)                                                     \
    do {                                                                     \
        ncclResult_t r__ = (expr);                                           \
        if (r__ != ncclSuccess) throw std::runtime_error(rccl().getErrorString(r__)); \
    } while (0)

static_assert(sizeof(ncclUniqueId) == MW_RCCL_ID_BYTES, "RCCL unique id size");

int mw_rccl_get_unique_id(void *id_out)
{
    MW_TRY({
        ncclUniqueId id;
        MW_NCCL_OK(rccl().getUniqueId(&id));
        memcpy(id_out, &id, sizeof(id));
        return 0;
    }, -1)
}

int mw_rccl_init(mw_exec *exec, const void *id, int32_t nranks, int32_t rank)
{
    MW_TRY({
        if (exec->comm) throw std::runtime_error("mw_rccl_init: communicator already set");
        ncclUniqueId uid;
        memcpy(&uid, id, sizeof(uid));
        // the communicator binds to the calling thread's current device:
        // the executor's for the call, the caller's again afterwards (also
        // when the init throws)
        int prev = 0;
        MW_HIP_OK(hipGetDevice(&prev));
        struct Restore {
            int dev;
            ~Restore() { (void)hipSetDevice(dev); }
        } restore { prev };
        MW_HIP_OK(hipSetDevice(exec->gpu));
        MW_NCCL_OK(rccl().commInitRank(&exec->comm, nranks, uid, rank));
        return 0;
    }, -1)
}

int mw_allgather_exported(mw_exec *exec, int32_t slot, void *dst, int64_t bytes_per_rank)
{
    MW_TRY({
        if (!exec->comm) throw std::runtime_error("mw_allgather_exported: call mw_rccl_init first");
        void *src = exec->exec->getExported(slot, nullptr);
        if (!src) throw std::runtime_error("mw_allgather_exported: no such export slot");
        const int64_t cap = exec->exec->exportBufferBytes(slot);
        if (bytes_per_rank < 0 || bytes_per_rank > cap) {
            throw std::runtime_error("mw_allgather_exported: bytes_per_rank exceeds the export buffer (" +
                                     std::to_string(cap) + " bytes)");
        }
        MW_NCCL_OK(rccl().allGather(src, dst, (size_t)bytes_per_rank, ncclChar, exec->comm,
                                 (hipStream_t)exec->exec->stream()));
        return 0;
    }, -1)
}

void *mw_device_alloc(mw_exec *exec, int64_t bytes)
{
    MW_TRY({
        (void)exec;
        void *p = nullptr;
        MW_HIP_OK(hipMalloc(&p, (size_t)std::max<int64_t>(bytes, 256)));
        return p;
    }, nullptr)
}

int mw_device_free(mw_exec *exec, void *ptr)
{
    MW_TRY({
        (void)exec;
        MW_HIP_OK(hipFree(ptr));
        return 0;
    }, -1)
}

#else
int mw_rccl_get_unique_id(void *)
{
    MW_TRY({ gfx950Only("mw_rccl_get_unique_id"); }, -1)
}

int mw_rccl_init(mw_exec *, const void *, int32_t, int32_t)
{
    MW_TRY({ gfx950Only("mw_rccl_init"); }, -1)
}

int mw_allgather_exported(mw_exec *, int32_t, void *, int64_t)
{
    MW_TRY({ gfx950Only("mw_allgather_exported"); }, -1)
}

// "Device" memory of the CPU back end is host memory.
void *mw_device_alloc(mw_exec *, int64_t bytes)
{
    MW_TRY({
        void *p = calloc(1, (size_t)std::max<int64_t>(bytes, 256));
        if (!p) throw std::runtime_error("mw_device_alloc: out of memory");
        return p;
    }, nullptr)
}

int mw_device_free(mw_exec *, void *ptr)
{
    free(ptr);
    return 0;
}

#endif

int32_t mw_num_worlds(mw_exec *exec) { return exec->exec->numWorlds(); }

int32_t mw_export_row_bytes(mw_exec *exec, int32_t slot)
{
    MW_TRY({
        const int32_t b = exec->exec->exportRowBytes(slot);
        if (b <= 0) throw std::runtime_error("mw_export_row_bytes: no such export slot");
        return b;
    }, -1)
}

int32_t mw_error_flags(mw_exec *exec)
{
    MW_TRY({ return exec->exec->errorFlags(); }, -1)
}

int32_t mw_num_archetypes(mw_exec *exec)
{
    return exec->exec->stateManager().numArchetypes();
}

int32_t mw_column_info(mw_exec *exec, int32_t archetype, int32_t column, int32_t *bytes,
                       int32_t *capacity)
{
    uint32_t b = 0;
    int32_t cap = 0;
    if (!exec->exec->columnBase(archetype, column, &cap, &b)) return -1;
    if (bytes) *bytes = (int32_t)b;
    if (capacity) *capacity = cap;
    return 0;
}

int32_t mw_entity_loc(mw_exec *exec, int32_t world, int32_t id, uint32_t gen, int32_t *archetype,
                      int32_t *row)
{
    MW_TRY({
        Loc l;
        if (!exec->exec->entityLoc(world, Entity { gen, id }, &l)) return 1;
        if (archetype) *archetype = (int32_t)l.archetype;
        if (row) *row = l.row;
        return 0;
    }, -1)
}

int32_t mw_read_column(mw_exec *exec, int32_t archetype, int32_t column, int32_t world, void *out,
                       int32_t max_rows)
{
    MW_TRY({
        int32_t cap = 0;
        uint32_t bytes = 0;
        char *base = (char *)exec->exec->columnBase(archetype, column, &cap, &bytes);
        if (!base || world < 0 || world >= exec->exec->numWorlds()) return -1;
        exec->exec->sync();
        int32_t n = exec->exec->numRows(archetype, world);
        int32_t copy = n < max_rows ? n : max_rows;
        if (copy > 0) {
            copyOut(out, base + (size_t)world * cap * bytes, (size_t)copy * bytes);
        }
        return n;
    }, -1)
}

int32_t mw_phys_read_candidates(mw_exec *exec, int32_t world, void *out, int32_t cap)
{
    MW_TRY({
        exec->exec->sync();
        phys::PhysArgs *P = phys::physicsArgs(exec->exec->stateManager());
        if (!P) return -1;
        int32_t n = 0;
        copyOut(&n, P->lastNumCands + world, 4);
        int32_t copy = n < cap ? n : cap;
        if (copy > 0) {
            copyOut(out, P->cands + (size_t)world * P->candCapacity,
                                sizeof(phys::CandidateCollision) * copy);
        }
        return n;
    }, -1)
}

int32_t mw_phys_read_contacts(mw_exec *exec, int32_t world, void *out, int32_t cap)
{
    MW_TRY({
        exec->exec->sync();
        phys::PhysArgs *P = phys::physicsArgs(exec->exec->stateManager());
        if (!P) return -1;
        int32_t n = 0;
        copyOut(&n, P->lastNumContacts + world, 4);
        std::vector<int32_t> order(n);
        if (n > 0) {
            copyOut(order.data(), P->contactOrder + (size_t)world * P->candCapacity,
                                4 * n);
        }
        std::vector<phys::Contact> slots(P->candCapacity);
        copyOut(slots.data(), P->candContacts + (size_t)world * P->candCapacity,
                            sizeof(phys::Contact) * P->candCapacity);
        phys::Contact *o = (phys::Contact *)out;
        for (int32_t i = 0; i < n && i < cap; i++) o[i] = slots[order[i]];
        return n;
    }, -1)
}

int32_t mw_phys_read_bvh(mw_exec *exec, int32_t world, void *nodes_out, float *leaf_aabbs_out,
                         int32_t cap_nodes)
{
    MW_TRY({
        exec->exec->sync();
        phys::PhysArgs *P = phys::physicsArgs(exec->exec->stateManager());
        if (!P) return -1;
        phys::broadphase::BVH bvh;
        copyOut(&bvh, P->bvh + world, sizeof(bvh));
        int32_t n = bvh.usedNodes < cap_nodes ? bvh.usedNodes : cap_nodes;
        if (nodes_out && n > 0) {
            copyOut(nodes_out, P->nodes + (size_t)world * P->maxNodes,
                                sizeof(phys::BVHNode) * n);
        }
        if (leaf_aabbs_out && bvh.numLeaves > 0) {
            copyOut(leaf_aabbs_out, P->leafAABBs + (size_t)world * P->maxLeaves,
                                sizeof(math::AABB) * bvh.numLeaves);
        }
        return bvh.usedNodes;
    }, -1)
}

double mw_phys_time_node(mw_exec *exec, const char *node_name, int32_t num_steps)
{
    MW_TRY({ return exec->exec->timeNode(node_name, num_steps); }, -1.0)
}

int32_t mw_num_nodes(mw_exec *exec)
{
    MW_TRY({ return exec->exec->numNodes(); }, -1)
}

int32_t mw_world_walk_runs(mw_exec *exec)
{
    MW_TRY({ return exec->exec->worldWalkRuns(); }, -1)
}

int32_t mw_walk_run_end(mw_exec *exec, int32_t node)
{
    MW_TRY({ return exec->exec->walkRunEnd(node); }, -1)
}

const char *mw_node_name(mw_exec *exec, int32_t node)
{
    MW_TRY({ return exec->exec->nodeName(node); }, nullptr)
}

int32_t mw_node_blocks_per_cu(mw_exec *exec, int32_t node)
{
    MW_TRY({ return exec->exec->nodeBlocksPerCU(node); }, -1)
}

int mw_set_node_blocks_per_cu(mw_exec *exec, int32_t node, int32_t blocks_per_cu)
{
    MW_TRY({
        exec->exec->setNodeBlocksPerCU(node, blocks_per_cu);
        return 0;
    }, -1)
}

int mw_parse_exec_config_override(const char *s, uint32_t *out)
{
    MW_TRY({
        if (!s || !out) throw std::runtime_error("mw_parse_exec_config_override: null argument");
        const madrona::ExecConfigOverride o = madrona::parseExecConfigOverride(s);
        out[0] = o.numThreads;
        out[1] = o.blocksPerCU;
        out[2] = o.numCUs;
        return 0;
    }, -1)
}

int32_t mw_parse_exec_config_file(const char *json, int32_t *nodes, int32_t *blocks, int32_t cap)
{
    MW_TRY({
        if (!json) throw std::runtime_error("mw_parse_exec_config_file: null argument");
        const auto v = madrona::parseExecConfigFile(json);
        for (int32_t i = 0; i < (int32_t)v.size() && i < cap; i++) {
            if (nodes) nodes[i] = v[i].node;
            if (blocks) blocks[i] = v[i].blocksPerCU;
        }
        return (int32_t)v.size();
    }, -1)
}

int32_t mw_set_timed_node(mw_exec *exec, const char *node_name)
{
    return mw_set_timed_node_every(exec, node_name, 1);
}

int32_t mw_set_timed_node_every(mw_exec *exec, const char *node_name, int32_t every)
{
    MW_TRY({
        if (every < 1) throw std::invalid_argument("mw_set_timed_node_every: every must be >= 1");
        exec->exec->setTimedNode(node_name, every);
        return 0;
    }, -1)
}

int32_t mw_set_timed_node_index(mw_exec *exec, int32_t node, int32_t every)
{
    MW_TRY({
        if (every < 1) throw std::invalid_argument("mw_set_timed_node_index: every must be >= 1");
        exec->exec->setTimedNodeIndex(node, every);
        return 0;
    }, -1)
}

double mw_timed_node_ms(mw_exec *exec, int64_t *launches)
{
    MW_TRY({ return exec->exec->timedNodeMs(launches); }, -1.0)
}

int mw_trace_enable(mw_exec *exec, int64_t max_records)
{
    MW_TRY({
        if (max_records < 0) throw std::runtime_error("mw_trace_enable: negative max_records");
        exec->exec->enableTracing(max_records);
        return 0;
    }, -1)
}

int mw_trace_block_records(void)
{
#if defined(MW_TRACING)
    return 1;
#else
    return 0;
#endif
}

int64_t mw_trace_read(mw_exec *exec, void *dst, int64_t max_bytes, int64_t *dropped)
{
    MW_TRY({
        const int64_t n = exec->exec->readTrace(dst, max_bytes, dropped);
        if (n < 0) throw std::runtime_error("mw_trace_read: tracing is not enabled");
        return n;
    }, (int64_t)-1)
}

const char *mw_trace_func_name(mw_exec *exec, int32_t func_id)
{
    MW_TRY({ return exec->exec->traceFuncName(func_id); }, (const char *)nullptr)
}

}

extern "C" int32_t mw_phys_counts(mw_exec *exec, int32_t *cands_out, int32_t *contacts_out)
{
    MW_TRY({
        exec->exec->sync();
        phys::PhysArgs *P = phys::physicsArgs(exec->exec->stateManager());
        if (!P) return -1;
        if (cands_out) {
            copyOut(cands_out, P->lastNumCands, 4 * P->numWorlds);
        }
        if (contacts_out) {
            copyOut(contacts_out, P->lastNumContacts, 4 * P->numWorlds);
        }
        return P->numWorlds;
    }, -1)
}

extern "C" int32_t mw_phys_take_units(mw_exec *exec, int64_t *out)
{
    MW_TRY({
        exec->exec->sync();
        phys::PhysArgs *P = phys::physicsArgs(exec->exec->stateManager());
        if (!P || !P->unitAccum || !out) return -1;
        copyOut(out, P->unitAccum, phys::kUnitSlots * sizeof(int64_t));
        zeroArena(P->unitAccum, phys::kUnitSlots * sizeof(int64_t));
        return phys::kUnitSlots;
    }, -1)
}

extern "C" int32_t mw_phys_kernel_variants(mw_exec *exec, int32_t *out, int32_t n)
{
    MW_TRY({
        phys::PhysArgs *P = phys::physicsArgs(exec->exec->stateManager());
        if (!P || !out) return -1;
        int32_t v[11];
        v[0] = P->refitGlobal != 0;
        v[1] = P->overlapImage != nullptr;
        v[2] = P->satImage != nullptr;
        v[3] = P->clipImage != nullptr;
        v[4] = P->solverImage != nullptr;
        v[5] = P->planeGeoBytes > 0;
        v[6] = P->satGeoBytes > 0;
        v[7] = P->objs.minkStride > 0;
        const phys::PhysicsModule &M = phys::physicsModule(exec->exec->stateManager());
        v[8] = M.solverLanes;
        v[9] = (int32_t)(M.solverItemsPerLevel * 100.0 + 0.5);
        v[10] = P->dfsChunks > 0;
        for (int32_t i = 0; i < n && i < 11; i++) out[i] = v[i];
        return 11;
    }, -1)
}
