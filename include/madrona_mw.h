/*
 * C ABI of the MI355X-native batched ECS world-stepper.
 *
 * This is the drop-in boundary for the reference's executor surface:
 *
 *   mw_create        <- madrona::MWCudaExecutor::MWCudaExecutor(StateConfig,
 *                       CompileConfig)  (reference include/madrona/mw_gpu.hpp:55-59,
 *                       src/mw/cuda_exec.cpp:1692-1763) and
 *                       TaskGraphExecutor::TaskGraphExecutor(cfg, user_cfg, inits)
 *                       (include/madrona/mw_cpu.hpp:53-60, mw_cpu.inl:8-44)
 *   mw_step          <- MWCudaExecutor::run()   (src/mw/cuda_exec.cpp:1777-1794),
 *                       TaskGraphExecutor::run() (include/madrona/mw_cpu.inl:46-50)
 *   mw_get_exported  <- getExported(slot)       (src/mw/cuda_exec.cpp:1796-1800,
 *                       include/madrona/mw_cpu.hpp:38); adds the packed row count
 *   mw_destroy       <- ~MWCudaExecutor()
 *
 * The reference reports errors by aborting (FATAL / REQ_CUDA,
 * include/madrona/cuda_utils.hpp:46-54); here every entry point returns a
 * status (0 = ok) or NULL and mw_last_error() describes the failure.
 * Environments are compiled ahead of time into the library and selected by
 * name (the reference JIT-compiles them with NVRTC instead).
 *
 * All pointers are plain host pointers except those documented as device
 * pointers (mw_get_exported, mw_stream).  No torch types cross this boundary.
 *
 * Two libraries export this ABI: libmadrona_mw.so (gfx950) and
 * libmadrona_cpu.so, the CPU back end built from the same world sources
 * with g++ (the reference's TaskGraphExecutor on a pinned thread pool,
 * include/madrona/mw_cpu.hpp:53-81, src/mw/cpu_exec.cpp:31-284).  In the
 * CPU library "device" pointers are host pointers, mw_step is synchronous
 * and the RCCL / tracing / launch-configuration entry points fail with a
 * status.
 */
#ifndef MADRONA_MW_H
#define MADRONA_MW_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mw_exec mw_exec;

/* ABI version of mw_config (bumped when a field changes meaning or place).
 * Version 1 = round 5: struct_size / abi_version added in front.           */
#define MW_ABI_VERSION 1u

/* Executor configuration (reference StateConfig, mw_gpu.hpp:20-32).  The
 * first two fields identify the layout the caller was compiled against:
 * mw_create refuses a struct_size / abi_version it does not know (status
 * NULL + mw_last_error), so a stale caller fails instead of being misread.
 * Initialise with MW_CONFIG_INIT (C: `mw_config c = MW_CONFIG_INIT;
 * c.num_worlds = ...`).  The environment's own config struct is checked the
 * same way through mw_create's user_cfg_bytes.                             */
typedef struct mw_config {
    uint32_t struct_size;      /* sizeof(mw_config)                          */
    uint32_t abi_version;      /* MW_ABI_VERSION                             */
    int32_t num_worlds;        /* worlds stepped by this executor (this GPU) */
    int32_t gpu_id;            /* HIP device ordinal                         */
    int32_t default_capacity;  /* rows per world for archetypes w/o a size   */
    int32_t use_graph;         /* 1: replay the step as one hipGraph         */
    int32_t tmp_alloc_bytes;   /* Context::tmpAlloc arena per world (reference
                                  StateManager::tmpAlloc) in bytes; 0: the
                                  default 16 KiB, -1: no arena (tmpAlloc
                                  returns null and flags the world)         */
    int32_t max_deferred_destroys; /* destroyEntityNow calls per world per
                                  row-parallel node (applied in the reference's
                                  order after the node); 0: 256              */
    int32_t num_workers;       /* CPU back end: worker threads, pinned one per
                                  core (reference ThreadPoolExecutor::Config::
                                  numWorkers, mw_cpu.hpp:20-27); 0: every core
                                  of the affinity mask.  Ignored on gfx950.   */
    int32_t serial_nodes;      /* 1: run every ParallelForNode /
                                  CustomParallelForNode world-serially (one
                                  invocation per world walks its rows in order,
                                  as the reference's ParallelForNode::run,
                                  taskgraph.inl:63-71); 0: row-parallel lanes
                                  with the ordered structural commit.  The CPU
                                  back end is always world-serial.          */
    int64_t tmp_pool_bytes;    /* tmpAlloc past a world's arena is chained, as
                                  the reference chains blocks (state.cpp:
                                  95-114): a device pool shared by all worlds
                                  (host: heap blocks), reset with the arenas.
                                  0: default (2 x the arenas, 16 MiB - 1 GiB),
                                  -1: none (exhaustion flags the world)     */
} mw_config;

#define MW_CONFIG_INIT { (uint32_t)sizeof(mw_config), MW_ABI_VERSION }

/* "collisions": rigid-body workload of SURVEY.md §8(d) C3/C4 (128 unit cube
 * hulls + one static plane per world, src/physics).                        */
typedef struct mw_collisions_config {
    int32_t num_cubes;
    int32_t num_substeps;
    float delta_t;
    float gravity_z;
    int32_t max_contacts;      /* SolverData::maxContacts per world          */
    int32_t max_candidates;    /* CandidateTemporary rows per world          */
    float cube_inv_mass;
    float cube_inv_inertia;
    float mu_s;
    float mu_d;
    int32_t num_joints;        /* ConstraintData rows per world: joint j ties
                                  cube 2j to 2j+1 (fixed joint); 0 = none  */
    int32_t num_hinge_joints;  /* the last num_hinge_joints joints are hinges
                                  instead (the reference's hinge diverges,
                                  DESIGN.md §4: short horizons only)       */
    const char *hull_paths;    /* NULL / "": every body is the built-in unit
                                  cube.  Otherwise ';'-separated .obj files
                                  loaded as convex hulls (PhysicsLoader);
                                  body i uses hull i % count, the ground
                                  plane comes after them                    */
} mw_collisions_config;

/* Per-world init (reference InitT): host pointers to num_cubes x 3 positions
 * and num_cubes x 4 quaternions (w, x, y, z).                              */
typedef struct mw_collisions_init {
    const float *pos;
    const float *rot;
} mw_collisions_init;

/* Synthetic inputs for worlds [first_world, first_world + num_worlds) of the
 * reference's serial mt19937(seed) draw (examples/collisions/collisions.cpp). */
void mw_gen_collisions_inits(int32_t first_world, int32_t num_worlds,
                             int32_t num_cubes, uint32_t seed,
                             float *pos_out, float *rot_out);

/* Physics asset path without a device (replaces PhysicsLoader::
 * loadHullFromDisk, src/physics/physics_assets.cpp:205-254): imports the
 * .obj, builds the half-edge hull and writes counts_out = {vertices, faces,
 * edges, half edges}, aabb_out = {min xyz, max xyz}, then up to the given
 * capacities the hull's vertices (xyz), face planes (normal xyz, d) and half
 * edges (next, twin, root vertex, polygon).  0 on success, -1 on a malformed
 * file (mw_last_error), -2 when a capacity is too small (counts still set). */
int mw_load_hull(const char *obj_path, int32_t *counts_out, float *aabb_out,
                 float *verts_out, int32_t vert_cap, float *planes_out, int32_t face_cap,
                 uint32_t *half_edges_out, int32_t half_edge_cap);

/* Create an executor for environment `env`.  `inits` points at num_worlds
 * records of `init_stride` bytes each (reference: const InitT *user_inits). */
mw_exec *mw_create(const char *env, const mw_config *cfg,
                   const void *user_cfg, size_t user_cfg_bytes,
                   const void *inits, size_t init_stride);

/* Load an environment compiled outside this library (reference: user
 * sources of CompileConfig, src/mw/cuda_exec.cpp:444-831, compiled ahead of
 * time here): a shared object built with hipcc against include/madrona,
 * linked to libmadrona_mw.so, whose worlds register themselves with
 * MADRONA_BUILD_MWGPU_ENTRY (include/madrona/mw_gpu_entry.hpp).  Returns the
 * number of environments it registered (-1 on error); mw_create then takes
 * their names.  mw_num_envs / mw_env_name list every registered name.     */
int32_t mw_load_env(const char *so_path);
int32_t mw_num_envs(void);
const char *mw_env_name(int32_t i);

/* Step every world `num_steps` times; blocks until done.
 * Growable tables (registerArchetype without a size) grow between any two
 * steps, here and in mw_step_async: behind each step the host is sent the
 * tables' largest row counts, and a table past half full doubles before
 * the next step is enqueued.  The host runs at most MADRONA_MW_GROW_LAG
 * (default 2, at most 7) steps ahead of the counts it has seen, so a table
 * that more than doubles within that many steps + 1 (or inside one step)
 * overflows and flags its worlds (mw_error_flags); growth itself waits for
 * the device.  Executors with growable tables launch one step graph per
 * step (no multi-step graphs).                                             */
int mw_step(mw_exec *exec, int32_t num_steps);

/* Enqueue `num_steps` steps on the executor stream without waiting (beyond
 * the bounded growth look-behind of mw_step above).                        */
int mw_step_async(mw_exec *exec, int32_t num_steps);

/* Wait for enqueued steps. */
int mw_sync(mw_exec *exec);

/* Device pointer of export slot `slot`: rows of all worlds packed
 * world-major (reference getExported).  *num_rows receives the row count of
 * the last enqueued step (waits for it).  The pointer is stable: the buffer
 * of a growable table is a reserved address range that a growth extends in
 * place, contents kept (HIP virtual memory; past 256x its first size, or
 * with MADRONA_MW_EXPORT_VMM=0, a growth moves it to a new buffer with the
 * contents copied, and earlier pointers are stale).                       */
void *mw_get_exported(mw_exec *exec, int32_t slot, int64_t *num_rows);

/* Copy up to max_bytes of export slot `slot` into buffer `dst` (device or
 * host; ordered on the executor stream after every enqueued step, then one
 * synchronisation).  Returns the bytes of packed rows copied; bytes of dst
 * past that count (up to max_bytes) are unspecified.                      */
int64_t mw_copy_exported(mw_exec *exec, int32_t slot, void *dst, int64_t max_bytes);

/* The training hand-off without a host round trip: a device-to-device copy
 * of min(max_bytes, the slot's buffer) bytes of export slot `slot` into
 * device memory `dst`, enqueued on the executor stream behind every step
 * enqueued so far; returns the bytes enqueued and does not wait (order a
 * consumer's stream after it with mw_stream_wait).  Bytes past the packed
 * rows are unspecified.                                                    */
int64_t mw_copy_exported_async(mw_exec *exec, int32_t slot, void *dst, int64_t max_bytes);

/* Bytes of one packed row of export slot `slot` (-1: no such slot). */
int32_t mw_export_row_bytes(mw_exec *exec, int32_t slot);

/* hipStream_t of the executor (device work ordering for callers). */
void *mw_stream(mw_exec *exec);

/* Make the caller's hipStream_t `stream` (e.g. torch's current stream) wait,
 * on the device and without a host sync, for every step enqueued so far.
 * Replaces CudaSync::wait (include/madrona/python.hpp:20-35,
 * src/python/utils.cpp:15-48), which waits on an external semaphore. */
int mw_stream_wait(mw_exec *exec, void *stream);

int mw_destroy(mw_exec *exec);
const char *mw_last_error(void);

/* ---- introspection (tests, tooling) ------------------------------------ */
int32_t mw_num_worlds(mw_exec *exec);
/* OR of per-world error flags: 1 id store full, 2 table full, 4 candidate
 * overflow, 8 contact overflow, 16 BVH stack overflow, 32 solver body
 * overflow, 64 index guard (site in bits 8..15), 128 joint overflow,
 * 1<<16 job dropped, 1<<17 tmpAlloc arena full, 1<<18 deferred log full,
 * 1<<19 op not available in a row-parallel node, 1<<20 commit limit,
 * 1<<21 static body written by a non-finite solve, 1<<22 row-parallel make
 * gave up waiting for its turn, 1<<23 row-parallel get of a query component
 * at another row (kErrFlagCrossRow, include/madrona/state.hpp).            */
int32_t mw_error_flags(mw_exec *exec);
int32_t mw_num_archetypes(mw_exec *exec);
/* Copy rows of (archetype, column) of one world to host `out` (capacity
 * max_rows); returns the world's row count or -1. */
int32_t mw_read_column(mw_exec *exec, int32_t archetype, int32_t column,
                       int32_t world, void *out, int32_t max_rows);
/* Entity lookup in world `world`'s ID store (reference getLoc): 0 and the
 * entity's (archetype, row) when (id, gen) is alive, 1 when it is not.   */
int32_t mw_entity_loc(mw_exec *exec, int32_t world, int32_t id, uint32_t gen,
                      int32_t *archetype, int32_t *row);
/* Column byte width and rows-per-world capacity. */
int32_t mw_column_info(mw_exec *exec, int32_t archetype, int32_t column,
                       int32_t *bytes, int32_t *capacity);

/* physics (collisions env): the last step's candidate pairs (4 x int32:
 * a.archetype, a.row, b.archetype, b.row), the last substep's contacts in
 * solver order (112-byte reference Contact records), the BVH (116-byte
 * nodes, used prefix) and leaf AABBs.  Each returns the element count.    */
int32_t mw_phys_read_candidates(mw_exec *exec, int32_t world, void *out, int32_t cap);
int32_t mw_phys_read_contacts(mw_exec *exec, int32_t world, void *out, int32_t cap);
int32_t mw_phys_read_bvh(mw_exec *exec, int32_t world, void *nodes_out,
                         float *leaf_aabbs_out, int32_t cap_nodes);

/* per-world candidate / contact counts of the last step / substep. */
int32_t mw_phys_counts(mw_exec *exec, int32_t *cands_out, int32_t *contacts_out);

/* Work units of the live-timed physics launches since the last call (then
 * zeroed): out[0] timed SolverNode / NarrowphaseNode launches, out[1] their
 * candidates summed over worlds, out[2] their substeps' contact manifolds,
 * out[3] how many of them also ran the next substep's integration + filter
 * (solver) or the first substep's filter (narrowphase), out[4] the
 * narrowphase launches' survivor pairs.  bench.py's roofline byte model uses
 * them so its units are the timed launches' own.  out holds 5 int64;
 * returns 5, or -1 without physics.  No reference counterpart.             */
int32_t mw_phys_take_units(mw_exec *exec, int64_t *out);

/* Which variant of each LDS-staging physics kernel the executor runs (mw_create
 * picks it: a world / hull image that does not fit a workgroup's LDS moves to
 * a global slab, same results).  out[0..5] = 1 for: refit on the global node
 * slab, findOverlaps / SAT / contact / solver with a global image, then the
 * plane kernel's and the SAT kernel's LDS hull tables, and (last) the SAT
 * edge query's Minkowski-test tables (hulls small enough; environment
 * MADRONA_MW_SAT_TABLES=0 at mw_create turns them off); out[8]: the solver's
 * lanes per world (64, or 32 once the executor has measured narrow
 * dependency levels; MADRONA_MW_SOLVER_LANES=32|64|auto), out[9]: the items
 * per dependency level (x100) the last lane check read, out[10] = 1 when
 * worlds past MADRONA_MW_OVERLAP_DFS_LEAVES leaves (default 512) can walk the
 * BVH (the traversal launches exist).  Returns 11, or -1 without physics.
 * MADRONA_MW_FORCE_GLOBAL_IMAGES=1 at mw_create forces the global variants. */
int32_t mw_phys_kernel_variants(mw_exec *exec, int32_t *out, int32_t n);

/* physics kernel timing hook for the bench: binds a HIP event pair to the
 * kernels of each launch of the named node kind ("SolverNode", ...): first
 * kernel start to last kernel end.
 * Returns the mean duration in ms over `num_steps` fresh steps.            */
double mw_phys_time_node(mw_exec *exec, const char *node_name, int32_t num_steps);

/* live timing inside the replayed step: the step graph is split at every
 * launch of the named node kind, which then runs directly on the executor
 * stream between graph segments with a HIP event pair bound to its kernels
 * (first kernel start to last kernel end); mw_timed_node_ms
 * returns the accumulated ms and the number of timed launches since the
 * last mw_set_timed_node (NULL/"" disables and restores the single graph). */
int32_t mw_set_timed_node(mw_exec *exec, const char *node_name);
/* the same, timing only every `every`-th step (the first of each run of
 * `every` steps is split and timed; the others replay the unsplit graph, so
 * the timing costs 1/every of the split's overhead). every >= 1.          */
int32_t mw_set_timed_node_every(mw_exec *exec, const char *node_name, int32_t every);
/* the same for one node of the step graph: `node` is its index in sorted
 * order (mw_node_name), e.g. one of several ParallelForNodes.  -1 and a
 * message on an index past the graph.                                      */
int32_t mw_set_timed_node_index(mw_exec *exec, int32_t node, int32_t every);
double mw_timed_node_ms(mw_exec *exec, int64_t *launches);

/* ---- job-API environments -----------------------------
 * The reference's examples written against its job API (ctx.submit /
 * ctx.parallelFor / ctx.archetype / currentJobID), run through the Context
 * job API: each world's jobs on the lane that owns it, in submission order.
 * "fantasy_vs_jobs": examples/fantasy_vs/fvs.cpp (mw_fvs_config /
 * mw_fvs_init, same game as "fantasy_vs").  "collisions_jobs":
 * examples/collisions/collisions.cpp:88-227 (brute-force pairs, pass-through
 * narrowphase, push-apart solver) with mw_collisions_init positions /
 * rotations of num_objects cubes (mw_gen_collisions_inits).              */
typedef struct mw_jobs_collisions_config {
    int32_t num_objects;       /* 100 in the reference (collisions.cpp:73) */
    int32_t max_candidates;    /* CollisionCandidate / Contact rows per world */
} mw_jobs_collisions_config;

/* ---- launch configuration (reference MADRONA_MWGPU_EXEC_CONFIG_OVERRIDE /
 * MADRONA_MWGPU_EXEC_CONFIG_FILE, src/mw/cuda_exec.cpp:1401-1560) ---------
 * Both environment variables are honoured when the step graph is built:
 * the override "threads,blocksPerCU,numCUs" sets the default blocks per CU
 * (threads: accepted, unused -- block sizes are per kernel here), the file
 * is a JSON object {"<node index>": <blocks per CU>, ...}.  Blocks per CU
 * caps the grid of a node's grid-stride kernels (ParallelForNode,
 * PerWorldNode) and sizes its persistent kernels (NarrowphaseNode's SAT and
 * contact kernels); 0 = the node's default grid.  Results do not depend on
 * it.  mw_set_node_blocks_per_cu: node -1 sets the default, value -1 on a
 * node reverts it to the default; re-captures the step graph.             */
int32_t mw_num_nodes(mw_exec *exec);
/* World walk (the persistent megakernel, reference src/mw/device/
 * megakernel_impl.inl:29-55): runs of consecutive world-local nodes (row
 * nodes over small tables with their ordered commits, world-serial row
 * nodes, per-world nodes, device nodes that declare kWorldLocal) are walked
 * by one kernel, a wave per world calling each node's world function in
 * graph order through the dispatch generated at build time from the world
 * source; same results.  On by default; MADRONA_MW_WORLD_WALK=0 in the
 * environment at mw_create launches every node on its own.  Returns the
 * walk launches per step (0: off / CPU back end).                          */
int32_t mw_world_walk_runs(mw_exec *exec);
/* The end of the walk run that node `node` starts: nodes [node, end) are one
 * walk launch (and one unit for mw_set_timed_node_index); node + 1 when it
 * starts none.  -1 on a bad index.                                         */
int32_t mw_walk_run_end(mw_exec *exec, int32_t node);
const char *mw_node_name(mw_exec *exec, int32_t node);
int32_t mw_node_blocks_per_cu(mw_exec *exec, int32_t node);
int mw_set_node_blocks_per_cu(mw_exec *exec, int32_t node, int32_t blocks_per_cu);
/* host-only parsers of the two formats (no GPU needed): 0 / the number of
 * entries on success, -1 on malformed input (mw_last_error says why).     */
int mw_parse_exec_config_override(const char *s, uint32_t *threads_blocks_cus);
int32_t mw_parse_exec_config_file(const char *json, int32_t *nodes, int32_t *blocks_per_cu,
                                  int32_t cap);

/* ---- device tracing (reference src/mw/device/include/madrona/mw_gpu/
 * tracing.hpp:14-128, MADRONA_TRACING + DeviceTracingManager::
 * transferLogToCPU, cuda_exec.cpp:1784) ----------------------------------
 * mw_trace_enable: log every following step -- a calibration record per
 * step, nodeStart / nodeFinish per node, blockStart / blockWait per block of
 * every kernel, blockExit at the step's end -- as 40-byte DeviceLog records
 * (event, funcID, numInvocations, nodeID, warpID, blockID, smID, logIndex,
 * ns timestamp), the input format of scripts/parse_device_tracing.py, up to
 * max_records in total (0 disables; re-captures the step graph).  One traced
 * executor per process.  mw_trace_read copies the records so far into dst
 * (up to max_bytes) and returns their total byte size (-1: tracing off);
 * *dropped counts records lost to a full buffer.  mw_trace_func_name maps a
 * funcID to its node kind ("SolverNode", ...), NULL past the last.        */
int mw_trace_enable(mw_exec *exec, int64_t max_records);
/* 1 when this library logs block records (the tracing build, -DMW_TRACING,
 * like the reference's MADRONA_TRACING); 0: node / step records only.     */
int mw_trace_block_records(void);
int64_t mw_trace_read(mw_exec *exec, void *dst, int64_t max_bytes, int64_t *dropped);
const char *mw_trace_func_name(mw_exec *exec, int32_t func_id);

/* ---- "fantasy_vs" environment (BASELINE.json configs[4]) -----------------
 * per world num_dragons casters + num_knights archers; dead entities are
 * destroyed every tick (examples/fantasy_vs/fvs.cpp, restated onto the
 * TaskGraph API).                                            */
typedef struct mw_fvs_config {
    int32_t num_dragons;       /* 50 in the reference benchmark (main.cpp:86) */
    int32_t num_knights;       /* 200 (main.cpp:87) */
} mw_fvs_config;

typedef struct mw_fvs_init {
    const float *dragon_pos;   /* num_dragons * 3 */
    const float *dragon_mana;  /* num_dragons */
    const float *knight_pos;   /* num_knights * 3 */
    const int32_t *knight_arrows; /* num_knights */
    int32_t world_index;       /* global world index (keys the per-world draws) */
    int32_t pad;
} mw_fvs_init;

/* Initial state of the reference example (fvs.cpp:88-108): one mt19937 drawn
 * serially over worlds; first_world selects a shard of that sequence.      */
void mw_gen_fvs_inits(int32_t first_world, int32_t num_worlds, int32_t num_dragons,
                      int32_t num_knights, uint32_t seed, float *dragon_pos,
                      float *dragon_mana, float *knight_pos, int32_t *knight_arrows);

/* ---- training hand-off across world shards (RCCL over xGMI) -------------
 * One process per GPU; rank 0 creates the id, the launcher distributes the
 * 128 bytes (e.g. over the torch.distributed TCP store), every rank calls
 * mw_rccl_init.  mw_allgather_exported enqueues an all-gather of the slot's
 * packed export buffer on the executor stream (after the step that wrote
 * it): dst receives nranks * bytes_per_rank bytes in rank order;
 * bytes_per_rank may not exceed the slot's export buffer (num_worlds x rows
 * per world x row bytes), else -1.  Replaces
 * the reference's host-side getExported gather for multi-GPU learners
 * (include/madrona/mw_gpu.hpp:71).                                         */
#define MW_RCCL_ID_BYTES 128
int mw_rccl_get_unique_id(void *id_out);
int mw_rccl_init(mw_exec *exec, const void *id, int32_t nranks, int32_t rank);
int mw_allgather_exported(mw_exec *exec, int32_t slot, void *dst, int64_t bytes_per_rank);
void *mw_device_alloc(mw_exec *exec, int64_t bytes);
int mw_device_free(mw_exec *exec, void *ptr);

#ifdef __cplusplus
}
#endif

#endif
