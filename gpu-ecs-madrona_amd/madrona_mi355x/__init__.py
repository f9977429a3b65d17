"""Python host mirror of the MI355X world-stepper (ctypes over the C ABI in
include/madrona_mw.h).

Mirrors the reference executor surface (TaskGraphExecutor / MWCudaExecutor:
construct with per-world inits, ``step()`` = ``run()``, ``exported(slot)`` =
``getExported(slot)``).  The HIP library is REQUIRED: importing this package
without ``gpu-ecs-madrona_amd/build/libmadrona_mw.so`` raises, and creating an
executor without a HIP device raises -- there is no CPU fallback.
"""
import ctypes
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MADRONA_MW_LIB") or os.path.join(os.path.dirname(PKG_DIR), "build", "libmadrona_mw.so")

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"madrona_mi355x: HIP library missing at {LIB_PATH}; "
        "build it with `make -C gpu-ecs-madrona_amd` (or __graft_entry__.build())")


def _mapped_hip_runtimes():
    try:
        with open("/proc/self/maps") as f:
            return sorted({os.path.realpath(l.split()[-1]) for l in f
                           if "libamdhip64" in l and "/" in l})
    except OSError:
        return []


# One HIP runtime per process.  PyTorch-ROCm wheels bundle their own
# libamdhip64 (soname libamdhip64.so.7, the same as the system ROCm's) and
# load it by path, so a process that loaded the system runtime first ends up
# with two runtimes and neither sees the device.  The library is built as
# code object v5 so it runs on either runtime; when torch is installed it is
# imported first and the library binds to torch's runtime (and, at first
# use, to torch's RCCL), so executor buffers are valid torch device memory.
# MADRONA_MW_NO_TORCH=1 skips this (C-ABI-only processes).
if not os.environ.get("MADRONA_MW_NO_TORCH"):
    try:
        import torch as _torch  # noqa: F401
    except ImportError:
        _torch = None

_lib = ctypes.CDLL(LIB_PATH)

if len(_mapped_hip_runtimes()) > 1:
    raise ImportError("madrona_mi355x: more than one HIP runtime mapped in this process "
                      f"({_mapped_hip_runtimes()}); import torch before loading the library")


MW_ABI_VERSION = 1     # include/madrona_mw.h


class MwConfig(ctypes.Structure):
    _fields_ = [("struct_size", ctypes.c_uint32), ("abi_version", ctypes.c_uint32),
                ("num_worlds", ctypes.c_int32), ("gpu_id", ctypes.c_int32),
                ("default_capacity", ctypes.c_int32), ("use_graph", ctypes.c_int32),
                ("tmp_alloc_bytes", ctypes.c_int32), ("max_deferred_destroys", ctypes.c_int32),
                ("num_workers", ctypes.c_int32), ("serial_nodes", ctypes.c_int32),
                ("tmp_pool_bytes", ctypes.c_int64)]


class CollisionsConfig(ctypes.Structure):
    _fields_ = [("num_cubes", ctypes.c_int32), ("num_substeps", ctypes.c_int32),
                ("delta_t", ctypes.c_float), ("gravity_z", ctypes.c_float),
                ("max_contacts", ctypes.c_int32), ("max_candidates", ctypes.c_int32),
                ("cube_inv_mass", ctypes.c_float), ("cube_inv_inertia", ctypes.c_float),
                ("mu_s", ctypes.c_float), ("mu_d", ctypes.c_float),
                ("num_joints", ctypes.c_int32), ("num_hinge_joints", ctypes.c_int32),
                ("hull_paths", ctypes.c_char_p)]


class FvsConfig(ctypes.Structure):
    _fields_ = [("num_dragons", ctypes.c_int32), ("num_knights", ctypes.c_int32)]


class FvsInit(ctypes.Structure):
    _fields_ = [("dragon_pos", ctypes.c_void_p), ("dragon_mana", ctypes.c_void_p),
                ("knight_pos", ctypes.c_void_p), ("knight_arrows", ctypes.c_void_p),
                ("world_index", ctypes.c_int32), ("pad", ctypes.c_int32)]


class CollisionsInit(ctypes.Structure):
    _fields_ = [("pos", ctypes.c_void_p), ("rot", ctypes.c_void_p)]


class JobsCollisionsConfig(ctypes.Structure):
    _fields_ = [("num_objects", ctypes.c_int32), ("max_candidates", ctypes.c_int32)]


# collisions_jobs CubeObject row: Entity, Translation, Rotation (w, x, y, z), PhysicsAABB
JC_ROW_DTYPE = np.dtype([("gen", np.uint32), ("id", np.int32), ("pos", np.float32, 3),
                         ("rot", np.float32, 4), ("aabb", np.float32, 6)])


RCCL_ID_BYTES = 128


def _declare(lib):
    """ctypes signatures of the C ABI (either library)."""
    lib.mw_create.restype = ctypes.c_void_p
    lib.mw_create.argtypes = [ctypes.c_char_p, ctypes.POINTER(MwConfig), ctypes.c_void_p,
                               ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
    lib.mw_step.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    lib.mw_step_async.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    lib.mw_sync.argtypes = [ctypes.c_void_p]
    lib.mw_get_exported.restype = ctypes.c_void_p
    lib.mw_get_exported.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_int64)]
    lib.mw_stream.restype = ctypes.c_void_p
    lib.mw_stream.argtypes = [ctypes.c_void_p]
    lib.mw_stream_wait.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.mw_destroy.argtypes = [ctypes.c_void_p]
    lib.mw_last_error.restype = ctypes.c_char_p
    lib.mw_num_worlds.argtypes = [ctypes.c_void_p]
    lib.mw_export_row_bytes.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    lib.mw_load_env.argtypes = [ctypes.c_char_p]
    lib.mw_entity_loc.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32,
                                   ctypes.c_void_p, ctypes.c_void_p]
    lib.mw_env_name.restype = ctypes.c_char_p
    lib.mw_env_name.argtypes = [ctypes.c_int32]
    lib.mw_error_flags.argtypes = [ctypes.c_void_p]
    lib.mw_num_archetypes.argtypes = [ctypes.c_void_p]
    lib.mw_read_column.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                    ctypes.c_void_p, ctypes.c_int32]
    lib.mw_column_info.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                    ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]
    lib.mw_phys_read_candidates.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32]
    lib.mw_phys_read_contacts.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32]
    lib.mw_phys_read_bvh.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_int32]
    lib.mw_phys_counts.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.mw_phys_take_units.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.mw_phys_kernel_variants.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32]
    lib.mw_copy_exported.restype = ctypes.c_int64
    lib.mw_copy_exported.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64]
    lib.mw_copy_exported_async.restype = ctypes.c_int64
    lib.mw_copy_exported_async.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                            ctypes.c_int64]
    lib.mw_gen_collisions_inits.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                             ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
    lib.mw_gen_fvs_inits.argtypes = [ctypes.c_int32] * 4 + [ctypes.c_uint32] + [ctypes.c_void_p] * 4
    lib.mw_phys_time_node.restype = ctypes.c_double
    lib.mw_phys_time_node.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int32]
    lib.mw_rccl_get_unique_id.argtypes = [ctypes.c_void_p]
    lib.mw_rccl_init.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32]
    lib.mw_allgather_exported.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                           ctypes.c_int64]
    lib.mw_device_alloc.restype = ctypes.c_void_p
    lib.mw_device_alloc.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    lib.mw_device_free.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.mw_load_hull.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                 ctypes.c_int32]
    lib.mw_trace_enable.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    lib.mw_trace_block_records.restype = ctypes.c_int
    lib.mw_trace_read.restype = ctypes.c_int64
    lib.mw_trace_read.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                   ctypes.POINTER(ctypes.c_int64)]
    lib.mw_trace_func_name.restype = ctypes.c_char_p
    lib.mw_trace_func_name.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    lib.mw_set_timed_node.restype = ctypes.c_int32
    lib.mw_set_timed_node.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
    lib.mw_set_timed_node_every.restype = ctypes.c_int32
    lib.mw_set_timed_node_every.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int32]
    lib.mw_set_timed_node_index.restype = ctypes.c_int32
    lib.mw_set_timed_node_index.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32]
    lib.mw_timed_node_ms.restype = ctypes.c_double
    lib.mw_timed_node_ms.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)]
    lib.mw_num_nodes.argtypes = [ctypes.c_void_p]
    lib.mw_world_walk_runs.argtypes = [ctypes.c_void_p]
    lib.mw_walk_run_end.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    lib.mw_node_name.restype = ctypes.c_char_p
    lib.mw_node_name.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    lib.mw_node_blocks_per_cu.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    lib.mw_set_node_blocks_per_cu.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32]
    lib.mw_parse_exec_config_override.argtypes = [ctypes.c_char_p, ctypes.c_void_p]
    lib.mw_parse_exec_config_file.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_int32]
    return lib


_declare(_lib)

CPU_LIB_PATH = os.environ.get("MADRONA_MW_CPU_LIB") or os.path.join(
    os.path.dirname(PKG_DIR), "build_cpu", "libmadrona_cpu.so")
_cpu_lib = None
# Back end of executors created without an explicit `backend`.
DEFAULT_BACKEND = os.environ.get("MADRONA_MW_BACKEND", "gpu")


def cpu_library():
    """The CPU back end (libmadrona_cpu.so: the same worlds and C ABI on a
    pinned host thread pool, the reference's TaskGraphExecutor); loaded on
    first use."""
    global _cpu_lib
    if _cpu_lib is None:
        if not os.path.exists(CPU_LIB_PATH):
            raise ImportError(f"madrona_mi355x: CPU library missing at {CPU_LIB_PATH}; "
                              "build it with `make -C gpu-ecs-madrona_amd cpu`")
        _cpu_lib = _declare(ctypes.CDLL(CPU_LIB_PATH))
    return _cpu_lib


# The symbols include/madrona_mw.h declares (checked by tests/test_capi_symbols.py).
C_ABI_SYMBOLS = (
    "mw_create", "mw_step", "mw_step_async", "mw_sync", "mw_get_exported", "mw_stream",
    "mw_destroy", "mw_last_error", "mw_num_worlds", "mw_error_flags", "mw_num_archetypes",
    "mw_read_column", "mw_column_info", "mw_phys_read_candidates", "mw_phys_read_contacts",
    "mw_phys_read_bvh", "mw_phys_time_node", "mw_phys_counts", "mw_phys_take_units",
    "mw_copy_exported",
    "mw_gen_collisions_inits", "mw_set_timed_node", "mw_set_timed_node_every", "mw_set_timed_node_index", "mw_timed_node_ms",
    "mw_rccl_get_unique_id", "mw_rccl_init", "mw_allgather_exported", "mw_device_alloc",
    "mw_device_free", "mw_gen_fvs_inits", "mw_stream_wait", "mw_load_hull",
    "mw_trace_enable", "mw_trace_read", "mw_trace_func_name", "mw_trace_block_records",
    "mw_num_nodes", "mw_world_walk_runs", "mw_walk_run_end", "mw_node_name", "mw_node_blocks_per_cu", "mw_set_node_blocks_per_cu",
    "mw_parse_exec_config_override", "mw_parse_exec_config_file",
    "mw_export_row_bytes", "mw_load_env", "mw_num_envs", "mw_env_name",
    "mw_entity_loc", "mw_copy_exported_async", "mw_phys_kernel_variants",
)


def parse_exec_config_override(s):
    """MADRONA_MWGPU_EXEC_CONFIG_OVERRIDE "threads,blocksPerCU,numCUs" ->
    (threads, blocks_per_cu, num_cus); MadronaError when malformed."""
    out = np.zeros(3, np.uint32)
    if _lib.mw_parse_exec_config_override(s.encode(), out.ctypes.data) != 0:
        raise _err()
    return tuple(int(v) for v in out)


def parse_exec_config_file(text):
    """MADRONA_MWGPU_EXEC_CONFIG_FILE contents -> [(node, blocks_per_cu)]."""
    n = _lib.mw_parse_exec_config_file(text.encode(), None, None, 0)
    if n < 0:
        raise _err()
    nodes = np.zeros(max(n, 1), np.int32)
    blocks = np.zeros(max(n, 1), np.int32)
    _lib.mw_parse_exec_config_file(text.encode(), nodes.ctypes.data, blocks.ctypes.data, n)
    return [(int(a), int(b)) for a, b in zip(nodes[:n], blocks[:n])]


def backend_library(backend=None):
    """The C-ABI library of a back end: "gpu" (libmadrona_mw.so, gfx950) or
    "cpu" (libmadrona_cpu.so)."""
    return cpu_library() if (backend or DEFAULT_BACKEND) == "cpu" else _lib


def load_env(so_path, backend=None):
    """Load an out-of-tree world (a shared object built against
    include/madrona that registers itself with MADRONA_BUILD_MWGPU_ENTRY,
    linked to the back end's library); returns the number of environments
    it registered."""
    lib = backend_library(backend)
    n = lib.mw_load_env(os.fsencode(so_path))
    if n < 0:
        raise _err(lib)
    return n


def env_names(backend=None):
    """Every registered environment name (built-in and loaded)."""
    lib = backend_library(backend)
    return [lib.mw_env_name(i).decode() for i in range(lib.mw_num_envs())]


def rccl_unique_id():
    """128-byte RCCL id (rank 0 creates it; the launcher distributes it)."""
    buf = ctypes.create_string_buffer(RCCL_ID_BYTES)
    if _lib.mw_rccl_get_unique_id(buf) != 0:
        raise _err()
    return buf.raw


def gen_collisions_inits(num_worlds, num_cubes=128, seed=0, first_world=0):
    """Product-side synthetic inputs (same serial mt19937 draw as the
    reference example; first_world selects a shard)."""
    pos = np.zeros((num_worlds, num_cubes, 3), np.float32)
    rot = np.zeros((num_worlds, num_cubes, 4), np.float32)
    _lib.mw_gen_collisions_inits(first_world, num_worlds, num_cubes, seed,
                                 pos.ctypes.data_as(ctypes.c_void_p),
                                 rot.ctypes.data_as(ctypes.c_void_p))
    return pos, rot

ERR_BITS = {1: "id store full", 2: "table full", 4: "candidate overflow",
            8: "contact overflow", 16: "BVH stack overflow", 32: "solver body overflow",
            64: "index guard (site in bits 8..15)", 128: "joint overflow",
            1 << 16: "job dropped", 1 << 17: "tmpAlloc arena full", 1 << 18: "deferred log full",
            1 << 19: "op not available in a row-parallel node", 1 << 20: "commit limit",
            1 << 21: "static body written by a non-finite solve",
            1 << 22: "row-parallel make gave up waiting for its turn",
            1 << 23: "row-parallel get/getUnsafe of a query component at another row"}
ERR_CROSS_ROW = 1 << 23


# DeviceLog (include/madrona/tracing.hpp; reference mw_gpu/tracing.hpp:30-41).
TRACE_DTYPE = np.dtype([("event", np.uint32), ("funcID", np.uint32),
                        ("numInvocations", np.uint32), ("nodeID", np.uint32),
                        ("warpID", np.uint32), ("blockID", np.uint32), ("smID", np.uint32),
                        ("logIndex", np.uint32), ("cycleCount", np.uint64)])
assert TRACE_DTYPE.itemsize == 40


def load_hull(path):
    """PhysicsLoader::loadHullFromDisk on the host (no device needed): the
    half-edge hull of an .obj file as numpy arrays -- vertices [V,3], face
    planes [F,4] (normal, d), half edges [H,4] (next, twin, root vertex,
    polygon), num_edges and the AABB [2,3]."""
    counts = np.zeros(4, np.int32)
    aabb = np.zeros((2, 3), np.float32)
    _lib.mw_load_hull(os.fspath(path).encode(), counts.ctypes.data, aabb.ctypes.data, None, 0,
                      None, 0, None, 0)
    if counts[0] == 0:
        raise _err()
    verts = np.zeros((counts[0], 3), np.float32)
    planes = np.zeros((counts[1], 4), np.float32)
    hes = np.zeros((counts[3], 4), np.uint32)
    if _lib.mw_load_hull(os.fspath(path).encode(), counts.ctypes.data, aabb.ctypes.data,
                         verts.ctypes.data, len(verts), planes.ctypes.data, len(planes),
                         hes.ctypes.data, len(hes)) != 0:
        raise _err()
    return {"vertices": verts, "planes": planes, "half_edges": hes,
            "num_edges": int(counts[2]), "aabb": aabb}


class MadronaError(RuntimeError):
    pass


def _err(lib=None):
    return MadronaError((lib or _lib).mw_last_error().decode())


def library():
    return _lib


CONTACT_DTYPE = np.dtype([
    ("ref", np.uint32, 2), ("alt", np.uint32, 2), ("points", np.float32, (4, 4)),
    ("numPoints", np.int32), ("normal", np.float32, 3), ("lambdaN", np.float32, 4),
])
BVH_NODE_DTYPE = np.dtype([
    ("minX", np.float32, 4), ("minY", np.float32, 4), ("minZ", np.float32, 4),
    ("maxX", np.float32, 4), ("maxY", np.float32, 4), ("maxZ", np.float32, 4),
    ("children", np.int32, 4), ("parentID", np.int32),
])

# Same record layout the oracle libraries return, for 1:1 comparisons.
BODY_DTYPE = np.dtype([
    ("gen", np.uint32), ("id", np.int32),
    ("pos", np.float32, 3), ("rot", np.float32, 4), ("vel", np.float32, 6),
    ("prevPos", np.float32, 3), ("prevRot", np.float32, 4),
    ("presolvePos", np.float32, 3), ("presolveRot", np.float32, 4),
    ("presolveVel", np.float32, 6),
    ("leafID", np.int32), ("objID", np.int32), ("responseType", np.uint32),
])

# physics body archetype id = registration order.
BODY_ARCHETYPE = 6
BODY_COLUMNS = {  # column index -> (BODY_DTYPE field(s), float/int words)
    0: ("entity", 2), 1: ("pos", 3), 2: ("rot", 4), 4: ("vel", 6), 5: ("objID", 1),
    6: ("responseType", 1), 7: ("prev", 7), 8: ("presolve", 7), 9: ("presolveVel", 6),
    12: ("leafID", 1),
}


class Executor:
    """A batch of worlds of one environment on one GPU."""

    def __init__(self, env, num_worlds, user_cfg, inits, init_stride, gpu_id=0,
                 default_capacity=64, use_graph=True, tmp_alloc_bytes=0,
                 max_deferred_destroys=0, backend=None, num_workers=0, serial_nodes=False,
                 tmp_pool_bytes=0):
        # backend "cpu": the same world on the CPU back end (num_workers
        # pinned host threads, 0 = every core of the affinity mask).
        # serial_nodes: every ParallelForNode walks each world's rows in
        # order (the reference's semantics for any node body)
        backend = backend or DEFAULT_BACKEND
        if backend not in ("gpu", "cpu"):
            raise ValueError(f"backend must be 'gpu' or 'cpu', not {backend!r}")
        self._lib = backend_library(backend)
        self.backend = backend
        cfg = MwConfig(ctypes.sizeof(MwConfig), MW_ABI_VERSION,
                       num_worlds, gpu_id, default_capacity, 1 if use_graph else 0,
                       tmp_alloc_bytes, max_deferred_destroys, num_workers,
                       1 if serial_nodes else 0, tmp_pool_bytes)
        self._keep = (user_cfg, inits)
        self.h = self._lib.mw_create(env.encode(), ctypes.byref(cfg), ctypes.byref(user_cfg),
                                ctypes.sizeof(user_cfg), ctypes.cast(inits, ctypes.c_void_p),
                                init_stride)
        if not self.h:
            raise _err(self._lib)
        self.num_worlds = num_worlds
        self.gpu_id = gpu_id

    def wait_on(self, stream):
        """Device-side ordering: `stream` (an int hipStream_t, e.g.
        torch.cuda.current_stream().cuda_stream) waits for every step
        enqueued so far; no host sync (reference CudaSync::wait)."""
        if self._lib.mw_stream_wait(self.h, ctypes.c_void_p(stream)) != 0:
            raise _err(self._lib)

    def exported_tensor(self, slot, element_type, dims):
        """Zero-copy view of export `slot` as a madrona_mi355x.python.Tensor
        (reference: getExported + madrona_python.Tensor(ptr, type, dims));
        dims must describe exactly the exported rows."""
        from .python import Tensor
        ptr, rows = self.exported(slot)
        if not ptr:
            raise MadronaError(f"no export slot {slot}")
        return Tensor.from_device_ptr(ptr, element_type, dims, self.gpu_id, owner=self)

    def step(self, n=1):
        if self._lib.mw_step(self.h, n) != 0:
            raise _err(self._lib)

    def step_async(self, n=1):
        if self._lib.mw_step_async(self.h, n) != 0:
            raise _err(self._lib)

    def sync(self):
        if self._lib.mw_sync(self.h) != 0:
            raise _err(self._lib)

    @property
    def stream(self):
        return self._lib.mw_stream(self.h)

    def exported(self, slot):
        rows = ctypes.c_int64(0)
        ptr = self._lib.mw_get_exported(self.h, slot, ctypes.byref(rows))
        return ptr, rows.value

    def exported_array(self, slot, dtype):
        """Host copy of export `slot` (packed [world-major, row] rows)."""
        dtype = np.dtype(dtype)
        _, rows = self.exported(slot)
        row_bytes = self._lib.mw_export_row_bytes(self.h, slot)
        if row_bytes <= 0:
            raise _err(self._lib)
        out = np.empty(max(rows, 1) * row_bytes, np.uint8)
        n = self.copy_exported(slot, out.ctypes.data, out.nbytes)
        return out[:n].view(dtype)

    def error_flags(self):
        return self._lib.mw_error_flags(self.h)

    def entity_loc(self, world, entity_id, gen):
        """(archetype, row) of a live entity, None when it is not alive."""
        a, r = ctypes.c_int32(), ctypes.c_int32()
        rc = self._lib.mw_entity_loc(self.h, world, entity_id, gen, ctypes.byref(a), ctypes.byref(r))
        if rc < 0:
            raise _err(self._lib)
        return None if rc else (a.value, r.value)

    def read_column(self, archetype, column, world, dtype, max_rows=4096):
        b = ctypes.c_int32()
        cap = ctypes.c_int32()
        if self._lib.mw_column_info(self.h, archetype, column, ctypes.byref(b), ctypes.byref(cap)) != 0:
            raise MadronaError(f"no column {archetype}:{column}")
        buf = np.zeros(max(cap.value, 1) * b.value, np.uint8)
        n = self._lib.mw_read_column(self.h, archetype, column, world,
                                buf.ctypes.data_as(ctypes.c_void_p), cap.value)
        if n < 0:
            raise _err(self._lib)
        return buf[: n * b.value].view(dtype)

    def copy_exported(self, slot, dst_ptr, max_bytes):
        n = self._lib.mw_copy_exported(self.h, slot, ctypes.c_void_p(dst_ptr), max_bytes)
        if n < 0:
            raise _err(self._lib)
        return n

    def copy_exported_async(self, slot, dst_ptr, max_bytes):
        """Enqueue the hand-off copy of export `slot` into device memory
        dst_ptr on the executor stream (no host wait)."""
        n = self._lib.mw_copy_exported_async(self.h, slot, ctypes.c_void_p(dst_ptr), max_bytes)
        if n < 0:
            raise _err(self._lib)
        return n

    def rccl_init(self, uid, nranks, rank):
        """Join the world-shard communicator (RCCL over xGMI)."""
        buf = ctypes.create_string_buffer(bytes(uid), RCCL_ID_BYTES)
        if self._lib.mw_rccl_init(self.h, buf, nranks, rank) != 0:
            raise _err(self._lib)

    def allgather_exported(self, slot, dst_ptr, bytes_per_rank):
        """Enqueue an all-gather of export `slot` into device memory dst_ptr
        (nranks * bytes_per_rank bytes, rank order) on the executor stream."""
        if self._lib.mw_allgather_exported(self.h, slot, ctypes.c_void_p(dst_ptr), bytes_per_rank) != 0:
            raise _err(self._lib)

    def device_alloc(self, nbytes):
        p = self._lib.mw_device_alloc(self.h, nbytes)
        if not p:
            raise _err(self._lib)
        return p

    def device_free(self, ptr):
        if self._lib.mw_device_free(self.h, ctypes.c_void_p(ptr)) != 0:
            raise _err(self._lib)

    def time_node(self, name, steps):
        """Eager timing of `steps` extra steps (advances the simulation)."""
        return self._lib.mw_phys_time_node(self.h, name.encode(), steps)

    def nodes(self):
        """Node kinds of the sorted step graph, by node index."""
        return [self._lib.mw_node_name(self.h, i).decode() for i in range(self._lib.mw_num_nodes(self.h))]

    def walk_run_end(self, node):
        """End of the walk run node `node` starts (node + 1: none)."""
        n = self._lib.mw_walk_run_end(self.h, node)
        if n < 0:
            raise _err(self._lib)
        return n

    def world_walk_runs(self):
        """World-walk launches per step (0 with MADRONA_MW_WORLD_WALK=0 at creation)."""
        n = self._lib.mw_world_walk_runs(self.h)
        if n < 0:
            raise _err(self._lib)
        return n

    def node_blocks_per_cu(self, node=-1):
        """Effective launch configuration (blocks per CU, 0 = full grid) of
        `node`; node -1: the default."""
        return self._lib.mw_node_blocks_per_cu(self.h, node)

    def set_node_blocks_per_cu(self, node, blocks_per_cu):
        """Per-node launch configuration (node -1: the default; value -1 on a
        node: back to the default).  Re-captures the step graph."""
        if self._lib.mw_set_node_blocks_per_cu(self.h, node, blocks_per_cu) != 0:
            raise _err(self._lib)

    def set_timed_node(self, name, every=1):
        """Bracket every launch of node kind `name` with HIP events inside the
        replayed step (None disables); resets the accumulators.  every > 1:
        only the first step of every run of `every` steps is timed."""
        if self._lib.mw_set_timed_node_every(self.h, name.encode() if name else None,
                                             int(every)) != 0:
            raise _err(self._lib)

    def set_timed_node_index(self, node, every=1):
        """set_timed_node for the one node at index `node` of node_names()."""
        if self._lib.mw_set_timed_node_index(self.h, int(node), int(every)) != 0:
            raise _err(self._lib)

    def timed_node(self):
        """(total ms, launches) accumulated since set_timed_node."""
        n = ctypes.c_int64(0)
        ms = self._lib.mw_timed_node_ms(self.h, ctypes.byref(n))
        return ms, n.value

    def enable_tracing(self, max_records=1 << 20):
        """Device tracing (reference MADRONA_TRACING, mw_gpu/tracing.hpp): every
        following step logs 40-byte DeviceLog records; 0 disables."""
        if self._lib.mw_trace_enable(self.h, int(max_records)) != 0:
            raise _err(self._lib)

    @staticmethod
    def trace_block_records():
        """True for the tracing build (block records compiled in)."""
        return bool(_lib.mw_trace_block_records())

    def trace_records(self):
        """(records as a TRACE_DTYPE array, number dropped to a full buffer)."""
        dropped = ctypes.c_int64(0)
        n = self._lib.mw_trace_read(self.h, None, 0, ctypes.byref(dropped))
        if n < 0:
            raise _err(self._lib)
        out = np.zeros(n // TRACE_DTYPE.itemsize, TRACE_DTYPE)
        if self._lib.mw_trace_read(self.h, out.ctypes.data, n, ctypes.byref(dropped)) < 0:
            raise _err(self._lib)
        return out, int(dropped.value)

    def trace_func_names(self):
        names, i = [], 0
        while True:
            s = self._lib.mw_trace_func_name(self.h, i)
            if s is None:
                return names
            names.append(s.decode())
            i += 1

    def dump_trace(self, path):
        """Writes the records as the flat binary file
        scripts/parse_device_tracing.py --trace_file reads."""
        recs, _ = self.trace_records()
        with open(path, "wb") as f:
            f.write(recs.tobytes())
        return len(recs)

    def close(self):
        if getattr(self, "h", None):
            self._lib.mw_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


def default_collisions_config(num_cubes=128, num_substeps=4, max_contacts=4096,
                              max_candidates=4096, num_joints=0, num_hinge_joints=0,
                              hull_paths=None):
    """dt 1/60, S=4, g=-9.8, unit mass cubes.  num_joints
    > 0 adds the joint workload: joint j ties cube 2j to 2j+1 with a fixed
    joint, or a hinge for the last num_hinge_joints.  hull_paths: .obj files
    loaded as convex hulls through PhysicsLoader (reference
    physics_assets.cpp:205-254); body i uses hull i % len(hull_paths)."""
    if 2 * num_joints > num_cubes or not 0 <= num_hinge_joints <= num_joints:
        raise ValueError("need 2 * num_joints <= num_cubes, 0 <= num_hinge_joints <= num_joints")
    paths = None
    if hull_paths:
        paths = ";".join(os.fspath(p) for p in hull_paths).encode()
    return CollisionsConfig(num_cubes, num_substeps, 1.0 / 60.0, -9.8, max_contacts,
                            max_candidates, 1.0, 1.5, 0.5, 0.5, num_joints, num_hinge_joints,
                            paths)


class CollisionsSim(Executor):
    """The `collisions` rigid-body environment (RigidBodyPhysicsSystem)."""

    def __init__(self, num_worlds, pos, rot, cfg=None, gpu_id=0, use_graph=True, **kw):
        cfg = cfg or default_collisions_config(num_cubes=pos.shape[1])
        self._pos = np.ascontiguousarray(pos, np.float32)
        self._rot = np.ascontiguousarray(rot, np.float32)
        assert self._pos.shape == (num_worlds, cfg.num_cubes, 3)
        assert self._rot.shape == (num_worlds, cfg.num_cubes, 4)
        inits = (CollisionsInit * num_worlds)()
        pbase = self._pos.ctypes.data
        rbase = self._rot.ctypes.data
        for w in range(num_worlds):
            inits[w].pos = pbase + w * cfg.num_cubes * 12
            inits[w].rot = rbase + w * cfg.num_cubes * 16
        self.cfg = cfg
        self.num_bodies = cfg.num_cubes + 1
        super().__init__("collisions", num_worlds, cfg, inits, ctypes.sizeof(CollisionsInit),
                         gpu_id=gpu_id, default_capacity=64, use_graph=use_graph, **kw)

    def bodies(self, w):
        """Per-body state of world w in the oracle's record layout."""
        return self._bodies_of(BODY_ARCHETYPE, w)

    def _bodies_of(self, A, w):
        out = np.zeros(self.num_bodies, BODY_DTYPE)
        ent = self.read_column(A, 0, w, np.uint32).reshape(-1, 2)
        n = len(ent)
        out = out[:n]
        out["gen"] = ent[:, 0]
        out["id"] = ent[:, 1].view(np.int32)
        out["pos"] = self.read_column(A, 1, w, np.float32).reshape(n, 3)
        out["rot"] = self.read_column(A, 2, w, np.float32).reshape(n, 4)
        out["vel"] = self.read_column(A, 4, w, np.float32).reshape(n, 6)
        out["objID"] = self.read_column(A, 5, w, np.int32)
        out["responseType"] = self.read_column(A, 6, w, np.uint32)
        prev = self.read_column(A, 7, w, np.float32).reshape(n, 7)
        out["prevPos"], out["prevRot"] = prev[:, :3], prev[:, 3:]
        ps = self.read_column(A, 8, w, np.float32).reshape(n, 7)
        out["presolvePos"], out["presolveRot"] = ps[:, :3], ps[:, 3:]
        out["presolveVel"] = self.read_column(A, 9, w, np.float32).reshape(n, 6)
        out["leafID"] = self.read_column(A, 12, w, np.int32)
        return out

    def candidates(self, w, cap=1 << 15):
        out = np.zeros((cap, 4), np.int32)
        n = self._lib.mw_phys_read_candidates(self.h, w, out.ctypes.data_as(ctypes.c_void_p), cap)
        if n < 0:
            raise _err(self._lib)
        return out[:n]

    def contacts(self, w, cap=1 << 14):
        out = np.zeros(cap, CONTACT_DTYPE)
        n = self._lib.mw_phys_read_contacts(self.h, w, out.ctypes.data_as(ctypes.c_void_p), cap)
        if n < 0:
            raise _err(self._lib)
        return out[:n]

    def counts(self):
        c = np.zeros(self.num_worlds, np.int32)
        k = np.zeros(self.num_worlds, np.int32)
        if self._lib.mw_phys_counts(self.h, c.ctypes.data_as(ctypes.c_void_p),
                               k.ctypes.data_as(ctypes.c_void_p)) < 0:
            raise _err(self._lib)
        return c, k

    def take_units(self):
        """(timed launches, candidates, contact manifolds, launches with the
        fused next-substep / first-substep filter work, narrowphase survivor
        pairs) summed over the live-timed physics launches since the last
        call; zeroes them."""
        out = np.zeros(5, np.int64)
        if self._lib.mw_phys_take_units(self.h, out.ctypes.data_as(ctypes.c_void_p)) < 0:
            raise _err(self._lib)
        return tuple(int(x) for x in out)

    def kernel_variants(self):
        """{kernel: True when it runs its global-image variant} (mw_create
        decides per LDS image; plane_lds / sat_lds: the plane / SAT kernel's
        LDS hull tables; sat_mink: the SAT edge query's Minkowski tables)."""
        out = np.zeros(11, np.int32)
        if self._lib.mw_phys_kernel_variants(self.h, out.ctypes.data_as(ctypes.c_void_p), 11) < 0:
            raise _err(self._lib)
        keys = ("refit", "find_overlaps", "sat", "contact", "solver", "plane_lds", "sat_lds", "sat_mink")
        d = {k: bool(v) for k, v in zip(keys, out)}
        d["solver_lanes"] = int(out[8])     # lanes per world the solver runs (64 or 32)
        d["solver_items_per_level"] = out[9] / 100.0   # what the last lane check read
        d["overlap_traversal"] = bool(out[10])  # worlds past the DFS threshold walk the BVH
        return d

    def bvh(self, w, cap=4096):
        nodes = np.zeros(cap, BVH_NODE_DTYPE)
        aabbs = np.zeros((self.num_bodies, 6), np.float32)
        n = self._lib.mw_phys_read_bvh(self.h, w, nodes.ctypes.data_as(ctypes.c_void_p),
                                  aabbs.ctypes.data_as(ctypes.c_void_p), cap)
        if n < 0:
            raise _err(self._lib)
        return nodes[:n], aabbs


# ---------------------------------------------------------------------------
# fantasy_vs (BASELINE.json configs[4])
# ---------------------------------------------------------------------------
FVS_ROW_DTYPE = np.dtype([("gen", np.uint32), ("id", np.int32), ("pos", np.float32, 3),
                          ("hp", np.int32), ("remaining", np.float32), ("extra", np.uint32)])


def gen_fvs_inits(num_worlds, num_dragons=50, num_knights=200, seed=0, first_world=0):
    """Reference example init (fvs.cpp:88-108), serial mt19937 over worlds;
    first_world selects a shard."""
    d = {"dragon_pos": np.zeros((num_worlds, num_dragons, 3), np.float32),
         "dragon_mana": np.zeros((num_worlds, num_dragons), np.float32),
         "knight_pos": np.zeros((num_worlds, num_knights, 3), np.float32),
         "knight_arrows": np.zeros((num_worlds, num_knights), np.int32)}
    _lib.mw_gen_fvs_inits(first_world, num_worlds, num_dragons, num_knights, seed,
                          *[d[k].ctypes.data_as(ctypes.c_void_p) for k in
                            ("dragon_pos", "dragon_mana", "knight_pos", "knight_arrows")])
    return d


class FvsSim(Executor):
    """The `fantasy_vs` environment: casters / archers, deaths destroy entities."""
    DRAGON, KNIGHT, TRACKER = 0, 1, 2

    def __init__(self, num_worlds, inits, first_world=0, gpu_id=0, use_graph=True,
                 env="fantasy_vs", **kw):
        # env "fantasy_vs_jobs": the same game written against the job API
        self._inits = {k: np.ascontiguousarray(v) for k, v in inits.items()}
        nd = self._inits["dragon_mana"].shape[1]
        nk = self._inits["knight_arrows"].shape[1]
        assert self._inits["dragon_mana"].shape[0] == num_worlds
        self.cfg = FvsConfig(nd, nk)
        arr = (FvsInit * num_worlds)()
        base = {k: v.ctypes.data for k, v in self._inits.items()}
        for w in range(num_worlds):
            arr[w].dragon_pos = base["dragon_pos"] + w * nd * 12
            arr[w].dragon_mana = base["dragon_mana"] + w * nd * 4
            arr[w].knight_pos = base["knight_pos"] + w * nk * 12
            arr[w].knight_arrows = base["knight_arrows"] + w * nk * 4
            arr[w].world_index = first_world + w
        super().__init__(env, num_worlds, self.cfg, arr, ctypes.sizeof(FvsInit),
                         gpu_id=gpu_id, default_capacity=64, use_graph=use_graph, **kw)

    def table(self, w, arch):
        """Rows of Dragon / Knight of world w in the oracle's record layout."""
        ent = self.read_column(arch, 0, w, np.uint32).reshape(-1, 2)
        n = len(ent)
        out = np.zeros(n, FVS_ROW_DTYPE)
        if n == 0:
            return out
        out["gen"] = ent[:, 0]
        out["id"] = ent[:, 1].view(np.int32)
        out["pos"] = self.read_column(arch, 1, w, np.float32).reshape(n, 3)
        out["hp"] = self.read_column(arch, 2, w, np.int32).reshape(n, 16)[:, 0]
        out["remaining"] = self.read_column(arch, 3, w, np.float32)
        out["extra"] = self.read_column(arch, 4, w, np.uint32)
        return out

    def num_rows(self, w, arch):
        return len(self.read_column(arch, 0, w, np.uint64))


class JobsCollisionsSim(Executor):
    """`collisions_jobs`: examples/collisions' own job-API toy (brute-force
    pairs, pass-through narrowphase, push-apart solver) on the Context job
    API; pos [W, N, 3] / rot [W, N, 4] from gen_collisions_inits."""
    CUBE, CANDIDATE, CONTACT = 0, 1, 2

    def __init__(self, num_worlds, pos, rot, max_candidates=1024, gpu_id=0, use_graph=True, **kw):
        self._pos = np.ascontiguousarray(pos, np.float32)
        self._rot = np.ascontiguousarray(rot, np.float32)
        n = self._pos.shape[1]
        assert self._pos.shape[0] == num_worlds and self._rot.shape[:2] == (num_worlds, n)
        self.num_objects = n
        self.cfg = JobsCollisionsConfig(n, max_candidates)
        arr = (CollisionsInit * num_worlds)()
        for w in range(num_worlds):
            arr[w].pos = self._pos.ctypes.data + w * n * 12
            arr[w].rot = self._rot.ctypes.data + w * n * 16
        super().__init__("collisions_jobs", num_worlds, self.cfg, arr, ctypes.sizeof(CollisionsInit),
                         gpu_id=gpu_id, default_capacity=64, use_graph=use_graph, **kw)

    def cubes(self, w):
        """CubeObject rows of world w (JC_ROW_DTYPE), table order."""
        ent = self.read_column(self.CUBE, 0, w, np.uint32).reshape(-1, 2)
        n = len(ent)
        out = np.zeros(n, JC_ROW_DTYPE)
        if n == 0:
            return out
        out["gen"] = ent[:, 0]
        out["id"] = ent[:, 1].view(np.int32)
        out["pos"] = self.read_column(self.CUBE, 1, w, np.float32).reshape(n, 3)
        out["rot"] = self.read_column(self.CUBE, 2, w, np.float32).reshape(n, 4)
        out["aabb"] = self.read_column(self.CUBE, 3, w, np.float32).reshape(n, 6)
        return out


class SimpleSim(CollisionsSim):
    """The `simple_taskgraph` environment: clamp + physics over two body
    archetypes (Sphere: objects + test object, Agent)."""
    SPHERE, AGENT = BODY_ARCHETYPE, BODY_ARCHETYPE + 1

    def __init__(self, num_worlds, pos, rot, cfg=None, gpu_id=0, use_graph=True,
                 env="simple_taskgraph", **kw):
        # env: a loaded world with simple_taskgraph's config, inits and body
        # archetypes (tests/ext_env/phys_grow.hip)
        cfg = cfg or default_collisions_config(num_cubes=pos.shape[1])
        self._pos = np.ascontiguousarray(pos, np.float32)
        self._rot = np.ascontiguousarray(rot, np.float32)
        inits = (CollisionsInit * num_worlds)()
        for w in range(num_worlds):
            inits[w].pos = self._pos.ctypes.data + w * cfg.num_cubes * 12
            inits[w].rot = self._rot.ctypes.data + w * cfg.num_cubes * 16
        self.cfg = cfg
        self.num_bodies = cfg.num_cubes + 2
        kw.setdefault("default_capacity", 64)
        Executor.__init__(self, env, num_worlds, cfg, inits,
                          ctypes.sizeof(CollisionsInit), gpu_id=gpu_id, use_graph=use_graph, **kw)

    def bodies(self, w):
        """Sphere rows then Agent rows (the reference query order)."""
        return np.concatenate([self._bodies_of(self.SPHERE, w), self._bodies_of(self.AGENT, w)])
