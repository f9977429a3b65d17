"""Both builds of the "cross_rows" test world (tests/ext_env/cross_rows_rules.hpp):

  * CrossSim  -- this framework, built out of tree into
    tests/ext_env/build/libcross_rows.so (libcross_rows_cpu.so for the CPU
    back end) and loaded through mw_load_env;
  * RefCross  -- the same world on the reference's own ECS
    (oracle/_ref/libmadrona_ref_cross.so, oracle/ref_cross.cpp).

Rows come back as numpy structured arrays with identical dtypes."""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV_SO = os.path.join(ROOT, "tests", "ext_env", "build", "libcross_rows.so")
ENV_SO_CPU = os.path.join(ROOT, "tests", "ext_env", "build", "libcross_rows_cpu.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libmadrona_ref_cross.so")
ENV_NAME = "CrossRows::World"
NUM_CELLS = 48

CELL_DTYPE = np.dtype([("gen", np.uint32), ("id", np.int32), ("value", np.int32),
                       ("heat", np.float32), ("next_gen", np.uint32), ("next_id", np.int32),
                       ("spark_gen", np.uint32), ("spark_id", np.int32), ("prefix", np.uint32),
                       ("pad", np.int32)])
SPARK_DTYPE = np.dtype([("gen", np.uint32), ("id", np.int32), ("src_gen", np.uint32),
                        ("src_id", np.int32), ("born", np.int32), ("energy", np.int32)])
STATS_DTYPE = np.dtype([("tick", np.int32), ("cells", np.int32), ("sparks", np.int32),
                        ("running", np.uint32)])
assert CELL_DTYPE.itemsize == 40 and SPARK_DTYPE.itemsize == 24

ARCH_CELL, ARCH_SPARK, ARCH_STATS = 0, 1, 2


def ref_available():
    return os.path.exists(REF_SO)


class CrossConfig(ctypes.Structure):
    _fields_ = [("numCells", ctypes.c_int32), ("perNodeSerial", ctypes.c_int32)]


class CrossInit(ctypes.Structure):
    _fields_ = [("worldIndex", ctypes.c_int32)]


def load_env(backend=None):
    import madrona_mi355x as mw
    backend = backend or mw.DEFAULT_BACKEND
    so = ENV_SO_CPU if backend == "cpu" else ENV_SO
    if ENV_NAME not in mw.env_names(backend):
        if not os.path.exists(so):
            raise FileNotFoundError(f"{so} not built (make -C tests/ext_env)")
        assert mw.load_env(so, backend) == 1
    return mw


class CrossSim:
    def __init__(self, num_worlds, per_node_serial=False, first_world=0, graph=None, **kw):
        # graph: None = the world's row nodes; "peek" / "poke" = the
        # cross-row check's one-node graphs (cross_rows.hip peekSystem /
        # pokeSystem)
        mw = load_env(kw.get("backend"))
        inits = (CrossInit * num_worlds)(*[CrossInit(first_world + w) for w in range(num_worlds)])
        mode = {None: 1 if per_node_serial else 0, "peek": 2, "poke": 3}[graph]
        self.exec = mw.Executor(ENV_NAME, num_worlds, CrossConfig(NUM_CELLS, mode),
                                inits, ctypes.sizeof(CrossInit), **kw)
        self.num_worlds = num_worlds

    def step(self, n=1):
        self.exec.step(n)

    def _rows(self, arch, world, dtype):
        parts = [self.exec.read_column(arch, c, world, np.uint8, max_rows=4096) for c in (0, 1)]
        n = len(parts[0]) // 8
        if n == 0:
            return np.zeros(0, dtype)
        return np.hstack([p.reshape(n, -1) for p in parts]).view(dtype).reshape(n)

    def cells(self, w):
        return self._rows(ARCH_CELL, w, CELL_DTYPE)

    def sparks(self, w):
        return self._rows(ARCH_SPARK, w, SPARK_DTYPE)

    def stats(self, w):
        s = self.exec.read_column(ARCH_STATS, 1, w, np.uint8)
        return s.view(STATS_DTYPE)[0]

    def error_flags(self):
        return self.exec.error_flags()

    def close(self):
        self.exec.close()


class RefCross:
    def __init__(self, num_worlds, first_world=0):
        lib = ctypes.CDLL(REF_SO)
        lib.ref_cross_create.restype = ctypes.c_void_p
        lib.ref_cross_create.argtypes = [ctypes.c_int32] * 3
        lib.ref_cross_step.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        for f in ("ref_cross_read_cells", "ref_cross_read_sparks"):
            getattr(lib, f).argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                        ctypes.c_int32]
        lib.ref_cross_read_stats.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]
        self.lib = lib
        self.h = lib.ref_cross_create(num_worlds, NUM_CELLS, first_world)
        self.num_worlds = num_worlds

    def step(self, n=1):
        self.lib.ref_cross_step(self.h, n)

    def _read(self, fn, w, dtype, cap=4096):
        out = np.zeros(cap, dtype)
        n = fn(self.h, w, out.ctypes.data, cap)
        return out[:n]

    def cells(self, w):
        return self._read(self.lib.ref_cross_read_cells, w, CELL_DTYPE)

    def sparks(self, w):
        return self._read(self.lib.ref_cross_read_sparks, w, SPARK_DTYPE)

    def stats(self, w):
        out = np.zeros(1, STATS_DTYPE)
        self.lib.ref_cross_read_stats(self.h, w, out.ctypes.data)
        return out[0]


def compare_world(sim, ref, w, where=""):
    """Bit-exact cells, sparks (entity IDs included) and stats."""
    a, b = sim.cells(w), ref.cells(w)
    assert len(a) == len(b), f"{where} world {w}: {len(a)} vs {len(b)} cells"
    assert a.tobytes() == b.tobytes(), f"{where} world {w}: cells differ"
    a, b = sim.sparks(w), ref.sparks(w)
    assert len(a) == len(b), f"{where} world {w}: {len(a)} vs {len(b)} sparks"
    assert a.tobytes() == b.tobytes(), f"{where} world {w}: sparks differ"
    sa, sb = sim.stats(w), ref.stats(w)
    assert sa.tobytes() == sb.tobytes(), f"{where} world {w}: stats {sa} vs {sb}"


def worlds_equal(sim, ref, w):
    return (sim.cells(w).tobytes() == ref.cells(w).tobytes() and
            sim.sparks(w).tobytes() == ref.sparks(w).tobytes() and
            sim.stats(w).tobytes() == ref.stats(w).tobytes())
