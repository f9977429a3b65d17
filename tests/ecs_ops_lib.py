"""Both builds of the "ecs_ops" test world (tests/ext_env/ecs_ops_rules.hpp):

  * EcsOpsSim -- this framework, the world built out of tree into
    tests/ext_env/build/libecs_ops.so and loaded through mw_load_env;
  * RefEcsOps -- the same world on the reference's own ECS
    (oracle/_ref/libmadrona_ref_ecs.so, oracle/ref_ecs.cpp).

Rows are returned as numpy structured arrays with identical dtypes."""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV_SO = os.path.join(ROOT, "tests", "ext_env", "build", "libecs_ops.so")
ENV_SO_CPU = os.path.join(ROOT, "tests", "ext_env", "build", "libecs_ops_cpu.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libmadrona_ref_ecs.so")
ENV_NAME = "EcsOps::World"
NUM_AGENTS = 40

AGENT_DTYPE = np.dtype([("gen", np.uint32), ("id", np.int32), ("pos", np.float32, 3),
                        ("vel", np.float32, 3), ("hits", np.int32), ("spawned", np.int32),
                        ("pairsMade", np.int32), ("destroyed", np.int32)])
PAIR_DTYPE = np.dtype([("a_gen", np.uint32), ("a_id", np.int32), ("b_gen", np.uint32),
                       ("b_id", np.int32), ("d2", np.float32), ("pad", np.int32)])
SPAWN_DTYPE = np.dtype([("gen", np.uint32), ("id", np.int32), ("p_gen", np.uint32),
                        ("p_id", np.int32), ("born", np.int32), ("hits", np.int32),
                        ("serial", np.int32), ("pad", np.int32)])
STATS_DTYPE = np.dtype([("tick", np.int32), ("numPairs", np.int32), ("numSpawns", np.int32),
                        ("sumHits", np.int32), ("sumD2", np.float32), ("dynTicks", np.int32)])
assert AGENT_DTYPE.itemsize == 48 and PAIR_DTYPE.itemsize == 24
assert SPAWN_DTYPE.itemsize == 32 and STATS_DTYPE.itemsize == 24

# archetype indices in the framework build (registration order)
ARCH_AGENT, ARCH_PAIR, ARCH_SPAWN, ARCH_STATS = 0, 1, 2, 3


def ref_available():
    return os.path.exists(REF_SO)


class EcsConfig(ctypes.Structure):
    _fields_ = [("numAgents", ctypes.c_int32), ("growSpawns", ctypes.c_int32)]


class EcsInit(ctypes.Structure):
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


class EcsOpsSim:
    def __init__(self, num_worlds, first_world=0, tmp_alloc_bytes=64 * 1024, grow_spawns=False, **kw):
        # grow_spawns: Spawn registered without a size (registerArchetype),
        # starting at default_capacity rows per world and grown by the
        # executor between steps
        mw = load_env(kw.get("backend"))
        inits = (EcsInit * num_worlds)(*[EcsInit(first_world + w) for w in range(num_worlds)])
        self.exec = mw.Executor(ENV_NAME, num_worlds, EcsConfig(NUM_AGENTS, 1 if grow_spawns else 0), inits,
                                ctypes.sizeof(EcsInit), tmp_alloc_bytes=tmp_alloc_bytes, **kw)
        self.num_worlds = num_worlds

    def step(self, n=1):
        self.exec.step(n)

    def _cols(self, arch, world, cols):
        return [self.exec.read_column(arch, c, world, np.uint8, max_rows=4096) for c in cols]

    def agents(self, w):
        parts = self._cols(ARCH_AGENT, w, (0, 1, 2, 3))
        n = len(parts[0]) // 8
        if n == 0:
            return np.zeros(0, AGENT_DTYPE)
        rows = np.hstack([p.reshape(n, -1) for p in parts])
        return rows.view(AGENT_DTYPE).reshape(n)

    def pairs(self, w):
        (p,) = self._cols(ARCH_PAIR, w, (1,))
        return p.view(PAIR_DTYPE)

    def spawns(self, w):
        parts = self._cols(ARCH_SPAWN, w, (0, 1))
        n = len(parts[0]) // 8
        if n == 0:
            return np.zeros(0, SPAWN_DTYPE)
        rows = np.hstack([p.reshape(n, -1) for p in parts])
        return rows.view(SPAWN_DTYPE).reshape(n)

    def stats(self, w):
        (s,) = self._cols(ARCH_STATS, w, (1,))
        return s.view(STATS_DTYPE)[0]

    def entity_row(self, w, entity_id, gen):
        loc = self.exec.entity_loc(w, int(entity_id), int(gen))
        return None if loc is None else loc[1]

    def error_flags(self):
        return self.exec.error_flags()

    def close(self):
        self.exec.close()


class RefEcsOps:
    def __init__(self, num_worlds, first_world=0):
        lib = ctypes.CDLL(REF_SO)
        lib.ref_ecs_create.restype = ctypes.c_void_p
        lib.ref_ecs_create.argtypes = [ctypes.c_int32] * 3
        lib.ref_ecs_step.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        for f in ("ref_ecs_read_agents", "ref_ecs_read_pairs", "ref_ecs_read_spawns"):
            getattr(lib, f).argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                        ctypes.c_int32]
        lib.ref_ecs_read_stats.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]
        lib.ref_ecs_entity_row.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                           ctypes.c_uint32, ctypes.c_void_p]
        self.lib = lib
        self.h = lib.ref_ecs_create(num_worlds, NUM_AGENTS, first_world)
        self.num_worlds = num_worlds

    def step(self, n=1):
        self.lib.ref_ecs_step(self.h, n)

    def _read(self, fn, w, dtype, cap=4096):
        out = np.zeros(cap, dtype)
        n = fn(self.h, w, out.ctypes.data, cap)
        return out[:n]

    def agents(self, w):
        return self._read(self.lib.ref_ecs_read_agents, w, AGENT_DTYPE)

    def pairs(self, w):
        return self._read(self.lib.ref_ecs_read_pairs, w, PAIR_DTYPE)

    def spawns(self, w):
        return self._read(self.lib.ref_ecs_read_spawns, w, SPAWN_DTYPE)

    def stats(self, w):
        out = np.zeros(1, STATS_DTYPE)
        self.lib.ref_ecs_read_stats(self.h, w, out.ctypes.data)
        return out[0]

    def entity_row(self, w, entity_id, gen):
        r = ctypes.c_int32()
        rc = self.lib.ref_ecs_entity_row(self.h, w, int(entity_id), int(gen), ctypes.byref(r))
        return None if rc else r.value


SPAWN_CONTENT = ("p_gen", "p_id", "born", "hits", "serial")


def compare_world(sim, ref, w, where="", exact_ids=False):
    """Bit-exact agents, pairs, stats and spawn contents / row order; spawn
    entity IDs (made by parallel lanes) checked for consistency: unique,
    alive, mapped to their own row (SURVEY.md §8c relabelling rule).
    exact_ids: the spawn rows' entity IDs equal the reference's too (a
    world-serial run: mw_config.serial_nodes or the CPU back end)."""
    if exact_ids:
        a, b = sim.spawns(w), ref.spawns(w)
        assert a.tobytes() == b.tobytes(), f"{where} world {w}: spawn rows / IDs differ"
    a, b = sim.agents(w), ref.agents(w)
    assert a.tobytes() == b.tobytes(), f"{where} world {w}: agents differ"
    a, b = sim.pairs(w), ref.pairs(w)
    assert len(a) == len(b), f"{where} world {w}: {len(a)} vs {len(b)} pairs"
    assert a.tobytes() == b.tobytes(), f"{where} world {w}: pairs differ"
    a, b = sim.spawns(w), ref.spawns(w)
    assert len(a) == len(b), f"{where} world {w}: {len(a)} vs {len(b)} spawns"
    for f in SPAWN_CONTENT:
        assert a[f].tobytes() == b[f].tobytes(), f"{where} world {w}: spawn {f} differs"
    assert len(set(a["id"].tolist())) == len(a), f"{where} world {w}: duplicate spawn ids"
    for r, (i, g) in enumerate(zip(a["id"], a["gen"])):
        assert sim.entity_row(w, i, g) == r, f"{where} world {w}: spawn row {r} lookup"
    sa, sb = sim.stats(w), ref.stats(w)
    assert sa.tobytes() == sb.tobytes(), f"{where} world {w}: stats {sa} vs {sb}"
