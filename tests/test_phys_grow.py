"""A physics world whose other table grows: every
growth of a table re-allocates the entity ID store, which the physics module
caches in its kernel arguments; PhysicsModule::stateResized (called by
StateManager::growArchetype) refreshes that copy.

tests/ext_env/phys_grow.hip is simple_taskgraph's world plus a growable Mark
table filled with 8 entities per step from a system ahead of physics.  The
marks never touch a body, so the bodies must stay bit-identical to the
built-in simple_taskgraph world stepping the same inits, through several
growths of Mark (and of the ID store), with no error flag -- on the HIP back
end and on the CPU back end."""
import ctypes
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SO = {"gpu": os.path.join(HERE, "ext_env", "build", "libphys_grow.so"),
      "cpu": os.path.join(HERE, "ext_env", "build", "libphys_grow_cpu.so")}
ENV = "phys_grow"
DECLARED = 16            # Mark's starting rows per world (mw_config.default_capacity)
MARKS_PER_STEP = 8


def _mw(backend):
    import madrona_mi355x as mw
    if ENV not in mw.env_names(backend):
        if not os.path.exists(SO[backend]):
            pytest.skip(f"{SO[backend]} not built (make -C tests/ext_env)")
        assert mw.load_env(SO[backend], backend) == 1
    return mw


def _capacity(sim, arch, col=1):
    b, c = ctypes.c_int32(), ctypes.c_int32()
    assert sim._lib.mw_column_info(sim.h, arch, col, ctypes.byref(b), ctypes.byref(c)) == 0
    return c.value


def _run(backend, W, n, steps, **kw):
    mw = _mw(backend)
    cfg = mw.default_collisions_config(num_cubes=n, max_contacts=1024, max_candidates=1024)
    pos, rot = mw.gen_collisions_inits(W, n, seed=4)
    grow = mw.SimpleSim(W, pos, rot, cfg, env=ENV, backend=backend, default_capacity=DECLARED, **kw)
    plain = mw.SimpleSim(W, pos, rot, cfg, backend=backend, **kw)
    mark = mw.SimpleSim.AGENT + 1
    assert _capacity(grow, mark) == DECLARED
    for s in range(1, steps + 1):
        grow.step(1)
        plain.step(1)
        assert grow.error_flags() == 0, (s, mw.ERR_BITS)
        for w in range(W):
            a, b = grow.bodies(w), plain.bodies(w)
            assert a.tobytes() == b.tobytes(), f"step {s} world {w}: bodies differ"
    rows = [len(grow.read_column(mark, 0, w, np.uint64)) for w in range(W)]
    assert rows == [MARKS_PER_STEP * steps] * W, rows
    assert _capacity(grow, mark) >= 8 * DECLARED       # grew at least three times
    grow.close()
    plain.close()


def test_physics_follows_id_store_growth_cpu():
    _run("cpu", 3, 24, 20, num_workers=2)


@pytest.mark.gpu
def test_physics_follows_id_store_growth_gpu():
    _run("gpu", 4, 40, 40)
