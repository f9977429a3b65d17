"""GPU parity for simple_taskgraph (BASELINE.json configs[0] / [1]): clamp
ParallelForNode + rigid-body physics over two body archetypes (Sphere,
Agent), against the reference itself (oracle/_ref simple worlds, live when
present) and the golden fixtures generated from it.  Bit-exact bodies."""
import os

import numpy as np
import pytest

import oracle_lib as ol
from test_collisions_gpu import _cfg_pair, _diff

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "simple_ref.npz")


def _mw():
    import madrona_mi355x as mw
    return mw


def test_simple_taskgraph_matches_reference_golden():
    mw = _mw()
    g = np.load(GOLDEN)
    gcfg, _ = _cfg_pair(num_cubes=100)
    W = g["pos"].shape[0]
    sim = mw.SimpleSim(W, g["pos"], g["rot"], gcfg)
    done = 0
    for s in (1, 10, 60):
        sim.step(s - done)
        done = s
        assert sim.error_flags() == 0, mw.ERR_BITS
        for w in range(W):
            d = _diff(sim.bodies(w), g[f"s{s}/w{w}"])
            assert d is None, f"step {s} world {w}: {d}"


@pytest.mark.skipif(not ol.ref_available(), reason="reference build absent")
def test_simple_taskgraph_matches_live_reference_long():
    mw = _mw()
    gcfg, ocfg = _cfg_pair(num_cubes=100)
    W = 6
    pos, rot = ol.gen_collisions_inits(W, 100, seed=9)
    sim = mw.SimpleSim(W, pos, rot, gcfg)
    ref = ol.ReferenceSimple(ocfg, pos, rot)
    for chunk in range(10):
        sim.step(20)
        ref.step(20)
        for w in range(W):
            d = _diff(sim.bodies(w), ref.bodies(w))
            assert d is None, f"step {20 * (chunk + 1)} world {w}: {d}"


def test_simple_taskgraph_full_size_runs_clean():
    # BASELINE.json configs[1] size (8192 worlds): no error flags, agents
    # exported through getExported slot 0 (one row per world).
    mw = _mw()
    gcfg, _ = _cfg_pair(num_cubes=100, max_contacts=4096)
    W = 8192
    pos, rot = mw.gen_collisions_inits(W, 100, seed=0)
    sim = mw.SimpleSim(W, pos, rot, gcfg)
    sim.step(30)
    assert sim.error_flags() == 0, mw.ERR_BITS
    agents = sim.exported_array(0, np.float32).reshape(-1, 3)
    assert agents.shape == (W, 3) and np.all(np.isfinite(agents))
