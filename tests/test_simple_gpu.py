"""GPU parity for simple_taskgraph (BASELINE.json configs[0] / [1]): clamp
ParallelForNode + rigid-body physics over two body archetypes (Sphere,
Agent).  Bit-exact bodies against

  * the reference's own golden snapshots (steps 1, 10, 50: before any face
    manifold whose reference value is undefined, see test_simple_oracle.py);
  * the live reference (oracle/_ref) on every step before the oracle reports
    the first such manifold in a world;
  * the oracle (oracle/mw_oracle.cpp simple mode, pinned to the reference
    above) on every step, through and past those manifolds, and its golden
    snapshot at step 150.
"""
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


def test_simple_taskgraph_matches_golden():
    mw = _mw()
    g = np.load(GOLDEN)
    gcfg, _ = _cfg_pair(num_cubes=100)
    W = g["pos"].shape[0]
    sim = mw.SimpleSim(W, g["pos"], g["rot"], gcfg)
    done = 0
    for s in (1, 10, 50, 150):
        sim.step(s - done)
        done = s
        assert sim.error_flags() == 0, mw.ERR_BITS
        for w in range(W):
            key = f"s{s}/w{w}" if f"s{s}/w{w}" in g else f"orc_s{s}/w{w}"
            d = _diff(sim.bodies(w), g[key])
            assert d is None, f"{key}: {d}"


@pytest.mark.parametrize("nsub,seed", [(4, 9), (1, 0)])
def test_simple_taskgraph_matches_oracle_and_reference(nsub, seed):
    mw = _mw()
    gcfg, ocfg = _cfg_pair(num_cubes=100, num_substeps=nsub)
    W, STEPS = 6, 200
    pos, rot = ol.gen_collisions_inits(W, 100, seed=seed)
    sim = mw.SimpleSim(W, pos, rot, gcfg)
    orc = ol.OracleSimple(ocfg, pos, rot)
    ref = ol.ReferenceSimple(ocfg, pos, rot) if ol.ref_available() else None
    live = [True] * W
    for s in range(1, STEPS + 1):
        sim.step(1)
        orc.step(1)
        if ref is not None and any(live):
            ref.step(1)
        for w in range(W):
            got = sim.bodies(w)
            d = _diff(got, orc.bodies(w))
            assert d is None, f"vs oracle, step {s} world {w}: {d}"
            if live[w] and orc.ub_manifolds(w):
                live[w] = False
            if ref is not None and live[w]:
                d = _diff(got, ref.bodies(w))
                assert d is None, f"vs reference, step {s} world {w}: {d}"
        if s % 50 == 0:
            assert sim.error_flags() == 0, mw.ERR_BITS
    assert not all(live), "no world reached an undefined manifold: UB path not covered"


def test_simple_taskgraph_full_size_sampled_worlds():
    # BASELINE.json configs[1] size (8192 worlds): no error flags, agents
    # exported through getExported slot 0 (one row per world), and sampled
    # worlds (first, middle, last) bit-exact against the oracle replaying
    # them from the same per-world seeds.
    mw = _mw()
    gcfg, ocfg = _cfg_pair(num_cubes=100, max_contacts=4096)
    W, STEPS = 8192, 60
    pos, rot = mw.gen_collisions_inits(W, 100, seed=0)
    sim = mw.SimpleSim(W, pos, rot, gcfg)
    sample = [0, 1, W // 2, W - 1]
    orc = ol.OracleSimple(ocfg, np.ascontiguousarray(pos[sample]), np.ascontiguousarray(rot[sample]))
    sim.step(STEPS)
    orc.step(STEPS, 4)
    assert sim.error_flags() == 0, mw.ERR_BITS
    for i, w in enumerate(sample):
        d = _diff(sim.bodies(w), orc.bodies(i))
        assert d is None, f"world {w}: {d}"
    agents = sim.exported_array(0, np.float32).reshape(-1, 3)
    assert agents.shape == (W, 3) and np.all(np.isfinite(agents))
    for i, w in enumerate(sample):
        b = orc.bodies(i)
        assert agents[w].tobytes() == b["pos"][-1].tobytes(), w
