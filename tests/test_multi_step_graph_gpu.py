"""GPU: runs of plain steps replayed as one multi-step graph
(MADRONA_MW_STEPS_PER_GRAPH = K, executor.hip captureMultiStep / runSteps).
K steps captured back to back must be the same K steps: fantasy_vs against
the oracle through its deaths (step counts that are not multiples of K, so
multi-step and single-step launches mix), and collisions with sampled live
node timing (every 10th step split, the others plain) bit-exact against the
single-step graph."""
import numpy as np
import pytest

import oracle_lib as ol
from oracle_lib import gen_collisions_inits

pytestmark = pytest.mark.gpu


def test_fvs_multi_step_graph_bit_exact(monkeypatch):
    monkeypatch.setenv("MADRONA_MW_STEPS_PER_GRAPH", "8")
    import madrona_mi355x as mw
    W = 4
    inits = ol.gen_fvs_inits(W, 50, 200, seed=3)
    sim = mw.FvsSim(W, inits)
    orc = ol.OracleFvs(inits)
    for n in (5, 37, 300, 411, 13):
        sim.step(n)
        orc.step(n)
        assert sim.error_flags() == 0
        for w in range(W):
            for arch in (0, 1):
                a, b = sim.table(w, arch), orc.table(w, arch)
                assert a.tobytes() == b.tobytes(), (n, w, arch)


def test_collisions_multi_step_graph_with_sampled_timing(monkeypatch):
    import madrona_mi355x as mw
    W, n = 16, 64
    pos, rot = gen_collisions_inits(W, n, seed=9)
    cfg = mw.default_collisions_config(n, 4, 4096, 4096)
    monkeypatch.setenv("MADRONA_MW_STEPS_PER_GRAPH", "1")
    ref = mw.CollisionsSim(W, pos, rot, cfg)
    monkeypatch.setenv("MADRONA_MW_STEPS_PER_GRAPH", "8")
    sim = mw.CollisionsSim(W, pos, rot, cfg)
    sim.set_timed_node("SolverNode", every=10)
    ref.step(47)
    sim.step(47)
    ms, launches = sim.timed_node()
    assert launches > 0
    for w in range(W):
        a, b = sim.bodies(w), ref.bodies(w)
        assert a.tobytes() == b.tobytes(), w
    assert np.array_equal(sim.counts()[0], ref.counts()[0])
