"""GPU: the refit kernel's LDS holds about two thirds of the BVH node
capacity (physics.hip refitLDSNodes, broadphase.hip refitKernel); a world
whose rebuild used more nodes refits its node slab in place in HBM inside
the same launch.  Both forms must give the same bits: runs with the LDS
capacity forced below every world's used nodes (all in place) and between
the worlds' counts (81-97 used nodes for 128 cubes: mixed) against the
default (all in LDS), every body and the candidate / contact counts."""
import numpy as np
import pytest

from oracle_lib import gen_collisions_inits

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cap", ["8", "88"])
def test_refit_in_place_worlds_bit_exact(monkeypatch, cap):
    import madrona_mi355x as mw
    W, n = 32, 128
    pos, rot = gen_collisions_inits(W, n, seed=5)
    cfg = mw.default_collisions_config(n, 4, 4096, 4096)
    monkeypatch.delenv("MADRONA_MW_REFIT_LDS_NODES", raising=False)
    ref = mw.CollisionsSim(W, pos, rot, cfg)
    monkeypatch.setenv("MADRONA_MW_REFIT_LDS_NODES", cap)
    sim = mw.CollisionsSim(W, pos, rot, cfg)
    for _ in range(3):
        ref.step(20)
        sim.step(20)
        assert sim.error_flags() == 0
        for w in range(W):
            assert sim.bodies(w).tobytes() == ref.bodies(w).tobytes(), (cap, w)
        for a, b in zip(sim.counts(), ref.counts()):
            assert np.array_equal(a, b), cap
