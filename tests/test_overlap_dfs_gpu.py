"""GPU: findOverlaps' BVH traversal (reference
include/madrona/physics.inl:61-100, BVH::findOverlaps, called per body by
src/physics/broadphase.cpp:897-932).

Worlds with more leaves than MADRONA_MW_OVERLAP_DFS_LEAVES (default 512) walk
the 4-wide BVH per body with an LDS stack; smaller worlds sweep the leaves in
the tree's emission order (broadphase.hip).  Both emit the reference's
candidates in the reference's order, so forcing either form on any world
must stay bit-exact against the oracle, and the traversal's cost per world
must grow with the bodies, not with bodies x leaves."""
import numpy as np
import pytest

from oracle_lib import gen_collisions_inits
from test_lds_fallback_gpu import _grid_world, _lockstep, _pair

pytestmark = pytest.mark.gpu


def test_dfs_forced_on_collisions_worlds_bit_exact(monkeypatch):
    """Threshold 0: the 128-cube collisions worlds take the traversal (their
    bodies pile up, so queries overlap several subtrees); candidates and
    contacts equal the oracle's every step."""
    monkeypatch.setenv("MADRONA_MW_OVERLAP_DFS_LEAVES", "0")
    W, n = 8, 128
    pos, rot = gen_collisions_inits(W, n, seed=5)
    sim, orc = _pair(W, n, pos, rot)
    _lockstep(sim, orc, W, 60)
    c, _ = sim.counts()
    assert np.all(c > 0), c


def test_dfs_forced_on_simple_worlds_spans_body_archetypes(monkeypatch):
    """Threshold 0 on simple_taskgraph: its bodies live in two archetypes
    (spheres, then the agent), so one 256-row chunk of the traversal kernels
    numbers rows across both, as the sweep does; bodies equal the oracle's
    every step (candidate order feeds the contact order, hence the bits)."""
    import madrona_mi355x as mw
    import oracle_lib as ol
    from test_collisions_gpu import _cfg_pair, _diff
    monkeypatch.setenv("MADRONA_MW_OVERLAP_DFS_LEAVES", "0")
    gcfg, ocfg = _cfg_pair(num_cubes=100)
    W = 4
    pos, rot = ol.gen_collisions_inits(W, 100, seed=3)
    sim = mw.SimpleSim(W, pos, rot, gcfg)
    assert sim.kernel_variants()["overlap_traversal"]
    orc = ol.OracleSimple(ocfg, pos, rot)
    for s in range(1, 121):
        sim.step(1)
        orc.step(1)
        for w in range(W):
            d = _diff(sim.bodies(w), orc.bodies(w))
            assert d is None, f"step {s} world {w}: {d}"
    assert sim.error_flags() == 0, mw.ERR_BITS


def test_default_small_worlds_do_not_launch_the_traversal():
    """129-leaf collisions worlds stay on the one-block sweep kernels: the
    traversal launches are not created below the threshold."""
    import madrona_mi355x as mw
    W, n = 2, 128
    pos, rot = gen_collisions_inits(W, n, seed=1)
    sim = mw.CollisionsSim(W, pos, rot, mw.default_collisions_config(n, 4, 2048, 2048))
    assert not sim.kernel_variants()["overlap_traversal"]


@pytest.mark.parametrize("dfs_leaves", ["512", "-1"])
def test_large_world_traversal_and_sweep_bit_exact(monkeypatch, dfs_leaves):
    """1200 cubes per world (past the default threshold): the traversal
    (default) and the leaf sweep (-1) each match the oracle."""
    monkeypatch.setenv("MADRONA_MW_OVERLAP_DFS_LEAVES", dfs_leaves)
    W, n = 2, 1200
    pos, rot = _grid_world(W, n, spacing=2.2)
    sim, orc = _pair(W, n, pos, rot, max_contacts=8192, max_candidates=8192)
    _lockstep(sim, orc, W, 8)


def test_world_past_16bit_indices_refused():
    """Leaf ranks (findOverlaps) and body slots (solver records) are 16-bit:
    a world past those limits is refused at creation with the limit named,
    not indexed wrongly (the body-slot limit, 32767, binds first)."""
    import madrona_mi355x as mw
    W, n = 1, 40000
    pos, rot = _grid_world(W, n, spacing=2.5)
    g = mw.default_collisions_config(n, 1, 1024, 1024)
    with pytest.raises(mw.MadronaError, match="per world must be <= 32767"):
        mw.CollisionsSim(W, pos, rot, g)
