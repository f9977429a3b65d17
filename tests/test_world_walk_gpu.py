"""GPU: the world walk (the persistent megakernel; reference
src/mw/device/megakernel_impl.inl:29-55).  By default (MADRONA_MW_WORLD_WALK=0
turns it off at creation) runs of consecutive world-local nodes are walked by
one kernel, a wave per world calling each node's world function in graph
order through the dispatch generated from the world source at build time
(tools/gen_walk_dispatch.py: direct calls, no function pointers); a world
with structural work stops at the commit point and worldResumeKernel commits
and finishes it.  Every state must equal the per-node launches bit for bit:
  * fantasy_vs through its deaths (every fvs node is world-local: the tick is
    one walk run), also against the oracle;
  * ecs_ops (row-parallel makeEntityNow / makeTemporary / destroyEntityNow /
    tmpAlloc, a dynamic-count node that splits the graph into runs);
  * cross_rows world-serially (serial row nodes inside a walk).
"""
import numpy as np
import pytest

import cross_rows_lib as cl
import ecs_ops_lib as el
import oracle_lib as ol

pytestmark = pytest.mark.gpu


def _walk(monkeypatch, on):
    monkeypatch.setenv("MADRONA_MW_WORLD_WALK", "1" if on else "0")


def test_fvs_walk_bit_exact_through_deaths(monkeypatch):
    import madrona_mi355x as mw
    W = 48
    inits = ol.gen_fvs_inits(W, 50, 200, seed=3)
    _walk(monkeypatch, True)
    a = mw.FvsSim(W, inits)
    _walk(monkeypatch, False)
    b = mw.FvsSim(W, inits)
    assert a.world_walk_runs() == 1 and b.world_walk_runs() == 0
    orc = ol.OracleFvs(inits)
    for chunk in range(8):
        a.step(100)
        b.step(100)
        orc.step(100)
        assert a.error_flags() == 0
        for w in range(W):
            for arch in (0, 1):
                same = a.table(w, arch).tobytes() == b.table(w, arch).tobytes()
                assert same, (chunk, w, arch)
        for w in range(0, W, 7):
            for arch in (0, 1):
                same = a.table(w, arch).tobytes() == orc.table(w, arch).tobytes()
                assert same, ("oracle", chunk, w, arch)
    assert sum(len(orc.table(w, 0)) for w in range(W)) < 50 * W   # dragons died


def test_ecs_ops_walk_bit_exact(monkeypatch):
    W, steps = 64, 30
    _walk(monkeypatch, True)
    a = el.EcsOpsSim(W)
    _walk(monkeypatch, False)
    b = el.EcsOpsSim(W)
    assert a.exec.world_walk_runs() >= 1
    for s in range(steps):
        a.step()
        b.step()
        assert a.error_flags() == 0 and b.error_flags() == 0
        for w in range(0, W, 5):
            for get in (a.agents, a.spawns, a.pairs, a.stats):
                other = getattr(b, get.__name__)
                same = get(w).tobytes() == other(w).tobytes()
                assert same, (s, w, get.__name__)


def test_cross_rows_serial_walk_matches_reference(monkeypatch):
    W, steps = 16, 20
    _walk(monkeypatch, True)
    sim = cl.CrossSim(W, serial_nodes=True)
    ref = cl.RefCross(W) if cl.ref_available() else None
    assert sim.exec.world_walk_runs() >= 1
    _walk(monkeypatch, False)
    plain = cl.CrossSim(W, serial_nodes=True)
    for s in range(steps):
        sim.step()
        plain.step()
        if ref is not None:
            ref.step()
        assert sim.error_flags() == 0
        for w in range(W):
            assert cl.worlds_equal(sim, plain, w), (s, w)
            if ref is not None:
                assert cl.worlds_equal(sim, ref, w), ("reference", s, w)


def test_walk_is_default_and_times_as_one_unit(monkeypatch):
    """The walk is on without the variable; timing the node that starts a
    walk run (mw_set_timed_node_index) times the whole run as one launch
    (walk + resume kernels bound to the event pair) and leaves the state
    bit-exact with the untimed per-node run."""
    import madrona_mi355x as mw
    monkeypatch.delenv("MADRONA_MW_WORLD_WALK", raising=False)
    W = 32
    inits = ol.gen_fvs_inits(W, 50, 200, seed=5)
    a = mw.FvsSim(W, inits)
    assert a.world_walk_runs() == 1
    end = a.walk_run_end(0)
    assert end == len(a.nodes())          # the whole tick is one run
    assert a.walk_run_end(end - 1) == end  # a node inside it starts none
    _walk(monkeypatch, False)
    b = mw.FvsSim(W, inits)
    assert b.world_walk_runs() == 0 and b.walk_run_end(0) == 1
    a.set_timed_node_index(0, every=3)
    a.step(30)
    b.step(30)
    ms, n = a.timed_node()
    assert n == 10 and ms > 0
    a.set_timed_node(None)
    a.step(20)
    b.step(20)
    for w in range(W):
        for arch in (0, 1):
            assert a.table(w, arch).tobytes() == b.table(w, arch).tobytes(), (w, arch)
