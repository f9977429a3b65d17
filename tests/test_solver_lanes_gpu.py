"""The solver's lane variant chosen per executor (VERDICT r5
#1): lanes64 (one world per wave) or lanes32 (two worlds per wave, the level
passes over both worlds' merged schedule).  By default the executor measures
the worlds' dependency-level widths (PhysArgs::solverLevelStats) at the
synchronisations from 24 steps in (at most every 64 steps) and takes 32
lanes when levels average at most 12 items, 64 from 20; MADRONA_MW_SOLVER_LANES
fixes either.  Both variants are the
same operations in the same per-world order, so switching mid-run changes
no bit: checked here against the fixed-64 executor and the oracle."""
import pytest

import oracle_lib as ol
from test_collisions_gpu import _cfg_pair, _contacts_equal, _diff

pytestmark = pytest.mark.gpu


def _mw():
    import madrona_mi355x as mw
    return mw


@pytest.mark.parametrize("workload,expect", [("simple", 32), ("collisions", 64)])
def test_auto_lanes_switch_is_bit_exact(monkeypatch, workload, expect):
    mw = _mw()
    n = 100 if workload == "simple" else 128
    gcfg, ocfg = _cfg_pair(num_cubes=n)
    W, STEPS = 16, 200
    pos, rot = ol.gen_collisions_inits(W, n, seed=3)
    Sim = mw.SimpleSim if workload == "simple" else mw.CollisionsSim
    monkeypatch.setenv("MADRONA_MW_SOLVER_LANES", "64")
    fixed = Sim(W, pos, rot, gcfg)
    monkeypatch.setenv("MADRONA_MW_SOLVER_LANES", "auto")
    auto = Sim(W, pos, rot, gcfg)
    assert auto.kernel_variants()["solver_lanes"] == 64       # measured first
    orc = (ol.OracleSimple if workload == "simple" else ol.OraclePhys)(ocfg, pos, rot)
    lanes = set()
    for s in range(1, STEPS + 1):
        fixed.step(1)
        auto.step(1)                                           # every step syncs: polls from step 24
        orc.step(1)
        if s % 4 and s != STEPS:
            continue
        for w in range(W):
            a = auto.bodies(w)
            assert a.tobytes() == fixed.bodies(w).tobytes(), (s, w)
            d = _diff(a, orc.bodies(w))
            assert d is None, (s, w, d)
        assert auto.error_flags() == 0
        lanes.add(auto.kernel_variants()["solver_lanes"])
    # settled: simple_taskgraph's chains are narrow, collisions' levels wide
    assert auto.kernel_variants()["solver_lanes"] == expect, lanes


def test_forced_32_lanes_collisions_bit_exact(monkeypatch):
    mw = _mw()
    monkeypatch.setenv("MADRONA_MW_SOLVER_LANES", "32")
    gcfg, ocfg = _cfg_pair()
    W = 9                                   # odd: a block's second world is absent
    pos, rot = ol.gen_collisions_inits(W, 128, seed=4)
    sim = mw.CollisionsSim(W, pos, rot, gcfg)
    assert sim.kernel_variants()["solver_lanes"] == 32
    orc = ol.OraclePhys(ocfg, pos, rot)
    for s in range(1, 31):
        sim.step(1)
        orc.step(1)
        for w in range(W):
            d = _diff(sim.bodies(w), orc.bodies(w))
            assert d is None, (s, w, d)
            ka, kb = sim.contacts(w), orc.contacts(w)
            assert len(ka) == len(kb), (s, w)
            assert all(_contacts_equal(ka[i], kb[i]) for i in range(len(ka))), (s, w)
