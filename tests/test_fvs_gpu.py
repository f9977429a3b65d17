"""GPU parity for fantasy_vs (BASELINE.json configs[4]): the HIP executor
(device ParallelForNodes + PerWorldNode with device-side makeEntityNow /
destroyEntityNow / clearArchetype) vs the oracle, bit-exact on every column
of the Dragon / Knight tables, including entity ids and generations after
destroys and ID reuse and the row order left by swap-removes."""
import numpy as np
import pytest

import oracle_lib as ol

pytestmark = pytest.mark.gpu


def _mw():
    import madrona_mi355x as mw
    return mw


def _compare(sim, orc, worlds, tag):
    for w in worlds:
        for arch in (0, 1):
            a, b = sim.table(w, arch), orc.table(w, arch)
            assert len(a) == len(b), f"{tag} world {w} arch {arch}: {len(a)} vs {len(b)} rows"
            assert a.tobytes() == b.tobytes(), f"{tag} world {w} arch {arch}: rows differ"


def test_fvs_bit_exact_through_deaths():
    mw = _mw()
    W = 6
    inits = ol.gen_fvs_inits(W, 50, 200, seed=0)
    sim = mw.FvsSim(W, inits)
    orc = ol.OracleFvs(inits)
    _compare(sim, orc, range(W), "init")
    for t in range(1, 17):
        sim.step(100)
        orc.step(100)
        assert sim.error_flags() == 0
        _compare(sim, orc, range(W), f"tick {100 * t}")
    assert sum(len(orc.table(w, 0)) for w in range(W)) < 50 * W   # dragons died


def test_fvs_every_tick_around_first_deaths():
    mw = _mw()
    W = 4
    inits = ol.gen_fvs_inits(W, 50, 200, seed=7)
    sim = mw.FvsSim(W, inits)
    orc = ol.OracleFvs(inits)
    sim.step(550)
    orc.step(550)
    for t in range(200):
        sim.step()
        orc.step()
        _compare(sim, orc, range(W), f"tick {551 + t}")


def test_fvs_golden_fixture_on_gpu():
    mw = _mw()
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "fvs_ref.npz"))
    inits = {k: g[f"base/init/{k}"] for k in
             ("dragon_pos", "dragon_mana", "knight_pos", "knight_arrows")}
    sim = mw.FvsSim(4, inits)
    done = 0
    for t in (250, 1000, 1500):
        sim.step(t - done)
        done = t
        for w in range(4):
            for arch in (0, 1):
                assert sim.table(w, arch).tobytes() == g[f"base/t{t}/w{w}/a{arch}"].tobytes()


def test_fvs_full_size_sampled_worlds():
    # BASELINE.json configs[4] size: 16384 worlds; the oracle replays a sample
    # of worlds with their global world indices.
    mw = _mw()
    W = 16384
    inits = mw.gen_fvs_inits(W, 50, 200, seed=0)
    sim = mw.FvsSim(W, inits)
    sample = [0, 1, 8191, W - 1]
    sub = {k: np.ascontiguousarray(v[sample]) for k, v in inits.items()}
    orcs = [ol.OracleFvs({k: v[i:i + 1] for k, v in sub.items()}, first_world_index=w)
            for i, w in enumerate(sample)]
    sim.step(1200)
    assert sim.error_flags() == 0
    for i, w in enumerate(sample):
        orcs[i].step(1200)
        for arch in (0, 1):
            assert sim.table(w, arch).tobytes() == orcs[i].table(0, arch).tobytes(), (w, arch)


@pytest.mark.parametrize("fuse", ["0", "1"])
def test_fvs_fused_and_per_archetype_launches_match_oracle(monkeypatch, fuse):
    # MADRONA_MW_FUSE_ARCHETYPES=1 (default): actionSelect / markDead run one
    # world-wave launch over dragons and knights (parallelForWorldMultiKernel);
    # 0: one launch per archetype.  Both bit-exact through the deaths.
    monkeypatch.setenv("MADRONA_MW_FUSE_ARCHETYPES", fuse)
    mw = _mw()
    W = 5
    inits = ol.gen_fvs_inits(W, 50, 200, seed=3)
    sim = mw.FvsSim(W, inits)
    orc = ol.OracleFvs(inits)
    for t in range(1, 9):
        sim.step(150)
        orc.step(150)
        assert sim.error_flags() == 0
        _compare(sim, orc, range(W), f"fuse={fuse} tick {150 * t}")
