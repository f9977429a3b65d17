"""GPU parity for joint constraints (ConstraintData rows solved after the
contacts of every substep, reference src/physics/physics.cpp:478-671): the
HIP solver (joints join the per-world level schedule as extra items) vs the
oracle and vs the reference's golden fixtures, through the C ABI."""
import os

import numpy as np
import pytest

from oracle_lib import OraclePhys, PhysConfig, gen_collisions_inits, joint_inits

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "joints_ref.npz")


def _mw():
    import madrona_mi355x as mw
    return mw


def _cfgs(n, j, h=0, max_contacts=1024, max_candidates=4096):
    mw = _mw()
    g = mw.default_collisions_config(n, 4, max_contacts, max_candidates, num_joints=j,
                                     num_hinge_joints=h)
    o = PhysConfig(n, 4, g.delta_t, g.gravity_z, max_contacts, g.cube_inv_mass,
                   g.cube_inv_inertia, g.mu_s, g.mu_d, j, h)
    return g, o


def _same(a, b):
    return all(a[f].tobytes() == b[f].tobytes() for f in a.dtype.names)


def _first_diff(a, b):
    for f in a.dtype.names:
        if a[f].tobytes() != b[f].tobytes():
            rows = np.nonzero((a[f] != b[f]).reshape(len(a), -1).any(1))[0]
            return f"{f}: rows {rows[:8]}"
    return None


def _parity(W, n, j, h, seed, steps, every=1, max_contacts=1024):
    mw = _mw()
    g, o = _cfgs(n, j, h, max_contacts)
    pos, rot = joint_inits(*gen_collisions_inits(W, n, seed=seed), j, h)
    sim = mw.CollisionsSim(W, pos, rot, g)
    orc = OraclePhys(o, pos, rot)
    for s in range(1, steps + 1):
        sim.step()
        orc.step(1, 4)
        if s % every and s != steps:
            continue
        assert sim.error_flags() == 0, mw.ERR_BITS
        for w in range(W):
            d = _first_diff(sim.bodies(w), orc.bodies(w))
            assert d is None, f"step {s} world {w}: {d}"
    return sim


def test_fixed_joints_bit_exact_vs_oracle_every_step():
    _parity(W=4, n=32, j=8, h=0, seed=13, steps=300)


def test_joints_match_reference_golden():
    mw = _mw()
    gld = np.load(GOLDEN, allow_pickle=False)
    g, _ = _cfgs(32, 8)
    sim = mw.CollisionsSim(4, gld["fixed/pos"], gld["fixed/rot"], g)
    done = 0
    for s in (1, 20, 50, 100, 150, 300):
        sim.step(s - done)
        done = s
        for w in range(4):
            key = f"fixed/s{s}/w{w}" if f"fixed/s{s}/w{w}" in gld else f"fixed/orc_s{s}/w{w}"
            assert _same(sim.bodies(w), gld[key]), f"{key}: {_first_diff(sim.bodies(w), gld[key])}"
    g, _ = _cfgs(8, 4, 2)
    sim = mw.CollisionsSim(2, gld["hinge/pos"], gld["hinge/rot"], g)
    for s in range(1, 13):
        sim.step()
        for w in range(2):
            assert _same(sim.bodies(w), gld[f"hinge/s{s}/w{w}"]), f"hinge step {s} world {w}"


def test_hinge_joints_bit_exact_while_finite():
    _parity(W=3, n=8, j=4, h=2, seed=4, steps=12)


def test_many_joints_take_the_global_record_path():
    # 64 fixed joints + contacts exceed the solver's 128 LDS-resident items
    # per world, so these worlds solve with global records
    _parity(W=4, n=128, j=64, h=0, seed=2, steps=40, every=5, max_contacts=2048)


def test_joints_full_size_sampled_worlds():
    mw = _mw()
    W, n, j, steps = 8192, 128, 16, 30
    g, o = _cfgs(n, j, max_contacts=4096)
    pos, rot = joint_inits(*mw.gen_collisions_inits(W, n, seed=0), j)
    sim = mw.CollisionsSim(W, pos, rot, g)
    sample = [0, 1, W // 2, W - 1]
    orc = OraclePhys(o, np.ascontiguousarray(pos[sample]), np.ascontiguousarray(rot[sample]))
    sim.step(steps)
    orc.step(steps, 4)
    assert sim.error_flags() == 0, mw.ERR_BITS
    for i, w in enumerate(sample):
        d = _first_diff(sim.bodies(w), orc.bodies(i))
        assert d is None, f"world {w}: {d}"
