"""CPU tests: pin the oracle's joint constraints (oracle/mw_oracle.cpp
handleJoint, restating src/physics/physics.cpp:247-279, 478-671) against the
reference -- its golden fixtures (tests/golden/make_golden_joints.py) and,
where present, the live reference build (oracle/_ref).

Workload: collisions worlds plus ConstraintData rows; joint j ties cube 2j to
2j+1 (fixed, or hinge for the last num_hinge_joints), starting satisfied
(oracle_lib.joint_inits).  The reference's hinge diverges (its positional
correction has the sign opposite to the fixed joint's), so hinge cases run
only the steps it stays finite.
"""
import os

import numpy as np
import pytest

from oracle_lib import (OraclePhys, ReferencePhys, default_phys_config,
                        gen_collisions_inits, joint_inits, ref_available)

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "joints_ref.npz")


def _eq(a, b):
    return all(a[f].tobytes() == b[f].tobytes() for f in a.dtype.names)


def joint_config(n, j, h=0):
    cfg = default_phys_config(n, 4, max_contacts=1024)
    cfg.numJoints = j
    cfg.numHingeJoints = h
    return cfg


def test_fixed_joints_oracle_matches_reference_golden():
    g = np.load(GOLDEN, allow_pickle=False)
    cfg = joint_config(32, 8)
    pos, rot = g["fixed/pos"], g["fixed/rot"]
    ip, ir = joint_inits(*gen_collisions_inits(4, 32, seed=13), 8)
    assert ip.tobytes() == pos.tobytes() and ir.tobytes() == rot.tobytes()
    orc = OraclePhys(cfg, pos, rot)
    done = 0
    for s in (1, 20, 50, 100, 150, 300):
        orc.step(s - done)
        done = s
        for w in range(4):
            key = f"fixed/s{s}/w{w}" if f"fixed/s{s}/w{w}" in g else f"fixed/orc_s{s}/w{w}"
            assert _eq(orc.bodies(w), g[key]), f"{key} differs"


def test_hinge_joints_oracle_matches_reference_golden():
    g = np.load(GOLDEN, allow_pickle=False)
    cfg = joint_config(8, 4, 2)
    orc = OraclePhys(cfg, g["hinge/pos"], g["hinge/rot"])
    for s in range(1, 13):
        orc.step(1)
        for w in range(2):
            assert _eq(orc.bodies(w), g[f"hinge/s{s}/w{w}"]), f"hinge step {s} world {w}"


def test_joints_change_the_simulation():
    """The ConstraintData rows are solved: without them the same inputs end
    elsewhere, and fixed pairs stay at their rest distance."""
    g = np.load(GOLDEN, allow_pickle=False)
    pos, rot = g["fixed/pos"], g["fixed/rot"]
    a = OraclePhys(joint_config(32, 8), pos, rot)
    b = OraclePhys(joint_config(32, 0), pos, rot)
    a.step(60)
    b.step(60)
    assert not _eq(a.bodies(0), b.bodies(0))
    p = a.bodies(0)["pos"]
    # fixed joint at rest, in cube 2j's frame: x2 - x1 = r1 + 0.5 fwd - R(-90 z) r2
    # = (0, 2, 0) - (-1.5, 0, 0), so |x2 - x1| = 2.5
    d = np.linalg.norm(p[1:16:2] - p[0:16:2], axis=1)
    assert np.all(np.abs(d - 2.5) < 0.05), d


def test_joint_entities_take_ids_after_the_plane():
    cfg = joint_config(8, 3)
    pos, rot = joint_inits(*gen_collisions_inits(1, 8, seed=2), 3)
    b = OraclePhys(cfg, pos, rot).bodies(0)
    plain = OraclePhys(joint_config(8, 0), pos, rot).bodies(0)
    assert b["id"].tobytes() == plain["id"].tobytes()


@pytest.mark.skipif(not ref_available(), reason="reference build absent (GPU box)")
@pytest.mark.parametrize("n,j,h,seed,steps", [(32, 8, 0, 13, 200), (128, 16, 0, 3, 60),
                                              (8, 4, 2, 4, 12)])
def test_joints_oracle_matches_live_reference_until_undefined(n, j, h, seed, steps):
    W = 3
    cfg = joint_config(n, j, h)
    pos, rot = joint_inits(*gen_collisions_inits(W, n, seed=seed), j, h)
    orc, ref = OraclePhys(cfg, pos, rot), ReferencePhys(cfg, pos, rot)
    ub_first = [0] * W
    checked = 0
    for s in range(1, steps + 1):
        orc.step()
        ref.step()
        for w in range(W):
            if not ub_first[w] and orc.ub_manifolds(w):
                ub_first[w] = s
            if not ub_first[w]:
                assert np.isfinite(ref.bodies(w)["pos"]).all()
                assert _eq(orc.bodies(w), ref.bodies(w)), f"oracle != reference at step {s} world {w}"
                checked += 1
    assert checked >= W * min(steps, 20)
