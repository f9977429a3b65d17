"""CPU tests: pin the simple_taskgraph oracle (oracle/mw_oracle.cpp simple
mode: clamp node, Sphere + Agent body archetypes, no plane) against the
reference (examples/simple_taskgraph/simple.cpp:22-117 on the reference
physics, oracle/ref_harness.cpp).

The reference's face manifold reduction leaves one slot of an uninitialised
Manifold unwritten when every clipped point lies on one side of the p0-p1
line (src/physics/narrowphase.cpp:797-853) and then hands all four slots to
the solver: its result from that step on is undefined (stack contents).
The oracle counts those manifolds and defines the slot as zero; bit-exact
parity with the reference is asserted on every step before the first one,
and the divergence is asserted to start exactly there.
"""
import os

import numpy as np
import pytest

from oracle_lib import (OracleSimple, ReferenceSimple, default_phys_config,
                        gen_collisions_inits, ref_available)

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "simple_ref.npz")


def _eq(a, b):
    return all(a[f].tobytes() == b[f].tobytes() for f in a.dtype.names)


def test_simple_oracle_matches_reference_golden():
    g = np.load(GOLDEN, allow_pickle=False)
    cfg = default_phys_config(100, 4, max_contacts=1024)
    W = g["pos"].shape[0]
    orc = OracleSimple(cfg, g["pos"], g["rot"])
    done = 0
    for s in (1, 10, 50, 150):
        orc.step(s - done)
        done = s
        for w in range(W):
            key = f"s{s}/w{w}" if f"s{s}/w{w}" in g else f"orc_s{s}/w{w}"
            assert _eq(orc.bodies(w), g[key]), f"{key} differs"
    # every fixture world went through at least one undefined manifold by 150
    assert np.all(g["ub_first"] > 50) and np.all(g["ub_first"] <= 150)
    for w in range(W):
        assert orc.ub_manifolds(w) > 0


def test_simple_layout_ids_and_leaves():
    """Creation order objects -> agent -> test (simple.cpp:94-117): IDs and
    leaf IDs follow it; body (query) order is Sphere rows then Agent."""
    n = 7
    cfg = default_phys_config(n, 4, max_contacts=256)
    pos, rot = gen_collisions_inits(2, n, seed=1)
    b = OracleSimple(cfg, pos, rot).bodies(1)
    assert len(b) == n + 2
    # Sphere rows: n objects then the test object; Agent row last
    assert list(b["leafID"]) == list(range(n)) + [n + 1, n]
    assert b["pos"][n].tolist() == [-10.0, 0.0, 0.0]
    assert b["pos"][n + 1].tolist() == [0.0, 0.0, 0.0]
    assert list(np.argsort(b["id"])) == list(range(n)) + [n + 1, n]


@pytest.mark.skipif(not ref_available(), reason="reference build absent (GPU box)")
@pytest.mark.parametrize("nsub,seed", [(4, 9), (1, 0)])
def test_simple_oracle_matches_live_reference_until_undefined(nsub, seed):
    W, N, STEPS = 4, 100, 120
    cfg = default_phys_config(N, nsub, max_contacts=2048)
    pos, rot = gen_collisions_inits(W, N, seed=seed)
    orc = OracleSimple(cfg, pos, rot)
    ref = ReferenceSimple(cfg, pos, rot)
    ub_first = [0] * W
    diverged = [0] * W
    for s in range(1, STEPS + 1):
        orc.step()
        ref.step()
        for w in range(W):
            if not ub_first[w] and orc.ub_manifolds(w):
                ub_first[w] = s
            if not diverged[w] and not _eq(orc.bodies(w), ref.bodies(w)):
                diverged[w] = s
            if not ub_first[w]:
                assert not diverged[w], f"oracle != reference at step {s} world {w}"
    # any divergence starts at or after the first undefined manifold
    for w in range(W):
        assert diverged[w] == 0 or diverged[w] >= ub_first[w] > 0, (w, diverged[w], ub_first[w])
    assert any(ub_first), "no undefined manifold reached: case does not cover the UB path"
