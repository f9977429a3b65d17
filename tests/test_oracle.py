"""CPU tests: pin the oracle (C++ restatement) against the reference.

* golden fixtures made by the reference itself (tests/golden/make_golden.py)
* the live reference build (oracle/_ref) when it is present in this container
"""
import os

import numpy as np
import pytest

from oracle_lib import (BODY_DTYPE, CONTACT_DTYPE, OraclePhys, PhysConfig,
                        ReferencePhys, default_phys_config,
                        gen_collisions_inits, ref_available)

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "collisions_ref.npz")


def _golden():
    return np.load(GOLDEN, allow_pickle=False)


def _cfg_from_golden(g):
    ci, cf = g["cfg"], g["cfg_f"]
    return PhysConfig(int(ci[0]), int(ci[1]), float(cf[0]), float(cf[1]), int(ci[2]),
                      float(cf[2]), float(cf[3]), float(cf[4]), float(cf[5]))


def contacts_equal(a, b):
    """Bit-exact equality on the meaningful part of two contact records."""
    n = int(a["numPoints"])
    return (a["ref"].tobytes() == b["ref"].tobytes()
            and a["alt"].tobytes() == b["alt"].tobytes()
            and n == int(b["numPoints"])
            and a["normal"].tobytes() == b["normal"].tobytes()
            and a["points"][:n].tobytes() == b["points"][:n].tobytes()
            and a["lambdaN"][:n].tobytes() == b["lambdaN"][:n].tobytes())


def test_init_generator_matches_golden_inputs():
    g = _golden()
    pos, rot = gen_collisions_inits(g["init_pos"].shape[0], 128, seed=0)
    assert pos.tobytes() == g["init_pos"].tobytes()
    assert rot.tobytes() == g["init_rot"].tobytes()


def test_oracle_bit_exact_vs_golden_bodies_and_contacts():
    g = _golden()
    cfg = _cfg_from_golden(g)
    W = g["init_pos"].shape[0]
    orc = OraclePhys(cfg, g["init_pos"], g["init_rot"])
    step = 0
    for target in g["snap_steps"]:
        orc.step(int(target) - step)
        step = int(target)
        want = g[f"bodies_{step}"].view(BODY_DTYPE).reshape(W, -1)
        for w in range(W):
            got = orc.bodies(w)
            assert got.tobytes() == want[w].tobytes(), f"bodies differ at step {step} world {w}"
        if step == 1:
            for w in range(W):
                _, aabbs, parents, sorted_l = orc.bvh(w)
                assert aabbs.tobytes() == g[f"bvh_leaf_aabbs_{w}"].tobytes()
                assert parents.tobytes() == g[f"bvh_leaf_parents_{w}"].tobytes()
                assert sorted_l.tobytes() == g[f"bvh_sorted_{w}"].tobytes()
        key = f"contacts_{step}_0"
        if key in g:
            for w in range(W):
                want_c = g[f"contacts_{step}_{w}"].view(CONTACT_DTYPE).reshape(-1)
                got_c = orc.contacts(w)
                # the last substep's manifolds, as many as the reference
                # counted (numContacts after that narrowphase node)
                assert len(got_c) == int(g[f"contact_count_{step}_{w}"]) == len(want_c), (step, w)
                for i in range(len(got_c)):
                    assert contacts_equal(got_c[i], want_c[i]), (step, w, i)


WINDOW = os.path.join(os.path.dirname(__file__), "golden", "collisions_window_ref.npz")


def _contact_prefix_equal(got, raw_ref):
    """Ours holds exactly the last substep's manifolds; the reference's array
    holds them as a prefix (an earlier substep may have written more)."""
    assert len(got) <= len(raw_ref), (len(got), len(raw_ref))
    for i in range(len(got)):
        if not contacts_equal(got[i], raw_ref[i]):
            return i
    return None


@pytest.mark.skipif(not ref_available(), reason="reference build absent (GPU box)")
def test_oracle_bit_exact_vs_live_reference():
    # Every step through the end of bench.py's default window (131-330):
    # bodies, the step's candidate pairs (harness candidate log), the last
    # substep's contacts and the BVH.  Each world is compared up to its first
    # manifold with an undefined reference value; the oracle
    # counts them, and collisions worlds of this seed have none.
    cfg = default_phys_config(num_cubes=128, max_contacts=2048)
    pos, rot = gen_collisions_inits(2, 128, seed=7)
    orc = OraclePhys(cfg, pos, rot)
    ref = ReferencePhys(cfg, pos, rot, log_candidates=True)
    for step in range(330):
        orc.step()
        ref.step()
        for w in range(2):
            assert orc.ub_manifolds(w) == 0, (step, w)
            assert orc.bodies(w).tobytes() == ref.bodies(w).tobytes(), (step, w)
            assert orc.candidates(w).tobytes() == ref.candidates(w).tobytes(), (step, w)
            raw = ref.contacts_raw(w)
            raw = raw[raw["ref"][:, 0] != 0xFFFFFFFF]
            got = orc.contacts(w)
            # the reference's own count of the last substep's manifolds
            assert len(got) == ref.last_contact_count(w), (step, w, len(got))
            assert _contact_prefix_equal(got, raw) is None, (step, w)
            if step % 10 == 0:
                n_o, a_o, p_o, s_o = orc.bvh(w)
                n_r, a_r, p_r, s_r = ref.bvh(w)
                assert n_o.tobytes() == n_r[:len(n_o)].tobytes()
                assert a_o.tobytes() == a_r.tobytes()


def test_oracle_bit_exact_vs_reference_window_golden():
    # BASELINE configs[2]'s own worlds (0, 1, 4095, 8191 of 8192, seed 0) at
    # steps 130 / 145 / 330, the bench's timed windows, against fixtures the
    # reference wrote (tests/golden/make_golden.py make_window).
    g = np.load(WINDOW, allow_pickle=False)
    worlds = [int(w) for w in g["worlds"]]
    pos, rot = gen_collisions_inits(int(g["num_worlds"]), 128, seed=0)
    assert pos[worlds].tobytes() == g["init_pos"].tobytes()
    assert rot[worlds].tobytes() == g["init_rot"].tobytes()
    ci = g["cfg"]
    cfg = default_phys_config(num_cubes=int(ci[0]), num_substeps=int(ci[1]),
                              max_contacts=int(ci[2]))
    orc = OraclePhys(cfg, g["init_pos"], g["init_rot"])
    done = 0
    for step in g["snap_steps"]:
        step = int(step)
        orc.step(step - done, 4)
        done = step
        for i in range(len(worlds)):
            # no undefined-manifold value in these worlds through step 330
            assert orc.ub_manifolds(i) == 0, (step, worlds[i])
            want = g[f"bodies_{step}_{i}"].view(BODY_DTYPE)
            assert orc.bodies(i).tobytes() == want.tobytes(), (step, worlds[i])
            assert orc.candidates(i).tobytes() == g[f"candidates_{step}_{i}"].tobytes()
            want_c = g[f"contacts_{step}_{i}"].view(CONTACT_DTYPE).reshape(-1)
            got = orc.contacts(i)
            assert len(got) == int(g[f"contact_count_{step}_{i}"]) == len(want_c) > 0
            assert _contact_prefix_equal(got, want_c) is None, (step, worlds[i])


def test_oracle_small_world_counts_and_threads_agree():
    """Ragged case: few bodies, 1 substep; the threaded driver must equal the
    serial one (worlds are independent)."""
    cfg = default_phys_config(num_cubes=5, num_substeps=1, max_contacts=256)
    pos, rot = gen_collisions_inits(6, 5, seed=3)
    a = OraclePhys(cfg, pos, rot)
    b = OraclePhys(cfg, pos, rot)
    a.step(20, threads=1)
    b.step(20, threads=3)
    for w in range(6):
        assert a.bodies(w).tobytes() == b.bodies(w).tobytes()
