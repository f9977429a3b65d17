"""GPU parity: the HIP physics path vs the oracle (C++ restatement pinned to
the reference) and vs the reference's own golden fixtures.

Bar (BASELINE.json north_star): integer ECS state (entity ids, generations,
Locs, candidate pairs, contact Locs / counts) bit-exact; float state within
1e-5 -- we additionally check bit-exactness, which the MI355X kernels reach
because they keep the reference's operation order.
"""
import numpy as np
import pytest

from oracle_lib import OraclePhys, PhysConfig, gen_collisions_inits

pytestmark = pytest.mark.gpu

FLOAT_FIELDS = ("pos", "rot", "vel", "prevPos", "prevRot", "presolvePos", "presolveRot",
                "presolveVel")
INT_FIELDS = ("gen", "id", "leafID", "objID", "responseType")


def _mw():
    import madrona_mi355x as mw
    return mw


def _cfg_pair(num_cubes=128, num_substeps=4, max_contacts=2048, max_candidates=4096):
    mw = _mw()
    g = mw.default_collisions_config(num_cubes, num_substeps, max_contacts, max_candidates)
    o = PhysConfig(num_cubes, num_substeps, g.delta_t, g.gravity_z, max_contacts,
                   g.cube_inv_mass, g.cube_inv_inertia, g.mu_s, g.mu_d)
    return g, o


def _diff(a, b):
    """Describe the first field mismatch between two body record arrays."""
    for f in INT_FIELDS + FLOAT_FIELDS:
        x, y = a[f], b[f]
        if x.tobytes() != y.tobytes():
            rows = np.nonzero((x != y).reshape(len(x), -1).any(1))[0]
            err = np.max(np.abs(x.astype(np.float64) - y.astype(np.float64)))
            return f"{f}: rows {rows[:8]} max|d|={err:.3e}"
    return None


def _contacts_equal(a, b):
    n = int(a["numPoints"])
    return (a["ref"].tobytes() == b["ref"].tobytes() and a["alt"].tobytes() == b["alt"].tobytes()
            and n == int(b["numPoints"]) and a["normal"].tobytes() == b["normal"].tobytes()
            and a["points"][:n].tobytes() == b["points"][:n].tobytes()
            and a["lambdaN"][:n].tobytes() == b["lambdaN"][:n].tobytes())


def _run_parity(W, steps, num_cubes=128, num_substeps=4, seed=0, check_every=1):
    mw = _mw()
    gcfg, ocfg = _cfg_pair(num_cubes, num_substeps)
    pos, rot = gen_collisions_inits(W, num_cubes, seed=seed)
    sim = mw.CollisionsSim(W, pos, rot, gcfg)
    orc = OraclePhys(ocfg, pos, rot)
    for w in range(W):
        assert _diff(sim.bodies(w), orc.bodies(w)) is None, "init state differs"
    max_err = 0.0
    for s in range(steps):
        sim.step()
        orc.step()
        if (s + 1) % check_every and s != steps - 1:
            continue
        assert sim.error_flags() == 0, mw.ERR_BITS
        for w in range(W):
            ca, cb = sim.candidates(w), orc.candidates(w)
            assert ca.tobytes() == cb.tobytes(), f"step {s} world {w}: candidates differ ({len(ca)} vs {len(cb)})"
            ka, kb = sim.contacts(w), orc.contacts(w)
            assert len(ka) == len(kb), f"step {s} world {w}: {len(ka)} vs {len(kb)} contacts"
            for i in range(len(ka)):
                assert _contacts_equal(ka[i], kb[i]), f"step {s} world {w}: contact {i} differs"
            ga, gb = sim.bodies(w), orc.bodies(w)
            for f in FLOAT_FIELDS:
                max_err = max(max_err, float(np.max(np.abs(ga[f].astype(np.float64) - gb[f]))))
            d = _diff(ga, gb)
            assert d is None, f"step {s} world {w}: {d}"
    return max_err


def test_collisions_bit_exact_vs_oracle_small():
    err = _run_parity(W=4, steps=30)
    assert err == 0.0


def test_collisions_bit_exact_ragged_worlds_one_substep():
    # few bodies, 1 substep: exercises empty / tiny candidate lists
    _run_parity(W=3, steps=20, num_cubes=5, num_substeps=1, seed=11)


def test_collisions_bvh_matches_oracle_after_first_step():
    mw = _mw()
    gcfg, ocfg = _cfg_pair()
    pos, rot = gen_collisions_inits(2, 128, seed=5)
    sim = mw.CollisionsSim(2, pos, rot, gcfg)
    orc = OraclePhys(ocfg, pos, rot)
    for _ in range(3):
        sim.step()
        orc.step()
        for w in range(2):
            na, aa = sim.bvh(w)
            nb, ab, _, _ = orc.bvh(w)
            assert len(na) == len(nb)
            assert na.tobytes() == nb.tobytes()
            assert aa.tobytes() == ab.tobytes()


def test_collisions_bit_exact_long_horizon_contacts():
    # 300 steps: every cube lands (z <= 10 falls for ~85 steps), stacks and
    # settles, so cube-cube face / edge manifolds and cube-plane contacts
    # dominate the tail of the run.
    mw = _mw()
    gcfg, ocfg = _cfg_pair()
    W, steps = 8, 300
    pos, rot = gen_collisions_inits(W, 128, seed=3)
    sim = mw.CollisionsSim(W, pos, rot, gcfg)
    orc = OraclePhys(ocfg, pos, rot)
    seen_contacts = 0
    for s in range(steps):
        sim.step()
        orc.step(1, 8)
        _, contacts = sim.counts()
        seen_contacts += int(contacts.sum())
        if (s + 1) % 25:
            continue
        assert sim.error_flags() == 0, mw.ERR_BITS
        for w in range(W):
            d = _diff(sim.bodies(w), orc.bodies(w))
            assert d is None, f"step {s} world {w}: {d}"
            ka, kb = sim.contacts(w), orc.contacts(w)
            assert len(ka) == len(kb)
            for i in range(len(ka)):
                assert _contacts_equal(ka[i], kb[i]), f"step {s} world {w}: contact {i} differs"
    assert seen_contacts > W * steps * 10, seen_contacts


def test_collisions_full_size_sampled_worlds():
    # BASELINE.json configs[2] size (8192 worlds) through bench.py's whole
    # window (settle 120 + warmup 10 + 200 timed steps): the oracle replays a
    # sample of worlds (first, middle, last) from the same per-world seeds;
    # bodies, candidate pairs and contacts are compared at the start and the
    # end of the timed window.
    mw = _mw()
    gcfg, ocfg = _cfg_pair(max_contacts=4096)
    W = 8192
    pos, rot = mw.gen_collisions_inits(W, 128, seed=0)
    sim = mw.CollisionsSim(W, pos, rot, gcfg)
    sample = [0, 1, W // 2, W - 1]
    orc = OraclePhys(ocfg, np.ascontiguousarray(pos[sample]), np.ascontiguousarray(rot[sample]))
    done = 0
    for checkpoint in (130, 330):
        sim.step(checkpoint - done)
        orc.step(checkpoint - done, 4)
        done = checkpoint
        assert sim.error_flags() == 0, mw.ERR_BITS
        cands, contacts = sim.counts()
        assert cands.mean() > 100 and contacts.mean() > 10, (cands.mean(), contacts.mean())
        for i, w in enumerate(sample):
            d = _diff(sim.bodies(w), orc.bodies(i))
            assert d is None, f"step {checkpoint} world {w}: {d}"
            assert sim.candidates(w).tobytes() == orc.candidates(i).tobytes(), (checkpoint, w)
            ka, kb = sim.contacts(w), orc.contacts(i)
            assert len(ka) == len(kb), (checkpoint, w)
            for k in range(len(ka)):
                assert _contacts_equal(ka[k], kb[k]), f"step {checkpoint} world {w}: contact {k}"


def test_collisions_full_size_vs_reference_window():
    # BASELINE configs[2] at full size (8192 worlds) against the fixtures
    # the reference itself wrote for worlds 0, 1, 4095 and 8191 at steps
    # 130, 145 (the driver's timed steps 126-145) and 330 (the end of
    # bench.py's default window): bodies, candidate pairs and the last
    # substep's contacts, bit for bit (tests/golden/make_golden.py
    # make_window).
    import os
    from oracle_lib import BODY_DTYPE, CONTACT_DTYPE
    mw = _mw()
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "collisions_window_ref.npz"),
                allow_pickle=False)
    worlds = [int(w) for w in g["worlds"]]
    W = int(g["num_worlds"])
    gcfg, _ = _cfg_pair(max_contacts=int(g["cfg"][2]))
    pos, rot = mw.gen_collisions_inits(W, 128, seed=0)
    assert pos[worlds].tobytes() == g["init_pos"].tobytes()
    sim = mw.CollisionsSim(W, pos, rot, gcfg)
    done = 0
    for step in (int(x) for x in g["snap_steps"]):
        sim.step(step - done)
        done = step
        assert sim.error_flags() == 0, mw.ERR_BITS
        for i, w in enumerate(worlds):
            want = g[f"bodies_{step}_{i}"].view(BODY_DTYPE)
            d = _diff(sim.bodies(w), want)
            assert d is None, f"step {step} world {w}: {d}"
            assert sim.candidates(w).tobytes() == g[f"candidates_{step}_{i}"].tobytes(), (step, w)
            # exactly the reference's last-substep manifolds: its own count
            # (SolverData::numContacts after that narrowphase node) is pinned
            want_c = g[f"contacts_{step}_{i}"].view(CONTACT_DTYPE).reshape(-1)
            got = sim.contacts(w)
            assert len(got) == int(g[f"contact_count_{step}_{i}"]) == len(want_c), (step, w, len(got))
            for k in range(len(got)):
                assert _contacts_equal(got[k], want_c[k]), f"step {step} world {w}: contact {k}"


def test_side_stream_plane_branch_is_bit_identical(monkeypatch):
    # MADRONA_MW_SIDE_STREAM=1 runs the hull-plane kernel on a second stream
    # beside SAT + contact clipping (a parallel branch of the step graph);
    # every body and contact stays bit-identical to the single-stream step.
    mw = _mw()
    gcfg, _ = _cfg_pair()
    pos, rot = gen_collisions_inits(16, 128, seed=6)
    b = mw.CollisionsSim(16, pos, rot, gcfg)
    monkeypatch.setenv("MADRONA_MW_SIDE_STREAM", "1")
    a = mw.CollisionsSim(16, pos, rot, gcfg)
    a.step(40)
    b.step(40)
    assert a.error_flags() == 0
    for w in range(16):
        assert a.bodies(w).tobytes() == b.bodies(w).tobytes()
        assert a.contacts(w).tobytes() == b.contacts(w).tobytes()


def test_live_node_timing_does_not_perturb_state():
    # set_timed_node splits the step graph at the named node kind and times
    # its launches with HIP events; state must stay bit-identical to an
    # untimed run.
    mw = _mw()
    gcfg, _ = _cfg_pair()
    pos, rot = gen_collisions_inits(16, 128, seed=2)
    a = mw.CollisionsSim(16, pos, rot, gcfg)
    b = mw.CollisionsSim(16, pos, rot, gcfg)
    a.set_timed_node("NarrowphaseNode")
    for _ in range(10):
        a.step()           # synchronous steps: each one's launches are counted
    b.step(10)
    ms, n = a.timed_node()
    assert n == 10 * gcfg.num_substeps and ms > 0
    for w in range(16):
        assert a.bodies(w).tobytes() == b.bodies(w).tobytes()
    a.set_timed_node(None)
    a.step(1)
    assert a.timed_node() == (0.0, 0)


def test_sampled_node_timing_counts_and_does_not_perturb_state():
    # set_timed_node(every=3): only the first of every 3 steps is split and
    # timed, the rest replay the unsplit graph (bench.py's --timed-every).
    mw = _mw()
    gcfg, _ = _cfg_pair()
    pos, rot = gen_collisions_inits(16, 128, seed=3)
    a = mw.CollisionsSim(16, pos, rot, gcfg)
    b = mw.CollisionsSim(16, pos, rot, gcfg)
    a.set_timed_node("SolverNode", every=3)
    a.step(10)             # steps 0, 3, 6, 9 are timed
    b.step(10)
    ms, n = a.timed_node()
    assert n == 4 * gcfg.num_substeps and ms > 0
    for w in range(16):
        assert a.bodies(w).tobytes() == b.bodies(w).tobytes()
        assert a.contacts(w).tobytes() == b.contacts(w).tobytes()


def test_node_index_timing_times_one_node():
    # set_timed_node_index: only the one node (the first of the four
    # SolverNodes) is split and timed; its event pair is bound to the
    # node's kernels, so the per-launch time stays within the step's.
    mw = _mw()
    gcfg, _ = _cfg_pair()
    pos, rot = gen_collisions_inits(16, 128, seed=5)
    a = mw.CollisionsSim(16, pos, rot, gcfg)
    b = mw.CollisionsSim(16, pos, rot, gcfg)
    kinds = a.nodes()
    first = kinds.index("SolverNode")
    assert kinds.count("SolverNode") == gcfg.num_substeps
    a.set_timed_node_index(first)
    a.step(6)
    b.step(6)
    ms, n = a.timed_node()
    assert n == 6 and ms > 0
    for w in range(16):
        assert a.bodies(w).tobytes() == b.bodies(w).tobytes()
    with pytest.raises(RuntimeError, match="past the graph"):
        a.set_timed_node_index(len(kinds))


def test_episode_return_export_matches_oracle():
    # CustomParallelForNode (one wave per world) over the EpisodeReturn
    # singleton + the packed export buffer (getExported slot 2, a singleton:
    # flat copy, fixed offsets).
    mw = _mw()
    gcfg, ocfg = _cfg_pair()
    W, steps = 5, 12
    pos, rot = gen_collisions_inits(W, 128, seed=4)
    sim = mw.CollisionsSim(W, pos, rot, gcfg)
    orc = OraclePhys(ocfg, pos, rot)
    ret = np.zeros(W, np.float32)
    for _ in range(steps):
        sim.step()
        orc.step()
        for w in range(W):
            b = orc.bodies(w)
            z = b["pos"][b["responseType"] == 0][:, 2].astype(np.float32)
            ret[w] = np.float32(ret[w] + np.cumsum(z, dtype=np.float32)[-1] / np.float32(len(z)))
    got = sim.exported_array(2, np.float32)
    assert got.shape == (W,)
    assert got.tobytes() == ret.tobytes()


def test_export_copy_is_ordered_after_async_steps():
    # mw_copy_exported / mw_get_exported(&rows) read the packed rows and
    # their total on the executor stream: right after step_async they see
    # that step's export, with no host sync by the caller.
    mw = _mw()
    gcfg, _ = _cfg_pair()
    pos, rot = gen_collisions_inits(64, 128, seed=6)
    a = mw.CollisionsSim(64, pos, rot, gcfg)
    b = mw.CollisionsSim(64, pos, rot, gcfg)
    for _ in range(3):
        a.step_async(1)
        got = a.exported_array(2, np.float32)
        b.step(1)
        assert got.shape == (64,)
        assert got.tobytes() == b.exported_array(2, np.float32).tobytes()
    dst = np.full(64 * 2, -7.0, np.float32)
    a.step_async(1)
    n = a.copy_exported(2, dst.ctypes.data, dst.nbytes)
    b.step(1)
    assert n == 64 * 4
    assert dst[:64].tobytes() == b.exported_array(2, np.float32).tobytes()
