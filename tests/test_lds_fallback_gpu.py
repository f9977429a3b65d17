"""GPU: kernels whose LDS image does not fit a workgroup run their
global-image variant and stay bit-exact; a launch shape that cannot run at all
is refused at mw_create with the kernel and the bytes named.

Background: a contact kernel built with 256-lane blocks
asked for more LDS than a workgroup holds, never ran, and the step still
returned success with error_flags() == 0 (0 vs 2 contacts at step 0).  Now
every launch is shape-checked on the host (csrc/runtime/hip_launch.hpp) and
every LDS-staging physics kernel has a global-image twin (physics.hip
upload()).  The reference handles hulls up to 512 faces on its stack
(src/physics/narrowphase.cpp:139-235) and any leaf count through its BVH walk
(include/madrona/physics.inl:61-100), so these shapes must work here too."""
import os

import numpy as np
import pytest

from oracle_lib import HullSet, OraclePhys, PhysConfig, gen_collisions_inits

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
DATA = os.path.join(os.path.dirname(HERE), "gpu-ecs-madrona_amd", "data")


def _eq(a, b):
    return all(a[f].tobytes() == b[f].tobytes() for f in a.dtype.names)


def _contacts_equal(a, b):
    n = int(a["numPoints"])
    return (a["ref"].tobytes() == b["ref"].tobytes() and a["alt"].tobytes() == b["alt"].tobytes()
            and n == int(b["numPoints"]) and a["normal"].tobytes() == b["normal"].tobytes()
            and a["points"][:n].tobytes() == b["points"][:n].tobytes()
            and a["lambdaN"][:n].tobytes() == b["lambdaN"][:n].tobytes())


def _pair(W, n, pos, rot, names=None, max_contacts=2048, max_candidates=4096):
    import madrona_mi355x as mw
    paths = [os.path.join(DATA, x + ".obj") for x in names] if names else None
    g = mw.default_collisions_config(n, 4, max_contacts, max_candidates, hull_paths=paths)
    o = PhysConfig(n, 4, g.delta_t, g.gravity_z, max_contacts, g.cube_inv_mass,
                   g.cube_inv_inertia, g.mu_s, g.mu_d)
    hs = HullSet.from_files(paths) if paths else None
    orc = OraclePhys(o, pos, rot, hs) if hs else OraclePhys(o, pos, rot)
    return mw.CollisionsSim(W, pos, rot, g), orc


def _lockstep(sim, orc, W, steps, contacts=True):
    for s in range(steps):
        sim.step()
        orc.step()
        assert sim.error_flags() == 0, f"step {s}: error flags {sim.error_flags():#x}"
        for w in range(W):
            ca, cb = sim.candidates(w), orc.candidates(w)
            assert ca.tobytes() == cb.tobytes(), f"step {s} world {w}: candidates differ"
            if contacts:
                ka, kb = sim.contacts(w), orc.contacts(w)
                assert len(ka) == len(kb), f"step {s} world {w}: {len(ka)} vs {len(kb)} contacts"
                for i in range(len(ka)):
                    assert _contacts_equal(ka[i], kb[i]), f"step {s} world {w}: contact {i} differs"
            assert _eq(sim.bodies(w), orc.bodies(w)), f"step {s} world {w}: bodies differ"


def test_disc64_hulls_take_global_clip_and_sat_images():
    """64-vertex caps: the contact kernel's clip buffers (2 x 128 points per
    lane, 458 KB per 128-lane block) and the SAT groups' hull staging exceed a
    workgroup; both run from global slabs, bit-exact every step -- the same
    failure class as the 256-lane contact build of r2 (gpurun_out/c256.log)."""
    W, n = 3, 32
    pos, rot = gen_collisions_inits(W, n, seed=3)
    sim, orc = _pair(W, n, pos, rot, names=("disc64", "cube"))
    v = sim.kernel_variants()
    assert v["contact"] and v["sat"], v
    assert not v["solver"] and not v["find_overlaps"], v
    _lockstep(sim, orc, W, 60)


def test_forced_global_images_bit_exact(monkeypatch):
    """Every LDS-staging kernel forced to its global variant
    (MADRONA_MW_FORCE_GLOBAL_IMAGES) on the benchmark's cube worlds and on a
    mixed hull set: the same bits as the oracle every step."""
    monkeypatch.setenv("MADRONA_MW_FORCE_GLOBAL_IMAGES", "1")
    W, n = 4, 128
    pos, rot = gen_collisions_inits(W, n, seed=0)
    sim, orc = _pair(W, n, pos, rot)
    v = sim.kernel_variants()
    assert all(v[k] for k in ("refit", "find_overlaps", "sat", "contact", "solver")), v
    _lockstep(sim, orc, W, 30)

    W, n = 3, 24
    pos, rot = gen_collisions_inits(W, n, seed=5)
    sim, orc = _pair(W, n, pos, rot, names=("cube", "wedge", "hex_prism", "disc16"))
    _lockstep(sim, orc, W, 40)


@pytest.mark.parametrize("tables", ["1", "0"])
def test_sat_edge_query_forms_bit_exact(monkeypatch, tables):
    """The SAT edge query's two forms (narrowphase.hip groupEdgeQueryTables:
    the Minkowski-test dot products tabulated per (edge, face), passes
    compacted per lane; groupEdgeQuery: the test per edge pair) on cube
    worlds and on a cube + wedge hull set: the same bits as the oracle every
    step (MADRONA_MW_SAT_TABLES=0 selects the per-pair form)."""
    monkeypatch.setenv("MADRONA_MW_SAT_TABLES", tables)
    W, n = 4, 128
    pos, rot = gen_collisions_inits(W, n, seed=11)
    sim, orc = _pair(W, n, pos, rot)
    v = sim.kernel_variants()
    assert v["sat_mink"] == (tables == "1") and v["sat_lds"], v
    _lockstep(sim, orc, W, 30)

    W, n = 3, 24
    pos, rot = gen_collisions_inits(W, n, seed=7)
    sim, orc = _pair(W, n, pos, rot, names=("cube", "wedge"))
    assert sim.kernel_variants()["sat_mink"] == (tables == "1")
    _lockstep(sim, orc, W, 40)


def _grid_world(W, n, spacing=3.0, z=0.95):
    side = int(np.ceil(np.sqrt(n)))
    pos = np.zeros((W, n, 3), np.float32)
    rot = np.zeros((W, n, 4), np.float32)
    rot[..., 0] = 1.0
    for w in range(W):
        i = np.arange(n)
        pos[w, :, 0] = (i % side) * spacing - side * spacing / 2 + 0.25 * w
        pos[w, :, 1] = (i // side) * spacing - side * spacing / 2
        pos[w, :, 2] = z + 0.01 * (i % 7)           # resting on the plane
    return pos, rot


def test_world_past_the_lds_images_bit_exact():
    """3200 cubes per world: more leaves than findOverlaps' LDS leaf image
    (~3000), more BVH nodes than refit's, more bodies than the solver's
    (~1100) and more contacts than its LDS records -- every broadphase and
    solver kernel runs its global variant; bodies, candidates and contacts
    are bit-exact against the oracle every step."""
    W, n = 2, 3200
    pos, rot = _grid_world(W, n)
    sim, orc = _pair(W, n, pos, rot, max_contacts=8192, max_candidates=8192)
    v = sim.kernel_variants()
    assert v["refit"] and v["find_overlaps"] and v["solver"], v
    _lockstep(sim, orc, W, 12)
    c, k = sim.counts()
    assert np.all(c >= n) and np.all(k >= n), (c, k)     # every cube on the plane


def test_commit_lds_overflow_refused_at_create():
    """The ordered commit's LDS (row indices + append keys + destroy keys)
    with 65536 deferred destroys per world exceeds a workgroup: mw_create
    fails and names the bytes, instead of a node whose structural ops are
    silently dropped."""
    import madrona_mi355x as mw
    import ecs_ops_lib as el
    with pytest.raises(mw.MadronaError, match="ordered commit needs .* B of LDS"):
        el.EcsOpsSim(2, max_deferred_destroys=65536)
    sim = el.EcsOpsSim(2, max_deferred_destroys=4096)       # fits: still works
    sim.step(2)
    assert sim.error_flags() == 0
