"""GPU parity for collisions worlds over OBJ hulls (the physics asset path,
SURVEY.md §8f-3): the product loads the .obj files itself (importer +
PhysicsLoader, mw_collisions_config.hull_paths) and steps them through the
HIP kernels; the oracle gets the same meshes from oracle_lib.parse_obj and is
pinned to the reference by tests/test_hulls_oracle.py.  Bar as for cubes:
bit-exact bodies, candidates and contacts."""
import os

import numpy as np
import pytest

from oracle_lib import HullSet, OraclePhys, PhysConfig, gen_collisions_inits

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
DATA = os.path.join(os.path.dirname(HERE), "gpu-ecs-madrona_amd", "data")
GOLDEN = os.path.join(HERE, "golden", "hulls_ref.npz")


def _obj(n):
    return os.path.join(DATA, n + ".obj")


def _eq(a, b):
    return all(a[f].tobytes() == b[f].tobytes() for f in a.dtype.names)


def _contacts_equal(a, b):
    n = int(a["numPoints"])
    return (a["ref"].tobytes() == b["ref"].tobytes() and a["alt"].tobytes() == b["alt"].tobytes()
            and n == int(b["numPoints"]) and a["normal"].tobytes() == b["normal"].tobytes()
            and a["points"][:n].tobytes() == b["points"][:n].tobytes()
            and a["lambdaN"][:n].tobytes() == b["lambdaN"][:n].tobytes())


def _pair(names, W, n, seed, max_contacts=2048, max_candidates=4096, pos=None, rot=None):
    import madrona_mi355x as mw
    paths = [_obj(x) for x in names]
    g = mw.default_collisions_config(n, 4, max_contacts, max_candidates, hull_paths=paths)
    o = PhysConfig(n, 4, g.delta_t, g.gravity_z, max_contacts, g.cube_inv_mass,
                   g.cube_inv_inertia, g.mu_s, g.mu_d)
    if pos is None:
        pos, rot = gen_collisions_inits(W, n, seed=seed)
    return mw.CollisionsSim(W, pos, rot, g), OraclePhys(o, pos, rot, HullSet.from_files(paths))


@pytest.mark.parametrize("names,n,seed,steps", [
    (("cube", "wedge", "hex_prism"), 24, 5, 60),
    (("octahedron",), 64, 7, 40),
    (("disc16", "octahedron"), 32, 7, 100),            # past undefined manifolds
    (("disc16", "hex_prism", "wedge", "cube", "octahedron"), 128, 3, 30),
])
def test_hull_worlds_bit_exact_vs_oracle_every_step(names, n, seed, steps):
    W = 3
    sim, orc = _pair(names, W, n, seed)
    for w in range(W):
        assert _eq(sim.bodies(w), orc.bodies(w)), "init state differs"
    for s in range(steps):
        sim.step()
        orc.step()
        assert sim.error_flags() == 0
        for w in range(W):
            ca, cb = sim.candidates(w), orc.candidates(w)
            assert ca.tobytes() == cb.tobytes(), f"step {s} world {w}: candidates differ"
            ka, kb = sim.contacts(w), orc.contacts(w)
            assert len(ka) == len(kb), f"step {s} world {w}: {len(ka)} vs {len(kb)} contacts"
            for i in range(len(ka)):
                assert _contacts_equal(ka[i], kb[i]), f"step {s} world {w}: contact {i} differs"
            assert _eq(sim.bodies(w), orc.bodies(w)), f"step {s} world {w}: bodies differ"


def test_hull_worlds_match_reference_golden():
    g = np.load(GOLDEN, allow_pickle=False)
    sim, _ = _pair(("cube", "wedge", "hex_prism"), 3, 24, 0, pos=g["mixed/pos"],
                   rot=g["mixed/rot"])
    done = 0
    for s in (1, 50, 150, 300):
        sim.step(s - done)
        done = s
        for w in range(3):
            assert _eq(sim.bodies(w), g[f"mixed/s{s}/w{w}"]), f"step {s} world {w}"


def test_hull_worlds_full_size_sampled():
    """8192 worlds x 128 bodies over five hulls; sampled worlds replayed by the
    oracle."""
    W, n = 8192, 128
    names = ("disc16", "hex_prism", "wedge", "cube", "octahedron")
    import madrona_mi355x as mw
    paths = [_obj(x) for x in names]
    g = mw.default_collisions_config(n, 4, 2048, 4096, hull_paths=paths)
    pos, rot = gen_collisions_inits(W, n, seed=0)
    sim = mw.CollisionsSim(W, pos, rot, g)
    sim.step(20)
    assert sim.error_flags() == 0
    o = PhysConfig(n, 4, g.delta_t, g.gravity_z, 2048, g.cube_inv_mass, g.cube_inv_inertia,
                   g.mu_s, g.mu_d)
    sample = [0, 1, 4095, 8191]
    orc = OraclePhys(o, pos[sample], rot[sample], HullSet.from_files(paths))
    orc.step(20, threads=4)
    for i, w in enumerate(sample):
        assert _eq(sim.bodies(w), orc.bodies(i)), f"world {w}"


def test_bad_hull_path_fails_loudly(tmp_path):
    import madrona_mi355x as mw
    g = mw.default_collisions_config(8, 4, 256, 512, hull_paths=[str(tmp_path / "none.obj")])
    pos, rot = gen_collisions_inits(2, 8, seed=0)
    with pytest.raises(mw.MadronaError, match="none.obj"):
        mw.CollisionsSim(2, pos, rot, g)
