"""CPU checks of oracle/jobs_oracle.cpp, the restatement of examples/
collisions' job-API toy (collisions.cpp:88-227) that pins the GPU
collisions_jobs environment.  The reference's job system is not compiled in
its snapshot, so the toy cannot run there: these are the
example's own invariants -- every overlapping pair is found in both orders,
every candidate becomes exactly one contact, candidates / contacts are
cleared each tick and their entity ids recycled, cube ids never change, and
the solver's pushes move every touched cube by whole unit normals."""
import numpy as np

import oracle_lib as ol


def _aabb_overlaps(a, b):
    return (a[:3] < b[3:]).all() and (b[:3] < a[3:]).all()


def test_toy_pairs_contacts_and_ids():
    W, N = 3, 100
    pos, rot = ol.gen_collisions_inits(W, N, seed=0)
    orc = ol.OracleJobsCollisions(pos, rot, max_candidates=4096)
    ids0 = [(orc.cubes(w)["gen"].copy(), orc.cubes(w)["id"].copy()) for w in range(W)]
    orc.step(1)
    for w in range(W):
        c = orc.cubes(w)
        pairs = sum(_aabb_overlaps(c["aabb"][i], c["aabb"][j])
                    for i in range(N) for j in range(N) if i != j)
        cands, contacts, overflow = orc.last_counts(w)
        assert not overflow
        assert cands == contacts == pairs and pairs % 2 == 0 and pairs > 0
    orc.step(20)
    for w in range(W):
        c = orc.cubes(w)
        assert (c["gen"] == ids0[w][0]).all() and (c["id"] == ids0[w][1]).all()
        assert np.isfinite(c["pos"]).all()
        assert not orc.last_counts(w)[2]


def test_toy_is_deterministic():
    pos, rot = ol.gen_collisions_inits(2, 100, seed=3)
    a = ol.OracleJobsCollisions(pos, rot)
    b = ol.OracleJobsCollisions(pos, rot)
    a.step(15)
    b.step(15)
    for w in range(2):
        assert a.cubes(w).tobytes() == b.cubes(w).tobytes()
