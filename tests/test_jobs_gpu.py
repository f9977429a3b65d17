"""The reference's job API (ctx.submit / ctx.parallelFor / ctx.archetype /
currentJobID) on the GPU, running the examples written
against it:

* fantasy_vs_jobs (csrc/envs/fvs_jobs.hip = examples/fantasy_vs/fvs.cpp
  with the edits listed there) matches the oracle (oracle/fvs_oracle.cpp,
  pinned to the reference ECS) and the TaskGraph restatement (fantasy_vs)
  bit for bit -- entity ids, generations, row order -- while both sides of a
  world have entities left (then the job loop stops, as the reference's
  gameLoop does);
* collisions_jobs (csrc/envs/collisions_jobs.hip = collisions.cpp:88-227)
  matches oracle/jobs_oracle.cpp bit for bit every tick (parity unpinned
  against the reference runtime, whose job system is not compiled)."""
import numpy as np
import pytest

import oracle_lib as ol

pytestmark = pytest.mark.gpu


def _mw():
    import madrona_mi355x as mw
    return mw


def test_fvs_jobs_matches_oracle_through_deaths():
    mw = _mw()
    W = 6
    inits = ol.gen_fvs_inits(W, 50, 200, seed=0)
    sim = mw.FvsSim(W, inits, env="fantasy_vs_jobs")
    orc = ol.OracleFvs(inits)
    compared = 0
    for t in range(1, 16):
        sim.step(100)
        orc.step(100)
        assert sim.error_flags() == 0
        for w in range(W):
            if len(orc.table(w, 0)) == 0 or len(orc.table(w, 1)) == 0:
                continue                       # a side is gone: the job loop stopped
            for arch in (0, 1):
                assert sim.table(w, arch).tobytes() == orc.table(w, arch).tobytes(), (t, w, arch)
            compared += 1
    assert compared > 60
    assert sum(len(orc.table(w, 0)) for w in range(W)) < 50 * W     # deaths happened


def test_fvs_jobs_every_tick_around_first_deaths():
    mw = _mw()
    W = 4
    inits = ol.gen_fvs_inits(W, 50, 200, seed=7)
    sim = mw.FvsSim(W, inits, env="fantasy_vs_jobs")
    orc = ol.OracleFvs(inits)
    sim.step(550)
    orc.step(550)
    for t in range(120):
        sim.step()
        orc.step()
        for w in range(W):
            for arch in (0, 1):
                assert sim.table(w, arch).tobytes() == orc.table(w, arch).tobytes(), (t, w, arch)


def test_fvs_jobs_matches_taskgraph_restatement_full_size():
    mw = _mw()
    W = 4096
    inits = mw.gen_fvs_inits(W, 50, 200, seed=11)
    a = mw.FvsSim(W, inits)
    b = mw.FvsSim(W, inits, env="fantasy_vs_jobs")
    a.step(400)
    b.step(400)
    assert a.error_flags() == 0 and b.error_flags() == 0
    for w in range(0, W, 61):
        ta = [a.table(w, k) for k in (0, 1)]
        if min(len(t) for t in ta) == 0:
            continue
        for k in (0, 1):
            assert ta[k].tobytes() == b.table(w, k).tobytes(), (w, k)


def test_collisions_jobs_matches_oracle_every_tick():
    mw = _mw()
    W, N = 6, 100
    pos, rot = ol.gen_collisions_inits(W, N, seed=0)
    sim = mw.JobsCollisionsSim(W, pos, rot, max_candidates=2048)
    orc = ol.OracleJobsCollisions(pos, rot, max_candidates=2048)
    for t in range(25):
        sim.step()
        orc.step()
        assert sim.error_flags() == 0
        for w in range(W):
            assert not orc.last_counts(w)[2]
            assert sim.cubes(w).tobytes() == orc.cubes(w).tobytes(), (t, w)
    assert sum(orc.last_counts(w)[0] for w in range(W)) >= 0


def test_collisions_jobs_many_worlds_sampled():
    mw = _mw()
    W, N = 2048, 100
    pos, rot = ol.gen_collisions_inits(W, N, seed=5)
    sim = mw.JobsCollisionsSim(W, pos, rot, max_candidates=2048)
    sim.step(5)
    assert sim.error_flags() == 0
    sample = list(range(0, W, 257))
    orc = ol.OracleJobsCollisions(pos[sample], rot[sample], max_candidates=2048)
    orc.step(5)
    for i, w in enumerate(sample):
        assert sim.cubes(w).tobytes() == orc.cubes(i).tobytes(), w
