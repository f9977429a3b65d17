"""configs[3] on the one GPU a test box has: the sharded HIP executor.

BASELINE.json configs[3] is 65 536 collisions worlds over 8 GPUs, rank g
owning worlds [8192 g, 8192 (g + 1)) (madrona_mi355x/sharding.py).  Eight
gloo ranks stand in for the node's 8 GPUs: each creates the HIP executor on
device 0 for its shard (inits drawn with the GLOBAL world index,
first_world = 8192 g; 8 x ~4.8 GB of HBM), steps it, and all-gathers the
per-world episode returns with sharding.gather_world_returns (the gloo form
of the RCCL hand-off; RCCL itself cannot put two ranks on one device, so the
RCCL nranks > 1 path stays unmeasured until the driver's 8-GPU run).
Checks:
  * the gathered 65 536 returns equal one process stepping all 8 shards in
    order;
  * sampled worlds of every shard, replayed by the oracle from their global
    index, are bit-exact (bodies, candidates, contacts).
Reference: SURVEY.md §8(e); per-executor init src/mw/cuda_exec.cpp:1692-1763.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

WORLDS_PER_RANK = 8192
SHARDS = tuple(range(8))  # the ranks of an 8-GPU node these processes play
STEPS = 48
SAMPLE = (0, 1, 4095, 8191)   # local indices checked against the oracle


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _cfg(mw):
    return mw.default_collisions_config(128, 4, max_contacts=4096, max_candidates=4096)


def _sim(mw, shard):
    from madrona_mi355x.sharding import world_shard
    first, n = world_shard(shard, WORLDS_PER_RANK)
    pos, rot = mw.gen_collisions_inits(n, 128, seed=0, first_world=first)
    return mw.CollisionsSim(n, pos, rot, _cfg(mw))


def _check_sample(mw, sim, shard):
    """Oracle replay of sampled worlds from their global index."""
    from oracle_lib import OraclePhys, PhysConfig
    from madrona_mi355x.sharding import world_shard
    import test_collisions_gpu as tc
    g = _cfg(mw)
    o = PhysConfig(128, 4, g.delta_t, g.gravity_z, 4096, g.cube_inv_mass, g.cube_inv_inertia,
                   g.mu_s, g.mu_d)
    first, n = world_shard(shard, WORLDS_PER_RANK)
    pos, rot = mw.gen_collisions_inits(n, 128, seed=0, first_world=first)
    sel = list(SAMPLE)
    orc = OraclePhys(o, np.ascontiguousarray(pos[sel]), np.ascontiguousarray(rot[sel]))
    orc.step(STEPS, 4)
    for k, w in enumerate(SAMPLE):
        d = tc._diff(sim.bodies(w), orc.bodies(k))
        assert d is None, f"shard {shard} world {first + w}: {d}"
        assert sim.candidates(w).tobytes() == orc.candidates(k).tobytes(), (shard, w)
        ka, kb = sim.contacts(w), orc.contacts(k)
        assert len(ka) == len(kb), (shard, w)
        for i in range(len(ka)):
            assert tc._contacts_equal(ka[i], kb[i]), (shard, w, i)


def _rank_main(rank, world_size, port, result_q):
    import madrona_mi355x as mw   # before torch (one HIP runtime)
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        from madrona_mi355x.sharding import gather_world_returns
        shard = SHARDS[rank]
        sim = _sim(mw, shard)
        sim.step(STEPS)
        assert sim.error_flags() == 0, mw.ERR_BITS
        local = torch.from_numpy(sim.exported_array(2, np.float32).copy())
        assert local.numel() == WORLDS_PER_RANK
        gathered = gather_world_returns(local).numpy().copy()
        _check_sample(mw, sim, shard)
        sim.close()
        result_q.put((rank, gathered))
    finally:
        dist.destroy_process_group()


def test_configs3_shards_on_one_gpu_gather_and_oracle():
    import torch.multiprocessing as tmp
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    n = len(SHARDS)
    procs = [ctx.Process(target=_rank_main, args=(r, n, port, q)) for r in range(n)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in procs:
            r, g = q.get(timeout=150)
            got[r] = g
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.exitcode is None:
                p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert all(got[r].tobytes() == got[0].tobytes() for r in range(n))
    assert got[0].size == n * WORLDS_PER_RANK
    # one process running every shard, in global world order
    import madrona_mi355x as mw
    want = []
    for shard in SHARDS:
        sim = _sim(mw, shard)
        sim.step(STEPS)
        want.append(sim.exported_array(2, np.float32))
        sim.close()
    want = np.concatenate(want)
    assert np.isfinite(want).all()
    assert got[0].tobytes() == want.tobytes()
