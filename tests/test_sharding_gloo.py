"""Multi-GPU path on CPU: world sharding + the episode-return all-gather
 with world_size 2 over gloo.  Each rank generates only its
shard's inits (product generator, first_world offset), steps its shard on the
framework's own executor (the CPU back end, libmadrona_cpu.so: the same world
sources, graph and export buffers as a GPU rank), reads the packed export
(getExported slot 2) and all-gathers it; the gathered returns must equal the
oracle's single-process run over all worlds, in world order."""
import os
import socket

import numpy as np
import pytest

import madrona_mi355x  # noqa: F401  (before torch, see madrona_mi355x/__init__.py)
import torch
import torch.distributed as dist
import torch.multiprocessing as tmp

WORLDS_PER_RANK = 3
STEPS = 4
CUBES = 12


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _returns(pos, rot, steps):
    """Per-world episode returns after each step: the collisions env's
    accumulateReturn (mean z of dynamic bodies, float32, row order)."""
    from oracle_lib import OraclePhys, default_phys_config
    sim = OraclePhys(default_phys_config(CUBES, 4, max_contacts=1024), pos, rot)
    ret = np.zeros(pos.shape[0], np.float32)
    out = []
    for _ in range(steps):
        sim.step(1)
        for w in range(pos.shape[0]):
            b = sim.bodies(w)
            z = b["pos"][b["responseType"] == 0][:, 2].astype(np.float32)
            s = np.cumsum(z, dtype=np.float32)[-1] if len(z) else np.float32(0)
            ret[w] = np.float32(ret[w] + (s / np.float32(len(z)) if len(z) else np.float32(0)))
        out.append(ret.copy())
    return out


def _rank_main(rank, world_size, port, result_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        import madrona_mi355x as mw
        from madrona_mi355x.sharding import gather_world_returns, world_shard
        first, n = world_shard(rank, WORLDS_PER_RANK)
        pos, rot = mw.gen_collisions_inits(n, CUBES, seed=0, first_world=first)
        cfg = mw.default_collisions_config(CUBES, 4, 1024, 1024)
        sim = mw.CollisionsSim(n, pos, rot, cfg, backend="cpu", num_workers=1)
        gathered = []
        for _ in range(STEPS):
            sim.step(1)
            r = sim.exported_array(2, np.float32).copy()
            gathered.append(gather_world_returns(torch.from_numpy(r)).numpy().copy())
        assert sim.error_flags() == 0
        sim.close()
        if rank == 0:
            result_q.put(np.stack(gathered))
    finally:
        dist.destroy_process_group()


def test_world_sharded_return_allgather_matches_single_process():
    ws = 2
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import madrona_mi355x as mw
    pos, rot = mw.gen_collisions_inits(ws * WORLDS_PER_RANK, CUBES, seed=0)
    want = np.stack(_returns(pos, rot, STEPS))
    assert got.shape == (STEPS, ws * WORLDS_PER_RANK)
    assert got.tobytes() == want.tobytes()


def test_world_shard_ranges_are_contiguous_and_disjoint():
    from madrona_mi355x.sharding import world_shard
    spans = [world_shard(r, 8192) for r in range(8)]
    assert spans[0] == (0, 8192) and spans[7] == (7 * 8192, 8192)
    covered = np.concatenate([np.arange(f, f + n) for f, n in spans])
    assert np.array_equal(covered, np.arange(8 * 8192))
    with pytest.raises(ValueError):
        world_shard(-1, 4)
