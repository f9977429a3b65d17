"""World sharding across GPUs.

Worlds are independent (a world's Context only reaches its own state,
reference include/madrona/context.hpp:152-156), so N GPUs hold contiguous
world ranges: rank r owns worlds [r * W, (r + 1) * W) and steps them with no
cross-GPU traffic.  The only collective is the training hand-off: the
per-world episode returns (an exported singleton column, state.hpp:128-129)
are all-gathered into world order -- RCCL over xGMI issued by the framework
on its step stream (bootstrap_rccl + Executor.allgather_exported) on the GPU
path; gather_world_returns is the same gather over any torch.distributed
backend (gloo in the CPU tests).
"""


def world_shard(rank, worlds_per_rank):
    """(first_world, num_worlds) of `rank` under contiguous weak-scaling
    sharding; init generation uses first_world so every world draws the same
    seeds it would in a single-process run."""
    if rank < 0 or worlds_per_rank <= 0:
        raise ValueError("rank must be >= 0 and worlds_per_rank > 0")
    return rank * worlds_per_rank, worlds_per_rank


def gather_world_returns(local, out=None, group=None):
    """All-gather each rank's [W] per-world returns into [world_size * W] in
    global world order.  Uses the single-buffer collective (one RCCL
    all-gather over xGMI); backends without it (gloo) fall back to the list
    form with identical results."""
    import torch
    import torch.distributed as dist

    ws = dist.get_world_size(group)
    if out is None:
        out = torch.empty(ws * local.numel(), dtype=local.dtype, device=local.device)
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, local, group=group)
    else:
        parts = [torch.empty_like(local) for _ in range(ws)]
        dist.all_gather(parts, local, group=group)
        torch.cat(parts, out=out)
    return out


def bootstrap_rccl(sim, rank, world_size, group=None):
    """Create the world-shard RCCL communicator of `sim` (an Executor): rank 0
    draws the 128-byte id, torch.distributed (any backend, e.g. gloo over the
    launcher's TCP store) broadcasts it, every rank joins."""
    import torch.distributed as dist
    import madrona_mi355x as mw

    uid = [mw.rccl_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0, group=group)
    sim.rccl_init(uid[0], world_size, rank)
