"""Env sharding across GPUs.

Envs are independent, so the batch partitions by global env id: rank r of a
world of G owns ids [r*N/G, (r+1)*N/G).  Every random draw is keyed by global
env id (Philox), so a rollout is identical for any G.  There is no per-step
collective; the only exchange is an optional gather of rollout tensors
``[T+1, n_local, 13]`` to rank 0 at the end (RCCL over xGMI with backend
"nccl", gloo on CPU).
"""
import numpy as np


def shard_range(total, world, rank):
    """[start, stop) of the global env ids rank `rank` owns (balanced, contiguous)."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    base, rem = divmod(total, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def shard_ids(total, world, rank):
    s, e = shard_range(total, world, rank)
    return np.arange(s, e)


def gather_rollouts(local, dst=0, group=None):
    """Gather per-rank rollouts [T+1, n_r, F] to `dst` as [T+1, sum n_r, F] (rank order = env id order).

    Shards may differ in size by one env; each rank sends its count first.  Uses
    torch.distributed.gather (RCCL point-to-point over xGMI under "nccl")."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n = torch.tensor([local.shape[1]], dtype=torch.int64, device=local.device)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n, group=group)
    counts = [int(c.item()) for c in counts]
    nmax = max(counts)
    pad = local
    if local.shape[1] < nmax:
        pad = torch.zeros((local.shape[0], nmax, local.shape[2]), dtype=local.dtype, device=local.device)
        pad[:, : local.shape[1]] = local
    pad = pad.contiguous()
    bufs = [torch.empty_like(pad) for _ in range(world)] if rank == dst else None
    dist.gather(pad, bufs, dst=dst, group=group)
    if rank != dst:
        return None
    return torch.cat([b[:, :c] for b, c in zip(bufs, counts)], dim=1)
