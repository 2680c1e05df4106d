"""Multi-GPU layer: one process per GPU, batches sharded across ranks, keys broadcast.

The path shards embarrassingly (every bfv_mul_and_relin / dbfv_mul in a batch is
independent), so there is NO data-path collective: each rank owns a
contiguous slice of the batch.  The only collective is the one-time RCCL broadcast of
the relinearisation key over xGMI (2.25 MiB at cfg3/4, 15 MiB at cfg5).  Results can be
gathered to one rank with ``gather_to`` (all_gather of equal-sized shards); an RCCL
ncclSum would overflow mod q and is never used.
"""

from __future__ import annotations

import torch
import torch.distributed as dist


def shard(total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [start, start+count) slice of ``total`` items for ``rank`` (sizes differ by <= 1)."""
    base, extra = divmod(total, world)
    count = base + (1 if rank < extra else 0)
    start = rank * base + min(rank, extra)
    return start, count


def broadcast_key(key: torch.Tensor, src: int = 0) -> torch.Tensor:
    """Broadcast the relinearisation key (``[G][2][L][n]`` int64 view of u64) from ``src``."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.broadcast(key, src=src)
    return key


def load_key_everywhere(ctx, key: torch.Tensor, num_keys: int, src: int = 0):
    """Broadcast ``key`` from ``src`` and make it the context's resident relinearisation key."""
    broadcast_key(key, src)
    ctx.load_relin_key_dev(key, num_keys)


def max_over_ranks(value: float, device=None) -> float:
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_to(shard_out: torch.Tensor, total: int, dst: int = 0):
    """Collect every rank's output shard on ``dst`` (returns the concatenation there, None elsewhere).
    Shards are padded to the largest shard size for the collective."""
    world = dist.get_world_size()
    rank = dist.get_rank()
    maxc = shard(total, 0, world)[1]
    pad = torch.zeros((maxc,) + tuple(shard_out.shape[1:]), dtype=shard_out.dtype, device=shard_out.device)
    pad[: shard_out.shape[0]] = shard_out
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad)
    if rank != dst:
        return None
    return torch.cat([parts[r][: shard(total, r, world)[1]] for r in range(world)])
