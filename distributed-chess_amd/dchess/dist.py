"""Data-parallel perft / replay across ranks (one process per GPU).

Perft shards the deterministic frontier at ply `split`: every rank rebuilds the
top plies identically, takes the contiguous slice [r*N/W, (r+1)*N/W) of that
ply (dc_perft_shard), counts its subtrees, and the per-root-move divide vectors
are summed with one all-reduce (RCCL over xGMI with the "nccl" backend; gloo on
CPU in the tests).  Replay partitions game ids: rank r replays games
[r*G, (r+1)*G) of the seeded generator; counters are all-reduced.
No other data crosses ranks.
"""
import numpy as np


def allreduce_sum_u64(vec, group=None, device=None):
    """Sums a uint64 vector over all ranks (values stay < 2^63)."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return np.asarray(vec, np.uint64)
    t = torch.tensor(np.asarray(vec, np.uint64).astype(np.int64), device=device or "cpu")
    dist.all_reduce(t, group=group)
    return t.cpu().numpy().astype(np.uint64)


def sharded_perft(shard_fn, pos, depth, split, rank, world, reduce=allreduce_sum_u64):
    """shard_fn(pos, depth, split, shard, n_shards) -> (total, divide, root_moves)
    for this rank's shard; returns the global (total, divide, root_moves)."""
    _, div, rm = shard_fn(pos, depth, split, rank, world)
    div = reduce(np.asarray(div, np.uint64))
    return int(div.sum(dtype=np.uint64)), div, rm


def game_range(rank, world, games_per_rank):
    """First game id and count of this rank's replay shard (weak scaling)."""
    return rank * games_per_rank, games_per_rank
