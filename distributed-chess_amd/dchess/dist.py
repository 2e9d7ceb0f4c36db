"""Data-parallel perft / replay across ranks (one process per GPU).

Perft.  Every rank rebuilds the top plies identically (their order is
deterministic) and counts the subtrees of its STRIDED shard of the ply-`split`
frontier: nodes rank, rank + world, rank + 2*world, ... (dc_perft_shard: the
front end selects the shard's nodes by index -- k_front for REF depth 6/7 at
split 3, k_make_count over the top kernel's move words otherwise; strided
shards carry equal leaf counts to ~1 %, contiguous eighths differed by 1.47x).  The per-root-move divide vectors are summed with
one all-reduce -- RCCL over xGMI with the "nccl" backend, gloo on CPU in the
tests.  (The A/B build's DC_SHARD=contig knob takes contiguous slices.)

Replay.  Game ids [0, n_total) are split into contiguous ranges of whole
64-game bitmap words (replay_range == dc_replay_shard_range).  Rank r
generates and replays its range; the exchange step is
  * the five counters: validated / accepted / rejected / digest_sum are sums
    mod 2^64 and digest_xor an xor (not an all-reduce op RCCL has), so the
    40-byte records are all-gathered and folded;
  * the per-rank ply-major accept bitmaps, gathered to rank 0 and placed at
    their word offsets of the whole batch's ply-major bitmap.
No other data crosses ranks.
"""
import numpy as np

STAT_KEYS = ("validated", "accepted", "rejected", "digest_sum", "digest_xor")


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


# ------------------------------------------------------------------- replay
def replay_range(n_total, rank, world):
    """(first game id, count) of rank's replay shard: contiguous, whole 64-game
    words (the contract of dc_replay_shard_range, include/dchess.h)."""
    words = (n_total + 63) // 64
    per = (words + world - 1) // world
    lo = min(n_total, min(words, rank * per) * 64)
    hi = min(n_total, min(words, (rank + 1) * per) * 64)
    return lo, max(hi - lo, 0)


def fold_stats(records):
    """Combines per-shard {validated, accepted, rejected, digest_sum, digest_xor}
    records (uint64 [k, 5]): the first four add mod 2^64, the last xors."""
    r = np.asarray(records, np.uint64).reshape(-1, 5)
    out = np.zeros(5, np.uint64)
    with np.errstate(over="ignore"):
        out[:4] = r[:, :4].sum(axis=0, dtype=np.uint64)
    out[4] = np.bitwise_xor.reduce(r[:, 4]) if len(r) else 0
    return dict(zip(STAT_KEYS, (int(x) for x in out)))


def combine_replay(stats, bitmap, n_total, rank, world, device="cpu"):
    """The replay exchange step.  stats: this rank's 5 counters (dict or uint64
    [5]); bitmap: this rank's ply-major bitmap, a torch int64 tensor
    [n_plies][words of its range] on `device` (or None: counters only).
    Returns (combined stats dict, whole-batch bitmap uint64 [n_plies][W] on
    rank 0 else None).  Collectives: one all_gather of 5 x u64 per rank, one
    gather of the (padded) bitmaps to rank 0."""
    import torch
    import torch.distributed as dist
    if isinstance(stats, dict):
        stats = [stats[k] for k in STAT_KEYS]
    mine = np.asarray(stats, np.uint64)
    if not dist.is_initialized() or world == 1:
        bm = None if bitmap is None else bitmap.cpu().numpy().view(np.uint64)
        return fold_stats(mine), bm
    t = torch.from_numpy(mine.view(np.int64).copy()).to(device)
    recs = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(recs, t)
    combined = fold_stats(np.stack([x.cpu().numpy().view(np.uint64) for x in recs]))
    if bitmap is None:
        return combined, None
    words = (n_total + 63) // 64
    per = (words + world - 1) // world
    plies = bitmap.shape[0]
    padded = torch.zeros((plies, per), dtype=torch.int64, device=device)
    padded[:, :bitmap.shape[1]] = bitmap
    gl = [torch.empty_like(padded) for _ in range(world)] if rank == 0 else None
    dist.gather(padded, gather_list=gl, dst=0)
    if rank != 0:
        return combined, None
    out = np.zeros((plies, words), np.uint64)
    for r, g in enumerate(gl):
        first, count = replay_range(n_total, r, world)
        w = (count + 63) // 64
        out[:, first // 64:first // 64 + w] = g[:, :w].cpu().numpy().view(np.uint64)
    return combined, out


def game_range(rank, world, games_per_rank):
    """First game id and count of a rank's shard when every rank replays its own
    `games_per_rank` games (weak scaling)."""
    return rank * games_per_rank, games_per_rank
