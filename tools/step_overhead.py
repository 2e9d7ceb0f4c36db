"""Times perft(startpos, d) steps with and without per-launch HIP-event profiling.
argv: depth [split n_shards shard] -- with shards, one rank's dc_perft_shard step."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "distributed-chess_amd"))
import dchess  # noqa: E402

eng = dchess.Engine(0)
pos = dchess.startpos()
depth = int(sys.argv[1]) if len(sys.argv) > 1 else 6
split, n_sh, shard = (int(x) for x in sys.argv[2:5]) if len(sys.argv) > 4 else (3, 1, 0)


def step():
    return eng.perft_shard(pos, depth, split, shard, n_sh) if n_sh > 1 else eng.perft(pos, depth)


for _ in range(5):
    step()
for prof in (False, True, False):
    eng.set_profiling(prof)
    eng.reset_stats()
    t0 = time.perf_counter()
    n = 50
    for _ in range(n):
        step()
    dt = (time.perf_counter() - t0) / n
    ks = {k: round(eng.kernel_stats(k)["total_ms"] / n, 4)
          for k in ("expand_top", "expand_count", "scan", "expand_write", "count2")}
    print(f"shards={n_sh} profiling={prof} step_ms={dt * 1e3:.3f} kernels_ms={sum(ks.values()):.3f} {ks}", flush=True)
