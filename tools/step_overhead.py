"""Times perft(startpos, d) steps with and without per-launch HIP-event profiling."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "distributed-chess_amd"))
import dchess  # noqa: E402

eng = dchess.Engine(0)
pos = dchess.startpos()
depth = int(sys.argv[1]) if len(sys.argv) > 1 else 6
for _ in range(5):
    eng.perft(pos, depth)
for prof in (False, True, False):
    eng.set_profiling(prof)
    eng.reset_stats()
    t0 = time.perf_counter()
    n = 50
    for _ in range(n):
        eng.perft(pos, depth)
    dt = (time.perf_counter() - t0) / n
    ks = {k: eng.kernel_stats(k)["total_ms"] / n for k in ("expand_top", "expand_count", "scan", "expand_write", "count2")}
    print(f"profiling={prof} step_ms={dt * 1e3:.3f} kernels_ms={sum(ks.values()):.3f} {ks}")
