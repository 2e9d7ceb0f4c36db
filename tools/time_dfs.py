"""Times REF perft(startpos, d) through K4 (k_perft_dfs) for d in argv (default 8):
total, wall ms per run, dfs kernel ms (HIP events) and the level memory used.
Prints one JSON line per depth.  GPU tool (no parity check beyond printing the
total; the tests hold the goldens)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "distributed-chess_amd"))
import dchess  # noqa: E402

eng = dchess.Engine(0)
s = dchess.startpos()
for d in [int(x) for x in sys.argv[1:]] or [8]:
    t0 = time.perf_counter()
    tot, div, rm = eng.perft(s, d)
    first = time.perf_counter() - t0
    reps = 3 if d <= 8 else 1
    t0 = time.perf_counter()
    for _ in range(reps):
        eng.perft(s, d)
    wall = time.perf_counter() - t0
    eng.reset_stats()
    eng.set_profiling(True)
    eng.perft(s, d)
    eng.set_profiling(False)
    k = {n: eng.kernel_stats(n) for n in ("dfs", "count2", "expand_write", "expand_top")}
    print(json.dumps({"depth": d, "total": tot, "first_run_s": first, "ms_per_run": 1e3 * wall / reps,
                      "leaves_per_s": tot / (wall / reps), "kernels_ms": {n: v["total_ms"] for n, v in k.items()},
                      "divide": {str(int(m)): int(v) for m, v in zip(rm, div)}}), flush=True)
