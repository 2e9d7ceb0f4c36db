"""Average k_count2* time of perft(startpos, D) over N runs (HIP events on the
context stream); no parity check, so it can time the DC_C2C_PHASE variants."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-chess_amd"))
import dchess  # noqa: E402

depth = int(os.environ.get("DEPTH", "7"))
n = int(os.environ.get("RUNS", "10"))
eng = dchess.Engine(0)
pos = dchess.startpos()
for _ in range(2):
    eng.perft(pos, depth)
eng.reset_stats()
eng.set_profiling(True)
for _ in range(n):
    tot, _, _ = eng.perft(pos, depth)
eng.set_profiling(False)
k = eng.kernel_stats("count2")
print(f"count2 {k['total_ms'] / max(k['launches'], 1):.4f} ms  total={tot}")
