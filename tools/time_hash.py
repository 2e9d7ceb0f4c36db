"""Kernel time of dc_state_hash_device on N seeded games x 80 plies (HIP events)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "distributed-chess_amd"))
import numpy as np  # noqa: E402

import dchess  # noqa: E402

n = int(os.environ.get("GAMES", "1000000"))
plies = 80
eng = dchess.Engine(0)
d_moves = eng.alloc(n * plies * 2)
d_h = eng.alloc(n * 32)
eng.gen_games_device(d_moves, 0x5EED20241022, 0, n, plies, 32)
blob, off = dchess.pack_names([(f"white{g}", f"black{g}") for g in range(n)])
d_names, d_off = eng.names_device(blob, off)
eng.state_hash_device(d_moves, n, plies, d_names, d_off, d_h)
eng.set_profiling(True)
for _ in range(3):
    eng.state_hash_device(d_moves, n, plies, d_names, d_off, d_h)
eng.set_profiling(False)
k = eng.kernel_stats("state_hash")
ms = k["total_ms"] / k["launches"]
print(f"state_hash {n} games: {ms:.3f} ms  {n / ms * 1e3:.3e} hashes/s  first 0x{bytes(d_h.download(np.uint8, 32)).hex()}")
