"""Child categories of k_count2c at perft(startpos, D) (run with DC_C2C_PHASE=7,
which replaces the counts by statistics: divide[0..3] = quiet special
children, full-recount children, simple children, parents; [4..8] the
full children by what changes for the opponent)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "distributed-chess_amd"))
import dchess  # noqa: E402

e = dchess.Engine(0)
tot, div, rm = e.perft(dchess.startpos(), int(os.environ.get("DEPTH", "7")))
q, f, s, p = (int(x) for x in div[:4])
n = s + q + f
c, o, d, b, z = (int(x) for x in div[4:9])
print(f"full children: captures {c / f:.3f}; O rays to redo: orth only {o / f:.3f}, diag only {d / f:.3f}, "
      f"both {b / f:.3f}, neither {z / f:.3f}")
print(f"parents {p}  children {n}  simple {s} ({s / n:.3f})  special quiet {q} ({q / n:.3f})  full {f} ({f / n:.3f})")
