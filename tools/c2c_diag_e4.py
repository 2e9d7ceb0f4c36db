"""Round-2 fault, grid-length vs side-to-move control:
perft(6) and perft(7) after 1.e4 (Black to move at the root), N runs each,
through one build (run from that build's tree).  perft(6) after 1.e4 runs the
final stage k_count3c<0, ...> on a short grid (ply 3, ~9k grandparents) and
perft(7) runs k_count3c<1, ...> on a long one -- the opposite pairing of
startpos, where perft(6) (<1>, short) fails and perft(7) (<0>, long) is exact.
Goldens: the startpos perft(7) / perft(8) divide entries of e2e4 (1804)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.getcwd(), "distributed-chess_amd"))
import dchess  # noqa: E402

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 3
gold = {6: 325340111, 7: 8764808383}
e = dchess.Engine(0)
p = dchess.pos_from_fen("rnbqkbnr/pppppppp/8/8/4P3/8/PPPP1PPP/RNBQKBNR b - - 0 1")
tag = os.environ.get("TAG", "?")
for d in (6, 7):
    for r in range(runs):
        tot = int(e.perft(p, d)[0])
        print(json.dumps({"tag": tag, "root": "startpos+e2e4", "depth": d, "run": r, "total": tot,
                          "golden": gold[d], "delta": tot - gold[d]}), flush=True)
