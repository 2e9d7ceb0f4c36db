"""Exhaustive CPU check of the FIDE simple-child identity (test infrastructure):
every position of each suite root's tree to the given depth, every simple
child (tools/fide_simple_proto.py) counted by fastcpu and compared with c0.
  python tools/fide_split_exhaustive.py kiwipete:3 pos6:3 pos3:4 startpos:4 pos4:4
Round 4's runs: profiles/r04/fide_split_exhaustive.jsonl."""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
import fide_simple_proto as F  # noqa: E402
import oracle_lib as O  # noqa: E402


def main():
    og = json.load(open(os.path.join(HERE, "..", "tests", "golden", "oracle_golden.json")))["perft_fide"]
    for arg in sys.argv[1:]:
        name, depth = arg.split(":")
        depth = int(depth)
        t0 = time.time()
        frontier = [O.Pos.from_fen(og[name]["fen"])]
        allpos = list(frontier)
        for _ in range(depth):
            frontier = [O.fast_make(p, int(m), O.FIDE) for p in frontier for m in O.fast_gen_moves(p, O.FIDE)]
            allpos += frontier
        tot = simp = bad = 0
        for pos in allpos:
            moves = O.fast_gen_moves(pos, O.FIDE)
            tot += len(moves)
            sm = F.simple_moves(pos, moves, F.sens(pos))
            if not sm:
                continue
            q = pos.copy()
            q.stm, q.ep = 1 - pos.stm, -1
            c0 = len(O.fast_gen_moves(q, O.FIDE))
            for m in sm:
                simp += 1
                bad += len(O.fast_gen_moves(O.fast_make(pos, m, O.FIDE), O.FIDE)) != c0
        print(json.dumps({"root": name, "depth": depth, "positions": len(allpos), "children": tot, "simple": simp,
                          "mismatches": bad, "s": round(time.time() - t0)}), flush=True)


if __name__ == "__main__":
    main()
