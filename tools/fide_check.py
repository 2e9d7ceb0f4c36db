"""FIDE suite counts of one library build (diagnostics):
DCHESS_LIB=... python tools/fide_check.py [--depth D] [names...]"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-chess_amd"))
import dchess  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("names", nargs="*", default=["kiwipete", "pos3", "pos4", "pos5", "pos6", "startpos"])
ap.add_argument("--depth", type=int, default=5)
ap.add_argument("--divide", action="store_true", help="per-root-move differences against fastcpu")
ap.add_argument("--repeat", type=int, default=1)
args = ap.parse_args()
og = json.load(open(os.path.join(REPO, "tests", "golden", "oracle_golden.json")))["perft_fide"]
eng = dchess.Engine(0)
out, divs = {}, {}
for k in args.names:
    for rep in range(args.repeat):
        t, div, rm = eng.perft(dchess.pos_from_fen(og[k]["fen"]), args.depth, rules=dchess.RULES_FIDE)
        out.setdefault(k, []).append(int(t) - og[k]["perft"][str(args.depth)])
        if args.divide and int(t) != og[k]["perft"][str(args.depth)]:
            sys.path.insert(0, os.path.join(REPO, "tests"))
            import oracle_lib as ol
            if k not in divs:
                _, fdiv, frm = ol.fast_perft(ol.Pos.from_fen(og[k]["fen"]), args.depth, ol.FIDE, threads=16)
                divs[k] = {int(m): int(v) for m, v in zip(frm, fdiv)}
            d = {int(m): int(v) - divs[k][int(m)] for m, v in zip(rm, div) if int(v) != divs[k][int(m)]}
            print(json.dumps({"pos": k, "rep": rep, "n_root": len(rm), "root_diffs": {str(m): v for m, v in d.items()}}))
print(json.dumps({"lib": os.environ.get("DCHESS_LIB", "product"), "cu_mask": os.environ.get("ROC_GLOBAL_CU_MASK"),
                  "grid": os.environ.get("DC_DIAG_GRID"), f"diff_vs_published_d{args.depth}": out}))
