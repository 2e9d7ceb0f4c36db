"""c2c_group investigation: perft(5/6/7) of startpos
through one build of libdchess.so (DCHESS_LIB), N runs each, printing the
total and the per-root-move divide entries that differ from the golden.
GPU tool:  TAG=soa DCHESS_LIB=.../lib_soa.so python tools/c2c_diag.py [runs]"""
import os, sys, json
sys.path.insert(0, os.path.join(os.getcwd(), "distributed-chess_amd"))
import dchess
runs = int(sys.argv[1]) if len(sys.argv) > 1 else 3
e = dchess.Engine(0)
s = dchess.startpos()
g = json.load(open("tests/golden/oracle_golden.json"))["perft_ref"]["startpos"]
tag = os.environ.get("TAG", "?")
for d in (5, 6, 7):
    gold = g[str(d)]
    gdiv = gold.get("divide")
    for r in range(runs):
        tot, div, rm = e.perft(s, d)
        out = {"tag": tag, "depth": d, "run": r, "total": int(tot), "golden": gold["total"],
               "delta": int(tot) - gold["total"]}
        if int(tot) != gold["total"]:
            # root-move index (the node order's tag) -> count delta
            out["divide_delta"] = {f"{i}:{int(m)}": int(div[i]) - int(gdiv[str(int(m))])
                                   for i, m in enumerate(rm) if int(div[i]) != int(gdiv[str(int(m))])}
        print(json.dumps(out), flush=True)
