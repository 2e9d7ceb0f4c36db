import os, sys, json
sys.path.insert(0, os.path.join(os.getcwd(), "distributed-chess_amd"))
import dchess
e = dchess.Engine(0)
s = dchess.startpos()
g = json.load(open("tests/golden/oracle_golden.json"))["perft_ref"]["startpos"]
for d in (5, 6, 7):
    tots = [int(e.perft(s, d)[0]) for _ in range(4)]
    print(os.environ.get("TAG"), d, tots, "golden", g[str(d)]["total"])
