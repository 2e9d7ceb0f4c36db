"""Determinism stress of the shipped perft build: 60 x perft(6), 30 x perft(7)
and 3 x each over 8 strided shards, all against the golden totals.  Round 2:
"runs ok" on MI355X.  GPU tool: python tools/perft_stress.py"""
import os, sys, json
sys.path.insert(0, os.path.join(os.getcwd(), "distributed-chess_amd"))
import dchess
e = dchess.Engine(0)
s = dchess.startpos()
g = json.load(open("tests/golden/oracle_golden.json"))["perft_ref"]["startpos"]
bad = 0
for d, n in ((6, 60), (7, 30)):
    for _ in range(n):
        t = int(e.perft(s, d)[0]); bad += t != g[str(d)]["total"]
for d in (6, 7):
    for _ in range(3):
        t = sum(int(e.perft_shard(s, d, 3, k, 8)[0]) for k in range(8)); bad += t != g[str(d)]["total"]
print("runs ok" if bad == 0 else f"MISMATCHES {bad}")
