"""Repeated perft(5/6/7) of startpos through one build of libdchess.so
(DCHESS_LIB; TAG labels the output): every run should equal the golden.
Round 2 used it on hand-built variants (-DDC_C2C_SOA=1, -DDC_C3C_MINW=3, ...)
to show that a struct-of-arrays LDS layout of c2c_group's parents gives
varying perft(6) counts at 4 waves/SIMD only.
GPU tool: TAG=x DCHESS_LIB=... python tools/lds_layout_check.py"""
import os, sys, json
sys.path.insert(0, os.path.join(os.getcwd(), "distributed-chess_amd"))
import dchess
e = dchess.Engine(0)
s = dchess.startpos()
g = json.load(open("tests/golden/oracle_golden.json"))["perft_ref"]["startpos"]
for d in (5, 6, 7):
    tots = [int(e.perft(s, d)[0]) for _ in range(4)]
    print(os.environ.get("TAG"), d, tots, "golden", g[str(d)]["total"])
