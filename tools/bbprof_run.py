#!/usr/bin/env python3
"""Run one workload on the instrumented library (tools/bbprof_build.sh) and
write the per-block wave-execution counts (tools/bbprof.py model input).
  DCHESS_LIB=.../build/bb/libdchess_bb.so python tools/bbprof_run.py perft7|fide7|replay|gen|hash OUT.json
The workload's result is checked against its golden value, so an
instrumentation that changed the kernel's behaviour fails here."""
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-chess_amd"))
import numpy as np  # noqa: E402

import dchess  # noqa: E402

work, out = sys.argv[1], sys.argv[2]
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 1
L = dchess.lib()
file = "moves" if work in ("replay", "gen") else "hash" if work == "hash" else "perft"
fn = getattr(C.CDLL(dchess.LIB_PATH), f"dc_ab_bbprof_{file}")
fn.argtypes = [C.c_void_p, C.c_int]
eng = dchess.Engine(0)
res = {}
if work == "fide7":  # FIDE final stage (k_count2b<FideRules>), published perft(7)
    pos = dchess.pos_from_fen("rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1")
    eng.perft(pos, 7, rules=dchess.RULES_FIDE)
    assert fn(None, 1) == 0
    for _ in range(reps):
        tot, _, _ = eng.perft(pos, 7, rules=dchess.RULES_FIDE)
        if tot != 3195901860:
            raise SystemExit(f"FIDE perft(7) = {tot}: the instrumented kernel changed the result")
    res["result"] = int(tot)
elif work.startswith("perft"):
    depth = int(work[5:])
    want = {6: 120909581, 7: 3282734510}[depth]
    eng.perft(dchess.startpos(), depth)  # warm (graphs, buffers)
    assert fn(None, 1) == 0
    for _ in range(reps):
        tot, _, _ = eng.perft(dchess.startpos(), depth)
        if tot != want:
            raise SystemExit(f"perft({depth}) = {tot}, want {want}: the instrumented kernel changed the result")
    res["result"] = int(tot)
elif work == "hash":  # k_state_hash_ref on the bench's workload; game 0's hash as the check
    n = 1_000_000
    d_mv, d_h = eng.alloc(n * 80 * 2), eng.alloc(n * 32)
    eng.gen_games_device(d_mv, 0x5EED20241022, 0, n, 80, 32)
    blob, off = dchess.pack_names([(f"white{g}", f"black{g}") for g in range(n)])
    d_names, d_off = eng.names_device(blob, off)
    eng.state_hash_device(d_mv, n, 80, d_names, d_off, d_h)
    eng.synchronize()
    assert fn(None, 1) == 0
    for _ in range(reps):
        eng.state_hash_device(d_mv, n, 80, d_names, d_off, d_h)
    h0 = bytes(d_h.download(np.uint8, 32)).hex()
    if not h0.startswith("384ec2c485379b44"):
        raise SystemExit(f"game 0 hash {h0}: the instrumented kernel changed the result")
    res["result"] = h0
elif work in ("replay", "gen"):
    g = json.load(open(os.path.join(REPO, "tests", "golden", "replay_golden.json")))
    n = 1_000_000
    mv = eng.gen_games(int(g["seed"], 0) if isinstance(g["seed"], str) else g["seed"], 0, n, 80, 32)
    assert fn(None, 1) == 0
    for _ in range(reps):
        if work == "gen":
            mv2 = eng.gen_games(int(g["seed"], 0) if isinstance(g["seed"], str) else g["seed"], 0, n, 80, 32)
            if not (mv2 == mv).all():
                raise SystemExit("generator output changed under instrumentation")
        else:
            bm, dg, st = eng.replay(mv)
    res["result"] = "ok"
buf = np.zeros(8192, np.uint64)
assert fn(buf.ctypes.data, 0) == 0
res.update({"work": work, "launches": reps, "lib": dchess.LIB_PATH, "wave_executions": [int(x) for x in buf]})
json.dump(res, open(out, "w"))
print(work, "blocks with executions:", int((buf > 0).sum()), "max", int(buf.max()))
