#!/usr/bin/env python3
"""Same-box A/B timing of perft legs across library builds (measurement only).
  python tools/ab_perft_time.py ROUNDS LIB_A LIB_B ...
Each round runs every library once, in order (ABAB...), each in its own child
process (DCHESS_LIB=<lib>), timing dc_perft_repeat_device steps of:
  ref7   perft(startpos, 7) under RULES_REF     (20 steps)
  fide7  perft(startpos, 7) under RULES_FIDE    (4 steps)
  suite  the six FIDE suite FENs at depth 5     (4 steps each)
with the golden count checked on every step.  Prints one JSON line per run and
a per-library median summary.  LEGS=ref7,fide7 selects legs."""
import json
import os
import statistics
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, os, sys, time
sys.path.insert(0, os.path.join(sys.argv[1], "distributed-chess_amd"))
import numpy as np
import dchess
og = json.load(open(os.path.join(sys.argv[1], "tests", "golden", "oracle_golden.json")))["perft_fide"]
REF7 = 3282734510
eng = dchess.Engine(0)
def timed(pos, depth, steps, rules, want):
    W = 258
    warm = eng.alloc(8 * W * 8)  # 8 runs: also captures the batch graph (kRepeatBatch)
    eng.perft_repeat_device(pos, depth, 3, 0, 1, 8, warm, rules=rules)
    eng.synchronize()
    warm.free()
    buf = eng.alloc(steps * W * 8)
    eng.synchronize()
    t0 = time.perf_counter()
    eng.perft_repeat_device(pos, depth, 3, 0, 1, steps, buf, rules=rules)
    eng.synchronize()
    dt = time.perf_counter() - t0
    res = buf.download(np.uint64, steps * W).reshape(steps, W)
    buf.free()
    if not (res[:, 257] == want).all():
        raise SystemExit(f"parity failure: {res[:, 257].tolist()} != {want}")
    return 1e3 * dt / steps
out = {}
legs = os.environ.get("LEGS", "ref7,fide7,suite").split(",")
if "ref7" in legs:
    out["ref7_ms"] = timed(dchess.startpos(), 7, 20, dchess.RULES_REF, REF7)
if "fide7" in legs:
    out["fide7_ms"] = timed(dchess.pos_from_fen(og["startpos"]["fen"]), 7, 4, dchess.RULES_FIDE, og["startpos"]["perft"]["7"])
if "suite" in legs:
    out["suite_d5_ms"] = sum(timed(dchess.pos_from_fen(og[k]["fen"]), 5, 4, dchess.RULES_FIDE, og[k]["perft"]["5"])
                             for k in ("startpos", "kiwipete", "pos3", "pos4", "pos5", "pos6"))
print(json.dumps(out))
'''


def main():
    rounds = int(sys.argv[1])
    libs = sys.argv[2:]
    res = {lib: [] for lib in libs}
    for r in range(rounds):
        for lib in libs:
            env = dict(os.environ, DCHESS_LIB=os.path.abspath(lib))
            p = subprocess.run([sys.executable, "-c", CHILD, REPO], env=env, capture_output=True, text=True,
                               timeout=300)
            if p.returncode:
                print(json.dumps({"lib": lib, "round": r, "error": p.stderr[-800:]}))
                sys.exit(1)
            rec = json.loads(p.stdout.strip().splitlines()[-1])
            res[lib].append(rec)
            print(json.dumps({"lib": lib, "round": r, **rec}), flush=True)
    summary = {lib: {k: statistics.median(x[k] for x in v) for k in v[0]} for lib, v in res.items()}
    print(json.dumps({"median": summary}))


if __name__ == "__main__":
    main()
