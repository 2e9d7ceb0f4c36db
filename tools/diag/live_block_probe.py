"""Which call blocks behind a resident live wave: times each step
of buffer growth / context churn with two contexts' waves resident."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "distributed-chess_amd"))
import dchess  # noqa: E402

out = {}


def step(name, f):
    t0 = time.time()
    r = f()
    out[name] = round(time.time() - t0, 4)
    return r


p = np.array([dchess.startpos()], dchess.POS_DTYPE)
mv = np.array([8 | (24 << 6)], np.uint16)
a = step("ctx_a", lambda: dchess.Engine(0))
b = step("ctx_b", lambda: dchess.Engine(0))
step("live_a_on", lambda: a.live_validator(8_000_000))
step("live_b_on", lambda: b.live_validator(8_000_000))
step("validate_a", lambda: a.validate_batch(p, mv))
step("validate_b", lambda: b.validate_batch(p, mv))
step("perft_a_d1", lambda: a.perft(dchess.startpos(), 1))
step("perft_a_d3", lambda: a.perft(dchess.startpos(), 3))
step("perft_a_d5", lambda: a.perft(dchess.startpos(), 5))
step("validate_a2", lambda: a.validate_batch(p, mv))
step("perft_b_d5", lambda: b.perft(dchess.startpos(), 5))
c = step("ctx_c", lambda: dchess.Engine(0))
step("perft_c_d3", lambda: c.perft(dchess.startpos(), 3))
step("close_c", lambda: c.close())
step("validate_b2", lambda: b.validate_batch(p, mv))
step("live_off", lambda: (a.live_validator(0), b.live_validator(0)))
print(json.dumps(out))
