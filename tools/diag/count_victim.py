"""Runs the minimal count victim (tools/diag/count_victim.hip) over recorded
final-stage children (a map from tools/fide_child_diag.py --save-map) beside
co-resident noise waves; prints one JSON line per (library, TAB, noise kind):
how many boards were counted wrong.
  python tools/diag/count_victim.py --map DIR --libs r4tab [--kinds=-1,12] [names...]"""
import argparse
import ctypes as C
import json
import os
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ap = argparse.ArgumentParser()
ap.add_argument("names", nargs="*", default=["kiwipete", "pos6"])
ap.add_argument("--map", required=True)
ap.add_argument("--libs", default="r4tab")
ap.add_argument("--kinds", default="-1,12")
ap.add_argument("--blocks", default="96,768")
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--max", type=int, default=1 << 20)
args = ap.parse_args()
N = C.CDLL(os.path.join(REPO, "tools", "diag", "libnoise.so"))
N.noise_start.argtypes = [C.c_int, C.c_int, C.c_double]
for name in args.names:
    m = np.load(os.path.join(args.map, f"{name}_d5.npz"))
    rows = m["rows"][: args.max]
    n = len(rows)
    boards = torch.from_numpy(np.ascontiguousarray(rows[:, 0:8]).view(np.int32)).cuda()
    meta = torch.from_numpy(np.ascontiguousarray(rows[:, 8]).view(np.int32)).cuda()
    want = rows[:, 9].astype(np.int64) * args.reps
    stm = 1 - int(rows[0, 11] >> 31)
    assert ((1 - (rows[:, 11] >> 31)) == stm).all()
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    for lib in args.libs.split(","):
        V = C.CDLL(os.path.join(REPO, "tools", "diag", f"libcountvictim_{lib}.so"))
        V.cv_run.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_int]
        for blocks in [int(b) for b in args.blocks.split(",")]:
            for tab in (1, 0):
                for kind in [int(k) for k in args.kinds.split(",")]:
                    out.zero_()
                    torch.cuda.synchronize()
                    if kind >= 0:
                        assert N.noise_start(kind, 512, 4000.0) == 0
                        time.sleep(0.05)
                    t0 = time.time()
                    r = V.cv_run(stm, tab, boards.data_ptr(), meta.data_ptr(), n, out.data_ptr(), args.reps, blocks)
                    dt = time.time() - t0
                    if kind >= 0:
                        N.noise_wait()
                    got = out.cpu().numpy().astype(np.int64)
                    bad = got != want
                    print(json.dumps({"pos": name, "lib": lib, "tab": tab, "blocks": blocks, "noise": kind, "rc": r,
                                      "boards": n, "wrong": int(bad.sum()), "lost": int((want - got)[bad].sum()),
                                      "victim_s": round(dt, 3)}), flush=True)
