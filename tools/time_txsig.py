#!/usr/bin/env python3
"""Times dc_verify_tx_batch_device on a resident batch: TXS transactions (the
1024 distinct signed transactions of tests/golden/txsig_batch.json tiled),
checked against the fixture's expected verdicts.  Prints one JSON line."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-chess_amd"))
import numpy as np  # noqa: E402

import dchess  # noqa: E402


def load_batch(n):
    fx = json.load(open(os.path.join(REPO, "tests", "golden", "txsig_batch.json")))
    txs = fx["txs"]
    reps = (n + len(txs) - 1) // len(txs)
    quads = [(t["white"], t["black"], t["sig"], t["pk"]) for t in txs] * reps
    acts = np.array([t["action"] for t in txs] * reps, np.uint32)[:n]
    turns = np.array([t["turn"] for t in txs] * reps, np.int8)[:n]
    want = np.array([t["verdict"] for t in txs] * reps, np.uint8)[:n]
    return dchess.pack_txs(quads[:n], acts, turns), want


def main():
    n = int(os.environ.get("TXS", "262144"))
    steps = int(os.environ.get("STEPS", "5"))
    (blob, off, acts, turns), want = load_batch(n)
    eng = dchess.Engine(0)
    bufs = []
    for arr in (np.frombuffer(blob, np.uint8), off, acts, turns):
        b = eng.alloc(max(arr.nbytes, 1))
        b.upload(arr)
        bufs.append(b)
    d_v = eng.alloc(n)
    eng.verify_txs_device(*bufs, n, d_v)  # warmup (+ G table)
    got = d_v.download(np.uint8, n)
    assert (got == want).all(), f"parity: {int((got != want).sum())} mismatches"
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.verify_txs_device(*bufs, n, d_v)
    dt = time.perf_counter() - t0
    eng.reset_stats()
    eng.set_profiling(True)
    eng.verify_txs_device(*bufs, n, d_v)
    eng.set_profiling(False)
    k = eng.kernel_stats("verify_tx")
    print(json.dumps({"txs": n, "verifies_per_s": n * steps / dt, "kernel_ms": k["total_ms"],
                      "kernel_verifies_per_s": n / (k["total_ms"] / 1e3)}), flush=True)


if __name__ == "__main__":
    main()
