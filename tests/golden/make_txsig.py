#!/usr/bin/env python3
"""Generates tests/golden/txsig_batch.json: 512 transactions signed the way the
client signs them (chess/src/app/play/page.tsx:37-44, :106-125) with keys
from a seeded RNG, about 1 in 6 corrupted (message, signature or key), each
with the verdict of oracle/txsig.py (App::validate_signature,
core/src/consensus/hotstuff.rs:168-208, plus the owner check :141-148).
Used by tools/time_txsig.py and bench.py's signature leg (inputs + expected
verdicts; the oracle is not imported at run time there)."""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import txsig as T  # noqa: E402


def main(n=512, seed=0x7A5161):
    rng = random.Random(seed)
    keys = [rng.randrange(1, T.N) for _ in range(32)]
    pubs = [T.pubkey_hex(d) for d in keys]
    txs = []
    for i in range(n):
        wi, bi = rng.randrange(32), rng.randrange(32)
        turn = rng.randrange(2)
        act = [rng.randrange(8) for _ in range(4)]
        w, b = pubs[wi], pubs[bi]
        d = keys[wi] if turn == 0 else keys[bi]
        r, s = T.sign(d, T.message_hash(w, b, tuple(act)))
        sig, pk = T.sig_hex(r, s), (w if turn == 0 else b)
        kind = rng.randrange(12)
        if kind == 0:
            act[0] ^= 1  # message changed after signing
        elif kind == 1:
            j = rng.randrange(128)
            sig = sig[:j] + ("1" if sig[j] == "0" else "0") + sig[j + 1:]
        elif kind == 2:
            pk = pubs[(wi + 1) % 32]
        v = T.check_tx(w, b, tuple(act), sig, pk)
        if v == T.SIG_OK and pk != (w if turn == 0 else b):
            v = 6
        txs.append({"white": w, "black": b, "action": act, "sig": sig, "pk": pk, "turn": turn, "verdict": v})
    out = {"generator": "tests/golden/make_txsig.py", "seed": seed, "txs": txs}
    json.dump(out, open(os.path.join(HERE, "txsig_batch.json"), "w"), separators=(",", ":"))
    print({v: sum(t["verdict"] == v for t in txs) for v in range(7)})


if __name__ == "__main__":
    main()
