"""Full-size replay goldens (BASELINE configs[3] = C4 and configs[4] = C5) -- TEST INFRASTRUCTURE.

Run:  python tests/golden/make_replay_golden.py [--games 100000000] [--threads 8]
      (~25 min for 100M games on 8 cores; the C4 10M-game block comes first)

The workload is SURVEY §8d C4/C5: seed 0x5EED20241022, game ids 0..N, 80 ply
slots, noise 32/256 (dc_gen_games).  Replay semantics are commit_block's
(/root/reference/core/src/consensus/hotstuff.rs:52-56): validate each ply,
apply only accepted moves.

Engines:
  * fastcpu (oracle/fastcpu.cpp, the mailbox engine) generates and replays
    every game, in 10M-game blocks;
  * refcpu (oracle/refcpu.cpp, the literal restatement of
    /root/reference/core/src/chess.rs) replays two 100k-game samples of C4 --
    the first 100,032 games (whole bitmap words) and 100,000 games strided
    across all 10M -- and must agree with fastcpu verdict for verdict and
    digest for digest.

Written to tests/golden/replay_golden.json:
  c4: the first 10M games as one batch: SHA-256 of the ply-major moves
      [80][10M] u16, of the ply-major accept bitmap [80][156250] u64 and of the
      per-game final-state digests [10M] u64, plus the 5 replay stats;
  c5: all N games as one batch (bitmap [80][ceil(N/64)] u64 assembled from the
      blocks, digests streamed), plus each block's own record.
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as O  # noqa: E402

SEED = 0x5EED20241022
PLIES = 80
NOISE = 32
BLOCK = 10_000_000  # a multiple of 64: block bitmaps are whole word columns of the global one


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def stats_dict(st):
    return {"validated": int(st[0]), "accepted": int(st[1]), "rejected": int(st[2]),
            "digest_sum": int(st[3]), "digest_xor": int(st[4])}


def refcpu_samples(mv, bm, dg, threads):
    """refcpu over two 100k-game samples of the block; asserts agreement."""
    out = []
    n = mv.shape[1]
    k = 1563 * 64  # first 100,032 games = 1563 whole bitmap words
    t0 = time.time()
    rbm, rdg, rst = O.ref_replay(mv[:, :k], threads=threads)
    assert (rbm == bm[:, :1563]).all(), "refcpu/fastcpu bitmap mismatch (prefix sample)"
    assert (rdg == dg[:k]).all(), "refcpu/fastcpu digest mismatch (prefix sample)"
    out.append({"kind": "prefix", "games": k, "agree": True, "stats": stats_dict(rst),
                "seconds": round(time.time() - t0, 1)})
    stride = n // 100_000
    idx = np.arange(100_000, dtype=np.int64) * stride + min(7, stride - 1)
    t0 = time.time()
    rbm, rdg, rst = O.ref_replay(np.ascontiguousarray(mv[:, idx]), threads=threads)
    bits = (bm[:, idx >> 6] >> (idx & 63).astype(np.uint64)) & np.uint64(1)  # [plies][100k]
    rbits = (rbm[:, np.arange(100_000) >> 6] >> (np.arange(100_000) & 63).astype(np.uint64)) & np.uint64(1)
    assert (bits == rbits).all(), "refcpu/fastcpu bitmap mismatch (strided sample)"
    assert (rdg == dg[idx]).all(), "refcpu/fastcpu digest mismatch (strided sample)"
    out.append({"kind": "strided", "games": 100_000, "first": int(idx[0]), "stride": int(stride), "agree": True,
                "stats": stats_dict(rst), "seconds": round(time.time() - t0, 1)})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=100_000_000)
    ap.add_argument("--threads", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--out", default=os.path.join(HERE, "replay_golden.json"))
    args = ap.parse_args()
    N = args.games
    assert N % BLOCK == 0 or N < BLOCK
    words = (N + 63) // 64
    gbm = np.zeros((PLIES, words), np.uint64)  # global ply-major bitmap (1 GB at 100M)
    dsha = hashlib.sha256()
    tot = np.zeros(5, np.uint64)
    blocks = []
    golden = {"seed": SEED, "n_plies": PLIES, "noise_per_256": NOISE, "engine": "fastcpu (all games); refcpu samples"}
    for first in range(0, N, BLOCK):
        n = min(BLOCK, N - first)
        t0 = time.time()
        mv = O.fast_gen_games(SEED, first, n, PLIES, NOISE, threads=args.threads)
        t1 = time.time()
        bm, dg, st = O.fast_replay(mv, threads=args.threads)
        t2 = time.time()
        rec = {"first_game": first, "n_games": n, "moves_sha256": sha(mv), "bitmap_sha256": sha(bm),
               "digests_sha256": sha(dg), "stats": stats_dict(st),
               "seconds": {"gen": round(t1 - t0, 1), "replay": round(t2 - t1, 1)}}
        if first == 0:
            c4 = dict(rec)
            c4["refcpu_samples"] = refcpu_samples(mv, bm, dg, args.threads)
            golden["c4"] = c4
        blocks.append(rec)
        gbm[:, first // 64:first // 64 + bm.shape[1]] = bm
        dsha.update(np.ascontiguousarray(dg).tobytes())
        tot[0:4] += st[0:4]  # u64 sums wrap mod 2^64 like the kernels'
        tot[4] ^= st[4]
        print(f"block {first}: {rec['stats']} gen {t1 - t0:.1f}s replay {t2 - t1:.1f}s", flush=True)
        del mv, bm, dg
        golden["c5"] = {"first_game": 0, "n_games": first + n, "bitmap_sha256": sha(gbm[:, :(first + n + 63) // 64])
                        if first + n == N else None, "digests_sha256": dsha.hexdigest(),
                        "stats": stats_dict(tot), "blocks": blocks}
        with open(args.out, "w") as f:  # partial results survive an interrupted run
            json.dump(golden, f, indent=1, sort_keys=True)
    print("wrote", args.out)


if __name__ == "__main__":
    main()
