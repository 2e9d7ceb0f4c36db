"""Per-child recount of the FIDE final stage -- diagnostics for DESIGN.md §3.6.

A library built with -DDC_DIAG_CHILD (tools/ab_build.sh) writes one 64-byte
record for every child `k_count2b` counts: the child board and meta, the count
k (and, with DC_DIAG_CHILD=2, a second count k2 of the same child by the same
code), the slot word, the parent index, HW_ID and XCC_ID.  This script runs
FIDE perft(5) of suite positions with such a library (DCHESS_LIB=...), recounts
every recorded child with fastcpu (oracle/, the checker) and prints one JSON
line per position: how many children are wrong, by how much, and where (XCC,
SE, CU, SIMD, wave, lane) they ran.

  DCHESS_LIB=$PWD/distributed-chess_amd/build/var/NAME/libdchess.so \
      python tools/fide_child_diag.py [--save-map DIR | --kmap DIR] [kiwipete pos5 ...]

--save-map DIR keeps each position's records and their positions (a full-record
build); --kmap DIR reads a -DDC_DIAG_CHILD=3 build's counts (one dword per
child, nothing else stored) at those positions and compares them with the
map's verified counts -- the layout depends only on (block, chunk, slot), so
the two builds' records line up.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time
from collections import Counter

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-chess_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import dchess  # noqa: E402
import oracle_lib as ol  # noqa: E402

KIND = ".PNKXBRQ"


def board_str(bb):
    """64-char board, a1 first; upper case white, lower case black."""
    out = []
    for s in range(64):
        code = ((int(bb[1]) >> s) & 1) | (((int(bb[2]) >> s) & 1) << 1) | (((int(bb[3]) >> s) & 1) << 2)
        c = KIND[code]
        out.append(c.lower() if code and (int(bb[0]) >> s) & 1 else c)
    return "/".join("".join(out[8 * r:8 * r + 8]) for r in range(7, -1, -1))


def hw(hwid):
    return {"wave": hwid & 15, "simd": (hwid >> 4) & 3, "cu": (hwid >> 8) & 15, "sh": (hwid >> 12) & 1,
            "se": (hwid >> 13) & 7, "tg": (hwid >> 16) & 15}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("names", nargs="*", default=["kiwipete", "pos5", "pos6", "pos4"])
    ap.add_argument("--save-map")
    ap.add_argument("--kmap")
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--noise", type=int, default=-1, help="co-resident noise kind (tools/diag/noise.hip)")
    ap.add_argument("--noise-blocks", type=int, default=512)
    args = ap.parse_args()
    noise = None
    if args.noise >= 0:
        noise = C.CDLL(os.path.join(REPO, "tools", "diag", "libnoise.so"))
        noise.noise_start.argtypes = [C.c_int, C.c_int, C.c_double]
    names = args.names
    og = json.load(open(os.path.join(REPO, "tests", "golden", "oracle_golden.json")))["perft_fide"]
    eng = dchess.Engine(0)
    L = dchess.lib()
    if not hasattr(L, "dc_diag_child_set"):
        raise SystemExit("DCHESS_LIB is not a -DDC_DIAG_CHILD build")
    L.dc_diag_child_set.argtypes = [C.c_void_p, C.c_uint64]
    L.dc_diag_child_set.restype = C.c_int
    cap = 24 << 20
    buf = torch.empty((cap, 16), dtype=torch.int32, device="cuda")
    for name in names:
        buf.fill_(-1)
        torch.cuda.synchronize()
        assert L.dc_diag_child_set(buf.data_ptr(), cap) == 0
        if noise is not None:
            eng.perft(dchess.pos_from_fen(og[name]["fen"]), args.depth, rules=dchess.RULES_FIDE)  # capture first
            buf.fill_(-1)
            torch.cuda.synchronize()
            assert noise.noise_start(args.noise, args.noise_blocks, 1500.0) == 0
            time.sleep(0.05)
        tot = eng.perft(dchess.pos_from_fen(og[name]["fen"]), args.depth, rules=dchess.RULES_FIDE)[0]
        torch.cuda.synchronize()
        if noise is not None:
            assert noise.noise_wait() == 0
        assert L.dc_diag_child_set(None, 0) == 0
        pub = og[name]["perft"][str(args.depth)]
        if args.kmap:
            m = np.load(os.path.join(args.kmap, f"{name}_d{args.depth}.npz"))
            flat = buf.view(-1)
            kv = flat[torch.from_numpy(m["idx"]).cuda()].cpu().numpy().view(np.uint32)
            stray = int((flat != -1).sum().item()) - len(kv)
            want = m["rows"][:, 9]
            bad = kv != want
            res = {"pos": name, "mode": "kmap", "lib": os.environ.get("DCHESS_LIB", "product"), "total": tot,
                   "published": pub, "diff_total": tot - pub, "records": int(len(kv)), "stray_writes": stray,
                   "unwritten": int((kv == 0xFFFFFFFF).sum()), "wrong": int(bad.sum())}
            if bad.any():
                rws = m["rows"][bad]
                d = kv[bad].astype(np.int64) - want[bad].astype(np.int64)
                res["delta_hist"] = Counter(d.tolist()).most_common(12)
                misc = rws[:, 15]
                res["by_lane_row"] = dict(Counter((((misc >> 8) & 0xFF) // 16).tolist()))
                res["by_block_wave"] = dict(Counter(((misc >> 16) & 0xFF).tolist()))
                res["by_active_lanes"] = dict(Counter(((misc & 0xFF) // 16).tolist()))
                res["wrong_parents"] = int(len(set(rws[:, 12].tolist())))
                ex = []
                for i in range(min(16, len(rws))):
                    r = rws[i]
                    bb = r[0:8].copy().view(np.uint64)
                    ex.append({"board": board_str(bb), "meta": int(r[8]), "expected": int(r[9]), "got": int(kv[bad][i]),
                               "from": int(r[11] & 63), "to": int((r[11] >> 6) & 63), "pl": int((r[11] >> 15) & 255),
                               "pidx": int(r[12]), "lane": int((r[15] >> 8) & 0xFF), "bwave": int((r[15] >> 16) & 0xFF),
                               "at": int(m["idx"][bad][i])})
                res["examples"] = ex
                os.makedirs(os.path.join(REPO, "gpurun_out", "r5"), exist_ok=True)
                np.savez(os.path.join(REPO, "gpurun_out", "r5", f"kmap_bad_{name}_d{args.depth}.npz"),
                         rows=rws, got=kv[bad], at=m["idx"][bad])
            print(json.dumps(res), flush=True)
            continue
        sel = (buf[:, 9] != -1).nonzero().squeeze(1)
        rows = buf[sel].cpu().numpy().view(np.uint32)
        n = len(rows)
        bb = rows[:, 0:8].copy().view(np.uint64).reshape(n, 4)
        cm, k, k2, e = rows[:, 8], rows[:, 9], rows[:, 10], rows[:, 11]
        pidx, hwid, xcc, misc = rows[:, 12], rows[:, 13], rows[:, 14], rows[:, 15]
        stm = (1 - (e >> 31)).astype(np.uint8)
        exp = ol.fast_count_quad(bb, stm, (cm & 0xFFFF).astype(np.uint16), ol.FIDE, threads=16)
        bad = k != exp
        bad2 = k2 != exp
        diff12 = k != k2
        if args.save_map:
            os.makedirs(args.save_map, exist_ok=True)
            np.savez(os.path.join(args.save_map, f"{name}_d{args.depth}.npz"), idx=sel.cpu().numpy(), rows=rows)
        res = {"pos": name, "lib": os.environ.get("DCHESS_LIB", "product"), "total": tot, "published": pub,
               "diff_total": tot - pub, "records": int(n), "sum_k": int(k.astype(np.int64).sum()),
               "sum_exp": int(exp.astype(np.int64).sum()), "wrong": int(bad.sum()), "wrong_k2": int(bad2.sum()),
               "k_ne_k2": int(diff12.sum())}
        if bad.any() or bad2.any():
            d = k.astype(np.int64) - exp.astype(np.int64)
            res["delta_hist"] = Counter(d[bad].tolist()).most_common(12)
            hwd = np.array([[hw(int(h))[f] for f in ("wave", "simd", "cu", "se")] for h in hwid])

            def by(col, vals):
                tot_c = Counter(vals.tolist())
                bad_c = Counter(vals[bad].tolist())
                return {str(v): [bad_c.get(v, 0), tot_c[v]] for v in sorted(tot_c)}
            res["by_xcc"] = by("xcc", xcc)
            res["by_se"] = by("se", hwd[:, 3])
            res["by_simd"] = by("simd", hwd[:, 1])
            res["by_wave_slot"] = by("wave", hwd[:, 0])
            res["by_block_wave"] = by("bw", (misc >> 16) & 0xFF)
            res["by_lane_row"] = by("row", ((misc >> 8) & 0xFF) // 16)
            res["by_active_lanes"] = by("act", (misc & 0xFF) // 16)
            res["by_window"] = by("win", (misc >> 24) & 1)
            # how many wrong children per parent, and per wave execution (same hwid+pidx//64 burst)
            res["wrong_parents"] = int(len(set(pidx[bad].tolist())))
            ex = []
            for i in np.nonzero(bad | bad2)[0][:16]:
                ex.append({"board": board_str(bb[i]), "stm": int(stm[i]), "meta": int(cm[i]), "expected": int(exp[i]),
                           "k": int(k[i]), "k2": int(k2[i]), "from": int(e[i] & 63), "to": int((e[i] >> 6) & 63),
                           "promo": int((e[i] >> 12) & 7), "pl": int((e[i] >> 15) & 255), "pidx": int(pidx[i]),
                           "xcc": int(xcc[i]), "hw": hw(int(hwid[i])), "active": int(misc[i] & 0xFF),
                           "lane": int((misc[i] >> 8) & 0xFF), "bwave": int((misc[i] >> 16) & 0xFF)})
            res["examples"] = ex
            os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
            tag = os.path.basename(os.path.dirname(os.environ.get("DCHESS_LIB", "x/product/y")))
            np.save(os.path.join(REPO, "gpurun_out", f"diag_{tag}_{name}_bad.npy"), rows[bad | bad2])
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
