"""dc_history_append (host) against refcpu's update_history (chess.rs:127-184):
random REF games played through or_ref_apply, the info bytes taken from the
cells before each move (as dc_apply_batch / dc_replay_info report them)."""
import numpy as np

import dchess
import oracle_lib as O


def play(seed, plies, start_hist):
    rng = np.random.default_rng(seed)
    cells, turn, hist = O.startpos_cells().copy(), 0, start_hist
    moves, info = [], []
    for _ in range(plies):
        ok = np.nonzero(O.ref_verdicts_all(cells, turn) == 0)[0]
        if len(ok) == 0:
            break
        # mostly legal moves, some rejected ones (they leave no history entry)
        e = int(rng.choice(ok)) if rng.random() < 0.85 else int(rng.integers(4096))
        f, t = e & 63, e >> 6
        code = int(cells[f] & 7) | (8 if cells[t] >= 0 else 0) if cells[f] >= 0 else 0
        v, cells, turn, hist = O.ref_apply(cells, turn, hist, f >> 3, f & 7, t >> 3, t & 7)
        moves.append(f | t << 6)
        info.append(code if v == 0 else 0xFF)
    return np.array(moves, np.uint16), np.array(info, np.uint8), hist


def test_history_append_matches_refcpu():
    for seed in range(12):
        for start in ("", "1. e4", "x　y\tz  "):  # split_whitespace counts Unicode White_Space
            mv, inf, hist = play(seed, 60, start)
            assert dchess.history_append(start, mv, inf) == hist, (seed, start)


def test_history_append_numbering_quirk_and_sizes():
    # "1. e4 3. d5 5. exd5": the move number is 1 + the tokens already present
    mv = np.array([12 | 28 << 6, 51 | 35 << 6, 0xFFFF, 28 | 35 << 6], np.uint16)
    inf = np.array([0, 0, 0xFF, 8], np.uint8)
    assert dchess.history_append("", mv, inf) == "1. e4 3. d5 5. exd5"
    assert dchess.history_append(None, mv[:0], inf[:0]) == ""
    import ctypes as C
    n = C.c_size_t()
    L = dchess.lib()
    # too small a buffer: DC_EINVAL with the needed length reported
    buf = C.create_string_buffer(4)
    r = L.dc_history_append(b"", mv.ctypes.data, inf.ctypes.data, 4, 1, buf, 4, C.byref(n))
    assert r == dchess.EINVAL and n.value == len("1. e4 3. d5 5. exd5")
    # an OTHER-kind piece never moves (chess.rs:210): its info code is refused
    bad = np.array([6], np.uint8)
    assert L.dc_history_append(b"", mv.ctypes.data, bad.ctypes.data, 1, 1, None, 0, C.byref(n)) == dchess.EUNSUPPORTED
