"""ctypes wrapper over oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The oracle (refcpu = literal restatement of /root/reference/core/src/chess.rs,
fastcpu = independent mailbox engine) is the checker for the HIP product.  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
"""
import ctypes as C
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
_LIB = None

REF, FIDE = 0, 1
OK, NO_PIECE, WRONG_TURN, ILLEGAL, OOR = 0, 1, 2, 3, 4
SENTINEL = 0xFFFF

_u8p = C.POINTER(C.c_uint8)
_i8p = C.POINTER(C.c_int8)
_u16p = C.POINTER(C.c_uint16)
_u32p = C.POINTER(C.c_uint32)
_u64p = C.POINTER(C.c_uint64)


def build():
    subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(ORACLE_DIR, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.or_startpos_cells.argtypes = [_i8p]
        L.or_ref_validate.argtypes = [_i8p, C.c_int32] + [C.c_uint32] * 4
        L.or_ref_message.restype = C.c_char_p
        L.or_ref_message.argtypes = [C.c_int]
        L.or_ref_apply.argtypes = [_i8p, C.POINTER(C.c_int32), C.c_char_p, C.c_size_t] + [C.c_uint32] * 4
        L.or_ref_verdicts_all.argtypes = [_i8p, C.c_int32, _u8p]
        L.or_ref_perft.restype = C.c_uint64
        L.or_ref_perft.argtypes = [_i8p, C.c_int32, C.c_uint, C.c_uint, _u64p]
        L.or_ref_replay.argtypes = [_u16p, C.c_uint32, C.c_uint32, C.c_uint, _u64p, _u64p, _u64p]
        L.or_fast_from_fen.argtypes = [C.c_char_p, _i8p, _u8p, _u8p, _i8p]
        L.or_fast_verdicts_all.argtypes = [_i8p, C.c_uint8, C.c_uint8, C.c_int8, C.c_int, _u8p]
        L.or_fast_validate.argtypes = [_i8p, C.c_uint8, C.c_uint8, C.c_int8, C.c_int, C.c_uint16]
        L.or_fast_gen_moves.argtypes = [_i8p, C.c_uint8, C.c_uint8, C.c_int8, C.c_int, _u16p]
        L.or_fast_make.argtypes = [_i8p, _u8p, _u8p, _i8p, C.c_int, C.c_uint16]
        L.or_fast_perft.restype = C.c_uint64
        L.or_fast_perft.argtypes = [_i8p, C.c_uint8, C.c_uint8, C.c_int8, C.c_int, C.c_uint, C.c_uint,
                                    _u64p, _u16p, _u32p]
        L.or_fast_gen_games.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int,
                                        _u16p, C.c_uint]
        L.or_fast_replay.argtypes = [_u16p, C.c_uint32, C.c_uint32, C.c_int, C.c_uint, _u64p, _u64p, _u64p]
        L.or_fast_quad.argtypes = [_i8p, _u64p]
        L.or_fast_digest.restype = C.c_uint64
        L.or_fast_digest.argtypes = [_i8p, C.c_uint8]
        L.or_fast_count_quad.argtypes = [_u64p, _u8p, _u16p, C.c_uint32, C.c_int, C.c_uint, _u32p]
        _LIB = L
    return _LIB


def _p(a, t):
    return a.ctypes.data_as(t)


class Pos:
    """Oracle-side position: cells[64] (-1 empty, color*8+kind), stm, castle, ep."""

    def __init__(self, cells=None, stm=0, castle=0, ep=-1):
        if cells is None:
            cells = startpos_cells()
            castle = 15
        self.cells = np.ascontiguousarray(cells, dtype=np.int8)
        self.stm, self.castle, self.ep = int(stm), int(castle), int(ep)

    @staticmethod
    def from_fen(fen):
        cells = np.zeros(64, np.int8)
        stm, castle, ep = C.c_uint8(), C.c_uint8(), C.c_int8()
        rc = lib().or_fast_from_fen(fen.encode(), _p(cells, _i8p), C.byref(stm), C.byref(castle), C.byref(ep))
        if rc != 0:
            raise ValueError(fen)
        return Pos(cells, stm.value, castle.value, ep.value)

    def copy(self):
        return Pos(self.cells.copy(), self.stm, self.castle, self.ep)


def startpos_cells():
    cells = np.zeros(64, np.int8)
    lib().or_startpos_cells(_p(cells, _i8p))
    return cells


def ref_validate(cells, turn, fx, fy, tx, ty):
    cells = np.ascontiguousarray(cells, dtype=np.int8)
    return lib().or_ref_validate(_p(cells, _i8p), turn, fx, fy, tx, ty)


def ref_message(v):
    return lib().or_ref_message(v).decode()


def ref_apply(cells, turn, history, fx, fy, tx, ty):
    """Returns (verdict, cells', turn', history')."""
    cells = np.ascontiguousarray(cells, dtype=np.int8).copy()
    t = C.c_int32(turn)
    buf = C.create_string_buffer(history.encode(), 4096)
    v = lib().or_ref_apply(_p(cells, _i8p), C.byref(t), buf, 4096, fx, fy, tx, ty)
    return v, cells, t.value, buf.value.decode()


def ref_verdicts_all(cells, turn):
    out = np.zeros(4096, np.uint8)
    cells = np.ascontiguousarray(cells, dtype=np.int8)
    lib().or_ref_verdicts_all(_p(cells, _i8p), turn, _p(out, _u8p))
    return out


def ref_perft(cells, turn, depth, threads=1):
    cells = np.ascontiguousarray(cells, dtype=np.int8)
    div = np.zeros(4096, np.uint64)
    tot = lib().or_ref_perft(_p(cells, _i8p), turn, depth, threads, _p(div, _u64p))
    return int(tot), div


def ref_replay(moves, threads=1):
    moves = np.ascontiguousarray(moves, dtype=np.uint16)
    n_plies, n_games = moves.shape
    words = (n_games + 63) // 64
    bitmap = np.zeros((n_plies, words), np.uint64)
    dig = np.zeros(n_games, np.uint64)
    st = np.zeros(5, np.uint64)
    lib().or_ref_replay(_p(moves, _u16p), n_games, n_plies, threads, _p(bitmap, _u64p), _p(dig, _u64p),
                        _p(st, _u64p))
    return bitmap, dig, st


def fast_verdicts_all(pos, rules=REF):
    out = np.zeros(4096, np.uint8)
    lib().or_fast_verdicts_all(_p(pos.cells, _i8p), pos.stm, pos.castle, pos.ep, rules, _p(out, _u8p))
    return out


def fast_validate(pos, move, rules=REF):
    return lib().or_fast_validate(_p(pos.cells, _i8p), pos.stm, pos.castle, pos.ep, rules, move)


def fast_gen_moves(pos, rules=REF):
    out = np.zeros(256, np.uint16)
    n = lib().or_fast_gen_moves(_p(pos.cells, _i8p), pos.stm, pos.castle, pos.ep, rules, _p(out, _u16p))
    return out[:n].copy()


def fast_make(pos, move, rules=REF):
    q = pos.copy()
    stm, castle, ep = C.c_uint8(q.stm), C.c_uint8(q.castle), C.c_int8(q.ep)
    lib().or_fast_make(_p(q.cells, _i8p), C.byref(stm), C.byref(castle), C.byref(ep), rules, move)
    q.stm, q.castle, q.ep = stm.value, castle.value, ep.value
    return q


def fast_perft(pos, depth, rules=REF, threads=None):
    threads = threads or min(8, os.cpu_count() or 1)
    div = np.zeros(256, np.uint64)
    rm = np.zeros(256, np.uint16)
    n = C.c_uint32()
    tot = lib().or_fast_perft(_p(pos.cells, _i8p), pos.stm, pos.castle, pos.ep, rules, depth, threads,
                              _p(div, _u64p), _p(rm, _u16p), C.byref(n))
    return int(tot), div[:n.value].copy(), rm[:n.value].copy()


def fast_gen_games(seed, first_game, n_games, n_plies, noise_per_256=32, rules=REF, threads=None):
    threads = threads or min(8, os.cpu_count() or 1)
    out = np.zeros((n_plies, n_games), np.uint16)
    lib().or_fast_gen_games(seed, first_game, n_games, n_plies, noise_per_256, rules, _p(out, _u16p), threads)
    return out


def fast_replay(moves, rules=REF, threads=None):
    threads = threads or min(8, os.cpu_count() or 1)
    moves = np.ascontiguousarray(moves, dtype=np.uint16)
    n_plies, n_games = moves.shape
    words = (n_games + 63) // 64
    bitmap = np.zeros((n_plies, words), np.uint64)
    dig = np.zeros(n_games, np.uint64)
    st = np.zeros(5, np.uint64)
    lib().or_fast_replay(_p(moves, _u16p), n_games, n_plies, rules, threads, _p(bitmap, _u64p), _p(dig, _u64p),
                         _p(st, _u64p))
    return bitmap, dig, st


def quad(cells):
    bb = np.zeros(4, np.uint64)
    cells = np.ascontiguousarray(cells, dtype=np.int8)
    lib().or_fast_quad(_p(cells, _i8p), _p(bb, _u64p))
    return bb


def digest(cells, stm):
    cells = np.ascontiguousarray(cells, dtype=np.int8)
    return int(lib().or_fast_digest(_p(cells, _i8p), stm))


def fast_count_quad(bb, stm, meta, rules=FIDE, threads=None):
    """Legal-move counts of quad-bitboard positions: bb (n, 4) u64, stm (n,) u8, meta (n,) u16."""
    bb = np.ascontiguousarray(bb, dtype=np.uint64)
    stm = np.ascontiguousarray(stm, dtype=np.uint8)
    meta = np.ascontiguousarray(meta, dtype=np.uint16)
    n = len(stm)
    out = np.zeros(n, dtype=np.uint32)
    lib().or_fast_count_quad(_p(bb, _u64p), _p(stm, _u8p), _p(meta, _u16p), n, rules,
                             threads or os.cpu_count() or 1, _p(out, _u32p))
    return out
