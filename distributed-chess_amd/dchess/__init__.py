"""dchess -- Python binding of libdchess.so (include/dchess.h) via ctypes.

This is plumbing for tests and bench.py: every call goes through the C ABI to
the gfx950 kernels.  There is no CPU fallback: if the shared library is missing
or no gfx950 device is present, the calls raise.

It also mirrors the reference's Rust call surface (core/src/chess.rs) in
`GameState` / `Position` / `AppError`, so parity tests read like the
reference's own unit tests (core/src/chess.rs:499-557).
"""
import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# DCHESS_LIB selects another build of the same ABI -- only tools/ab_*.sh use it,
# for libdchess_ab.so (the A/B-knob build, `make ab`).
LIB_PATH = os.environ.get("DCHESS_LIB") or os.path.join(os.path.dirname(PKG_DIR), "libdchess.so")

SUCCESS, EINVAL, EHIP, ENOMEM, ENODEV, ERCCL, EUNSUPPORTED = 0, -1, -2, -3, -4, -5, -6
V_OK, V_NO_PIECE, V_WRONG_TURN, V_ILLEGAL, V_OOR = 0, 1, 2, 3, 4
RULES_REF, RULES_FIDE = 0, 1
MOVE_OOR, MOVE_NONE = 0x8000, 0xFFFF
CELL_EMPTY = -1
KINDS = "PNBRQKX"  # cell kind order of the ABI (X = unknown kind string)

POS_DTYPE = np.dtype([("bb", "<u8", (4,)), ("stm", "u1"), ("castle", "u1"), ("ep", "i1"), ("r0", "u1"),
                      ("r1", "<u4")])
assert POS_DTYPE.itemsize == 40


class DChessError(RuntimeError):
    def __init__(self, status, what=""):
        self.status = status
        super().__init__(f"{what}: {lib().dc_strerror(status).decode()} ({status})")


class _Stats(C.Structure):
    _fields_ = [("validated", C.c_uint64), ("accepted", C.c_uint64), ("rejected", C.c_uint64),
                ("digest_sum", C.c_uint64), ("digest_xor", C.c_uint64)]


class _KStats(C.Structure):
    _fields_ = [("launches", C.c_uint64), ("total_ms", C.c_double), ("units", C.c_uint64)]


_LIB = None
_vp = C.c_void_p


def lib():
    """Loads libdchess.so (built by __graft_entry__.build()); raises if absent."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libdchess.so not built ({LIB_PATH}); run __graft_entry__.build()")
    L = C.CDLL(LIB_PATH)
    sig = {
        "dc_ctx_create": (C.c_int, [C.c_int, C.POINTER(_vp)]),
        "dc_ctx_destroy": (C.c_int, [_vp]),
        "dc_ctx_device": (C.c_int, [_vp]),
        "dc_ctx_stream": (_vp, [_vp]),
        "dc_strerror": (C.c_char_p, [C.c_int]),
        "dc_verdict_message": (C.c_char_p, [C.c_uint8]),
        "dc_version": (C.c_int, []),
        "dc_ctx_set_profiling": (C.c_int, [_vp, C.c_int]),
        "dc_ctx_kernel_stats": (C.c_int, [_vp, C.c_char_p, C.POINTER(_KStats)]),
        "dc_ctx_reset_stats": (C.c_int, [_vp]),
        "dc_device_alloc": (C.c_int, [_vp, C.c_size_t, C.POINTER(_vp)]),
        "dc_device_free": (C.c_int, [_vp, _vp]),
        "dc_memcpy_h2d": (C.c_int, [_vp, _vp, _vp, C.c_size_t]),
        "dc_memcpy_d2h": (C.c_int, [_vp, _vp, _vp, C.c_size_t]),
        "dc_startpos": (C.c_int, [_vp]),
        "dc_pos_from_cells": (C.c_int, [_vp, C.c_uint8, _vp]),
        "dc_pos_to_cells": (C.c_int, [_vp, _vp, C.POINTER(C.c_uint8)]),
        "dc_pos_from_fen": (C.c_int, [C.c_char_p, _vp]),
        "dc_move_pack": (C.c_uint16, [C.c_uint32] * 4),
        "dc_move_pack_batch": (C.c_int, [_vp, C.c_uint32, _vp]),
        "dc_validate_batch": (C.c_int, [_vp, C.c_uint32, _vp, _vp, C.c_uint32, _vp]),
        "dc_apply_batch": (C.c_int, [_vp, C.c_uint32, _vp, _vp, C.c_uint32, _vp, _vp]),
        "dc_live_validator": (C.c_int, [_vp, C.c_uint32]),
        "dc_replay": (C.c_int, [_vp, C.c_uint32, _vp, _vp, C.c_uint32, C.c_uint32, _vp, _vp, C.POINTER(_Stats)]),
        "dc_replay_device": (C.c_int, [_vp, C.c_uint32, _vp, _vp, C.c_uint32, C.c_uint32, _vp, _vp,
                                       C.POINTER(_Stats)]),
        "dc_replay_info": (C.c_int, [_vp, C.c_uint32, _vp, _vp, C.c_uint32, C.c_uint32, _vp, _vp, _vp,
                                     C.POINTER(_Stats)]),
        "dc_replay_info_device": (C.c_int, [_vp, C.c_uint32, _vp, _vp, C.c_uint32, C.c_uint32, _vp, _vp, _vp,
                                            C.POINTER(_Stats)]),
        "dc_history_append": (C.c_int, [C.c_char_p, _vp, _vp, C.c_uint32, C.c_size_t, _vp, C.c_size_t,
                                        C.POINTER(C.c_size_t)]),
        "dc_gen_games": (C.c_int, [_vp, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32,
                                   _vp]),
        "dc_gen_games_device": (C.c_int, [_vp, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32,
                                          C.c_uint32, _vp]),
        "dc_perft": (C.c_int, [_vp, C.c_uint32, _vp, C.c_uint32, _vp, _vp, C.POINTER(C.c_uint32),
                               C.POINTER(C.c_uint64)]),
        "dc_perft_shard": (C.c_int, [_vp, C.c_uint32, _vp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, _vp,
                                     _vp, C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)]),
        "dc_perft_repeat_device": (C.c_int, [_vp, C.c_uint32, _vp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                             C.c_uint32, _vp]),
        "dc_perft_batch": (C.c_int, [_vp, C.c_uint32, _vp, C.c_uint32, C.c_uint32, _vp, _vp, _vp, _vp,
                                     C.POINTER(C.c_uint32)]),
        "dc_perft_batch_repeat_device": (C.c_int, [_vp, C.c_uint32, _vp, C.c_uint32, C.c_uint32, C.c_uint32,
                                                   C.c_uint32, _vp]),
        "dc_ctx_synchronize": (C.c_int, [_vp]),
        "dc_multi_perft": (C.c_int, [_vp, C.c_int, C.c_uint32, _vp, C.c_uint32, _vp, _vp, C.POINTER(C.c_uint32),
                                     C.POINTER(C.c_uint64)]),
        "dc_replay_shard_range": (C.c_int, [C.c_uint64, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint64),
                                            C.POINTER(C.c_uint64)]),
        "dc_replay_scatter_shards": (C.c_int, [C.c_uint64, C.c_uint32, C.c_uint32, _vp, _vp]),
        "dc_multi_replay": (C.c_int, [_vp, C.c_int, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32,
                                      _vp, C.POINTER(_Stats)]),
        "dc_keccak256": (C.c_int, [_vp, C.c_size_t, _vp]),
        "dc_state_hash": (C.c_int, [_vp, _vp, C.c_char_p, C.c_char_p, _vp, _vp, C.c_uint32, C.c_uint32, _vp]),
        "dc_state_hash_device": (C.c_int, [_vp, _vp, C.c_char_p, _vp, _vp, _vp, C.c_uint32, C.c_uint32, _vp]),
        "dc_verify_tx_batch": (C.c_int, [_vp, C.c_char_p, _vp, _vp, _vp, C.c_uint32, _vp]),
        "dc_verify_tx_batch_device": (C.c_int, [_vp, _vp, _vp, _vp, _vp, C.c_uint32, _vp]),
        "dc_sig_verdict_message": (C.c_char_p, [C.c_uint8]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    _LIB = L
    return L


def history_append(history, moves, info):
    """dc_history_append: update_history (chess.rs:127-184) over one game's
    plies (moves/info 1-D, one entry per ply).  Returns the new history."""
    moves = np.ascontiguousarray(moves, np.uint16)
    info = np.ascontiguousarray(info, np.uint8)
    assert moves.shape == info.shape and moves.ndim == 1
    n = C.c_size_t()
    h = history.encode() if history is not None else None
    _check(lib().dc_history_append(h, _ptr(moves), _ptr(info), len(moves), 1, None, 0, C.byref(n)),
           "dc_history_append")
    buf = C.create_string_buffer(n.value + 1)
    _check(lib().dc_history_append(h, _ptr(moves), _ptr(info), len(moves), 1, buf, n.value + 1, C.byref(n)),
           "dc_history_append")
    return buf.value.decode()


def exported_symbols():
    """Names the header declares; tests check the library exports each."""
    hdr = os.path.join(os.path.dirname(os.path.dirname(PKG_DIR)), "include", "dchess.h")
    import re
    names = re.findall(r"^\s*(?:int|uint16_t|void\s*\*|const char\s*\*)\s+(dc_\w+)\s*\(", open(hdr).read(), re.M)
    return sorted(set(names))


def _check(status, what):
    if status != SUCCESS:
        raise DChessError(status, what)


def _ptr(a):
    return C.c_void_p(a.ctypes.data) if a is not None else None


def _dptr(d):
    """A DeviceBuffer, a raw device address (int) or None -> c_void_p."""
    if d is None:
        return None
    return d.ptr if hasattr(d, "ptr") else _vp(int(d))


def verdict_message(v):
    return lib().dc_verdict_message(v).decode()


def keccak256(data):
    """alloy_primitives::keccak256 of a byte string (host side of libdchess)."""
    data = bytes(data)
    buf = C.create_string_buffer(data, len(data)) if data else None
    out = C.create_string_buffer(32)
    _check(lib().dc_keccak256(C.cast(buf, _vp) if buf is not None else None, len(data), C.cast(out, _vp)),
           "dc_keccak256")
    return out.raw


def pack_names(pairs):
    """[(white, black), ...] -> (utf-8 blob, uint32 offsets[2n+1]) for dc_state_hash."""
    blob, off = bytearray(), [0]
    for w, b in pairs:
        for name in (w, b):
            blob += name.encode()
            off.append(len(blob))
    return bytes(blob), np.array(off, np.uint32)


SIG_OK, SIG_BAD_SIG_HEX, SIG_BAD_SIG, SIG_BAD_PK_HEX, SIG_BAD_PK, SIG_INVALID, SIG_WRONG_OWNER = range(7)


def pack_txs(strings, actions, turns=None):
    """[(white, black, signature_hex, pub_key_hex), ...] + uint32 actions [n, 4]
    (+ optional int8 turns, -1 = no owner check) -> the dc_verify_tx_batch inputs
    (utf-8 blob, uint32 offsets [4n+1], actions, turns)."""
    blob, off = bytearray(), [0]
    for quad in strings:
        for s in quad:
            blob += s.encode()
            off.append(len(blob))
    actions = np.ascontiguousarray(actions, np.uint32).reshape(-1, 4)
    assert len(actions) == len(strings)
    if turns is not None:
        turns = np.ascontiguousarray(turns, np.int8)
        assert len(turns) == len(strings)
    return bytes(blob), np.array(off, np.uint32), actions, turns


def sig_verdict_message(v):
    return lib().dc_sig_verdict_message(v).decode()


def _json_str(text):
    """serde_json string literal (escape table of serde_json 1.0 ser.rs)."""
    out = ['"']
    for ch in text:
        o = ord(ch)
        if ch == '"':
            out.append('\\"')
        elif ch == "\\":
            out.append("\\\\")
        elif o < 0x20:
            out.append({8: "\\b", 9: "\\t", 10: "\\n", 12: "\\f", 13: "\\r"}.get(o, "\\u%04x" % o))
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def game_state_json(turn, white, black, history, board):
    """serde_json::to_string(&GameState) (core/proto/game.proto:7-40 via prost +
    the serde derives of core/build.rs:2-32): fields in proto order, Option::None
    as null, the i32 enum fields as numbers.  board[x][y] is None or a Piece."""
    rows = []
    for x in range(8):
        cells = []
        for y in range(8):
            pc = board[x][y]
            cells.append('{"piece":null}' if pc is None else
                         '{"piece":{"color":%d,"kind":%s}}' % (pc.color, _json_str(pc.kind)))
        rows.append('{"cells":[' + ",".join(cells) + "]}")
    hist = "null" if history is None else _json_str(history)
    return ('{"turn":%d,"white_player":%s,"black_player":%s,"history":%s,"board":{"rows":[%s]}}'
            % (turn, _json_str(white), _json_str(black), hist, ",".join(rows)))


# ---------------------------------------------------------------- positions
def startpos():
    p = np.zeros(1, POS_DTYPE)
    _check(lib().dc_startpos(_ptr(p)), "dc_startpos")
    return p[0]


def pos_from_cells(cells, turn):
    cells = np.ascontiguousarray(cells, dtype=np.int8)
    p = np.zeros(1, POS_DTYPE)
    _check(lib().dc_pos_from_cells(_ptr(cells), int(turn), _ptr(p)), "dc_pos_from_cells")
    return p[0]


def pos_to_cells(pos):
    p = np.array([pos], POS_DTYPE)
    cells = np.zeros(64, np.int8)
    turn = C.c_uint8()
    _check(lib().dc_pos_to_cells(_ptr(p), _ptr(cells), C.byref(turn)), "dc_pos_to_cells")
    return cells, turn.value


def pos_from_fen(fen):
    p = np.zeros(1, POS_DTYPE)
    _check(lib().dc_pos_from_fen(fen.encode(), _ptr(p)), "dc_pos_from_fen")
    return p[0]


def move_pack(fx, fy, tx, ty):
    return int(lib().dc_move_pack(fx, fy, tx, ty))


def move_pack_batch(actions):
    """uint32 actions [n, 4] (from.x, from.y, to.x, to.y per transaction) ->
    uint16 move words (dc_move_pack_batch)."""
    actions = np.ascontiguousarray(actions, np.uint32).reshape(-1, 4)
    out = np.zeros(len(actions), np.uint16)
    _check(lib().dc_move_pack_batch(_ptr(actions), len(actions), _ptr(out)), "dc_move_pack_batch")
    return out


class DeviceBuffer:
    """Caller-owned device memory on an Engine's device (dc_device_alloc)."""

    def __init__(self, engine, nbytes):
        self.engine, self.nbytes = engine, int(nbytes)
        p = _vp()
        _check(lib().dc_device_alloc(engine.ctx, self.nbytes, C.byref(p)), "dc_device_alloc")
        self.ptr = p

    def upload(self, arr):
        arr = np.ascontiguousarray(arr)
        assert arr.nbytes <= self.nbytes
        _check(lib().dc_memcpy_h2d(self.engine.ctx, self.ptr, _ptr(arr), arr.nbytes), "dc_memcpy_h2d")

    def download(self, dtype, count):
        out = np.empty(count, dtype)
        assert out.nbytes <= self.nbytes
        _check(lib().dc_memcpy_d2h(self.engine.ctx, _ptr(out), self.ptr, out.nbytes), "dc_memcpy_d2h")
        return out

    def free(self):
        if self.ptr:
            lib().dc_device_free(self.engine.ctx, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Engine:
    """One dc_ctx: one gfx950 device, one HIP stream."""

    def __init__(self, device=0):
        ctx = _vp()
        _check(lib().dc_ctx_create(int(device), C.byref(ctx)), f"dc_ctx_create({device})")
        self.ctx = ctx
        self.device = device

    def close(self):
        if self.ctx:
            lib().dc_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -------------------------------------------------------------- timing
    def set_profiling(self, on=True):
        _check(lib().dc_ctx_set_profiling(self.ctx, 1 if on else 0), "dc_ctx_set_profiling")

    def reset_stats(self):
        _check(lib().dc_ctx_reset_stats(self.ctx), "dc_ctx_reset_stats")

    def kernel_stats(self, name):
        s = _KStats()
        _check(lib().dc_ctx_kernel_stats(self.ctx, name.encode(), C.byref(s)), "dc_ctx_kernel_stats")
        return {"launches": s.launches, "total_ms": s.total_ms, "units": s.units}

    def alloc(self, nbytes):
        return DeviceBuffer(self, nbytes)

    # ---------------------------------------------------------- validation
    def live_validator(self, lease_us):
        """dc_live_validator: calls of <= 64 moves on this engine are served by
        a resident wave (no launch per call) while the lease lasts; 0 stops it."""
        _check(lib().dc_live_validator(self.ctx, int(lease_us)), "dc_live_validator")

    def validate_batch(self, pos, moves, rules=RULES_REF):
        pos = np.ascontiguousarray(pos, POS_DTYPE)
        moves = np.ascontiguousarray(moves, np.uint16)
        assert pos.shape == moves.shape
        out = np.zeros(len(moves), np.uint8)
        _check(lib().dc_validate_batch(self.ctx, rules, _ptr(pos), _ptr(moves), len(moves), _ptr(out)),
               "dc_validate_batch")
        return out

    def apply_batch(self, pos, moves, rules=RULES_REF):
        """Returns (new positions, verdicts, info)."""
        pos = np.array(pos, POS_DTYPE, copy=True)
        moves = np.ascontiguousarray(moves, np.uint16)
        ver = np.zeros(len(moves), np.uint8)
        info = np.zeros(len(moves), np.uint8)
        _check(lib().dc_apply_batch(self.ctx, rules, _ptr(pos), _ptr(moves), len(moves), _ptr(ver), _ptr(info)),
               "dc_apply_batch")
        return pos, ver, info

    # -------------------------------------------------------------- replay
    def replay(self, moves, rules=RULES_REF, start=None, want_bitmap=True, want_digests=True):
        """moves: uint16 [n_plies, n_games] ply-major.  Returns (bitmap, digests, stats dict)."""
        moves = np.ascontiguousarray(moves, np.uint16)
        n_plies, n_games = moves.shape
        words = (n_games + 63) // 64
        bitmap = np.zeros((n_plies, words), np.uint64) if want_bitmap else None
        dig = np.zeros(n_games, np.uint64) if want_digests else None
        st = _Stats()
        sp = None
        if start is not None:
            sp = np.array([start], POS_DTYPE)
        _check(lib().dc_replay(self.ctx, rules, _ptr(sp) if sp is not None else None, _ptr(moves), n_games, n_plies,
                               _ptr(bitmap), _ptr(dig), C.byref(st)), "dc_replay")
        return bitmap, dig, {k: int(getattr(st, k)) for k, _ in _Stats._fields_}

    def replay_info(self, moves, start=None, want_bitmap=True, want_digests=True):
        """dc_replay_info (RULES_REF): replay plus per-ply move info.  Returns
        (bitmap, digests, info uint8 [n_plies, n_games], stats dict)."""
        moves = np.ascontiguousarray(moves, np.uint16)
        n_plies, n_games = moves.shape
        words = (n_games + 63) // 64
        bitmap = np.zeros((n_plies, words), np.uint64) if want_bitmap else None
        dig = np.zeros(n_games, np.uint64) if want_digests else None
        info = np.zeros((n_plies, n_games), np.uint8)
        st = _Stats()
        sp = np.array([start], POS_DTYPE) if start is not None else None
        _check(lib().dc_replay_info(self.ctx, RULES_REF, _ptr(sp), _ptr(moves), n_games, n_plies, _ptr(bitmap),
                                    _ptr(dig), _ptr(info), C.byref(st)), "dc_replay_info")
        return bitmap, dig, info, {k: int(getattr(st, k)) for k, _ in _Stats._fields_}

    def replay_device(self, d_moves, n_games, n_plies, d_bitmap=None, d_digests=None, rules=RULES_REF):
        """d_* are DeviceBuffers or raw device addresses (e.g. a torch tensor's
        data_ptr(), for buffers that a torch.distributed collective reads)."""
        st = _Stats()
        _check(lib().dc_replay_device(self.ctx, rules, None, _dptr(d_moves), n_games, n_plies, _dptr(d_bitmap),
                                      _dptr(d_digests), C.byref(st)), "dc_replay_device")
        return {k: int(getattr(st, k)) for k, _ in _Stats._fields_}

    def state_hash(self, moves, names, start=None, history=""):
        """keccak256(serde_json(final GameState)) of every game of a replay batch
        (dc_state_hash).  moves: uint16 [n_plies, n_games]; names: [(white, black)]
        per game.  Returns uint8 [n_games, 32]."""
        moves = np.ascontiguousarray(moves, np.uint16)
        n_plies, n_games = moves.shape
        blob, off = pack_names(names)
        assert len(off) == 2 * n_games + 1
        out = np.zeros((n_games, 32), np.uint8)
        sp = np.array([start], POS_DTYPE) if start is not None else None
        _check(lib().dc_state_hash(self.ctx, _ptr(sp) if sp is not None else None, history.encode(), blob,
                                   _ptr(off), _ptr(moves), n_games, n_plies, _ptr(out)), "dc_state_hash")
        return out

    def names_device(self, blob, off):
        """pack_names' (blob, offsets) uploaded once: the resident inputs of
        state_hash_device.  Returns (d_names, d_names_off)."""
        d_names = self.alloc(max(len(blob), 1))
        if blob:
            d_names.upload(np.frombuffer(blob, np.uint8))
        d_off = self.alloc(off.nbytes)
        d_off.upload(np.ascontiguousarray(off, np.uint32))
        return d_names, d_off

    def state_hash_device(self, d_moves, n_games, n_plies, d_names, d_names_off, d_hashes, history="", start=None):
        """dc_state_hash_device: every buffer resident on the device (DeviceBuffer);
        d_names / d_names_off hold pack_names' raw blob and offsets."""
        sp = np.array([start], POS_DTYPE) if start is not None else None
        _check(lib().dc_state_hash_device(self.ctx, _ptr(sp) if sp is not None else None, history.encode(),
                                          d_names.ptr, d_names_off.ptr, d_moves.ptr, n_games, n_plies, d_hashes.ptr),
               "dc_state_hash_device")

    def verify_txs(self, blob, off, actions, turns=None):
        """App::validate_signature (+ the owner check when turns is given) for a
        batch of transactions (dc_verify_tx_batch); inputs from pack_txs.
        Returns uint8 DC_SIG_* verdicts."""
        n = len(actions)
        out = np.zeros(n, np.uint8)
        if n == 0:
            return out
        _check(lib().dc_verify_tx_batch(self.ctx, blob, _ptr(off), _ptr(actions), _ptr(turns), n, _ptr(out)),
               "dc_verify_tx_batch")
        return out

    def verify_txs_device(self, d_blob, d_off, d_actions, d_turns, n, d_verdicts):
        _check(lib().dc_verify_tx_batch_device(self.ctx, d_blob.ptr, d_off.ptr, d_actions.ptr,
                                               d_turns.ptr if d_turns else None, n, d_verdicts.ptr),
               "dc_verify_tx_batch_device")

    def gen_games(self, seed, first_game, n_games, n_plies, noise_per_256=32, rules=RULES_REF):
        out = np.zeros((n_plies, n_games), np.uint16)
        _check(lib().dc_gen_games(self.ctx, rules, seed, first_game, n_games, n_plies, noise_per_256, _ptr(out)),
               "dc_gen_games")
        return out

    def gen_games_device(self, d_out, seed, first_game, n_games, n_plies, noise_per_256=32, rules=RULES_REF):
        _check(lib().dc_gen_games_device(self.ctx, rules, seed, first_game, n_games, n_plies, noise_per_256,
                                         _dptr(d_out)), "dc_gen_games_device")

    # --------------------------------------------------------------- perft
    def perft(self, pos, depth, rules=RULES_REF):
        """Returns (total, divide[n_root], root_moves[n_root])."""
        p = np.array([pos], POS_DTYPE)
        div = np.zeros(256, np.uint64)
        rm = np.zeros(256, np.uint16)
        nr, tot = C.c_uint32(), C.c_uint64()
        _check(lib().dc_perft(self.ctx, rules, _ptr(p), depth, _ptr(div), _ptr(rm), C.byref(nr), C.byref(tot)),
               "dc_perft")
        return int(tot.value), div[:nr.value].copy(), rm[:nr.value].copy()

    def perft_shard(self, pos, depth, split_depth, shard, n_shards, rules=RULES_REF):
        p = np.array([pos], POS_DTYPE)
        div = np.zeros(256, np.uint64)
        rm = np.zeros(256, np.uint16)
        nr, tot = C.c_uint32(), C.c_uint64()
        _check(lib().dc_perft_shard(self.ctx, rules, _ptr(p), depth, split_depth, shard, n_shards, _ptr(div),
                                    _ptr(rm), C.byref(nr), C.byref(tot)), "dc_perft_shard")
        return int(tot.value), div[:nr.value].copy(), rm[:nr.value].copy()

    def perft_repeat_device(self, pos, depth, split_depth, shard, n_shards, n_runs, d_out, rules=RULES_REF):
        """dc_perft_repeat_device: n_runs perfts enqueued back to back, run i's
        result at device address d_out + 8 * 258 * i (divide[256], n_root |
        overflow << 32, total); d_out is a DeviceBuffer or a raw device address.
        Returns once enqueued (see synchronize)."""
        p = np.array([pos], POS_DTYPE)
        ptr = d_out.ptr if hasattr(d_out, "ptr") else _vp(int(d_out))
        _check(lib().dc_perft_repeat_device(self.ctx, rules, _ptr(p), depth, split_depth, shard, n_shards, n_runs,
                                            ptr), "dc_perft_repeat_device")

    def perft_batch(self, positions, depth, rules=RULES_REF):
        """dc_perft_batch: the positions (same side to move) counted as one tree.
        Returns (totals[n_pos], divide[n_root], root_moves[n_root], root_pos[n_root])."""
        p = np.array(list(positions), POS_DTYPE)
        tot = np.zeros(len(p), np.uint64)
        div = np.zeros(256, np.uint64)
        rm = np.zeros(256, np.uint16)
        rp = np.zeros(256, np.uint8)
        nr = C.c_uint32()
        _check(lib().dc_perft_batch(self.ctx, rules, _ptr(p), len(p), depth, _ptr(tot), _ptr(div), _ptr(rm), _ptr(rp),
                                    C.byref(nr)), "dc_perft_batch")
        n = nr.value
        return tot, div[:n].copy(), rm[:n].copy(), rp[:n].copy()

    def perft_batch_repeat_device(self, positions, depth, split_depth, n_runs, d_out, rules=RULES_REF):
        """dc_perft_batch_repeat_device: n_runs batch perfts enqueued back to back,
        records as perft_repeat_device (per-position totals: sum divide over
        perft_batch's root_pos)."""
        p = np.array(list(positions), POS_DTYPE)
        ptr = d_out.ptr if hasattr(d_out, "ptr") else _vp(int(d_out))
        _check(lib().dc_perft_batch_repeat_device(self.ctx, rules, _ptr(p), len(p), depth, split_depth, n_runs, ptr),
               "dc_perft_batch_repeat_device")

    def synchronize(self):
        _check(lib().dc_ctx_synchronize(self.ctx), "dc_ctx_synchronize")

    def stream(self):
        """The context's hipStream_t as an int (for torch.cuda.ExternalStream)."""
        return int(lib().dc_ctx_stream(self.ctx) or 0)


def multi_perft(devices, pos, depth, rules=RULES_REF):
    devs = (C.c_int * len(devices))(*devices)
    p = np.array([pos], POS_DTYPE)
    div = np.zeros(256, np.uint64)
    rm = np.zeros(256, np.uint16)
    nr, tot = C.c_uint32(), C.c_uint64()
    _check(lib().dc_multi_perft(devs, len(devices), rules, _ptr(p), depth, _ptr(div), _ptr(rm), C.byref(nr),
                                C.byref(tot)), "dc_multi_perft")
    return int(tot.value), div[:nr.value].copy(), rm[:nr.value].copy()


def replay_shard_range(n_games, shard, n_shards):
    """(first game id, count) of one replay shard (dc_replay_shard_range)."""
    first, count = C.c_uint64(), C.c_uint64()
    _check(lib().dc_replay_shard_range(int(n_games), int(shard), int(n_shards), C.byref(first), C.byref(count)),
           "dc_replay_shard_range")
    return int(first.value), int(count.value)


def multi_replay(devices, seed, n_games, n_plies, noise_per_256=32, rules=RULES_REF, want_bitmap=True):
    """dc_multi_replay: the seeded games [0, n_games) over several devices of this
    process.  Returns (bitmap [n_plies][ceil(n_games/64)] or None, stats dict)."""
    devs = (C.c_int * len(devices))(*devices)
    words = (n_games + 63) // 64
    bitmap = np.zeros((n_plies, words), np.uint64) if want_bitmap else None
    st = _Stats()
    _check(lib().dc_multi_replay(devs, len(devices), rules, seed, n_games, n_plies, noise_per_256, _ptr(bitmap),
                                 C.byref(st)), "dc_multi_replay")
    return bitmap, {k: int(getattr(st, k)) for k, _ in _Stats._fields_}


# ---------------------------------------------------------------------------
# Mirror of the reference's Rust surface (core/src/chess.rs), backed by the GPU.
class AppError(Exception):
    """AppError::InternalGameError(String) -- core/src/errors.rs:9."""


class Position:
    """proto query.Position{x, y} (core/proto/query.proto)."""

    def __init__(self, x, y):
        self.x, self.y = int(x), int(y)


class Piece:
    """proto game.Piece{color, kind} (core/proto/game.proto:15-18)."""

    def __init__(self, color, kind):
        self.color, self.kind = int(color), str(kind)

    def __eq__(self, o):
        return isinstance(o, Piece) and (self.color, self.kind) == (o.color, o.kind)

    def __repr__(self):
        return f"Piece({self.color}, {self.kind!r})"


_DEFAULT_ENGINE = None


def default_engine():
    global _DEFAULT_ENGINE
    if _DEFAULT_ENGINE is None:
        _DEFAULT_ENGINE = Engine(0)
    return _DEFAULT_ENGINE


class GameState:
    """GameState (core/proto/game.proto:7-13) with the chess.rs methods.

    The board is kept as the proto's 8x8 grid of optional Pieces; every
    validate/apply is one dc_validate_batch / dc_apply_batch call (n = 1).
    """

    def __init__(self, white_player, black_player, engine=None):  # chess.rs:12-20
        self.white_player, self.black_player = white_player, black_player
        self.turn = 0
        self.history = ""
        self.engine = engine or default_engine()
        cells, _ = pos_to_cells(startpos())
        self.board = [[None] * 8 for _ in range(8)]
        for s in range(64):
            if cells[s] >= 0:
                self.board[s // 8][s % 8] = Piece(cells[s] >> 3, KINDS[cells[s] & 7])

    def _pos(self):
        cells = np.full(64, CELL_EMPTY, np.int8)
        for x in range(8):
            for y in range(8):
                p = self.board[x][y]
                if p is not None:
                    k = KINDS.index(p.kind) if p.kind in KINDS[:6] else 6
                    cells[8 * x + y] = p.color * 8 + k
        return pos_from_cells(cells, self.turn)

    def to_json(self):
        """serde_json::to_string(&GameState)."""
        return game_state_json(self.turn, self.white_player, self.black_player, self.history, self.board)

    def state_hash(self):
        """calculate_game_state_hash (core/src/consensus/hotstuff.rs:153-166): keccak256 of
        the JSON, as alloy's B256 Display string."""
        return "0x" + keccak256(self.to_json().encode()).hex()

    def validate_move(self, frm, to):  # chess.rs:82-98
        v = self.engine.validate_batch(np.array([self._pos()], POS_DTYPE),
                                       np.array([move_pack(frm.x, frm.y, to.x, to.y)], np.uint16))[0]
        if v == V_OOR:
            raise IndexError("index out of bounds")  # the reference panics here
        if v != V_OK:
            raise AppError(verdict_message(v))

    def apply_move(self, frm, to):  # chess.rs:43-80
        pos = np.array([self._pos()], POS_DTYPE)
        new, ver, info = self.engine.apply_batch(pos, np.array([move_pack(frm.x, frm.y, to.x, to.y)], np.uint16))
        v = int(ver[0])
        if v == V_OOR:
            raise IndexError("index out of bounds")
        if v != V_OK:
            raise AppError(verdict_message(v))
        kind, capture = KINDS[info[0] & 7], bool(info[0] & 8)
        mover = self.board[frm.x][frm.y]
        self._update_history(frm, to, mover.kind if kind == "X" else kind, capture)
        cells, turn = pos_to_cells(new[0])
        # Unknown-kind pieces never move (chess.rs:210): keep their original kind strings.
        old = self.board
        self.board = [[None] * 8 for _ in range(8)]
        for s in range(64):
            if cells[s] >= 0:
                k = KINDS[cells[s] & 7]
                if k == "X":
                    k = old[s // 8][s % 8].kind
                self.board[s // 8][s % 8] = Piece(cells[s] >> 3, k)
        self.turn = turn

    def _update_history(self, frm, to, kind, capture):  # chess.rs:127-184 (GPU supplies kind/capture)
        code = "PNBRQK".index(kind) | (8 if capture else 0)
        self.history = history_append(self.history, np.array([move_pack(frm.x, frm.y, to.x, to.y)], np.uint16),
                                      np.array([code], np.uint8))
