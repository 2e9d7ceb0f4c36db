"""CPU tests of the C-ABI library: it loads, exports every symbol include/dchess.h
declares, its host-side data-layout adapters agree with the oracle's layout,
and compute entry points fail loudly (DC_ENODEV) when no gfx950 device is
present -- there is no CPU fallback."""
import ctypes as C
import json
import os

import numpy as np
import pytest

import dchess
import oracle_lib as O

OG = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "oracle_golden.json")))


def test_library_exports_every_header_symbol():
    L = dchess.lib()
    names = dchess.exported_symbols()
    assert len(names) >= 25
    for n in names:
        assert hasattr(L, n), n


_C2RS = {"int": "c_int", "uint8_t": "u8", "int8_t": "i8", "uint16_t": "u16", "uint32_t": "u32",
         "uint64_t": "u64", "size_t": "usize", "char": "c_char", "void": "c_void", "dc_ctx": "dc_ctx",
         "dc_pos": "dc_pos", "dc_replay_stats": "dc_replay_stats", "dc_kernel_stats": "dc_kernel_stats"}


def _c_to_rust(t):
    """C parameter/return type (name stripped) -> the Rust FFI type it must be."""
    t = " ".join(t.split())
    arr = t.endswith("]")
    if arr:  # `const int8_t cells[64]` decays to a pointer
        t = t[:t.index("[")].rsplit(" ", 1)[0] + " *"
    stars = t.count("*")
    base = t.replace("*", " ").split()
    const = base[0] == "const"
    name = base[-1] if not const else base[1]
    rs = _C2RS[name]
    if stars == 0:
        return rs
    out = ("*const " if const else "*mut ") + rs
    for _ in range(stars - 1):
        out = "*mut " + out
    return out


def test_rust_binding_matches_header():
    """integration/rust/src/lib.rs (unverified: no cargo here) declares EVERY
    function of include/dchess.h, each parameter and the return value with the
    Rust type the C type maps to; and its safe layer has no panicking calls."""
    import re
    root = os.path.join(os.path.dirname(dchess.LIB_PATH), "..")
    hdr = re.sub(r"/\*.*?\*/", "", open(os.path.join(root, "include", "dchess.h")).read(), flags=re.S)
    rs = open(os.path.join(root, "integration", "rust", "src", "lib.rs")).read()
    decls = {}
    for m in re.finditer(r"^\s*((?:const\s+)?\w+\s*\**)\s*(dc_\w+)\s*\(([^)]*)\)\s*;", hdr, re.M):
        ret, name, args = m.group(1), m.group(2), " ".join(m.group(3).split())
        params = [] if args in ("", "void") else [a.strip() for a in args.split(",")]
        types = []
        for a in params:  # drop the parameter name (keep an array suffix)
            mm = re.match(r"(.*?)(\w+)(\[\d+\])?$", a)
            types.append(_c_to_rust(mm.group(1) + ("x" + mm.group(3) if mm.group(3) else "")).strip()
                         if mm.group(3) else _c_to_rust(mm.group(1)))
        decls[name] = (_c_to_rust(ret), types)
    assert len(decls) >= 40
    rs_fns = {}
    for m in re.finditer(r"pub fn (dc_\w+)\(([^)]*)\)\s*(?:->\s*([^;]+))?;", rs):
        args = [a.strip() for a in " ".join(m.group(2).split()).split(",") if a.strip()]
        rs_fns[m.group(1)] = ((m.group(3) or "()").strip(), [a.split(":", 1)[1].strip() for a in args])
    missing = sorted(set(decls) - set(rs_fns))
    assert not missing, missing
    for name, (ret, types) in decls.items():
        rret, rtypes = rs_fns[name]
        assert rret == ret, (name, rret, ret)
        assert rtypes == types, (name, rtypes, types)
    safe = rs[rs.index("pub struct DcError"):]
    for bad in ("assert!(", "assert_eq!(", ".unwrap()", ".expect(", "panic!(", "unreachable!("):
        assert bad not in safe, bad


def test_version_and_messages():
    assert dchess.lib().dc_version() >= 100
    # exact reference strings, chess.rs:104-121
    assert dchess.verdict_message(1) == "No piece at the source location"
    assert dchess.verdict_message(2) == "It's not this piece's turn to move"
    assert dchess.verdict_message(3) == "Invalid move for the piece"


def test_startpos_layout_matches_oracle():
    p = dchess.startpos()
    assert [int(x) for x in p["bb"]] == OG["startpos_quad"]
    cells, turn = dchess.pos_to_cells(p)
    assert (cells == O.startpos_cells()).all() and turn == 0


def test_cells_roundtrip_random():
    rng = np.random.default_rng(3)
    for _ in range(50):
        cells = np.full(64, -1, np.int8)
        k = int(rng.integers(0, 40))
        sq = rng.choice(64, k, replace=False)
        cells[sq] = rng.integers(0, 2, k) * 8 + rng.integers(0, 7, k)
        p = dchess.pos_from_cells(cells, 1)
        assert [int(x) for x in p["bb"]] == [int(x) for x in O.quad(cells)]
        back, turn = dchess.pos_to_cells(p)
        assert (back == cells).all() and turn == 1


def test_cells_reject_bad_input():
    cells = O.startpos_cells().copy()
    with pytest.raises(dchess.DChessError):
        dchess.pos_from_cells(cells, 2)  # turn outside {0,1}: Color::from_i32 panics (chess.rs:110)
    cells[20] = 2 * 8  # colour 2 is not representable
    with pytest.raises(dchess.DChessError):
        dchess.pos_from_cells(cells, 0)


def test_fen_parser_matches_oracle():
    for name, e in OG["perft_fide"].items():
        p = dchess.pos_from_fen(e["fen"])
        q = O.Pos.from_fen(e["fen"])
        assert [int(x) for x in p["bb"]] == [int(x) for x in O.quad(q.cells)], name
        assert (int(p["stm"]), int(p["castle"]), int(p["ep"])) == (q.stm, q.castle, q.ep)
    with pytest.raises(dchess.DChessError):
        dchess.pos_from_fen("not a fen")


def test_move_pack_batch():
    """Transaction.action u32 coordinates (query.proto:46-49) -> move words: in range
    packs f | t << 6, any coordinate >= 8 (up to 2^32 - 1) is DC_MOVE_OOR."""
    rng = np.random.default_rng(7)
    a = rng.integers(0, 8, (500, 4), dtype=np.uint32)
    big = rng.integers(8, 2**32, (500, 4), dtype=np.uint64).astype(np.uint32)
    pick = rng.random((500, 4)) < 0.1
    a = np.where(pick, big, a)
    got = dchess.move_pack_batch(a)
    want = [dchess.move_pack(*map(int, r)) for r in a]
    assert got.tolist() == want
    ok = ~pick.any(axis=1)
    assert (got[ok] == (a[ok, 0] * 8 + a[ok, 1]) | ((a[ok, 2] * 8 + a[ok, 3]) << 6)).all()
    assert (got[~ok] == dchess.MOVE_OOR).all()
    assert dchess.move_pack_batch(np.zeros((0, 4), np.uint32)).size == 0


def test_move_pack():
    assert dchess.move_pack(1, 0, 3, 0) == (8 | (24 << 6))
    assert dchess.move_pack(8, 0, 0, 0) == dchess.MOVE_OOR
    assert dchess.move_pack(0, 0, 0, 9) == dchess.MOVE_OOR


def test_no_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    ctx = C.c_void_p()
    assert dchess.lib().dc_ctx_create(0, C.byref(ctx)) == dchess.ENODEV
    with pytest.raises(dchess.DChessError):
        dchess.Engine(0)
