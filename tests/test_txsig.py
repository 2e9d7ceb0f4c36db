"""Transaction-signature check (App::validate_signature,
core/src/consensus/hotstuff.rs:168-208).

CPU tests (no GPU):
  - the oracle (oracle/txsig.py) pinned to published secp256k1 facts: the
    domain parameters, G on the curve, n G = infinity, the x coordinates of
    2G and 3G, hashlib SHA-256, sign/verify round trips;
  - the kernel's arithmetic and per-transaction function (dc_secp.h /
    dc_txsig.h, compiled for the host as build/test_secp) against the oracle.
GPU tests (-m gpu): dc_verify_tx_batch through the C ABI against the oracle,
including every reject class and the owner check.
"""
import os
import random
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import txsig as T  # noqa: E402

BIN = os.path.join(REPO, "distributed-chess_amd", "build", "test_secp")


# ------------------------------------------------------------ fixtures
def make_tx(rng, d_white, d_black, turn=0, compressed=True, action=None):
    """A Transaction signed the way the client does (chess/src/app/play/page.tsx:37-44,
    :106-125): players are hex public keys, pub_key is the mover's."""
    w = T.pubkey_hex(d_white, compressed)
    b = T.pubkey_hex(d_black, compressed)
    act = action or (rng.randrange(8), rng.randrange(8), rng.randrange(8), rng.randrange(8))
    d = d_white if turn == 0 else d_black
    r, s = T.sign(d, T.message_hash(w, b, act))
    return dict(white=w, black=b, action=act, sig=T.sig_hex(r, s), pk=w if turn == 0 else b, turn=turn)


def tamper_cases(rng):
    """One transaction per reject class of validate_signature plus edge cases."""
    d1, d2 = 0x1234567, 0xABCDEF987654321
    base = make_tx(rng, d1, d2)
    out = [base]
    t = dict(base); t["action"] = (base["action"][0] ^ 1,) + base["action"][1:]; out.append(t)  # message changed
    t = dict(base); t["sig"] = base["sig"][:-1]; out.append(t)                  # odd-length hex
    t = dict(base); t["sig"] = "zz" + base["sig"][2:]; out.append(t)            # bad hex char
    t = dict(base); t["sig"] = base["sig"] + "00"; out.append(t)                # 65-byte signature
    t = dict(base); t["sig"] = "%064x" % T.N + base["sig"][64:]; out.append(t)  # r = n (overflow)
    t = dict(base); t["sig"] = base["sig"][:64] + "%064x" % (T.N + 5); out.append(t)  # s >= n
    t = dict(base); t["sig"] = "0" * 64 + base["sig"][64:]; out.append(t)       # r = 0
    t = dict(base); t["sig"] = base["sig"][:64] + "0" * 64; out.append(t)       # s = 0
    r, s = int(base["sig"][:64], 16), int(base["sig"][64:], 16)
    t = dict(base); t["sig"] = T.sig_hex(r, T.N - s); out.append(t)             # high s: still valid
    t = dict(base); t["pk"] = base["pk"][:-2]; out.append(t)                    # 32-byte key
    t = dict(base); t["pk"] = "04" + base["pk"][2:]; out.append(t)              # tag mismatch length
    t = dict(base); t["pk"] = "05" + base["pk"][2:]; out.append(t)              # bad tag
    t = dict(base); t["pk"] = base["pk"][:5] + "g" + base["pk"][6:]; out.append(t)  # bad hex
    t = dict(base); t["pk"] = base["pk"].upper(); out.append(t)                 # upper-case hex: same key
    t = dict(base); t["pk"] = "02" + "%064x" % T.P; out.append(t)               # x >= p
    t = dict(base); t["pk"] = "02" + "%064x" % 5; out.append(t)                 # x = 5: no square root
    full = T.pubkey_hex(d1, False)
    t = dict(base); t["pk"] = full; out.append(t)                               # uncompressed form
    t = dict(base); t["pk"] = full[2:]; out.append(t)                           # raw 64-byte form
    y_odd = int(full[-64:], 16) & 1
    t = dict(base); t["pk"] = ("07" if y_odd else "06") + full[2:]; out.append(t)  # hybrid, right parity
    t = dict(base); t["pk"] = ("06" if y_odd else "07") + full[2:]; out.append(t)  # hybrid, wrong parity
    t = dict(base); t["pk"] = full[:-1] + ("0" if full[-1] != "0" else "1"); out.append(t)  # off the curve
    t = dict(base); t["pk"] = T.pubkey_hex(d2); out.append(t)                   # someone else's key
    t = dict(base); t["turn"] = 1; out.append(t)                                # not the mover
    t = make_tx(rng, d1, d2, turn=1); out.append(t)                             # black to move
    odd = make_tx(rng, d1, d2)
    odd["white"] = 'we"ird\\\n\x01é'                                         # escapes + UTF-8
    r, s = T.sign(d1, T.message_hash(odd["white"], odd["black"], odd["action"]))
    odd["sig"] = T.sig_hex(r, s); odd["pk"] = T.pubkey_hex(d1); odd["turn"] = -1; out.append(odd)
    big = make_tx(rng, d1, d2, action=(4294967295, 8, 123456, 0)); out.append(big)  # u32 coordinates
    return out


def expected(tx):
    v = T.check_tx(tx["white"], tx["black"], tx["action"], tx["sig"], tx["pk"])
    if v == T.SIG_OK and tx["turn"] >= 0:
        owner = tx["white"] if tx["turn"] == 0 else tx["black"]
        if tx["pk"] != owner:
            v = 6
    return v


# ------------------------------------------------------------- oracle pins
def test_oracle_curve_facts():
    assert T.on_curve(T.G)
    assert T.mul(T.N, T.G) is None
    # published x coordinates of 2G and 3G
    assert T.mul(2, T.G)[0] == 0xC6047F9441ED7D6D3045406E95C07CD85C778E4B8CEF3CA7ABAC09B95C709EE5
    assert T.mul(3, T.G)[0] == 0xF9308A019258C31049344F85F89D5229B531C845836F99B08601F113BCE036F9
    assert T.pubkey_hex(1) == "0279be667ef9dcbbac55a06295ce870b07029bfcdb2dce28d959f2815b16f81798"
    assert T.P == 2 ** 256 - 2 ** 32 - 977


LAMBDA = 0x5363AD4CC05C30E0A5261C028812645A122E22EA20816678DF02967C1B23BD72
BETA = 0x7AE96A2B657C07106E64479EAC3434E99CF0497512F58995C1396C28719501EE


def test_glv_constants():
    """The endomorphism constants dc_secp.h's ecmult uses (sc_split_lambda, fe_beta)."""
    assert pow(LAMBDA, 3, T.N) == 1 and pow(BETA, 3, T.P) == 1
    assert T.mul(LAMBDA, T.G) == (BETA * T.GX % T.P, T.GY)
    a1, b1 = 0x3086D221A7D46BCDE86C90E49284EB15, -0xE4437ED6010E88286F547FA90ABFE4C3
    a2, b2 = 0x114CA50F7A8E2F3F657C1108D9D44CFD8, a1
    assert (a1 + b1 * LAMBDA) % T.N == 0 and (a2 + b2 * LAMBDA) % T.N == 0
    g1 = (2 ** 384 * b2 + T.N // 2) // T.N
    g2 = (2 ** 384 * -b1 + T.N // 2) // T.N
    assert g1 == 0x3086D221A7D46BCDE86C90E49284EB153DAA8A1471E8CA7FE893209A45DBB031
    assert g2 == 0xE4437ED6010E88286F547FA90ABFE4C4221208AC9DF506C61571B4AE8AC47F71
    rng = random.Random(9)
    for k in [0, 1, T.N - 1, LAMBDA, T.N // 2] + [rng.randrange(T.N) for _ in range(2000)]:
        c1 = (k * g1 + 2 ** 383) >> 384
        c2 = (k * g2 + 2 ** 383) >> 384
        r2 = (c1 * -b1 + c2 * -b2) % T.N
        r1 = (k - r2 * LAMBDA) % T.N
        assert (r1 + LAMBDA * r2) % T.N == k
        for r in (r1, r2):
            assert min(r, T.N - r) < 2 ** 128


def test_oracle_message_json():
    # serde_json with preserve_order: keys in json! order, no whitespace
    assert T.message_json("ab", "cd", (1, 0, 3, 0)) == \
        '{"whitePlayer":"ab","blackPlayer":"cd","action":[{"x":1,"y":0},{"x":3,"y":0}]}'
    assert T.json_escape('a"b\\c\nd\x01\x7f') == 'a\\"b\\\\c\\nd\\u0001\x7f'


def test_oracle_sign_verify_roundtrip():
    rng = random.Random(7)
    for k in range(4):
        tx = make_tx(rng, rng.randrange(1, T.N), rng.randrange(1, T.N), turn=k & 1, compressed=bool(k & 2))
        assert expected(tx) == T.SIG_OK
    cases = tamper_cases(random.Random(1))
    got = [expected(t) for t in cases]
    assert got[:3] == [0, 5, 1] and 2 in got and 3 in got and 4 in got and 6 in got


# ---------------------------------------------- host build of the kernel code
@pytest.fixture(scope="module")
def secp_bin():
    if not os.path.exists(BIN):
        pytest.skip("build/test_secp not built (make -C distributed-chess_amd test_secp)")
    p = subprocess.Popen([BIN], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, bufsize=1)

    def ask(line):
        p.stdin.write(line + "\n")
        p.stdin.flush()
        return p.stdout.readline().strip()
    yield ask
    p.stdin.close()
    p.wait(timeout=30)


def _h(x):
    return "%064x" % x


def _s(s):
    return s.encode("utf-8").hex() or "-"


def test_host_field_scalar_ops(secp_bin):
    rng = random.Random(3)
    vals = [0, 1, 2, T.P - 1, T.P - 2, 2 ** 255, 2 ** 32 + 977, T.N - 1] + [rng.randrange(T.P) for _ in range(40)]
    for i, a in enumerate(vals):
        b = vals[(i * 7 + 3) % len(vals)]
        assert int(secp_bin(f"fe_mul {_h(a)} {_h(b)}"), 16) == a * b % T.P
        assert int(secp_bin(f"fe_sqr {_h(a)}"), 16) == a * a % T.P
        assert int(secp_bin(f"fe_add {_h(a)} {_h(b)}"), 16) == (a + b) % T.P
        assert int(secp_bin(f"fe_sub {_h(a)} {_h(b)}"), 16) == (a - b) % T.P
        if a:
            assert int(secp_bin(f"fe_inv {_h(a)}"), 16) == pow(a, T.P - 2, T.P)
        assert int(secp_bin(f"fe_sqrt {_h(a)}"), 16) == pow(a, (T.P + 1) // 4, T.P)
    svals = [1, 2, T.N - 1, 2 ** 255, 2 ** 256 - 1 - T.N] + [rng.randrange(1, T.N) for _ in range(30)]
    for i, a in enumerate(svals):
        b = svals[(i * 5 + 1) % len(svals)]
        assert int(secp_bin(f"sc_mul {_h(a)} {_h(b)}"), 16) == a * b % T.N
    for a in svals[:8]:
        assert int(secp_bin(f"sc_inv {_h(a)}"), 16) == pow(a, T.N - 2, T.N)


def test_host_point_mul(secp_bin):
    rng = random.Random(5)
    # GLV edge scalars: lambda, -lambda, 2^128 +- 1, n / 2, large negative split parts
    edge = [LAMBDA, T.N - LAMBDA, 2 ** 128 - 1, 2 ** 128, 2 ** 128 + 1, T.N // 2, T.N // 2 + 1, T.N - 2 ** 127,
            (2 ** 127 + LAMBDA * (2 ** 127 - 1)) % T.N]
    for k in [1, 2, 3, 255, 256, T.N - 1, 2 ** 200 + 12345] + edge + [rng.randrange(1, T.N) for _ in range(12)]:
        x, y = T.mul(k, T.G)
        assert secp_bin(f"mulg {_h(k)}") == f"{_h(x)} {_h(y)}"
        q = T.mul(rng.randrange(1, T.N), T.G)
        x, y = T.mul(k, q)
        assert secp_bin(f"mulq {_h(k)} {_h(q[0])} {_h(q[1])}") == f"{_h(x)} {_h(y)}"
    assert secp_bin(f"mulg {_h(T.N)}") == "inf"


def test_host_message_hash(secp_bin):
    for w, b, act in [("ab", "cd", (1, 0, 3, 0)), ("", "", (0, 0, 0, 0)), ('q"\\\x1f\t', "éx" * 40, (9, 10, 99, 4294967295))]:
        assert secp_bin(f"hash {_s(w)} {_s(b)} {' '.join(map(str, act))}") == T.message_hash(w, b, act).hex()


def test_host_check_tx(secp_bin):
    for tx in tamper_cases(random.Random(11)):
        line = (f"tx {_s(tx['white'])} {_s(tx['black'])} {' '.join(map(str, tx['action']))} "
                f"{_s(tx['sig'])} {_s(tx['pk'])} {tx['turn']}")
        assert int(secp_bin(line)) == expected(tx), tx


# ------------------------------------------------------------------ GPU
def pack_txs(txs):
    import dchess
    return dchess.pack_txs([(t["white"], t["black"], t["sig"], t["pk"]) for t in txs],
                           np.array([t["action"] for t in txs], np.uint32).reshape(-1, 4),
                           np.array([t["turn"] for t in txs], np.int8))


@pytest.mark.gpu
def test_gpu_verify_tx_cases(engine):
    txs = tamper_cases(random.Random(11)) * 3
    got = engine.verify_txs(*pack_txs(txs))
    assert got.tolist() == [expected(t) for t in txs]


@pytest.mark.gpu
def test_gpu_verify_tx_random_batch(engine):
    rng = random.Random(2024)
    keys = [rng.randrange(1, T.N) for _ in range(16)]
    txs = []
    for i in range(300):
        tx = make_tx(rng, keys[i % 16], keys[(i * 5 + 3) % 16], turn=i & 1, compressed=(i % 3 != 0))
        if i % 7 == 3:  # corrupt one signature hex digit
            j = rng.randrange(128)
            tx["sig"] = tx["sig"][:j] + ("0" if tx["sig"][j] != "0" else "1") + tx["sig"][j + 1:]
        txs.append(tx)
    got = engine.verify_txs(*pack_txs(txs))
    assert got.tolist() == [expected(t) for t in txs]
    assert engine.verify_txs(*pack_txs([])).size == 0


def _fixture():
    import json
    return json.load(open(os.path.join(HERE, "golden", "txsig_batch.json")))["txs"]


def test_fixture_matches_oracle():
    for t in _fixture()[:24]:
        tx = dict(t, action=tuple(t["action"]))
        assert expected(tx) == t["verdict"]


def test_host_fixture(secp_bin):
    for t in _fixture()[:48]:
        line = (f"tx {_s(t['white'])} {_s(t['black'])} {' '.join(map(str, t['action']))} "
                f"{_s(t['sig'])} {_s(t['pk'])} {t['turn']}")
        assert int(secp_bin(line)) == t["verdict"]


@pytest.mark.gpu
def test_gpu_verify_tx_fixture(engine):
    txs = _fixture()
    got = engine.verify_txs(*pack_txs(txs))
    assert got.tolist() == [t["verdict"] for t in txs]
