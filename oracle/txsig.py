"""oracle/txsig.py -- CPU restatement of the reference's transaction-signature
check (TEST INFRASTRUCTURE ONLY: imported by tests/ and bench.py's CPU leg as
the checker, never by the product path).

Reference: App::validate_signature, core/src/consensus/hotstuff.rs:168-208.

  message  = serde_json::json!({"whitePlayer", "blackPlayer",
             "action": [{"x","y"}, {"x","y"}]})            hotstuff.rs:169-176
             (key order kept: serde_json "preserve_order", core/Cargo.toml:27;
             the client signs JSON.stringify of the same object,
             chess/src/app/play/page.tsx:37-44, :106-113)
  hash     = Sha256::digest(serde_json::to_string(message))  hotstuff.rs:178-180
  Message::parse_slice(hash)                                  hotstuff.rs:181
  signature = hex::decode(tx.signature)                       hotstuff.rs:183
  Signature::parse_standard_slice(bytes)                      hotstuff.rs:186
  public_key = hex::decode(tx.pub_key)                        hotstuff.rs:193
  PublicKey::parse_slice(bytes, None)                         hotstuff.rs:195
  verify(&message, &signature, &public_key)                   hotstuff.rs:202

The curve arithmetic is libsecp256k1 0.7.1 (core/Cargo.lock), a third-party
crate absent from /root/reference; its published algorithm is restated here:
  - Message: 32 bytes read big-endian as a scalar, reduced mod n.
  - Signature::parse_standard_slice: 64 bytes = r || s, each big-endian;
    length != 64 or r >= n or s >= n -> error.  (r = 0 / s = 0 parse, then
    fail verification.)  No low-s requirement.
  - PublicKey::parse_slice(p, None): by length -- 65 full (tag 0x04, or
    hybrid 0x06/0x07 whose tag parity must match y), 33 compressed (tag
    0x02/0x03), 64 raw (x || y, treated as tag 0x04); other lengths -> error.
    x, y >= p -> error; the point must be on y^2 = x^3 + 7; compressed x with
    no square root -> error.
  - verify: r = 0 or s = 0 -> false; sn = s^-1 mod n, u1 = z sn, u2 = r sn;
    R = u1 G + u2 Q; R at infinity -> false; accept iff R.x == r, or
    r + n < p and R.x == r + n (the x coordinate is compared mod p).
  - hex::decode (hex 0.4.3): upper and lower case digits; odd length or a
    non-hex character -> error.

Parity: the reference has no test of this path and its Rust code cannot be
built here, so the restatement is pinned by (1) hashlib SHA-256,
(2) the published secp256k1 domain parameters and multiples of G (k = 1, 2, 3,
tests/test_txsig.py), (3) n G = infinity, and (4) sign/verify round trips with
RFC 6979-style deterministic nonces.  Beyond that: parity unpinned.
"""
import hashlib
import hmac

P = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEFFFFFC2F
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
GX = 0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798
GY = 0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8
G = (GX, GY)

# verdict codes (include/dchess.h DC_SIG_*), in the reference's check order
SIG_OK = 0
SIG_BAD_SIG_HEX = 1   # hex::decode(tx.signature) failed           hotstuff.rs:183-184
SIG_BAD_SIG = 2       # Signature::parse_standard_slice failed     hotstuff.rs:186-191
SIG_BAD_PK_HEX = 3    # hex::decode(tx.pub_key) failed             hotstuff.rs:193-194
SIG_BAD_PK = 4        # PublicKey::parse_slice failed              hotstuff.rs:195-200
SIG_INVALID = 5       # verify() returned false: "invalid signature" hotstuff.rs:202-206


# ------------------------------------------------------------ JSON (serde_json)
def json_escape(s):
    """serde_json's string escaping (ESCAPE table of serde_json 1.0.120):
    '"' and '\\' backslashed, \\b \\f \\n \\r \\t short forms, other bytes < 0x20
    as \\u00XX (lower-case hex); everything else (DEL, non-ASCII) raw UTF-8."""
    out = []
    for ch in s:
        o = ord(ch)
        if ch == '"':
            out.append('\\"')
        elif ch == '\\':
            out.append('\\\\')
        elif o < 0x20:
            short = {8: '\\b', 12: '\\f', 10: '\\n', 13: '\\r', 9: '\\t'}
            out.append(short.get(o, '\\u%04x' % o))
        else:
            out.append(ch)
    return ''.join(out)


def message_json(white, black, action):
    """serde_json::to_string of the json! object at hotstuff.rs:169-176.
    action = (fx, fy, tx, ty), u32 each (Position, query.proto:46-49)."""
    fx, fy, tx, ty = action
    return ('{"whitePlayer":"%s","blackPlayer":"%s","action":[{"x":%d,"y":%d},{"x":%d,"y":%d}]}'
            % (json_escape(white), json_escape(black), fx, fy, tx, ty))


def message_hash(white, black, action):
    return hashlib.sha256(message_json(white, black, action).encode("utf-8")).digest()


# ------------------------------------------------------------------- hex crate
def hex_decode(s):
    """hex::decode: None on an odd length or a non-hex character."""
    if len(s) % 2:
        return None
    out = bytearray()
    for i in range(0, len(s), 2):
        a, b = s[i], s[i + 1]
        if a not in "0123456789abcdefABCDEF" or b not in "0123456789abcdefABCDEF":
            return None
        out.append(int(a + b, 16))
    return bytes(out)


# ---------------------------------------------------------------- curve (affine)
def _add(p1, p2):
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    (x1, y1), (x2, y2) = p1, p2
    if x1 == x2:
        if (y1 + y2) % P == 0:
            return None
        lam = 3 * x1 * x1 * pow(2 * y1, P - 2, P) % P
    else:
        lam = (y2 - y1) * pow(x2 - x1, P - 2, P) % P
    x3 = (lam * lam - x1 - x2) % P
    return (x3, (lam * (x1 - x3) - y1) % P)


def mul(k, pt):
    r = None
    while k:
        if k & 1:
            r = _add(r, pt)
        pt = _add(pt, pt)
        k >>= 1
    return r


def on_curve(pt):
    x, y = pt
    return (y * y - x * x * x - 7) % P == 0


def parse_pubkey(b):
    """PublicKey::parse_slice(b, None) -> affine point or None (error)."""
    if len(b) == 64:
        b = b"\x04" + b
    if len(b) == 65:
        if b[0] not in (4, 6, 7):
            return None
        x, y = int.from_bytes(b[1:33], "big"), int.from_bytes(b[33:], "big")
        if x >= P or y >= P:
            return None
        if b[0] in (6, 7) and (y & 1) != (b[0] == 7):
            return None
        return (x, y) if on_curve((x, y)) else None
    if len(b) == 33:
        if b[0] not in (2, 3):
            return None
        x = int.from_bytes(b[1:], "big")
        if x >= P:
            return None
        y2 = (x * x * x + 7) % P
        y = pow(y2, (P + 1) // 4, P)
        if y * y % P != y2:
            return None
        if (y & 1) != (b[0] == 3):
            y = P - y
        return (x, y)
    return None


def verify_raw(z, r, s, q):
    if r == 0 or s == 0:
        return False
    sn = pow(s, N - 2, N)
    u1, u2 = z * sn % N, r * sn % N
    pt = _add(mul(u1, G), mul(u2, q))
    if pt is None:
        return False
    if pt[0] == r:
        return True
    return r + N < P and pt[0] == r + N


def check_tx(white, black, action, sig_hex, pk_hex):
    """Verdict of validate_signature for one Transaction (SIG_* code)."""
    z = int.from_bytes(message_hash(white, black, action), "big") % N
    sb = hex_decode(sig_hex)
    if sb is None:
        return SIG_BAD_SIG_HEX
    if len(sb) != 64:
        return SIG_BAD_SIG
    r, s = int.from_bytes(sb[:32], "big"), int.from_bytes(sb[32:], "big")
    if r >= N or s >= N:
        return SIG_BAD_SIG
    pb = hex_decode(pk_hex)
    if pb is None:
        return SIG_BAD_PK_HEX
    q = parse_pubkey(pb)
    if q is None:
        return SIG_BAD_PK
    return SIG_OK if verify_raw(z, r, s, q) else SIG_INVALID


# ------------------------------------------------- signing (fixture generation)
def _nonce(d, z, extra=b""):
    """Deterministic nonce, HMAC-SHA256 DRBG in the manner of RFC 6979 §3.2."""
    x = d.to_bytes(32, "big")
    h = (z % N).to_bytes(32, "big")
    v, k = b"\x01" * 32, b"\x00" * 32
    k = hmac.new(k, v + b"\x00" + x + h + extra, hashlib.sha256).digest()
    v = hmac.new(k, v, hashlib.sha256).digest()
    k = hmac.new(k, v + b"\x01" + x + h + extra, hashlib.sha256).digest()
    v = hmac.new(k, v, hashlib.sha256).digest()
    while True:
        v = hmac.new(k, v, hashlib.sha256).digest()
        t = int.from_bytes(v, "big")
        if 1 <= t < N:
            return t
        k = hmac.new(k, v + b"\x00", hashlib.sha256).digest()
        v = hmac.new(k, v, hashlib.sha256).digest()


def sign(d, msg_hash, low_s=True):
    z = int.from_bytes(msg_hash, "big") % N
    k = _nonce(d, z)
    R = mul(k, G)
    r = R[0] % N
    s = pow(k, N - 2, N) * (z + r * d) % N
    if low_s and s > N // 2:
        s = N - s
    return r, s


def pubkey_hex(d, compressed=True):
    x, y = mul(d, G)
    if compressed:
        return ("%02x" % (2 + (y & 1))) + x.to_bytes(32, "big").hex()
    return "04" + x.to_bytes(32, "big").hex() + y.to_bytes(32, "big").hex()


def sig_hex(r, s):
    return r.to_bytes(32, "big").hex() + s.to_bytes(32, "big").hex()
