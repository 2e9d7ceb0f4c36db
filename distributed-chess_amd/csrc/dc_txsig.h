// dc_txsig.h -- one transaction's signature check (App::validate_signature,
// core/src/consensus/hotstuff.rs:168-208) as a __host__ __device__ function:
// the body of k_verify_tx (dc_txsig.hip), also compiled into a host unit-test
// binary (tests/cpp/test_secp.cpp) so it is checked against oracle/txsig.py on
// a CPU.
//
//   message = serde_json::to_string(json!({"whitePlayer": W, "blackPlayer": B,
//             "action": [{"x","y"}, {"x","y"}]}))            hotstuff.rs:169-179
//   z       = Sha256(message) as a scalar (mod n)             hotstuff.rs:180-182
//   (r, s)  = hex::decode(signature), parse_standard_slice    hotstuff.rs:183-191
//   Q       = hex::decode(pub_key), PublicKey::parse_slice    hotstuff.rs:193-200
//   verify(z, (r, s), Q)                                      hotstuff.rs:202-207
// and, when the caller passes the game's turn, is_valid_tx's owner check
// (pub_key must be the string of the player to move, hotstuff.rs:141-148).
//
// The JSON bytes are produced one at a time by a small stream state machine
// (templates, the two names with serde_json's escapes, four decimal u32s,
// then the SHA-256 padding) and consumed by one compress call site, so the
// compression code appears once per kernel.
#pragma once
#include "dc_secp.h"

namespace dc {
namespace secp {

enum : u32 {
  SIG_OK = 0,
  SIG_BAD_SIG_HEX = 1,  // hex::decode(tx.signature) failed
  SIG_BAD_SIG = 2,      // Signature::parse_standard_slice failed (length, r or s >= n)
  SIG_BAD_PK_HEX = 3,   // hex::decode(tx.pub_key) failed
  SIG_BAD_PK = 4,       // PublicKey::parse_slice failed
  SIG_INVALID = 5,      // verify() == false: "invalid signature"
  SIG_WRONG_OWNER = 6,  // pub_key is not the player to move: "invalud turn"
};

// ---------------------------------------------------------------- SHA-256
SECP_HD u32 rotr32(u32 x, int n) { return (x >> n) | (x << (32 - n)); }

SECP_HD void sha256_init(u32 (&h)[8]) {
  h[0] = 0x6a09e667u;
  h[1] = 0xbb67ae85u;
  h[2] = 0x3c6ef372u;
  h[3] = 0xa54ff53au;
  h[4] = 0x510e527fu;
  h[5] = 0x9b05688cu;
  h[6] = 0x1f83d9abu;
  h[7] = 0x5be0cd19u;
}

// Byte k of one lane's 64-byte SHA-256 block: byte k & 3 of the block's dword
// k >> 2, dwords `stride` bytes apart.  Host: one contiguous block (stride 4).
// Device: the block's 16 dwords are rows of a [16][threads] LDS array, so the
// 64 lanes of a wave touching the same byte position hit 64 different banks
// (a contiguous 64-byte block per lane put lanes l, l + 4, ... on one bank:
// ~15 conflict cycles per LDS cycle, round 2).
struct BlkRef {
  uint8_t* p;
  u32 stride;
  SECP_HD uint8_t& operator[](u32 k) const { return p[(k >> 2) * stride + (k & 3)]; }
};

SECP_HD void sha256_compress(u32 (&h)[8], const BlkRef& blk) {
  constexpr u32 K[64] = {
      0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
      0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
      0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
      0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
      0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
      0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
      0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
      0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
  u32 w[16];
#pragma unroll
  for (int i = 0; i < 16; ++i)
    w[i] = ((u32)blk[4 * i] << 24) | ((u32)blk[4 * i + 1] << 16) | ((u32)blk[4 * i + 2] << 8) | (u32)blk[4 * i + 3];
  u32 a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], k = h[7];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    if (i >= 16) {
      const u32 w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      const u32 s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
      const u32 s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
      w[i & 15] += s0 + w[(i - 7) & 15] + s1;
    }
    const u32 S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
    const u32 ch = (e & f) ^ (~e & g);
    const u32 t1 = k + S1 + ch + K[i] + w[i & 15];
    const u32 S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
    const u32 mj = (a & b) ^ (a & c) ^ (b & c);
    const u32 t2 = S0 + mj;
    k = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  h[0] += a;
  h[1] += b;
  h[2] += c;
  h[3] += d;
  h[4] += e;
  h[5] += f;
  h[6] += g;
  h[7] += k;
}

// -------------------------------------------------- the signed JSON message
// Stages: 0 T0, 1 white, 2 T1, 3 black, 4 T2, 5 fx, 6 T3, 7 fy, 8 T4, 9 tx,
// 10 T3, 11 ty, 12 T5, 13 end.
struct MsgStream {
  const char* str[2];
  u32 len[2];
  u32 num[4];
  u32 stage, pos;
  u64 pend;  // queued escape bytes (low byte first)
  u32 npend;

  SECP_HD static const char* tpl(u32 stage, u32& n) {
    switch (stage) {
      case 0: n = 16; return "{\"whitePlayer\":\"";
      case 2: n = 17; return "\",\"blackPlayer\":\"";
      case 4: n = 17; return "\",\"action\":[{\"x\":";
      case 6:
      case 10: n = 5; return ",\"y\":";
      case 8: n = 7; return "},{\"x\":";
      default: n = 3; return "}]}";
    }
  }
  SECP_HD static u32 ndigits(u32 v) {
    u32 d = 1;
    while (v >= 10) {
      v /= 10;
      ++d;
    }
    return d;
  }
  // next byte of the message, or -1 at its end
  SECP_HD int next() {
    if (npend) {
      const int c = (int)(pend & 0xFF);
      pend >>= 8;
      --npend;
      return c;
    }
    for (;;) {
      if (stage >= 13) return -1;
      if (stage == 1 || stage == 3) {  // a player name, JSON-escaped (serde_json ESCAPE)
        const bool second = stage == 3;  // selects, not a runtime index: no scratch array
        const u32 ln = second ? len[1] : len[0];
        if (pos < ln) {
          const u32 c = (uint8_t)(second ? str[1] : str[0])[pos++];
          if (c == '"' || c == '\\') {
            pend = c;
            npend = 1;
            return '\\';
          }
          if (c < 0x20) {
            const u32 sh = c == 8 ? 'b' : c == 12 ? 'f' : c == 10 ? 'n' : c == 13 ? 'r' : c == 9 ? 't' : 0u;
            if (sh) {
              pend = sh;
              npend = 1;
            } else {  // \u00XX, lower-case hex
              const char* hx = "0123456789abcdef";
              pend = (u64)'u' | ((u64)'0' << 8) | ((u64)'0' << 16) | ((u64)(uint8_t)hx[c >> 4] << 24) |
                     ((u64)(uint8_t)hx[c & 15] << 32);
              npend = 5;
            }
            return '\\';
          }
          return (int)c;
        }
      } else if (stage == 5 || stage == 7 || stage == 9 || stage == 11) {  // a coordinate
        const u32 v = stage == 5 ? num[0] : stage == 7 ? num[1] : stage == 9 ? num[2] : num[3];
        const u32 nd = ndigits(v);
        if (pos < nd) {
          u32 q = v;
          for (u32 i = pos + 1; i < nd; ++i) q /= 10;
          ++pos;
          return (int)('0' + q % 10);
        }
      } else {
        u32 n;
        const char* t = tpl(stage, n);
        if (pos < n) return (int)(uint8_t)t[pos++];
      }
      ++stage;
      pos = 0;
    }
  }
};

// SHA-256 of the message.  blk: the lane's 64-byte block (LDS on the device).
SECP_HD void message_hash(u32 (&h)[8], const char* white, u32 wl, const char* black, u32 bl, const u32 (&act)[4],
                          const BlkRef& blk) {
  MsgStream ms;
  ms.str[0] = white;
  ms.str[1] = black;
  ms.len[0] = wl;
  ms.len[1] = bl;
#pragma unroll
  for (int i = 0; i < 4; ++i) ms.num[i] = act[i];
  ms.stage = 0;
  ms.pos = 0;
  ms.pend = 0;
  ms.npend = 0;
  sha256_init(h);
  u64 total = 0;
  u32 fill = 0, pad = 0;  // pad: 0 message, 1 zeros, 2 length bytes, 3 done
  for (;;) {
    int c;
    if (pad == 0) {
      c = ms.next();
      if (c < 0) {
        pad = 1;
        c = 0x80;
      } else {
        ++total;
      }
    } else if (pad == 1 && fill != 56) {
      c = 0;
    } else {
      if (pad == 1) pad = 2;
      const u64 bits = total * 8;
      c = (int)((bits >> (8 * (63 - fill))) & 0xFF);
    }
    blk[fill++] = (uint8_t)c;
    if (fill == 64) {
      sha256_compress(h, blk);
      fill = 0;
      if (pad == 2) break;
    }
  }
}

// ------------------------------------------------------------------- hex
SECP_HD int hexval(u32 c) {
  if (c >= '0' && c <= '9') return (int)(c - '0');
  if (c >= 'a' && c <= 'f') return (int)(c - 'a' + 10);
  if (c >= 'A' && c <= 'F') return (int)(c - 'A' + 10);
  return -1;
}
SECP_HD bool hex_ok(const char* s, u32 n) {
  if (n & 1u) return false;
  bool ok = true;
  for (u32 i = 0; i < n; ++i) ok &= hexval((uint8_t)s[i]) >= 0;
  return ok;
}
// 64 hex chars (already validated) -> 256-bit big-endian number as limbs
SECP_HD void hex_limbs(u32 (&r)[8], const char* s) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    u32 v = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) v = (v << 4) | (u32)hexval((uint8_t)s[8 * (7 - i) + k]);
    r[i] = v;
  }
}

// PublicKey::parse_slice(bytes, None) on the hex text (validated, even length)
SECP_HD bool parse_pubkey(Ge& q, const char* s, u32 nchars) {
  const u32 nb = nchars / 2;
  if (nb != 33 && nb != 64 && nb != 65) return false;
  u32 tag = 4, off = 0;
  if (nb != 64) {
    tag = (u32)(hexval((uint8_t)s[0]) << 4 | hexval((uint8_t)s[1]));
    off = 2;
  }
  Fe x;
  hex_limbs(x.v, s + off);
  if (!fe_lt_p(x.v)) return false;
  if (nb == 33) {
    if (tag != 2 && tag != 3) return false;
    return ge_set_xo(q, x, tag == 3);
  }
  if (tag != 4 && tag != 6 && tag != 7) return false;
  Fe y;
  hex_limbs(y.v, s + off + 64);
  if (!fe_lt_p(y.v)) return false;
  if (tag != 4 && ((y.v[0] & 1u) != 0) != (tag == 7)) return false;
  q.x = x;
  q.y = y;
  return ge_on_curve(q);
}

SECP_HD bool str_eq(const char* a, u32 al, const char* b, u32 bl) {
  if (al != bl) return false;
  bool eq = true;
  for (u32 i = 0; i < al; ++i) eq &= a[i] == b[i];
  return eq;
}

// One transaction: the SIG_* verdict.  turn < 0 skips the owner check.
SECP_HD u32 check_tx(const char* white, u32 wl, const char* black, u32 bl, const u32 (&act)[4], const char* sig,
                     u32 sl, const char* pk, u32 pl, int turn, const Ge* gtab, const BlkRef& blk) {
  u32 h[8];
  message_hash(h, white, wl, black, bl, act, blk);
  if (!hex_ok(sig, sl)) return SIG_BAD_SIG_HEX;
  if (sl != 128) return SIG_BAD_SIG;
  Sc r, s;
  hex_limbs(r.v, sig);
  hex_limbs(s.v, sig + 64);
  if (sc_ge_n(r.v) || sc_ge_n(s.v)) return SIG_BAD_SIG;
  if (!hex_ok(pk, pl)) return SIG_BAD_PK_HEX;
  Ge q;
  if (!parse_pubkey(q, pk, pl)) return SIG_BAD_PK;
  // Message::parse_slice: the digest as a scalar, reduced mod n
  u32 zl[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) zl[i] = h[7 - i];
  Sc z;
  sc_canon(z, zl);
  if (!ecdsa_verify(r, s, z, q, gtab)) return SIG_INVALID;
  if (turn >= 0) {
    const bool own = turn == 0 ? str_eq(pk, pl, white, wl) : str_eq(pk, pl, black, bl);
    if (!own) return SIG_WRONG_OWNER;
  }
  return SIG_OK;
}

// gtab[256 i + j] = j 2^(8 i) G (j = 0: zero, unused)
SECP_HD void gtab_entry(Ge& out, int i, int j) {
  if (j == 0) {
    set_zero(out.x.v);
    set_zero(out.y.v);
    return;
  }
  Ge g;
  ge_generator(g);
  Gej b;
  gej_set_ge(b, g);
  for (int k = 0; k < 8 * i; ++k) gej_double(b, b);
  Gej acc;
  gej_set_inf(acc);
  for (int bit = 7; bit >= 0; --bit) {
    gej_double(acc, acc);
    if ((j >> bit) & 1) {
      Gej t;
      gej_add(t, acc, b);
      acc = t;
    }
  }
  gej_to_ge(out, acc);
}

}  // namespace secp
}  // namespace dc
