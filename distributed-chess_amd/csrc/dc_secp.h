// dc_secp.h -- secp256k1 field, scalar and point arithmetic for the batched
// transaction-signature check (k_verify_tx, dc_txsig.hip).
//
// What it restates: libsecp256k1 0.7.1 (core/Cargo.lock), as called by
// App::validate_signature (core/src/consensus/hotstuff.rs:168-208):
//   field  F_p, p = 2^256 - 2^32 - 977       (2^256 = 2^32 + 977 mod p)
//   scalar Z_n, n = 2^256 - C, C = 0x14551231950B75FC4402DA1732FC9BEBF
//   curve  y^2 = x^3 + 7, generator G
//
// Representation for a 32-bit VALU: 8 little-endian u32 limbs, always
// canonical (< p resp. < n) after every operation, so equality is limb
// equality and parity is bit 0.  Products are operand-scanned with 64-bit
// multiply-adds (v_mad_u64_u32: a*b + c + d never overflows 64 bits) and
// folded with the special form of p (one 977-multiply pass plus a shifted
// add) or of n (four passes of the 129-bit C).
//
// Every function is __host__ __device__: the same code runs in the gfx950
// kernel and in a host unit-test binary (tests/cpp/test_secp.cpp) that checks
// it against oracle/txsig.py on the CPU of this container.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#define SECP_HD __host__ __device__ __forceinline__

namespace dc {
namespace secp {

typedef uint32_t u32;
typedef uint64_t u64;

struct Fe {
  u32 v[8];
};
struct Sc {
  u32 v[8];
};
struct Ge {  // affine point (never the point at infinity)
  Fe x, y;
};
struct Gej {  // Jacobian point: (X / Z^2, Y / Z^3), or infinity
  Fe x, y, z;
  u32 inf;
};

// ------------------------------------------------------------------ limbs
SECP_HD void set_zero(u32 (&a)[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = 0;
}
SECP_HD bool is_zero8(const u32 (&a)[8]) {
  u32 o = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) o |= a[i];
  return o == 0;
}
SECP_HD bool eq8(const u32 (&a)[8], const u32 (&b)[8]) {
  u32 o = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) o |= a[i] ^ b[i];
  return o == 0;
}
SECP_HD void sel8(u32 (&r)[8], bool c, const u32 (&a)[8], const u32 (&b)[8]) {  // r = c ? a : b
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = c ? a[i] : b[i];
}
// 32 big-endian bytes -> limbs (no reduction)
SECP_HD void from_be32(u32 (&r)[8], const uint8_t* b) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint8_t* q = b + 28 - 4 * i;
    r[i] = ((u32)q[0] << 24) | ((u32)q[1] << 16) | ((u32)q[2] << 8) | (u32)q[3];
  }
}
SECP_HD void to_be32(const u32 (&a)[8], uint8_t* b) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint8_t* q = b + 28 - 4 * i;
    q[0] = (uint8_t)(a[i] >> 24);
    q[1] = (uint8_t)(a[i] >> 16);
    q[2] = (uint8_t)(a[i] >> 8);
    q[3] = (uint8_t)a[i];
  }
}

// ------------------------------------------------------------- field F_p
constexpr u32 kP977 = 977u;

// 32-bit add/subtract with carry: v_add_co / v_addc_co chains on the device
// (a u64 formulation costs a zero-extension v_mov per limb).
SECP_HD u32 addc32(u32 x, u32 y, u32 cin, u32* cout) {
#if defined(__clang__)
  return __builtin_addc(x, y, cin, cout);
#else
  const u64 d = (u64)x + y + cin;
  *cout = (u32)(d >> 32);
  return (u32)d;
#endif
}
SECP_HD u32 subb32(u32 x, u32 y, u32 bin, u32* bout) {
#if defined(__clang__)
  return __builtin_subc(x, y, bin, bout);
#else
  const u64 d = (u64)x - y - bin;
  *bout = (u32)(d >> 63);
  return (u32)d;
#endif
}

// r = a + (2^32 + 977) mod 2^256; returns the carry out (1 iff a >= p).
SECP_HD u32 add_k(u32 (&r)[8], const u32 (&a)[8]) {
  u32 c;
  r[0] = addc32(a[0], kP977, 0u, &c);
  r[1] = addc32(a[1], 1u, c, &c);
#pragma unroll
  for (int i = 2; i < 8; ++i) r[i] = addc32(a[i], 0u, c, &c);
  return c;
}

SECP_HD bool fe_lt_p(const u32 (&a)[8]) {
  u32 t[8];
  return add_k(t, a) == 0;
}

// a (< 2^256) -> a mod p (one conditional subtraction suffices: a < 2p)
SECP_HD void fe_canon(Fe& r, const u32 (&a)[8]) {
  u32 t[8];
  const u32 ge = add_k(t, a);
  sel8(r.v, ge != 0, t, a);
}

SECP_HD void fe_set_u32(Fe& r, u32 x) {
  set_zero(r.v);
  r.v[0] = x;
}

SECP_HD void fe_add(Fe& r, const Fe& a, const Fe& b) {
  u32 s[8], t[8], c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s[i] = addc32(a.v[i], b.v[i], c, &c);
  // a + b < 2p: if it overflowed 2^256 or s >= p, the result is s + (2^256 - p)
  const u32 d = add_k(t, s);
  sel8(r.v, (c | d) != 0, t, s);
}

SECP_HD void fe_sub(Fe& r, const Fe& a, const Fe& b) {
  u32 s[8], br = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s[i] = subb32(a.v[i], b.v[i], br, &br);
  // borrow: add p, i.e. subtract 2^32 + 977 modulo 2^256
  u32 b2;
  r.v[0] = subb32(s[0], br * kP977, 0u, &b2);
  r.v[1] = subb32(s[1], br, b2, &b2);
#pragma unroll
  for (int i = 2; i < 8; ++i) r.v[i] = subb32(s[i], 0u, b2, &b2);
}

SECP_HD void fe_neg(Fe& r, const Fe& a) {
  Fe z;
  set_zero(z.v);
  fe_sub(r, z, a);
}

#if defined(__HIP_DEVICE_COMPILE__)
// gfx950: acc (64 bits) += a * b, the carry out of bit 64 added into hi.  The
// carry comes from v_mad_u64_u32's VOP3b carry-out (an SGPR lane mask), which C
// cannot name: 2 VALU per partial product, where the operand-scanned C form
// costs ~6 (the u64 zero extensions are v_mov; tools/ubench/mul_rate.hip).
__device__ __forceinline__ void mac_c(u64& acc, u32& hi, u32 a, u32 b) {
  u64 cc;
  asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32_e64 %2, %1, %2, 0, %1"
      : "+v"(acc), "=&s"(cc), "+v"(hi)
      : "v"(a), "v"(b));
}
// acc + x (no carry out of bit 64 possible at the call sites): one v_mad_u64_u32
// by 1 instead of a zero-extension v_mov plus a 64-bit add.
__device__ __forceinline__ u64 mad1(u64 acc, u32 x) {
  u64 cc;
  asm("v_mad_u64_u32 %0, %1, %2, 1, %0" : "+v"(acc), "=s"(cc) : "v"(x));
  return acc;
}
#endif

// 512-bit product a * b.  Device: product scanning (Comba) on a 96-bit column
// accumulator; host: operand scanning (each step a*b + t + c < 2^64).
SECP_HD void mul_wide(u32 (&t)[16], const u32 (&a)[8], const u32 (&b)[8]) {
#if defined(__HIP_DEVICE_COMPILE__)
  u64 acc = 0;
#pragma unroll
  for (int k = 0; k < 15; ++k) {
    u32 hi = 0;
#pragma unroll
    for (int i = (k < 8 ? 0 : k - 7); i <= (k < 8 ? k : 7); ++i) mac_c(acc, hi, a[i], b[k - i]);
    t[k] = (u32)acc;
    acc = (acc >> 32) | ((u64)hi << 32);
  }
  t[15] = (u32)acc;
#else
#pragma unroll
  for (int i = 0; i < 16; ++i) t[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    u64 c = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const u64 x = (u64)a[i] * b[j] + t[i + j] + c;
      t[i + j] = (u32)x;
      c = x >> 32;
    }
    t[i + 8] = (u32)c;
  }
#endif
}

// 512-bit square.  Device: Comba with each cross product accumulated twice
// (no 97-bit doubling step); host: cross products once, doubled, plus the diagonal.
SECP_HD void sqr_wide(u32 (&t)[16], const u32 (&a)[8]) {
#if defined(__HIP_DEVICE_COMPILE__)
  u64 acc = 0;
#pragma unroll
  for (int k = 0; k < 15; ++k) {
    u32 hi = 0;
#pragma unroll
    for (int i = (k < 8 ? 0 : k - 7); 2 * i < k; ++i) {
      mac_c(acc, hi, a[i], a[k - i]);
      mac_c(acc, hi, a[i], a[k - i]);
    }
    if ((k & 1) == 0) mac_c(acc, hi, a[k >> 1], a[k >> 1]);
    t[k] = (u32)acc;
    acc = (acc >> 32) | ((u64)hi << 32);
  }
  t[15] = (u32)acc;
  return;
#endif
#pragma unroll
  for (int i = 0; i < 16; ++i) t[i] = 0;
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    u64 c = 0;
#pragma unroll
    for (int j = i + 1; j < 8; ++j) {
      const u64 x = (u64)a[i] * a[j] + t[i + j] + c;
      t[i + j] = (u32)x;
      c = x >> 32;
    }
    t[i + 8] = (u32)c;
  }
  // double the cross products
  u32 hi = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const u32 x = t[i];
    t[i] = (x << 1) | hi;
    hi = x >> 31;
  }
  // add the squares a[i]^2 at limb 2i
  u64 c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const u64 sq = (u64)a[i] * a[i];
    c += (u64)t[2 * i] + (u32)sq;
    t[2 * i] = (u32)c;
    c >>= 32;
    c += (u64)t[2 * i + 1] + (u32)(sq >> 32);
    t[2 * i + 1] = (u32)c;
    c >>= 32;
  }
}

// t (< 2^512) mod p: t = H 2^256 + L = L + 977 H + (H << 32) (mod p), twice.
SECP_HD void fe_reduce(Fe& r, const u32 (&t)[16]) {
  u32 s[8];
  u64 c = 0;
#if defined(__HIP_DEVICE_COMPILE__)
  // each 32-bit addend is one v_mad_u64_u32 by 1 into the 64-bit column (< 2^43)
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    c = (u64)t[8 + k] * kP977 + c;
    c = mad1(c, t[k]);
    if (k > 0) c = mad1(c, t[7 + k]);
    s[k] = (u32)c;
    c >>= 32;
  }
  const u64 top = mad1(c, t[15]);  // < 2^34
#else
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    u64 x = (u64)t[8 + k] * kP977 + t[k] + c;
    if (k > 0) x += t[7 + k];
    s[k] = (u32)x;
    c = x >> 32;
  }
  const u64 top = c + t[15];  // < 2^34
#endif
  // + top (2^32 + 977): two carry chains; the sum is < 2^256 + 2^67, so a
  // carry out leaves s < 2^67 and one more (2^32 + 977) cannot overflow
  const u64 m = top * kP977;
  u32 c1, c2;
  s[0] = addc32(s[0], (u32)m, 0u, &c1);
  s[1] = addc32(s[1], (u32)(m >> 32), c1, &c1);
  s[1] = addc32(s[1], (u32)top, 0u, &c2);
  s[2] = addc32(s[2], (u32)(top >> 32), c2, &c2);
  s[2] = addc32(s[2], 0u, c1, &c1);
#pragma unroll
  for (int k = 3; k < 8; ++k) {
    s[k] = addc32(s[k], 0u, c1, &c1);
    s[k] = addc32(s[k], 0u, c2, &c2);
  }
  const u32 w = c1 + c2;
  s[0] = addc32(s[0], w * kP977, 0u, &c1);
  s[1] = addc32(s[1], w, c1, &c1);
  s[2] = addc32(s[2], 0u, c1, &c1);
  s[3] = addc32(s[3], 0u, c1, &c1);
  fe_canon(r, s);
}

SECP_HD void fe_mul(Fe& r, const Fe& a, const Fe& b) {
  u32 t[16];
  mul_wide(t, a.v, b.v);
  fe_reduce(r, t);
}
SECP_HD void fe_sqr(Fe& r, const Fe& a) {
  u32 t[16];
  sqr_wide(t, a.v);
  fe_reduce(r, t);
}
SECP_HD void fe_sqr_n(Fe& r, const Fe& a, int n) {
  r = a;
  for (int i = 0; i < n; ++i) fe_sqr(r, r);
}

// a^((p+1)/4): libsecp256k1's addition chain (x2 .. x223 blocks of ones).
// r^2 == a iff a is a quadratic residue.
SECP_HD void fe_pow_sqrt(Fe& r, const Fe& a) {
  Fe x2, x3, x6, x9, x11, x22, x44, x88, x176, x220, x223, t;
  fe_sqr(x2, a);
  fe_mul(x2, x2, a);
  fe_sqr(x3, x2);
  fe_mul(x3, x3, a);
  fe_sqr_n(x6, x3, 3);
  fe_mul(x6, x6, x3);
  fe_sqr_n(x9, x6, 3);
  fe_mul(x9, x9, x3);
  fe_sqr_n(x11, x9, 2);
  fe_mul(x11, x11, x2);
  fe_sqr_n(x22, x11, 11);
  fe_mul(x22, x22, x11);
  fe_sqr_n(x44, x22, 22);
  fe_mul(x44, x44, x22);
  fe_sqr_n(x88, x44, 44);
  fe_mul(x88, x88, x44);
  fe_sqr_n(x176, x88, 88);
  fe_mul(x176, x176, x88);
  fe_sqr_n(x220, x176, 44);
  fe_mul(x220, x220, x44);
  fe_sqr_n(x223, x220, 3);
  fe_mul(x223, x223, x3);
  fe_sqr_n(t, x223, 23);
  fe_mul(t, t, x22);
  fe_sqr_n(t, t, 6);
  fe_mul(t, t, x2);
  fe_sqr(t, t);
  fe_sqr(r, t);
}

// a^(p-2) = a^-1 (a != 0): the same chain with the inverse's tail.
SECP_HD void fe_inv(Fe& r, const Fe& a) {
  Fe x2, x3, x6, x9, x11, x22, x44, x88, x176, x220, x223, t;
  fe_sqr(x2, a);
  fe_mul(x2, x2, a);
  fe_sqr(x3, x2);
  fe_mul(x3, x3, a);
  fe_sqr_n(x6, x3, 3);
  fe_mul(x6, x6, x3);
  fe_sqr_n(x9, x6, 3);
  fe_mul(x9, x9, x3);
  fe_sqr_n(x11, x9, 2);
  fe_mul(x11, x11, x2);
  fe_sqr_n(x22, x11, 11);
  fe_mul(x22, x22, x11);
  fe_sqr_n(x44, x22, 22);
  fe_mul(x44, x44, x22);
  fe_sqr_n(x88, x44, 44);
  fe_mul(x88, x88, x44);
  fe_sqr_n(x176, x88, 88);
  fe_mul(x176, x176, x88);
  fe_sqr_n(x220, x176, 44);
  fe_mul(x220, x220, x44);
  fe_sqr_n(x223, x220, 3);
  fe_mul(x223, x223, x3);
  fe_sqr_n(t, x223, 23);
  fe_mul(t, t, x22);
  fe_sqr_n(t, t, 5);
  fe_mul(t, t, a);
  fe_sqr_n(t, t, 3);
  fe_mul(t, t, x2);
  fe_sqr_n(t, t, 2);
  fe_mul(r, t, a);
}

// ---------------------------------------------------------- scalars Z_n
// C = 2^256 - n (129 bits)
SECP_HD u32 kC(int j) {
  return j == 0 ? 0x2FC9BEBFu : j == 1 ? 0x402DA173u : j == 2 ? 0x50B75FC4u : j == 3 ? 0x45512319u : 1u;
}

// r = a + C mod 2^256; returns the carry out (1 iff a >= n)
SECP_HD u32 add_c(u32 (&r)[8], const u32 (&a)[8]) {
  u32 c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = addc32(a[i], i < 5 ? kC(i) : 0u, c, &c);
  return c;
}

SECP_HD bool sc_ge_n(const u32 (&a)[8]) {
  u32 t[8];
  return add_c(t, a) != 0;
}

// a (< 2^256) -> a mod n
SECP_HD void sc_canon(Sc& r, const u32 (&a)[8]) {
  u32 t[8];
  const u32 ge = add_c(t, a);
  sel8(r.v, ge != 0, t, a);
}

// out = in[0..8) + in[8..NI) * C  (NO limbs; the caller's bound keeps it in range)
template <int NI, int NO>
SECP_HD void sc_fold(const u32 (&in)[NI], u32 (&out)[NO]) {
#if defined(__HIP_DEVICE_COMPILE__)
  // product scanning on the 96-bit column accumulator (mac_c), as mul_wide
  u64 acc = 0;
#pragma unroll
  for (int k = 0; k < NO; ++k) {
    u32 hi = 0;
    if (k < 8) acc = mad1(acc, in[k]);
#pragma unroll
    for (int i = 0; i < NI - 8; ++i) {
      const int j = k - i;
      if (j >= 0 && j < 5) mac_c(acc, hi, in[8 + i], kC(j));
    }
    out[k] = (u32)acc;
    acc = (acc >> 32) | ((u64)hi << 32);
  }
  return;
#endif
#pragma unroll
  for (int i = 0; i < NO; ++i) out[i] = i < 8 ? in[i] : 0u;
#pragma unroll
  for (int i = 0; i < NI - 8; ++i) {
    u64 c = 0;
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      if (i + j < NO) {
        const u64 x = (u64)in[8 + i] * kC(j) + out[i + j] + c;
        out[i + j] = (u32)x;
        c = x >> 32;
      }
    }
#pragma unroll
    for (int k = i + 5; k < NO; ++k) {
      const u64 x = (u64)out[k] + c;
      out[k] = (u32)x;
      c = x >> 32;
    }
  }
}

SECP_HD void sc_reduce(Sc& r, const u32 (&t)[16]) {
  u32 a[13], b[9], c[9], d[9];
  sc_fold<16, 13>(t, a);  // < 2^256 + 2^385
  sc_fold<13, 9>(a, b);   // < 2^256 + 2^259
  sc_fold<9, 9>(b, c);    // < 2^256 + 2^133
  sc_fold<9, 9>(c, d);    // < 2^256
  u32 e[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) e[i] = d[i];
  sc_canon(r, e);
}

SECP_HD void sc_mul(Sc& r, const Sc& a, const Sc& b) {
  u32 t[16];
  mul_wide(t, a.v, b.v);
  sc_reduce(r, t);
}

// a^(n-2) = a^-1 (a != 0): left-to-right sliding 4-bit windows over the
// constant exponent, odd powers a, a^3, .., a^15 precomputed: 252 squarings +
// 57 multiplications (the binary method takes 254 + 127).  kInvSched holds
// (squarings, odd-power index) per window after the first (a^15); generated
// from n - 2 and checked against pow(a, n - 2, n) by test_host_field_scalar_ops.
SECP_HD void sc_inv(Sc& r, const Sc& a) {
  constexpr int kWin = 57;
  constexpr uint8_t kInvSched[2 * kWin] = {4, 7, 4, 7, 4, 7, 4, 7, 4, 7, 4, 7, 4, 7, 4, 7, 4, 7, 4, 7, 4, 7, 4, 7, 4, 7, 4, 7, 4, 7, 4, 7, 4, 7, 4, 7, 4, 7, 4, 7, 4, 7, 4, 7, 4, 7, 4, 7, 4, 7, 4, 7, 4, 7, 4, 7, 4, 7, 4, 7, 3, 3, 5, 5, 3, 2, 4, 2, 4, 3, 5, 6, 2, 1, 5, 3, 6, 6, 5, 5, 4, 6, 3, 0, 6, 2, 10, 3, 4, 3, 5, 7, 4, 7, 5, 4, 6, 5, 4, 6, 5, 1, 6, 6, 10, 6, 4, 4, 9, 4, 4, 7, 1, 0};
  Sc tbl[8], a2;
  tbl[0] = a;
  {
    u32 t[16];
    sqr_wide(t, a.v);
    sc_reduce(a2, t);
  }
#pragma unroll
  for (int i = 1; i < 8; ++i) sc_mul(tbl[i], tbl[i - 1], a2);
  Sc x = tbl[7];
  for (int k = 0; k < kWin; ++k) {
    for (int q = 0; q < kInvSched[2 * k]; ++q) {
      u32 t[16];
      sqr_wide(t, x.v);
      sc_reduce(x, t);
    }
    // the odd power by select over the 8 entries, not by a runtime index:
    // an indexed Sc[8] lives in scratch (round 2: part of 992 B/lane)
    const int j = kInvSched[2 * k + 1];
    Sc m = tbl[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) sel8(m.v, j == i, tbl[i].v, m.v);
    sc_mul(x, x, m);
  }
  r = x;
}

// (a + b) mod n
SECP_HD void sc_add(Sc& r, const Sc& a, const Sc& b) {
  u32 s[8], t[8], c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s[i] = addc32(a.v[i], b.v[i], c, &c);
  const u32 d = add_c(t, s);
  sel8(r.v, (c | d) != 0, t, s);
}

// ---------------------------------------------------- GLV endomorphism
// lambda (Q.x, Q.y) = (beta Q.x, Q.y) with lambda^3 = 1 mod n, beta^3 = 1 mod p.
// libsecp256k1's scalar_split_lambda: k = r1 + lambda r2 (mod n) with
// |r1|, |r2| < 2^128, from c_i = round(k g_i / 2^384) and the short lattice
// basis (b1, b2).  Constants checked in tests/test_txsig.py
// (test_glv_constants): lambda^3 = 1, beta^3 = 1, lambda G = (beta Gx, Gy),
// g_i = round(2^384 b_i / n).
SECP_HD void fe_beta(Fe& r) {
  const u32 b[8] = {0x719501EEu, 0xC1396C28u, 0x12F58995u, 0x9CF04975u, 0xAC3434E9u, 0x6E64479Eu, 0x657C0710u, 0x7AE96A2Bu};
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = b[i];
}

// round(k g / 2^384) (< 2^128 + 1)
SECP_HD void sc_mul_shift384(Sc& r, const Sc& k, const u32 (&g)[8]) {
  u32 t[16];
  mul_wide(t, k.v, g);
  u32 c = t[11] >> 31;
#pragma unroll
  for (int i = 0; i < 4; ++i) r.v[i] = addc32(t[12 + i], 0u, c, &c);
  r.v[4] = c;
  r.v[5] = r.v[6] = r.v[7] = 0;
}

SECP_HD void sc_split_lambda(Sc& r1, Sc& r2, const Sc& k) {
  const u32 g1[8] = {0x45DBB031u, 0xE893209Au, 0x71E8CA7Fu, 0x3DAA8A14u, 0x9284EB15u, 0xE86C90E4u, 0xA7D46BCDu, 0x3086D221u};
  const u32 g2[8] = {0x8AC47F71u, 0x1571B4AEu, 0x9DF506C6u, 0x221208ACu, 0x0ABFE4C4u, 0x6F547FA9u, 0x010E8828u, 0xE4437ED6u};
  Sc mb1, mb2, ml, c1, c2;
  const u32 vb1[8] = {0x0ABFE4C3u, 0x6F547FA9u, 0x010E8828u, 0xE4437ED6u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u};
  const u32 vb2[8] = {0x3DB1562Cu, 0xD765CDA8u, 0x0774346Du, 0x8A280AC5u, 0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
  const u32 vml[8] = {0xB51283CFu, 0xE0CFC810u, 0x8EC739C2u, 0xA880B9FCu, 0x77ED9BA4u, 0x5AD9E3FDu, 0x3FA3CF1Fu, 0xAC9C52B3u};
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    mb1.v[i] = vb1[i];
    mb2.v[i] = vb2[i];
    ml.v[i] = vml[i];
  }
  sc_mul_shift384(c1, k, g1);
  sc_mul_shift384(c2, k, g2);
  sc_mul(c1, c1, mb1);
  sc_mul(c2, c2, mb2);
  sc_add(r2, c1, c2);
  sc_mul(r1, r2, ml);
  sc_add(r1, r1, k);
}

// r (mod n) with |r| < 2^128 as sign + 128-bit magnitude (limbs 0..3)
SECP_HD bool sc_signed128(u32 (&m)[4], const Sc& r) {
  const bool neg = (r.v[4] | r.v[5] | r.v[6] | r.v[7]) != 0;
  const u32 nl[4] = {0xD0364141u, 0xBFD25E8Cu, 0xAF48A03Bu, 0xBAAEDCE6u};
  u32 b = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const u32 d = subb32(nl[i], r.v[i], b, &b);  // n - r (its high limbs cancel)
    m[i] = neg ? d : r.v[i];
  }
  return neg;
}

// ------------------------------------------------------------------ points
SECP_HD void gej_set_ge(Gej& r, const Ge& a) {
  r.x = a.x;
  r.y = a.y;
  fe_set_u32(r.z, 1);
  r.inf = 0;
}

SECP_HD void gej_set_inf(Gej& r) {
  set_zero(r.x.v);
  set_zero(r.y.v);
  set_zero(r.z.v);
  r.inf = 1;
}

// 2a  (dbl-2009-l, a = 0: 2M + 5S).  y = 0 cannot occur on secp256k1.
SECP_HD void gej_double(Gej& r, const Gej& a) {
  Fe A, B, C, D, E, F, t;
  fe_sqr(A, a.x);
  fe_sqr(B, a.y);
  fe_sqr(C, B);
  fe_add(t, a.x, B);
  fe_sqr(t, t);
  fe_sub(t, t, A);
  fe_sub(t, t, C);
  fe_add(D, t, t);
  fe_add(E, A, A);
  fe_add(E, E, A);
  fe_sqr(F, E);
  Fe z3;
  fe_mul(z3, a.y, a.z);
  fe_add(r.z, z3, z3);
  fe_sub(t, F, D);
  fe_sub(r.x, t, D);
  fe_sub(t, D, r.x);
  fe_mul(t, E, t);
  fe_add(C, C, C);
  fe_add(C, C, C);
  fe_add(C, C, C);
  fe_sub(r.y, t, C);
  r.inf = a.inf;
}

// a + b, b affine  (madd-2007-bl: 7M + 4S); every special case handled.
SECP_HD void gej_add_ge(Gej& r, const Gej& a, const Ge& b) {
  if (a.inf) {
    gej_set_ge(r, b);
    return;
  }
  Fe z1z1, u2, s2, h, hh, i4, j, rr, v, t;
  fe_sqr(z1z1, a.z);
  fe_mul(u2, b.x, z1z1);
  fe_mul(s2, b.y, a.z);
  fe_mul(s2, s2, z1z1);
  fe_sub(h, u2, a.x);
  fe_sub(rr, s2, a.y);
  if (is_zero8(h.v)) {  // same x: doubling or the point at infinity (rare: branch)
    if (is_zero8(rr.v)) gej_double(r, a);
    else gej_set_inf(r);
    return;
  }
  fe_add(rr, rr, rr);
  fe_sqr(hh, h);
  fe_add(i4, hh, hh);
  fe_add(i4, i4, i4);
  fe_mul(j, h, i4);
  fe_mul(v, a.x, i4);
  Fe x3, y3, z3;
  fe_sqr(x3, rr);
  fe_sub(x3, x3, j);
  fe_sub(x3, x3, v);
  fe_sub(x3, x3, v);
  fe_sub(t, v, x3);
  fe_mul(y3, rr, t);
  fe_mul(t, a.y, j);
  fe_add(t, t, t);
  fe_sub(y3, y3, t);
  fe_add(z3, a.z, h);
  fe_sqr(z3, z3);
  fe_sub(z3, z3, z1z1);
  fe_sub(z3, z3, hh);
  r.x = x3;
  r.y = y3;
  r.z = z3;
  r.inf = 0;
}

// a + b, both Jacobian  (add-2007-bl: 11M + 5S); every special case handled.
SECP_HD void gej_add(Gej& r, const Gej& a, const Gej& b) {
  if (a.inf) {
    r = b;
    return;
  }
  if (b.inf) {
    r = a;
    return;
  }
  Fe z1z1, z2z2, u1, u2, s1, s2, h, i, j, rr, v, t;
  fe_sqr(z1z1, a.z);
  fe_sqr(z2z2, b.z);
  fe_mul(u1, a.x, z2z2);
  fe_mul(u2, b.x, z1z1);
  fe_mul(s1, a.y, b.z);
  fe_mul(s1, s1, z2z2);
  fe_mul(s2, b.y, a.z);
  fe_mul(s2, s2, z1z1);
  fe_sub(h, u2, u1);
  fe_sub(rr, s2, s1);
  if (is_zero8(h.v)) {
    if (is_zero8(rr.v)) gej_double(r, a);
    else gej_set_inf(r);
    return;
  }
  fe_add(rr, rr, rr);
  fe_add(i, h, h);
  fe_sqr(i, i);
  fe_mul(j, h, i);
  fe_mul(v, u1, i);
  Fe x3, y3, z3;
  fe_sqr(x3, rr);
  fe_sub(x3, x3, j);
  fe_sub(x3, x3, v);
  fe_sub(x3, x3, v);
  fe_sub(t, v, x3);
  fe_mul(y3, rr, t);
  fe_mul(t, s1, j);
  fe_add(t, t, t);
  fe_sub(y3, y3, t);
  fe_add(z3, a.z, b.z);
  fe_sqr(z3, z3);
  fe_sub(z3, z3, z1z1);
  fe_sub(z3, z3, z2z2);
  fe_mul(z3, z3, h);
  r.x = x3;
  r.y = y3;
  r.z = z3;
  r.inf = 0;
}

SECP_HD void gej_to_ge(Ge& r, const Gej& a) {  // a not at infinity
  Fe zi, zi2, zi3;
  fe_inv(zi, a.z);
  fe_sqr(zi2, zi);
  fe_mul(zi3, zi2, zi);
  fe_mul(r.x, a.x, zi2);
  fe_mul(r.y, a.y, zi3);
}

SECP_HD void ge_generator(Ge& g) {
  const u32 gx[8] = {0x16F81798u, 0x59F2815Bu, 0x2DCE28D9u, 0x029BFCDBu,
                     0xCE870B07u, 0x55A06295u, 0xF9DCBBACu, 0x79BE667Eu};
  const u32 gy[8] = {0xFB10D4B8u, 0x9C47D08Fu, 0xA6855419u, 0xFD17B448u,
                     0x0E1108A8u, 0x5DA4FBFCu, 0x26A3C465u, 0x483ADA77u};
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    g.x.v[i] = gx[i];
    g.y.v[i] = gy[i];
  }
}

// y^2 == x^3 + 7
SECP_HD bool ge_on_curve(const Ge& a) {
  Fe l, r, seven;
  fe_sqr(l, a.y);
  fe_sqr(r, a.x);
  fe_mul(r, r, a.x);
  fe_set_u32(seven, 7);
  fe_add(r, r, seven);
  return eq8(l.v, r.v);
}

// Compressed-key decompression: y with parity `odd` for x; false if x^3 + 7
// has no square root (libsecp256k1 set_xo_var).
SECP_HD bool ge_set_xo(Ge& r, const Fe& x, bool odd) {
  Fe c, seven, y, y2;
  fe_sqr(c, x);
  fe_mul(c, c, x);
  fe_set_u32(seven, 7);
  fe_add(c, c, seven);
  fe_pow_sqrt(y, c);
  fe_sqr(y2, y);
  if (!eq8(y2.v, c.v)) return false;
  if (((y.v[0] & 1u) != 0) != odd) fe_neg(y, y);
  r.x = x;
  r.y = y;
  return true;
}

// The G table: gtab[256 i + j] = j 2^(8 i) G (affine; j = 0 unused), so
// u G = sum over the 32 bytes b_i of u of gtab[256 i + b_i] -- 32 mixed
// additions and no doublings.
constexpr int kGTabRows = 32;
constexpr int kGTabEntries = kGTabRows * 256;

// u1 G + u2 Q.  Q part: GLV (u2 = k1 + lambda k2, |k_i| < 2^128), signed
// radix-2^W Booth digits in [-2^(W-1), 2^(W-1)] over a table of Q's first
// K = 2^(W-1) multiples, lambda applied per lookup as beta x.  The table is
// made affine with one batch inversion (Montgomery's trick) so every Q
// addition is a mixed one (7M + 4S instead of 11M + 5S), and it is read by a
// select over all K entries (v_cndmask), never by a per-lane index: a
// per-lane-indexed table lives in scratch (round 1: 8 Jacobian entries,
// 848 B/lane, 13 GB of HBM traffic per 262k-transaction launch).
// W = 3: 4 entries (64 VGPRs), 43 windows x 2 halves; W = 4: 8 entries (128 VGPRs),
// 33 windows.  G part: the byte table (32 mixed additions, no doublings).
#ifndef DC_SECP_QW
#define DC_SECP_QW 3
#endif
constexpr int kQWindow = DC_SECP_QW;

// bits [pos, pos + len) of the 128-bit magnitude m (zero beyond bit 127)
// (limbs picked by select: a runtime index would put m in scratch)
SECP_HD u32 pick4(const u32 (&m)[4], int i) { return i == 0 ? m[0] : i == 1 ? m[1] : i == 2 ? m[2] : i == 3 ? m[3] : 0u; }
SECP_HD u32 bits128(const u32 (&m)[4], int pos, int len) {
  const int i = pos >> 5, s = pos & 31;
  u32 v = pick4(m, i) >> s;
  if (s + len > 32) v |= pick4(m, i + 1) << (32 - s);
  return v & ((1u << len) - 1u);
}

// radix-2^W Booth digit w of m: d_w = b[Ww..Ww+W-1] + b[Ww-1] - 2^W b[Ww+W-1]
template <int W>
SECP_HD int booth_digit(const u32 (&m)[4], int w) {
  const u32 lo = bits128(m, W * w, W);
  const u32 below = w > 0 ? bits128(m, W * w - 1, 1) : 0u;
  return (int)(lo + below) - (int)((lo >> (W - 1)) << W);
}

// f(integral_constant<int, I>) for I = B, B + S, ... while I != E: a loop whose
// index is a compile-time constant in every iteration.  `#pragma unroll` did
// not unroll the table build (gej_add_ge's special-case branches): X/Y/Z, the
// prefix products and the table were then indexed by an SGPR and lived in
// scratch (992 B/lane, most of k_verify_tx's HBM traffic).
template <int B, int E, int S = 1, class F>
SECP_HD void static_for(F&& f) {
  if constexpr (B != E) {
    f(std::integral_constant<int, B>{});
    static_for<B + S, E, S>(f);
  }
}

template <int W>
SECP_HD void ecmult_w(Gej& r, const Ge& q, const Sc& u2, const Sc& u1, const Ge* gtab) {
  constexpr int K = 1 << (W - 1);
  constexpr int NW = (129 + W - 1) / W;  // windows: |k| < 2^128 plus the Booth sign bit
  Sc k1, k2;
  sc_split_lambda(k1, k2, u2);
  u32 m1[4], m2[4];
  const bool n1 = sc_signed128(m1, k1), n2 = sc_signed128(m2, k2);
  // (i + 1) Q, i < K, Jacobian (none is infinity: Q has order n), then affine
  Ge tab[K];
  {
    Fe X[K], Y[K], Z[K];
    Gej a, t;
    gej_set_ge(a, q);
    X[0] = a.x;
    Y[0] = a.y;
    Z[0] = a.z;
    if (K > 1) {
      gej_double(t, a);
      X[1] = t.x;
      Y[1] = t.y;
      Z[1] = t.z;
    }
    static_for<2, K>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      gej_add_ge(a, t, q);
      X[i] = a.x;
      Y[i] = a.y;
      Z[i] = a.z;
      t = a;
    });
    // batch inversion of Z[0..K): prefix products, one inversion, back-substitution
    Fe c[K];
    c[0] = Z[0];
    static_for<1, K>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      fe_mul(c[i], c[i - 1], Z[i]);
    });
    Fe inv;
    fe_inv(inv, c[K - 1]);
    static_for<K - 1, -1, -1>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      Fe zi;
      if constexpr (i > 0) {
        fe_mul(zi, inv, c[i - 1]);
        fe_mul(inv, inv, Z[i]);
      } else {
        zi = inv;
      }
      Fe zi2, zi3;
      fe_sqr(zi2, zi);
      fe_mul(zi3, zi2, zi);
      fe_mul(tab[i].x, X[i], zi2);
      fe_mul(tab[i].y, Y[i], zi3);
    });
  }
  Fe beta;
  fe_beta(beta);
  Gej acc;
  gej_set_inf(acc);
  for (int w = NW - 1; w >= 0; --w) {
    if (w < NW - 1) {
#pragma unroll
      for (int k = 0; k < W; ++k) gej_double(acc, acc);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int d = booth_digit<W>(h ? m2 : m1, w);
      if (d) {
        const int ad = d < 0 ? -d : d;
        Ge p = tab[0];
        static_for<1, K>([&](auto ic) {  // select, not an index: the table stays in VGPRs
          constexpr int i = decltype(ic)::value;
          sel8(p.x.v, ad == i + 1, tab[i].x.v, p.x.v);
          sel8(p.y.v, ad == i + 1, tab[i].y.v, p.y.v);
        });
        if (h) fe_mul(p.x, p.x, beta);
        if ((d < 0) != (h ? n2 : n1)) fe_neg(p.y, p.y);
        Gej t;
        gej_add_ge(t, acc, p);
        acc = t;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < kGTabRows; ++i) {
    // (the loop stays rolled: the limb by select, not u1.v[i >> 2], which
    // would put u1 in scratch)
    const int l = i >> 2;
    u32 limb = u1.v[0];
    static_for<1, 8>([&](auto ic) { limb = l == decltype(ic)::value ? u1.v[decltype(ic)::value] : limb; });
    const u32 b = (limb >> (8 * (i & 3))) & 255u;
    if (b) {
      const Ge g = gtab[256 * i + b];
      Gej t;
      gej_add_ge(t, acc, g);
      acc = t;
    }
  }
  r = acc;
}

SECP_HD void ecmult(Gej& r, const Ge& q, const Sc& u2, const Sc& u1, const Ge* gtab) {
  ecmult_w<kQWindow>(r, q, u2, u1, gtab);
}

// libsecp256k1 verify_raw: r, s in [1, n); z the message scalar.
SECP_HD bool ecdsa_verify(const Sc& r, const Sc& s, const Sc& z, const Ge& q, const Ge* gtab) {
  if (is_zero8(r.v) || is_zero8(s.v)) return false;
  Sc sn, u1, u2;
  sc_inv(sn, s);
  sc_mul(u1, z, sn);
  sc_mul(u2, r, sn);
  Gej R;
  ecmult(R, q, u2, u1, gtab);
  if (R.inf) return false;
  // x(R) == r (as field elements, r < n < p) <=> X == r Z^2
  Fe z2, xr, rz;
  fe_sqr(z2, R.z);
#pragma unroll
  for (int i = 0; i < 8; ++i) xr.v[i] = r.v[i];
  fe_mul(rz, xr, z2);
  if (eq8(rz.v, R.x.v)) return true;
  // r + n < p: the x coordinate may have been reduced mod n
  // p - n = 0x14551231950B75FC4402DA1732FC9BEBE ... compare r < p - n <=> r + n < p
  u32 t[8];
  u64 c = 0;
  const u32 nl[8] = {0xD0364141u, 0xBFD25E8Cu, 0xAF48A03Bu, 0xBAAEDCE6u,
                     0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c += (u64)r.v[i] + nl[i];
    t[i] = (u32)c;
    c >>= 32;
  }
  if (c || !fe_lt_p(t)) return false;
#pragma unroll
  for (int i = 0; i < 8; ++i) xr.v[i] = t[i];
  fe_mul(rz, xr, z2);
  return eq8(rz.v, R.x.v);
}

}  // namespace secp
}  // namespace dc
