// dc_bits.h -- gfx950 device primitives on 64-bit boards (one lane = one position).
//
// Square s = 8*x + y (x = row, 0 = White's back rank; y = column), as in
// core/src/chess.rs:127-131 / :394-431.  All arithmetic is integer VALU work:
// a 64-bit logic op is two v_*_b32, a 64-bit shift is one v_lshlrev_b64 /
// v_lshrrev_b64, a popcount is two v_bcnt_u32_b32 (the second accumulates).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dc {

typedef unsigned long long u64;
typedef uint32_t u32;

constexpr u64 kFileA = 0x0101010101010101ull;  // y == 0
constexpr u64 kFileB = kFileA << 1;
constexpr u64 kFileG = kFileA << 6;
constexpr u64 kFileH = kFileA << 7;  // y == 7
constexpr u64 kNotA = ~kFileA;
constexpr u64 kNotH = ~kFileH;
constexpr u64 kNotAB = ~(kFileA | kFileB);
constexpr u64 kNotGH = ~(kFileG | kFileH);
constexpr u64 kRow(int x) { return 0xFFull << (8 * x); }
constexpr u64 kAll = ~0ull;
constexpr u64 kDiagMain = 0x8040201008040201ull;  // a1..h8 (x - y == 0)
constexpr u64 kDiagAnti = 0x0102040810204080ull;  // h1..a8 (x + y == 7)

// Generalised shift: S > 0 toward higher squares.  Emitted as one
// v_lshlrev_b64 / v_lshrrev_b64: on gfx950 every shift issues at half rate,
// so one 64-bit shift (4 cycles per wave) beats the compiler's habit of
// splitting it into v_alignbit_b32 + v_lshlrev_b32 once the halves feed
// 32-bit bitop3s (tools/ubench/vop_rate.hip, profiles/r01/ubench_vop.txt).
// DC_SHIFT_PAD selects how the shift is written: 0 (shipped) the inline-asm
// shift; A/B diagnostics only: 4 = an opaque SGPR shift amount (shift_amount;
// measured slower in round 4), 1 = s_nop 1 ahead of the asm shift, 2 = s_nop 1
// after it, 3 = plain C shifts.
#ifndef DC_SHIFT_PAD
#define DC_SHIFT_PAD 0
#endif
#if DC_SHIFT_PAD == 1
#define DC_SHL_ASM "s_nop 1\n\tv_lshlrev_b64 %0, %1, %2"
#define DC_SHR_ASM "s_nop 1\n\tv_lshrrev_b64 %0, %1, %2"
#elif DC_SHIFT_PAD == 2
#define DC_SHL_ASM "v_lshlrev_b64 %0, %1, %2\n\ts_nop 1"
#define DC_SHR_ASM "v_lshrrev_b64 %0, %1, %2\n\ts_nop 1"
#else
#define DC_SHL_ASM "v_lshlrev_b64 %0, %1, %2"
#define DC_SHR_ASM "v_lshrrev_b64 %0, %1, %2"
#endif
// The shift amount as an opaque SGPR constant (DC_SHIFT_PAD == 4, round 4):
// the compiler cannot split a shift by an unknown amount into 32-bit halves,
// so it emits the one v_lshlrev_b64 itself -- and, unlike after an inline-asm
// shift, it knows that instruction's hazards, so no conservative s_nop 0
// follows each shift (15M s_nop per perft(7) launch of k_count3c,
// tools/bbprof.py).
template <int A>
__device__ __forceinline__ u32 shift_amount() {
  u32 k;
  asm("s_mov_b32 %0, %1" : "=s"(k) : "i"(A));
  return k;
}
template <int S>
__device__ __forceinline__ u64 sh(u64 x) {
  u64 r;
#if DC_SHIFT_PAD == 4
  if constexpr (S >= 32) r = (u64)((u32)x << (S - 32)) << 32;
  else if constexpr (S <= -32) r = (u64)((u32)(x >> 32) >> (-S - 32));
  else if constexpr (S > 0) r = x << shift_amount<S>();
  else if constexpr (S < 0) r = x >> shift_amount<-S>();
#elif DC_SHIFT_PAD == 3
  if constexpr (S > 0) r = x << S;
  else if constexpr (S < 0) r = x >> -S;
#else
  // |S| >= 32 (the fills' 4 x 8 and 4 x 9 steps): one half moves, so a 32-bit
  // shift (S = 32: a register copy) instead of the half-rate 64-bit one
  if constexpr (S >= 32) r = (u64)((u32)x << (S - 32)) << 32;
  else if constexpr (S <= -32) r = (u64)((u32)(x >> 32) >> (-S - 32));
  else if constexpr (S > 0) asm(DC_SHL_ASM : "=v"(r) : "i"(S), "v"(x));
  else if constexpr (S < 0) asm(DC_SHR_ASM : "=v"(r) : "i"(-S), "v"(x));
#endif
  else r = x;
  return r;
}

__device__ __forceinline__ u32 pc(u64 x) { return (u32)__popcll(x); }

// gfx950 v_bitop3_b32: any 3-input bitwise function in one full-rate
// instruction per 32-bit half (v_and_or_b32 is half rate).  IMM is the truth
// table f(0xF0, 0xCC, 0xAA).
template <unsigned IMM>
__device__ __forceinline__ u64 bop3(u64 a, u64 b, u64 c) {
  const u32 lo = __builtin_amdgcn_bitop3_b32((u32)a, (u32)b, (u32)c, IMM);
  const u32 hi = __builtin_amdgcn_bitop3_b32((u32)(a >> 32), (u32)(b >> 32), (u32)(c >> 32), IMM);
  return ((u64)hi << 32) | lo;
}
__device__ __forceinline__ u64 and3(u64 a, u64 b, u64 c) { return bop3<0x80>(a, b, c); }     // a & b & c
__device__ __forceinline__ u64 or_and(u64 a, u64 b, u64 c) { return bop3<0xF8>(a, b, c); }   // a | (b & c)
__device__ __forceinline__ u64 and_andn(u64 a, u64 b, u64 c) { return bop3<0x40>(a, b, c); } // a & b & ~c
__device__ __forceinline__ int lsb(u64 x) { return __ffsll((long long)x) - 1; }
__device__ __forceinline__ int msb(u64 x) { return 63 - __clzll((long long)x); }

// Kogge-Stone occluded fill + one step: the attack set of all sliders in
// `gen` toward direction S (wrap guard M applied after every step).  In one
// direction each target has exactly one source (the first piece behind it),
// so popcount(attacks & ~own) counts moves with multiplicity.
template <int S, u64 M>
__device__ __forceinline__ u64 ray_attacks(u64 gen, u64 empty) {
  u64 pro = empty & M;
  gen = or_and(gen, pro, sh<S>(gen));
  pro &= sh<S>(pro);
  gen = or_and(gen, pro, sh<2 * S>(gen));
  pro &= sh<2 * S>(pro);
  gen = or_and(gen, pro, sh<4 * S>(gen));
  return sh<S>(gen) & M;
}

// Same fill, returning the attacks already masked by `allowed` (one bitop3).
template <int S, u64 M>
__device__ __forceinline__ u64 ray_moves(u64 gen, u64 empty, u64 allowed) {
  u64 pro = empty & M;
  gen = or_and(gen, pro, sh<S>(gen));
  pro &= sh<S>(pro);
  gen = or_and(gen, pro, sh<2 * S>(gen));
  pro &= sh<2 * S>(pro);
  gen = or_and(gen, pro, sh<4 * S>(gen));
  return and3(sh<S>(gen), M, allowed);
}

// Per-square attack and line tables (5 KB in device global memory, resident
// in each CU's vector L1): one vector load replaces a variable 64-bit shift
// pair, its select and the wrap-file select.  Round 4 (tools/bbprof_inline.py
// on k_count3c): king_moves was 5.6 % of the kernel's VALU issue cycles and
// slider_source ~7 %, almost all of it that arithmetic.  DC_ATT_TAB=0 keeps
// the arithmetic forms (A/B).
#ifndef DC_ATT_TAB
#define DC_ATT_TAB 1
#endif
struct AttTables {
  u64 king[64], knight[64];
  u64 behind[8][64];  // line_behind<D>(t)
  constexpr AttTables() : king{}, knight{}, behind{} {
    constexpr int kStep[8][2] = {{1, 0}, {-1, 0}, {0, 1}, {0, -1}, {1, 1}, {-1, -1}, {1, -1}, {-1, 1}};
    for (int s = 0; s < 64; ++s) {
      const int x = s >> 3, y = s & 7;
      for (int dx = -2; dx <= 2; ++dx)
        for (int dy = -2; dy <= 2; ++dy) {
          const int X = x + dx, Y = y + dy, ax = dx < 0 ? -dx : dx, ay = dy < 0 ? -dy : dy;
          if (X < 0 || X > 7 || Y < 0 || Y > 7) continue;
          if (ax <= 1 && ay <= 1 && (ax | ay)) king[s] |= 1ull << (8 * X + Y);
          if (ax + ay == 3 && ax && ay) knight[s] |= 1ull << (8 * X + Y);
        }
      for (int d = 0; d < 8; ++d)  // walk back from s against the slide direction
        for (int X = x - kStep[d][0], Y = y - kStep[d][1]; X >= 0 && X < 8 && Y >= 0 && Y < 8;
             X -= kStep[d][0], Y -= kStep[d][1])
          behind[d][s] |= 1ull << (8 * X + Y);
    }
  }
};
__constant__ constexpr AttTables kAtt{};

// The squares of the line through t in direction class D, strictly on the
// side the source of a slider move toward direction D lies (i.e. "behind" t).
// D: 0 N(+8) 1 S(-8) 2 E(+1) 3 W(-1) 4 NE(+9) 5 SW(-9) 6 NW(+7) 7 SE(-7).
// TAB false: the arithmetic form (the FIDE generator's single-workgroup top
// plies are latency-bound, and a table load sits on their dependency chain:
// FIDE suite at depth 5 2.65 -> 2.79 ms with the table, round 4 A/B)
template <int D, bool TAB = (DC_ATT_TAB != 0)>
__device__ __forceinline__ u64 line_behind(int t) {
  if constexpr (TAB) return kAtt.behind[D][t];
  const int x = t >> 3, y = t & 7;
  u64 line;
  if constexpr (D == 0 || D == 1) line = kFileA << y;
  else if constexpr (D == 2 || D == 3) line = 0xFFull << (8 * x);
  else if constexpr (D == 4 || D == 5) {
    const int d = x - y;
    line = d >= 0 ? (kDiagMain << (8 * d)) : (kDiagMain >> (-8 * d));
  } else {
    const int a = x + y - 7;
    line = a >= 0 ? (kDiagAnti << (8 * a)) : (kDiagAnti >> (-8 * a));
  }
  const u64 bit = 1ull << t;
  // even D: positive shift, source below t; odd D: source above t
  if constexpr ((D & 1) == 0) return line & (bit - 1);
  else return line & ~(bit | (bit - 1));
}

// Source square of a slider move toward D that lands on t: the nearest
// occupied square behind t.
template <int D, bool TAB = (DC_ATT_TAB != 0)>
__device__ __forceinline__ int slider_source(u64 occ, int t) {
  const u64 c = occ & line_behind<D, TAB>(t);
  if constexpr ((D & 1) == 0) return msb(c);
  else return lsb(c);
}

// Squares strictly between two squares that share a rank, file or diagonal;
// 0 otherwise (table-free obstruction difference, LERF mapping).
__device__ __forceinline__ u64 between(int s1, int s2) {
  const u64 m1 = ~0ull;
  const u64 a2a7 = 0x0001010101010100ull;
  const u64 b2g7 = 0x0040201008040200ull;
  const u64 h1b7 = 0x0002040810204080ull;
  const u64 btwn = (m1 << s1) ^ (m1 << s2);
  const u64 file = (u64)((s2 & 7) - (s1 & 7));
  const u64 rank = (u64)(((s2 | 7) - s1) >> 3);
  u64 line = ((file & 7) - 1) & a2a7;
  line += 2 * (((rank & 7) - 1) >> 58);
  line += (((rank - file) & 15) - 1) & b2g7;
  line += (((rank + file) & 15) - 1) & h1b7;
  line *= btwn & (0 - btwn);
  return line & btwn;
}

__device__ __forceinline__ u64 fmix64(u64 k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

__device__ __forceinline__ u64 splitmix_next(u64& s) {
  u64 z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// k-th (0-based) set bit of x; x must have more than k bits set.
__device__ __forceinline__ int select_bit(u64 x, u32 k) {
  const u32 lo = (u32)x;
  const u32 nlo = (u32)__popc(lo);
  int base = 0;
  u32 w = lo;
  if (k >= nlo) {
    k -= nlo;
    w = (u32)(x >> 32);
    base = 32;
  }
  for (u32 i = 0; i < k; ++i) w &= w - 1;
  return base + __ffs(w) - 1;
}

// k-th (0-based) set bit of x without a data-dependent loop: five halving
// steps on popcounts, then the last bit (x must have more than k bits set).
__device__ __forceinline__ u32 select_bit_bf(u64 x, u32 k) {
  u32 base = 0;
  u32 w = (u32)x;
  {
    const u32 n = (u32)__popc(w);
    const bool hi = k >= n;
    k = hi ? k - n : k;
    w = hi ? (u32)(x >> 32) : w;
    base = hi ? 32u : 0u;
  }
#pragma unroll
  for (u32 half = 16; half; half >>= 1) {
    const u32 low = w & ((1u << half) - 1);
    const u32 n = (u32)__popc(low);
    const bool hi = k >= n;
    k = hi ? k - n : k;
    w = hi ? (w >> half) : low;
    base += hi ? half : 0u;
  }
  return base;
}

// ---------------------------------------------------------------- wave ops
__device__ __forceinline__ u64 ballot(bool p) { return __ballot(p); }

__device__ __forceinline__ u32 lane_id() { return __lane_id(); }
// Number of set bits of the wave mask m below this lane: two v_mbcnt with the
// mask read straight from its SGPRs (no copy of the mask into VGPRs, no
// popcount of m & below).
__device__ __forceinline__ u32 mask_rank(u64 m) {
  return __builtin_amdgcn_mbcnt_hi((u32)(m >> 32), __builtin_amdgcn_mbcnt_lo((u32)m, 0u));
}

// DPP lane moves (gfx9 encodings: row_shr:n = 0x110 + n, row_bcast:15 =
// 0x142, row_bcast:31 = 0x143).  Lanes whose source is outside the row, and
// lanes of rows masked off by ROWM, read 0.  Scans and reductions built from
// these stay in the VALU: __shfl_up / __shfl_xor lower to ds_bpermute_b32,
// an LDS round trip per step that the profiles counted as LDS traffic and
// bank-conflict cycles (k_count2c's block scans, round 2).
template <int CTRL, int ROWM = 0xF>
__device__ __forceinline__ u32 dpp_z(u32 v) {
  return (u32)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWM, 0xF, true);
}

// Inclusive prefix sum over the 64 lanes of a wave: Hillis-Steele inside each
// 16-lane row (row_shr 1, 2, 4, 8), then row 0's total into row 1 and row 2's
// into row 3 (row_bcast:15), then rows 0-1's into rows 2-3 (row_bcast:31).
__device__ __forceinline__ u32 wave_incl_scan(u32 v) {
  v += dpp_z<0x111>(v);
  v += dpp_z<0x112>(v);
  v += dpp_z<0x114>(v);
  v += dpp_z<0x118>(v);
  v += dpp_z<0x142, 0xA>(v);
  v += dpp_z<0x143, 0xC>(v);
  return v;
}

// The same on 64-bit values (both halves moved, one 64-bit add per step).
__device__ __forceinline__ u64 wave_incl_scan64(u64 v) {
  auto step = [&](auto mv) {
    const u64 o = ((u64)mv((u32)(v >> 32)) << 32) | mv((u32)v);
    v += o;
  };
  step([](u32 x) { return dpp_z<0x111>(x); });
  step([](u32 x) { return dpp_z<0x112>(x); });
  step([](u32 x) { return dpp_z<0x114>(x); });
  step([](u32 x) { return dpp_z<0x118>(x); });
  step([](u32 x) { return dpp_z<0x142, 0xA>(x); });
  step([](u32 x) { return dpp_z<0x143, 0xC>(x); });
  return v;
}

// Wave-uniform value of lane `l` (l uniform).
__device__ __forceinline__ u32 lane_bcast(u32 v, u32 l) { return (u32)__builtin_amdgcn_readlane((int)v, (int)l); }
__device__ __forceinline__ u64 lane_bcast64(u64 v, u32 l) {
  return ((u64)lane_bcast((u32)(v >> 32), l) << 32) | lane_bcast((u32)v, l);
}

// Sum over the wave's 64 lanes, wave-uniform (every lane active).
__device__ __forceinline__ u64 wave_sum64(u64 v) { return lane_bcast64(wave_incl_scan64(v), 63); }
// The same when every lane's value is below 2^26 (the sum fits 32 bits): one
// DPP add per step instead of two moves and a 64-bit add
__device__ __forceinline__ u32 wave_sum32(u32 v) { return lane_bcast(wave_incl_scan(v), 63); }

}  // namespace dc
