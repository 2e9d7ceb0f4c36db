// dc_keccak.h -- Keccak-f[1600] and keccak256 (host and gfx950 device).
//
// The reference hashes serde_json(GameState) with alloy-primitives 0.7.7's
// keccak256 (tiny-keccak 2.0.2: the original Keccak padding 0x01 .. 0x80,
// rate 136 B, 32-byte digest; core/src/consensus/hotstuff.rs:153-166,
// core/src/consensus/types.rs:45-55).  The permutation is FIPS 202's
// Keccak-f[1600]: 24 rounds of theta, rho, pi, chi, iota on 25 64-bit lanes
// A[x + 5y]; round constants and rotation offsets below are derived from the
// spec's LFSR and (t+1)(t+2)/2 schedule.  On the device each lane of a wave
// runs its own permutation (one game per lane): a 64-bit rotate is two
// v_alignbit_b32, chi's a ^ (~b & c) is one v_bitop3_b32 per half.
#pragma once
#include <stddef.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define DC_HD __host__ __device__ __forceinline__
#else
#define DC_HD inline
#endif

namespace dc {

struct KeccakRC {
  uint64_t v[24];
};
DC_HD constexpr KeccakRC keccak_rc() {
  return KeccakRC{{0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
                   0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
                   0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
                   0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
                   0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
                   0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull}};
}

template <int N>
DC_HD uint64_t rotl64(uint64_t x) {
  if constexpr (N == 0) return x;
  else return (x << N) | (x >> (64 - N));
}

// One round on A[x + 5y].  rho offsets r[x][y]: (0,0) 0, (1,0) 1, (2,0) 62,
// (3,0) 28, (4,0) 27, (0,1) 36, (1,1) 44, (2,1) 6, (3,1) 55, (4,1) 20,
// (0,2) 3, (1,2) 10, (2,2) 43, (3,2) 25, (4,2) 39, (0,3) 41, (1,3) 45,
// (2,3) 15, (3,3) 21, (4,3) 8, (0,4) 18, (1,4) 2, (2,4) 61, (3,4) 56, (4,4) 14;
// pi: B[y + 5((2x + 3y) mod 5)] = rot(A[x + 5y], r[x][y]).
DC_HD void keccak_round(uint64_t* a, uint64_t rc) {
  uint64_t c0 = a[0] ^ a[5] ^ a[10] ^ a[15] ^ a[20];
  uint64_t c1 = a[1] ^ a[6] ^ a[11] ^ a[16] ^ a[21];
  uint64_t c2 = a[2] ^ a[7] ^ a[12] ^ a[17] ^ a[22];
  uint64_t c3 = a[3] ^ a[8] ^ a[13] ^ a[18] ^ a[23];
  uint64_t c4 = a[4] ^ a[9] ^ a[14] ^ a[19] ^ a[24];
  const uint64_t d0 = c4 ^ rotl64<1>(c1), d1 = c0 ^ rotl64<1>(c2), d2 = c1 ^ rotl64<1>(c3);
  const uint64_t d3 = c2 ^ rotl64<1>(c4), d4 = c3 ^ rotl64<1>(c0);
  uint64_t b[25];
  b[0] = a[0] ^ d0;
  b[10] = rotl64<1>(a[1] ^ d1);
  b[20] = rotl64<62>(a[2] ^ d2);
  b[5] = rotl64<28>(a[3] ^ d3);
  b[15] = rotl64<27>(a[4] ^ d4);
  b[16] = rotl64<36>(a[5] ^ d0);
  b[1] = rotl64<44>(a[6] ^ d1);
  b[11] = rotl64<6>(a[7] ^ d2);
  b[21] = rotl64<55>(a[8] ^ d3);
  b[6] = rotl64<20>(a[9] ^ d4);
  b[7] = rotl64<3>(a[10] ^ d0);
  b[17] = rotl64<10>(a[11] ^ d1);
  b[2] = rotl64<43>(a[12] ^ d2);
  b[12] = rotl64<25>(a[13] ^ d3);
  b[22] = rotl64<39>(a[14] ^ d4);
  b[23] = rotl64<41>(a[15] ^ d0);
  b[8] = rotl64<45>(a[16] ^ d1);
  b[18] = rotl64<15>(a[17] ^ d2);
  b[3] = rotl64<21>(a[18] ^ d3);
  b[13] = rotl64<8>(a[19] ^ d4);
  b[14] = rotl64<18>(a[20] ^ d0);
  b[24] = rotl64<2>(a[21] ^ d1);
  b[9] = rotl64<61>(a[22] ^ d2);
  b[19] = rotl64<56>(a[23] ^ d3);
  b[4] = rotl64<14>(a[24] ^ d4);
#pragma unroll
  for (int y = 0; y < 25; y += 5) {
    const uint64_t t0 = b[y], t1 = b[y + 1], t2 = b[y + 2], t3 = b[y + 3], t4 = b[y + 4];
    a[y] = t0 ^ (~t1 & t2);
    a[y + 1] = t1 ^ (~t2 & t3);
    a[y + 2] = t2 ^ (~t3 & t4);
    a[y + 3] = t3 ^ (~t4 & t0);
    a[y + 4] = t4 ^ (~t0 & t1);
  }
  a[0] ^= rc;
}

#if defined(__HIP_DEVICE_COMPILE__)
// gfx950 form of the same round: 64-bit lanes as (lo, hi) halves so that
// xor3 and chi's a ^ (~b & c) are one v_bitop3_b32 per half and a rotate is
// two v_alignbit_b32 (the generic form compiled to 64-bit shift pairs).
struct K64 {
  uint32_t lo, hi;
};
template <unsigned IMM>
__device__ __forceinline__ uint32_t kb3(uint32_t a, uint32_t b, uint32_t c) {
  return (uint32_t)__builtin_amdgcn_bitop3_b32(a, b, c, IMM);
}
__device__ __forceinline__ uint32_t kal(uint32_t a, uint32_t b, uint32_t s) {
  return (uint32_t)__builtin_amdgcn_alignbit(a, b, s);
}
__device__ __forceinline__ K64 kx3(K64 a, K64 b, K64 c) {  // a ^ b ^ c
  return K64{kb3<0x96>(a.lo, b.lo, c.lo), kb3<0x96>(a.hi, b.hi, c.hi)};
}
__device__ __forceinline__ K64 kx2(K64 a, K64 b) { return K64{a.lo ^ b.lo, a.hi ^ b.hi}; }
__device__ __forceinline__ K64 kchi(K64 a, K64 b, K64 c) {  // a ^ (~b & c)
  return K64{kb3<0xD2>(a.lo, b.lo, c.lo), kb3<0xD2>(a.hi, b.hi, c.hi)};
}
template <int N>
__device__ __forceinline__ K64 krot(K64 x) {
  if constexpr (N == 0) return x;
  else if constexpr (N == 32) return K64{x.hi, x.lo};
  else if constexpr (N < 32)
    return K64{kal(x.lo, x.hi, 32 - N), kal(x.hi, x.lo, 32 - N)};
  else
    return K64{kal(x.hi, x.lo, 64 - N), kal(x.lo, x.hi, 64 - N)};
}

__device__ __forceinline__ void keccak_f1600_dev(uint64_t* a64) {
  constexpr KeccakRC rc = keccak_rc();
  K64 a[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) a[i] = K64{(uint32_t)a64[i], (uint32_t)(a64[i] >> 32)};
// DC_KECCAK_UNROLL (round 6 A/B): rounds per loop trip.  2 and 4 fit the same
// 3 waves/SIMD (142-144 VGPRs) and measured slower: hash kernel 3.90-3.93 ->
// 3.99-4.00 ms (2) and 3.93-4.00 ms (4) (profiles/r06/ab_keccak_unroll.txt).
#ifndef DC_KECCAK_UNROLL
#define DC_KECCAK_UNROLL 1
#endif
// DC_KECCAK_FUSE (round 6): theta without D (see the round body): same box,
// alternating, hash kernel 3.18-3.20 -> 3.10-3.12 ms (profiles/r06/ab_keccak_fuse.txt).
#ifndef DC_KECCAK_FUSE
#define DC_KECCAK_FUSE 1
#endif
#pragma unroll DC_KECCAK_UNROLL
  for (int r = 0; r < 24; ++r) {
    const K64 c0 = kx3(kx3(a[0], a[5], a[10]), a[15], a[20]);
    const K64 c1 = kx3(kx3(a[1], a[6], a[11]), a[16], a[21]);
    const K64 c2 = kx3(kx3(a[2], a[7], a[12]), a[17], a[22]);
    const K64 c3 = kx3(kx3(a[3], a[8], a[13]), a[18], a[23]);
    const K64 c4 = kx3(kx3(a[4], a[9], a[14]), a[19], a[24]);
#if DC_KECCAK_FUSE
    // theta's D[x] = C[x-1] ^ rot1(C[x+1]) is never formed: each lane takes
    // a ^ C[x-1] ^ rot1(C[x+1]) as one three-input xor (180 VALU a round, not 190)
    const K64 r0 = krot<1>(c0), r1 = krot<1>(c1), r2 = krot<1>(c2), r3 = krot<1>(c3), r4 = krot<1>(c4);
#define DC_KTH(i, cm, rp) kx3(a[i], cm, rp)
#define DC_KD0 c4, r1
#define DC_KD1 c0, r2
#define DC_KD2 c1, r3
#define DC_KD3 c2, r4
#define DC_KD4 c3, r0
#else
    const K64 d0 = kx2(c4, krot<1>(c1)), d1 = kx2(c0, krot<1>(c2)), d2 = kx2(c1, krot<1>(c3));
    const K64 d3 = kx2(c2, krot<1>(c4)), d4 = kx2(c3, krot<1>(c0));
#define DC_KTH(i, d) kx2(a[i], d)
#define DC_KD0 d0
#define DC_KD1 d1
#define DC_KD2 d2
#define DC_KD3 d3
#define DC_KD4 d4
#endif
#define DC_KT(i, D) DC_KTH(i, D)
    K64 b[25];
    b[0] = DC_KT(0, DC_KD0);
    b[10] = krot<1>(DC_KT(1, DC_KD1));
    b[20] = krot<62>(DC_KT(2, DC_KD2));
    b[5] = krot<28>(DC_KT(3, DC_KD3));
    b[15] = krot<27>(DC_KT(4, DC_KD4));
    b[16] = krot<36>(DC_KT(5, DC_KD0));
    b[1] = krot<44>(DC_KT(6, DC_KD1));
    b[11] = krot<6>(DC_KT(7, DC_KD2));
    b[21] = krot<55>(DC_KT(8, DC_KD3));
    b[6] = krot<20>(DC_KT(9, DC_KD4));
    b[7] = krot<3>(DC_KT(10, DC_KD0));
    b[17] = krot<10>(DC_KT(11, DC_KD1));
    b[2] = krot<43>(DC_KT(12, DC_KD2));
    b[12] = krot<25>(DC_KT(13, DC_KD3));
    b[22] = krot<39>(DC_KT(14, DC_KD4));
    b[23] = krot<41>(DC_KT(15, DC_KD0));
    b[8] = krot<45>(DC_KT(16, DC_KD1));
    b[18] = krot<15>(DC_KT(17, DC_KD2));
    b[3] = krot<21>(DC_KT(18, DC_KD3));
    b[13] = krot<8>(DC_KT(19, DC_KD4));
    b[14] = krot<18>(DC_KT(20, DC_KD0));
    b[24] = krot<2>(DC_KT(21, DC_KD1));
    b[9] = krot<61>(DC_KT(22, DC_KD2));
    b[19] = krot<56>(DC_KT(23, DC_KD3));
    b[4] = krot<14>(DC_KT(24, DC_KD4));
#undef DC_KT
#undef DC_KTH
#undef DC_KD0
#undef DC_KD1
#undef DC_KD2
#undef DC_KD3
#undef DC_KD4
#pragma unroll
    for (int y = 0; y < 25; y += 5) {
      a[y] = kchi(b[y], b[y + 1], b[y + 2]);
      a[y + 1] = kchi(b[y + 1], b[y + 2], b[y + 3]);
      a[y + 2] = kchi(b[y + 2], b[y + 3], b[y + 4]);
      a[y + 3] = kchi(b[y + 3], b[y + 4], b[y]);
      a[y + 4] = kchi(b[y + 4], b[y], b[y + 1]);
    }
    a[0].lo ^= (uint32_t)rc.v[r];
    a[0].hi ^= (uint32_t)(rc.v[r] >> 32);
  }
#pragma unroll
  for (int i = 0; i < 25; ++i) a64[i] = ((uint64_t)a[i].hi << 32) | a[i].lo;
}
#endif

DC_HD void keccak_f1600(uint64_t* a) {
#if defined(__HIP_DEVICE_COMPILE__)
  keccak_f1600_dev(a);
#else
  constexpr KeccakRC rc = keccak_rc();
  for (int r = 0; r < 24; ++r) keccak_round(a, rc.v[r]);
#endif
}

constexpr int kKeccakRate = 136;  // bytes: 1600 - 2 x 256 bits of capacity

// Streaming keccak256 over bytes (host side; the device kernels absorb 8-byte
// words themselves).
struct Keccak256 {
  uint64_t a[25] = {};
  uint8_t buf[kKeccakRate] = {};
  int n = 0;
  void absorb_block() {
    for (int i = 0; i < kKeccakRate / 8; ++i) {
      uint64_t w = 0;
      for (int k = 0; k < 8; ++k) w |= (uint64_t)buf[8 * i + k] << (8 * k);
      a[i] ^= w;
    }
    keccak_f1600(a);
    n = 0;
  }
  void update(const void* data, size_t len) {
    const uint8_t* p = static_cast<const uint8_t*>(data);
    for (size_t i = 0; i < len; ++i) {
      buf[n++] = p[i];
      if (n == kKeccakRate) absorb_block();
    }
  }
  void final(uint8_t out[32]) {
    for (int i = n; i < kKeccakRate; ++i) buf[i] = 0;
    buf[n] ^= 0x01;  // Keccak padding (not SHA-3's 0x06)
    buf[kKeccakRate - 1] ^= 0x80;
    absorb_block();
    for (int i = 0; i < 32; ++i) out[i] = (uint8_t)(a[i / 8] >> (8 * (i % 8)));
  }
};

}  // namespace dc
