// dc_moves.hip -- single-move kernels for gfx950, one lane per position or game.
//
//   k_validate_{ref,fide}   K2: one lane per (position, move)      -> verdict byte
//   k_apply_{ref,fide}      K2': validate + make in place           -> verdict, info
//   k_replay_{ref,fide}     K1: one lane per game, loop over plies  -> ply-major accept bitmap
//   k_gen_games_{ref,fide}  K5: one lane per game, seeded games     -> ply-major moves
#include <algorithm>
#include <cstdlib>
#include <hip/hip_runtime.h>

#include "dc_common.h"

DC_BBPROF_DEFINE(moves)  // measurement builds only (tools/bbprof.py)

namespace dc {

// ------------------------------------------------------------- validation
// done != nullptr (a one-block launch whose I/O is pinned host memory, dc_api
// HostIo): once the block's results are stored, thread 0 publishes seq to the
// host flag with a system-scope release, so the caller can spin on the flag
// instead of synchronising the stream (the live n = 1 consensus call).
// Every thread makes its own stores visible at system scope before the
// barrier (a fence orders only the issuing wave's stores, and up to four
// waves write results), so the flag cannot overtake any wave's verdicts.
__device__ __forceinline__ void publish_done(u32* done, u32 seq) {
  if (!done) return;
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {  // a divergent (vector) store
    __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ __launch_bounds__(256) void k_validate_ref(const DevPos* __restrict__ pos, const uint16_t* __restrict__ moves,
                                                      u32 n, uint8_t* __restrict__ out, u32* done, u32 seq) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const DevPos p = pos[i];
    const Board b{p.bb[0], p.bb[1], p.bb[2], p.bb[3]};
    out[i] = (uint8_t)ref_verdict(b, p.stm & 1, moves[i]);
  }
  publish_done(done, seq);
}

__device__ __forceinline__ void apply_ref_one(DevPos* __restrict__ pos, const uint16_t* __restrict__ moves, u32 i,
                                              uint8_t* __restrict__ verdicts, uint8_t* __restrict__ info) {
  DevPos p = pos[i];
  Board b{p.bb[0], p.bb[1], p.bb[2], p.bb[3]};
  const u32 m = moves[i];
  const u32 v = ref_verdict(b, p.stm & 1, m);
  verdicts[i] = (uint8_t)v;
  if (v != V_OK) {
    if (info) info[i] = 0xFF;
    return;
  }
  const int f = (int)(m & 63), t = (int)((m >> 6) & 63);
  if (info) {
    // cell kind of the mover (P0 N1 B2 R3 Q4 K5 X6) | 8 if the target was occupied
    const u32 code = nibble(b, f) >> 1;
    const u32 cell_kind = (code == KC_P) ? 0 : (code == KC_N) ? 1 : (code == KC_B) ? 2 : (code == KC_R) ? 3
                        : (code == KC_Q) ? 4 : (code == KC_K) ? 5 : 6;
    info[i] = (uint8_t)(cell_kind | (((occupied(b) >> t) & 1) << 3));
  }
  ref_make(b, f, t);
  p.bb[0] = b.b0;
  p.bb[1] = b.b1;
  p.bb[2] = b.b2;
  p.bb[3] = b.b3;
  p.stm ^= 1;
  pos[i] = p;
}

__global__ __launch_bounds__(256) void k_apply_ref(DevPos* __restrict__ pos, const uint16_t* __restrict__ moves, u32 n,
                                                   uint8_t* __restrict__ verdicts, uint8_t* __restrict__ info, u32* done,
                                                   u32 seq) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) apply_ref_one(pos, moves, i, verdicts, info);
  publish_done(done, seq);
}

// Replay counters: one partial record {validated, accepted, rejected, digest
// sum, digest xor} per block, combined by k_reduce_stats -- per-wave global
// atomics on five addresses serialised at the memory side (rocprofv3, round 1).
__device__ __forceinline__ void block_stats(u32 validated, u32 accepted, u64 d, u64* partial) {
  __shared__ u64 ws[4][4];
  const u64 sv = wave_sum64(validated), sa = wave_sum64(accepted), sd = wave_sum64(d);
  u64 x = d;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x ^= __shfl_xor(x, o, 64);
  const u32 w = threadIdx.x >> 6;
  if (lane_id() == 0) {
    ws[w][0] = sv;
    ws[w][1] = sa;
    ws[w][2] = sd;
    ws[w][3] = x;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    u64 r[5] = {0, 0, 0, 0, 0};
    for (u32 k = 0; k < blockDim.x / 64; ++k) {
      r[0] += ws[k][0];
      r[1] += ws[k][1];
      r[3] += ws[k][2];
      r[4] ^= ws[k][3];
    }
    r[2] = r[0] - r[1];
    for (int k = 0; k < 5; ++k) partial[(size_t)blockIdx.x * 5 + k] = r[k];
  }
}

// stats_host (pinned, may be null): the same five counters stored straight
// into host memory, so a synchronous replay call needs no memset and no copy
// (they cost ~38 us of a ~0.9 ms call, round 2).  Folding this reduction into
// the replay kernel's last block instead needed an agent-scope release per
// block (an L2 writeback on gfx950): 0.86 -> 1.0 ms.
__global__ __launch_bounds__(256) void k_reduce_stats(const u64* __restrict__ partial, u32 n_blocks, u64* __restrict__ stats,
                                                      u64* __restrict__ stats_host = nullptr) {
  __shared__ u64 ws[4][5];
  u64 r[5] = {0, 0, 0, 0, 0};
  for (u32 b = threadIdx.x; b < n_blocks; b += blockDim.x) {
    for (int k = 0; k < 4; ++k) r[k] += partial[(size_t)b * 5 + k];
    r[4] ^= partial[(size_t)b * 5 + 4];
  }
  for (int k = 0; k < 5; ++k) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const u64 y = __shfl_xor(r[k], o, 64);
      r[k] = (k == 4) ? (r[k] ^ y) : (r[k] + y);
    }
  }
  if (lane_id() == 0)
    for (int k = 0; k < 5; ++k) ws[threadIdx.x >> 6][k] = r[k];
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 0; k < 5; ++k) {
      u64 v = ws[0][k];
      for (int w = 1; w < 4; ++w) v = (k == 4) ? (v ^ ws[w][k]) : (v + ws[w][k]);
      stats[k] = v;
      if (stats_host) __hip_atomic_store(stats_host + k, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// ------------------------------------------------------------------ replay
// One lane per game; the wave's 64 verdicts of a ply are one ballot word, so
// bitmap stores are one u64 per wave per ply (ply-major, no transpose).
constexpr int kReplayPrefetch = 4;

__global__ __launch_bounds__(256) void k_replay_ref(Board start, u32 stm0, const uint16_t* __restrict__ moves,
                                                    u32 n_games, u32 n_plies, u64* __restrict__ bitmap,
                                                    u64* __restrict__ digests, u64* __restrict__ partial) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = g < n_games;
  const u32 words = (n_games + 63) >> 6;
  Board b = start;
  u32 stm = stm0;
  u32 validated = 0, accepted = 0;
  uint16_t buf[kReplayPrefetch];
#pragma unroll
  for (int k = 0; k < kReplayPrefetch; ++k)
    buf[k] = (active && (u32)k < n_plies) ? moves[(size_t)k * n_games + g] : (uint16_t)0xFFFF;
  for (u32 ply = 0; ply < n_plies; ply += kReplayPrefetch) {
#pragma unroll
    for (int k = 0; k < kReplayPrefetch; ++k) {
      const u32 pl = ply + k;
      const u32 m = buf[k];
      const u32 nxt = pl + kReplayPrefetch;
      buf[k] = (active && nxt < n_plies) ? moves[(size_t)nxt * n_games + g] : (uint16_t)0xFFFF;
      bool ok = false;
      if (m != 0xFFFFu) {
        ++validated;
        ok = ref_verdict(b, stm, m) == V_OK;
        if (ok) {
          ref_make(b, (int)(m & 63), (int)((m >> 6) & 63));
          stm ^= 1;
          ++accepted;
        }
      }
      const u64 word = ballot(ok);
      if (bitmap && pl < n_plies && lane_id() == 0 && (g >> 6) < words) bitmap[(size_t)pl * words + (g >> 6)] = word;
    }
  }
  u64 d = 0;
  if (active) {
    d = board_digest(b, stm);
    if (digests) digests[g] = d;
  }
  block_stats(validated, accepted, d, partial);
}

// ------------------------------------------- replay, LDS table + LDS mailbox
// k_replay_ref3 gives the verdicts of ref_verdict with the geometry of every
// (from, to) pair read from a 48 KB table staged in LDS, indexed by the move
// word's low 12 bits (m & 0xFFF = f | t << 6):
//   btw[e]  squares strictly between f and t when aligned (the path walks of
//           chess.rs:272-284 / :322-332; the mid square of a double push,
//           :240-246), 0 otherwise -- so "path clear" is (btw & occ) == 0 for
//           every kind, and one test covers sliders and double pushes
//   geo[e]  bit n set iff a piece of nibble n (black | kind << 1) may move
//           f -> t onto an empty t; bit 16 + n iff onto an enemy piece.  Pawns
//           differ between the two (push / double from row 1 or 6 vs the
//           forward diagonal, chess.rs:235-251); knights, kings and sliders
//           do not (chess.rs:289-360).  Empty squares and unknown kinds have
//           no bits (chess.rs:101-108, :211).
// The mover's colour (WRONG_TURN, chess.rs:112-116) and an own piece on t
// (chess.rs:286, :334, :299, :359, :236) are two 16-entry bit LUTs on
// nibble(t) ^ stm.  Each game's board is a nibble mailbox in LDS (8 dwords per
// lane, dword-major [j][thread] so every lane owns its bank: conflict-free)
// beside an occupancy bitboard in registers: the nibbles of f and t are two
// ds_read_b32 + v_bfe, and make-move (chess.rs:72-77) is two ds_xor_b32 (XOR
// deltas commute, so f and t in one dword need no special case) plus the
// occupancy update.  The quad-bitboard is rebuilt once per game for the digest.
// Per ply: ~40 VALU ops against ~175 for ref_verdict on registers.
constexpr u32 kR3Threads = 1024;
constexpr u32 kR3TabBytes = 4096 * 8 + 4096 * 4;  // btw (32 KB) + geo (16 KB)
constexpr u32 kR3MbBytes = 8 * kR3Threads * 4;      // 32 KB: two blocks fill a CU's 160 KB
constexpr u32 kEnemyLut = 0xAAA8u;  // x = nibble(t) ^ stm: occupied (x >= 2) by the other side (x odd)
constexpr u32 kOwnLut = 0x5554u;    // ... by the side to move (x even)

__device__ __forceinline__ u32 replay_geo(u32 e) {
  const int f = (int)(e & 63), t = (int)(e >> 6);
  const int dx = (t >> 3) - (f >> 3), dy = (t & 7) - (f & 7);
  const int ax = dx < 0 ? -dx : dx, ay = dy < 0 ? -dy : dy;
  const bool knight = (ax == 1 && ay == 2) || (ax == 2 && ay == 1);
  const bool king = ax <= 1 && ay <= 1 && (ax | ay) != 0;
  const bool diag = ax == ay && ax != 0;
  const bool orth = (dx == 0) != (dy == 0);
  u32 both = 0;  // kinds whose quiet and capture geometry agree, both colours
  auto cls = [](u32 kind) { return 3u << (kind << 1); };
  if (knight) both |= cls(KC_N);
  if (king) both |= cls(KC_K);
  if (diag) both |= cls(KC_B) | cls(KC_Q);
  if (orth) both |= cls(KC_R) | cls(KC_Q);
  const u32 wp = 1u << (KC_P << 1), bp = wp << 1;
  u32 quiet = both, cap = both;
  if (dy == 0 && (dx == 1 || (dx == 2 && (f >> 3) == 1))) quiet |= wp;
  if (dy == 0 && (dx == -1 || (dx == -2 && (f >> 3) == 6))) quiet |= bp;
  if (ay == 1 && dx == 1) cap |= wp;
  if (ay == 1 && dx == -1) cap |= bp;
  return quiet | (cap << 16);
}

// v_writelane_b32: lane `sel` (wave-uniform) of `old` <- the uniform `val`.
__device__ __forceinline__ u32 writelane(u32 old, u32 val, u32 sel) {
  // gfx9's constant bus takes one SGPR per VALU op: the lane select goes through M0
  asm volatile("s_mov_b32 m0, %2\n\tv_writelane_b32 %0, %1, m0" : "+v"(old) : "s"(val), "s"(sel) : "m0");
  return old;
}

// Nibble-spaced bits (0, 4, ..., 28) of x gathered into bits 0..7.
__device__ __forceinline__ u32 gather_nibble_bits(u32 x) {
  x &= 0x11111111u;
  x = (x | (x >> 3)) & 0x03030303u;
  x = (x | (x >> 6)) & 0x000F000Fu;
  return (x | (x >> 12)) & 0xFFu;
}

// The start position's mailbox, packed on the host (kernel argument: SGPRs).
struct Mailbox {
  u32 d[8];
};

__global__ __launch_bounds__(kR3Threads) void k_replay_ref3(Mailbox mb0, u64 occ0, u32 stm0, const uint16_t* __restrict__ moves,
                                                           u32 n_games, u32 n_plies, u64* __restrict__ bitmap,
                                                           u64* __restrict__ digests, u64* __restrict__ partial) {
  // static (not extern) LDS: its base is the constant 0, folded into the ds offsets
  __shared__ __attribute__((aligned(16))) unsigned char r3_smem[kR3TabBytes + kR3MbBytes];
  u64* btw = reinterpret_cast<u64*>(r3_smem);
  u32* mb = reinterpret_cast<u32*>(r3_smem + kR3TabBytes);  // mb[j * kR3Threads + tid]
  const u32 tid = threadIdx.x;
  for (u32 e = tid; e < 4096; e += kR3Threads) {
    btw[e] = between((int)(e & 63), (int)(e >> 6));
    reinterpret_cast<u32*>(r3_smem + 4096 * 8)[e] = replay_geo(e);
  }
  __syncthreads();
  const u32 lane = lane_id();
  const u32 words = (n_games + 63) >> 6;
  const u32 tid4 = tid * 4;       // byte offset of this lane's mailbox column
  const u32 last = n_plies - 1;   // n_plies >= 1 (the launcher routes n_plies == 0 elsewhere)
  u32* my = mb + tid;
  u32 validated = 0, accepted = 0;
  u64 dsum = 0, dxor = 0;
  // Block-contiguous chunks: in round r, block b's 16 waves take the 16
  // consecutive 64-game chunks (r * grid + b) * 16 + w, so a block reads 2 KB
  // runs of every ply row and concurrently running blocks sweep one region of
  // each row.  Per-wave dynamic chunks scattered the 128-B reads over DRAM
  // pages: 1.65x slower.
  for (u32 round = 0;; ++round) {
    const u32 c = (round * gridDim.x + blockIdx.x) * (kR3Threads / 64) + (tid >> 6);
    if (c >= words) break;
    const u32 g = (c << 6) | lane;
    const bool active = g < n_games;
    // byte offset of this lane's game in a ply row; inactive lanes (last chunk
    // only) read game n-1 and are masked, so every load is unconditional
    const u32 goff = (active ? g : n_games - 1) * 2;
    // buffer_load with the ply row's base in an SGPR descriptor and the lane's
    // 32-bit offset in a VGPR: no 64-bit address arithmetic per ply
    auto load_move = [&](u32 p) -> u32 {
      const uint16_t* row = moves + (size_t)min(p, last) * n_games;  // uniform
      const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)row, 0, n_games * 2, 0x00020000);
      return __builtin_amdgcn_raw_buffer_load_b16(r, goff, 0, 0);
    };
#pragma unroll
    for (u32 j = 0; j < 8; ++j) my[j * kR3Threads] = mb0.d[j];
    u64 occ = occ0;
    u32 stm = stm0;
    u32 buf[kReplayPrefetch];
#pragma unroll
    for (int k = 0; k < kReplayPrefetch; ++k) buf[k] = load_move((u32)k);
    u32 bw_lo = 0, bw_hi = 0;  // lane j holds the ballot word of ply 64q + j
    for (u32 ply = 0; ply < n_plies; ply += kReplayPrefetch) {
#pragma unroll
      for (int k = 0; k < kReplayPrefetch; ++k) {
        const u32 pl = ply + k;
        const u32 m = (active && pl < n_plies) ? buf[k] : 0xFFFFu;
        buf[k] = load_move(pl + kReplayPrefetch);
        const u32 m2 = m << 2, m3 = m << 3;
        const u64 bt = *reinterpret_cast<const u64*>(r3_smem + (m3 & 0x7FF8u));             // btw[m & 0xFFF]
        const u32 gw = *reinterpret_cast<const u32*>(r3_smem + 4096 * 8 + (m2 & 0x3FFCu));  // geo[m & 0xFFF]
        // mailbox dwords of f and t: ((square >> 3) << 12) | tid4, one bitop3 each
        const u32 af = __builtin_amdgcn_bitop3_b32(m << 9, tid4, 0x7000u, 0xE4);  // (a & c) | (b & ~c)
        const u32 at = __builtin_amdgcn_bitop3_b32(m3, tid4, 0x7000u, 0xE4);
        const u32 wf = *reinterpret_cast<const u32*>(r3_smem + kR3TabBytes + af);
        const u32 wt = *reinterpret_cast<const u32*>(r3_smem + kR3TabBytes + at);
        const u32 st = (m >> 4) & 28;
        const u32 nib = __builtin_amdgcn_ubfe(wf, m2, 4);  // v_bfe reads offset bits 4:0 = (f & 7) * 4
        const u32 nibt = __builtin_amdgcn_ubfe(wt, st, 4);
        const u32 x = nibt ^ stm;
        const u32 shift = nib | (__builtin_amdgcn_ubfe(kEnemyLut, x, 1) << 4);
        // bit 0 of bad: wrong geometry for the target's state, own piece on t,
        // mover not of the side to move (or no piece), or an OOR/sentinel word
        const u32 geo_ok = __builtin_amdgcn_ubfe(gw, shift, 1), own = __builtin_amdgcn_ubfe(kOwnLut, x, 1);
        const u32 okb = __builtin_amdgcn_bitop3_b32(geo_ok, own, __builtin_amdgcn_bitop3_b32(nib, stm, m >> 15, 0xBE),
                                                    0x10);  // a & ~b & ~c, c = (nib ^ stm) | m >> 15 (0xBE): only bit 0 can be set
        const bool ok = okb != 0 && (bt & occ) == 0;
        const u64 w = ballot(ok);  // before the branch: the mask is the compare's own result
        if (ok) {
          atomicXor(reinterpret_cast<u32*>(r3_smem + kR3TabBytes + af), nib << m2);  // ds_xor_b32: f empties
          atomicXor(reinterpret_cast<u32*>(r3_smem + kR3TabBytes + at), (nib ^ nibt) << st);  // t <- mover
          occ = bop3<0xBA>(occ, 1ull << (m & 63), 1ull << ((m >> 6) & 63));  // (occ & ~f) | t
          stm ^= 1;
        }
        // per-lane counters: ballot popcounts (s_bcnt1 + 64-bit s_add) put ~8 SALU
        // on every ply's critical issue path and cost 20 % (A/B)
        validated += (m != 0xFFFFu);
        accepted += ok;
        const u32 slot = pl & 63;
        bw_lo = writelane(bw_lo, (u32)w, slot);
        bw_hi = writelane(bw_hi, (u32)(w >> 32), slot);
      }
      // every 64 plies (and at the end) lane j stores the word of ply base + j
      const u32 done = min(ply + kReplayPrefetch, n_plies);
      if (bitmap && ((done & 63) == 0 || done == n_plies)) {
        const u32 base = (done - 1) & ~63u;
        if (lane < done - base) bitmap[(size_t)(base + lane) * words + c] = ((u64)bw_hi << 32) | bw_lo;
      }
    }
    if (active) {
      Board b{0, 0, 0, 0};
#pragma unroll
      for (u32 j = 0; j < 8; ++j) {
        const u32 d = my[j * kR3Threads];
        b.b0 |= (u64)gather_nibble_bits(d) << (8 * j);
        b.b1 |= (u64)gather_nibble_bits(d >> 1) << (8 * j);
        b.b2 |= (u64)gather_nibble_bits(d >> 2) << (8 * j);
        b.b3 |= (u64)gather_nibble_bits(d >> 3) << (8 * j);
      }
      const u64 dg = board_digest(b, stm);
      if (digests) digests[g] = dg;
      dsum += dg;
      dxor ^= dg;
    }
  }
  // block partial {validated, accepted, rejected, digest sum, digest xor}
  const u64 sv = wave_sum64(validated), sa = wave_sum64(accepted), sd = wave_sum64(dsum);
  u64 xx = dxor;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) xx ^= __shfl_xor(xx, o, 64);
  __syncthreads();  // the table's LDS is reused for the per-wave sums
  u64* ws = btw;
  const u32 w = tid >> 6;
  if (lane == 0) {
    ws[w * 4 + 0] = sv;
    ws[w * 4 + 1] = sa;
    ws[w * 4 + 2] = sd;
    ws[w * 4 + 3] = xx;
  }
  __syncthreads();
  if (tid == 0) {
    u64 r[5] = {0, 0, 0, 0, 0};
    for (u32 k = 0; k < kR3Threads / 64; ++k) {
      r[0] += ws[k * 4 + 0];
      r[1] += ws[k * 4 + 1];
      r[3] += ws[k * 4 + 2];
      r[4] ^= ws[k * 4 + 3];
    }
    r[2] = r[0] - r[1];
    for (int k = 0; k < 5; ++k) partial[(size_t)blockIdx.x * 5 + k] = r[k];
  }
}

// ------------------------------------------- replay, round 3 (k_replay_ref4)
// k_replay_ref3's table + mailbox scheme with the per-ply issue trimmed
// (profiles/r02: ref3 issued 45 VALU + 23 SALU per wave and ply and waited 36 %
// of its cycles):
//   - the four LDS reads of a ply (btw, geo, the f and t mailbox dwords) issue
//     together: ref3's `okb && (btw & occ) == 0` let the compiler sink the btw
//     read behind a branch, a second dependent LDS round trip per ply plus an
//     exec-mask save/restore;
//   - one buffer descriptor spans the whole ply-major move array (the launcher
//     takes this kernel when it is < 4 GiB) and a ply's row is the SGPR
//     soffset min(p, last) * row_bytes: 2 SALU per load instead of 8;
//   - inactive lanes (the last chunk only) replay game n-1 unmasked: their
//     counters are dropped per chunk and their bitmap bits masked at the
//     64-ply store, so no per-ply select;
//   - both ballot halves go into the lanes' words under one M0 write;
//   - LOOK = 1: the two table reads (btw, geo) of ply p + 1 issue before ply
//     p's mailbox reads, so only the (conflict-free) mailbox round trip is on
//     a ply's dependency chain; the random, bank-conflicted table gathers
//     overlap the previous ply's logic.
// INFO (dc_replay_info, the resync path): per ply and game one byte, the
// moved piece's cell kind | 8 if the target held a piece (dc_apply_batch's
// info, what update_history needs, chess.rs:156-167), 0xFF for a rejected ply;
// ply-major like the moves.  Compiled out of the plain replay.
// DC_R4_LAZY = 1 (round-3 experiment, off): a vacated square is not cleared
// in the mailbox; the occupancy bitboard masks its stale nibble when read, so
// a make-move is one LDS read-modify-write instead of two.  Measured slower
// (10M x 80: 0.865 -> 0.998 ms, same box, profiles/r03/ab_replay_lazy.txt):
// the kernel is bound by its per-ply dependency chain, not by LDS cycles,
// and the occupancy test puts a 64-bit shift on that chain.
#ifndef DC_R4_LAZY
#define DC_R4_LAZY 0
#endif
template <int LOOK, int PF, bool DW, bool INFO = false>
__global__ __launch_bounds__(kR3Threads) void k_replay_ref4(Mailbox mb0, u64 occ0, u32 stm0, const uint16_t* __restrict__ moves,
                                                           u32 n_games, u32 n_plies, u64* __restrict__ bitmap,
                                                           u64* __restrict__ digests, u64* __restrict__ partial,
                                                           uint8_t* __restrict__ info = nullptr,
                                                           Board* __restrict__ boards = nullptr) {
  __shared__ __attribute__((aligned(16))) unsigned char r4_smem[kR3TabBytes + kR3MbBytes];
  u64* btw = reinterpret_cast<u64*>(r4_smem);
  u32* mb = reinterpret_cast<u32*>(r4_smem + kR3TabBytes);
  const u32 tid = threadIdx.x;
  for (u32 e = tid; e < 4096; e += kR3Threads) {
    btw[e] = between((int)(e & 63), (int)(e >> 6));
    reinterpret_cast<u32*>(r4_smem + 4096 * 8)[e] = replay_geo(e);
  }
  __syncthreads();
  const u32 lane = lane_id();
  const u32 words = (n_games + 63) >> 6;
  const u32 tid4 = tid * 4;
  const u32 last = n_plies - 1;
  const u32 row_bytes = n_games * 2;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)moves, 0, n_plies * row_bytes, 0x00020000);
  u32* my = mb + tid;
  u32 validated = 0, accepted = 0;
  u64 dsum = 0, dxor = 0;
  for (u32 round = 0;; ++round) {
    const u32 c = (round * gridDim.x + blockIdx.x) * (kR3Threads / 64) + (tid >> 6);
    if (c >= words) break;
    const u32 g = (c << 6) | lane;
    const bool active = g < n_games;
    const u64 amask = ballot(active);
    const u32 goff = (active ? g : n_games - 1) * 2;
    // DW (even n_games: every row dword-aligned): the lane loads the dword
    // holding its move and its neighbour's and rotates its own into the low
    // half where it is used.  A u16 load is zero-extended by the compiler
    // right after the load, i.e. at the loop's back edge, where that forces
    // s_waitcnt vmcnt(0) on all PF prefetched moves, the youngest issued one
    // ply earlier.  Every use of m reads only its low 16 bits (12-bit
    // indices, 16-bit compares), so the neighbour's half is harmless.
    const u32 rot = DW ? (goff & 2u) << 3 : 0u;
    auto load_move = [&](u32 p) -> u32 {
      const u32 so = min(p, last) * row_bytes;
      if constexpr (DW) return __builtin_amdgcn_raw_buffer_load_b32(rs, goff & ~3u, so, 0);
      else return __builtin_amdgcn_raw_buffer_load_b16(rs, goff, so, 0);
    };
    auto move_of = [&](u32 d) -> u32 { return DW ? __builtin_amdgcn_alignbit(d, d, rot) : d; };
#pragma unroll
    for (u32 j = 0; j < 8; ++j) my[j * kR3Threads] = mb0.d[j];
    u64 occ = occ0;
    u32 stm = stm0;
    u32 nvalw = 0, nacc = 0;
    u32 buf[PF];
#pragma unroll
    for (int k = 0; k < PF; ++k) buf[k] = load_move((u32)k);
    u32 bw_lo = 0, bw_hi = 0;  // lane j holds the ballot word of ply 64q + j
    struct Tab {
      u64 bt;
      u32 gw;
    };
    auto tab = [&](u32 m) {
      return Tab{*reinterpret_cast<const u64*>(r4_smem + ((m << 3) & 0x7FF8u)),
                 *reinterpret_cast<const u32*>(r4_smem + 4096 * 8 + ((m << 2) & 0x3FFCu))};
    };
    // LOOK: `nx` holds ply p's tables on entry and ply p + 1's (move mnext) on
    // exit; their reads issue after ply p's mailbox reads, which LDS returns
    // first (in order), so the wait for the mailbox never waits on them
    Tab nx{0, 0};
    auto ply_step = [&](u32 m, u32 slot, u32 mnext, u32 p) {
      const u32 m2 = m << 2, m3 = m << 3;
      const u32 af = __builtin_amdgcn_bitop3_b32(m << 9, tid4, 0x7000u, 0xE4);
      const u32 at = __builtin_amdgcn_bitop3_b32(m3, tid4, 0x7000u, 0xE4);
      const Tab t0 = LOOK ? nx : tab(m);
      const u32 wf = *reinterpret_cast<const u32*>(r4_smem + kR3TabBytes + af);
      const u32 wt = *reinterpret_cast<const u32*>(r4_smem + kR3TabBytes + at);
      if (LOOK) nx = tab(mnext);
      const u64 bt = t0.bt;
      const u32 gw = t0.gw;
      const u32 st = (m >> 4) & 28;
      const u32 rawt = __builtin_amdgcn_ubfe(wt, st, 4);
#if DC_R4_LAZY
      // a square's nibble is live only while occ has it (v_lshrrev_b64 takes
      // the shift's low 6 bits: f = m & 63 needs no mask)
      const u32 nib = ((u32)(occ >> (m & 63)) & 1u) ? __builtin_amdgcn_ubfe(wf, m2, 4) : 0u;
      const u32 nibt = ((u32)(occ >> ((m >> 6) & 63)) & 1u) ? rawt : 0u;
#else
      const u32 nib = __builtin_amdgcn_ubfe(wf, m2, 4);
      const u32 nibt = rawt;
#endif
      const u32 x = nibt ^ stm;
      const u32 shift = nib | (__builtin_amdgcn_ubfe(kEnemyLut, x, 1) << 4);
      const u32 geo_ok = __builtin_amdgcn_ubfe(gw, shift, 1), own = __builtin_amdgcn_ubfe(kOwnLut, x, 1);
      const u32 okb = __builtin_amdgcn_bitop3_b32(geo_ok, own, nib ^ stm, 0x10);  // a & ~b & ~c: only bit 0
      // okb has only bit 0; blocked != 0 iff a square between f and t is
      // occupied, so ok = blocked < okb is one compare (the btw read issues
      // with the other three for every lane).  OOR (bit 15) and the sentinel
      // are 16-bit compares whose masks combine in SALU; every other use of m
      // reads only its low 12 bits, so the u16 load needs no zero-extension.
      const u32 blocked = __builtin_amdgcn_bitop3_b32((u32)bt, (u32)occ, (u32)(bt >> 32) & (u32)(occ >> 32), 0xEA);  // (a & b) | c
      const bool geo_pass = blocked < okb, in_range = (uint16_t)m < 0x8000u;
      const bool ok = geo_pass & in_range;
      const u64 w = ballot(geo_pass) & ballot(in_range);  // two compare masks, one s_and (ballot(ok) rematerialises)
      // the lanes' ballot words are written before the make-move branch, so the
      // compare's own mask feeds both (no mask rematerialised after the branch)
      asm volatile("s_mov_b32 m0, %4\n\tv_writelane_b32 %0, %2, m0\n\tv_writelane_b32 %1, %3, m0"
                   : "+v"(bw_lo), "+v"(bw_hi)
                   : "s"((u32)w), "s"((u32)(w >> 32)), "s"(slot)
                   : "m0");
      if constexpr (INFO) {
        // cell kind by kind code (P0 N1 B2 R3 Q4 K5 X6; code 0 never moves)
        constexpr u32 kCellKind = (0u << 4) | (1u << 8) | (5u << 12) | (6u << 16) | (2u << 20) | (3u << 24) | (4u << 28);
        const u32 code = __builtin_amdgcn_ubfe(kCellKind, (nib >> 1) << 2, 4) | (nibt ? 8u : 0u);
        if (active) info[(size_t)p * n_games + g] = (uint8_t)(ok ? code : 0xFFu);
      }
      if (ok) {
#if !DC_R4_LAZY
        atomicXor(reinterpret_cast<u32*>(r4_smem + kR3TabBytes + af), nib << m2);
#endif
        atomicXor(reinterpret_cast<u32*>(r4_smem + kR3TabBytes + at), (nib ^ rawt) << st);
        occ = bop3<0xBA>(occ, 1ull << (m & 63), 1ull << ((m >> 6) & 63));
        stm ^= 1;
      }
      nvalw += (u32)__popcll(ballot((uint16_t)m != 0xFFFFu) & amask);  // wave-uniform (SALU)
    };
    // accepted moves are counted from the ballot words (one popcount pair per
    // lane per 64 plies) instead of per ply and lane
    auto flush = [&](u32 base, u32 n) {
      if (lane < n) {
        const u64 word = (((u64)bw_hi << 32) | bw_lo) & amask;
        nacc += (u32)__popcll(word);
        if (bitmap) bitmap[(size_t)(base + lane) * words + c] = word;
      }
    };
    u32 ply = 0;
    if (LOOK) nx = tab(move_of(buf[0]));
    for (; ply + PF <= n_plies; ply += PF) {
      const u32 s0 = ply & 63;
#pragma unroll
      for (int k = 0; k < PF; ++k) {
        const u32 m = move_of(buf[k]);
        buf[k] = load_move(ply + PF + k);
        ply_step(m, s0 + k, LOOK ? move_of(buf[(k + 1) % PF]) : 0u, ply + k);  // k = PF - 1: ply + PF, reloaded at k = 0
      }
      if (((ply + PF) & 63) == 0) flush(ply + PF - 64, 64);
    }
#pragma unroll
    for (int k = 0; k < PF - 1; ++k)
      if (ply + k < n_plies) ply_step(move_of(buf[k]), (ply + k) & 63, LOOK ? move_of(buf[k + 1]) : 0u, ply + k);
    if ((n_plies & 63) != 0) flush(n_plies & ~63u, n_plies & 63);
    accepted += nacc;  // a wave-level count: only the block sum is used
    if (lane == 0) validated += nvalw;  // wave-level count, added once per wave
    if (active) {
      Board b{0, 0, 0, 0};
#pragma unroll
      for (u32 j = 0; j < 8; ++j) {
        const u32 d = my[j * kR3Threads];
        b.b0 |= (u64)gather_nibble_bits(d) << (8 * j);
        b.b1 |= (u64)gather_nibble_bits(d >> 1) << (8 * j);
        b.b2 |= (u64)gather_nibble_bits(d >> 2) << (8 * j);
        b.b3 |= (u64)gather_nibble_bits(d >> 3) << (8 * j);
      }
      if (DC_R4_LAZY) b = Board{b.b0 & occ, b.b1 & occ, b.b2 & occ, b.b3 & occ};  // stale nibbles of vacated squares
      const u64 dg = board_digest(b, stm);
      if (digests) digests[g] = dg;
      if (INFO && boards) boards[g] = b;  // the state hash's final boards (round 6)
      dsum += dg;
      dxor ^= dg;
    }
  }
  const u64 sv = wave_sum64(validated), sa = wave_sum64(accepted), sd = wave_sum64(dsum);
  u64 xx = dxor;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) xx ^= __shfl_xor(xx, o, 64);
  __syncthreads();
  u64* ws = btw;
  const u32 w = tid >> 6;
  if (lane == 0) {
    ws[w * 4 + 0] = sv;
    ws[w * 4 + 1] = sa;
    ws[w * 4 + 2] = sd;
    ws[w * 4 + 3] = xx;
  }
  __syncthreads();
  if (tid == 0) {
    u64 r[5] = {0, 0, 0, 0, 0};
    for (u32 k = 0; k < kR3Threads / 64; ++k) {
      r[0] += ws[k * 4 + 0];
      r[1] += ws[k * 4 + 1];
      r[3] += ws[k * 4 + 2];
      r[4] ^= ws[k * 4 + 3];
    }
    r[2] = r[0] - r[1];
    for (int k = 0; k < 5; ++k) partial[(size_t)blockIdx.x * 5 + k] = r[k];
  }
}

// --------------------------------------------------------------- generator
// k-th accepted move in (from, to) order: own pieces by ascending square, each
// piece's targets ascending.
__device__ __forceinline__ u32 ref_kth_move(const Board& b, u32 stm, u32 k) {
  const u64 occ = occupied(b);
  u64 own = stm ? b.b0 : (occ & ~b.b0);
  while (own) {
    const int f = lsb(own);
    own &= own - 1;
    const u64 t = ref_piece_targets(b, f, stm, nibble(b, f) >> 1);
    const u32 c = pc(t);
    if (k < c) return (u32)f | ((u32)select_bit(t, k) << 6);
    k -= c;
  }
  return 0xFFFFu;  // unreachable when k < count
}

// K5, round 2.  The k-th move in (from, to) order without a per-piece loop:
// every lane evaluates its position in the side-to-move view (white_view), so
// one code path serves lanes of either colour; the source square of the k-th
// move is found by a 6-step binary search over square prefixes, each step a
// source-restricted bulk count (ref_count_from; prefix masks are built in real
// square order and flipped into the view), and its target is the kk-th set bit
// of that one piece's target set (ref_piece_targets_w).  The round-1 kernel
// (k_gen_games_ref_v1: a per-piece loop with a per-kind switch) issued 3,842
// VALU per wave and ply with 22 % of lanes active.  Same games, bit for bit
// (tests/golden: C4 moves SHA-256).
#ifdef DC_AB_KNOBS  // round-2 generator, kept for A/B measurement only (DC_GEN=2)
__global__ __launch_bounds__(256) void k_gen_games_ref_v2(u64 seed, u64 first_game, u32 n_games, u32 n_plies,
                                                          u32 noise_per_256, uint16_t* __restrict__ out) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_games) return;
  u64 s = seed ^ (first_game + g);
  Board b{0, 0, 0, 0};
  startpos_board(b);
  u32 stm = 0;
  bool over = false;
  for (u32 ply = 0; ply < n_plies; ++ply) {
    uint16_t* slot = out + (size_t)ply * n_games + g;
    const Board w = view_sel(b, stm);
    const u32 flip = stm ? 56u : 0u;
    const Sides sw = sides<0>(w);
    const Props pr = make_props(sw.empty);
    const u32 n = over ? 0u : ref_count_from_w(sw, pr, ~0ull);
    over = n == 0;
    u64 r = 0;
    if (!over) r = splitmix_next(s);
    const bool noise = (u32)(r & 0xFF) < noise_per_256;
    // the k-th move of the (from, to)-ordered list.  Own pieces in real square
    // order p_0 < p_1 < ...; c(j) = #moves of p_0..p_{j-1}.  Games start at
    // startpos and REF never adds a piece, so there are at most 16: four
    // halving steps find the largest j with c(j) <= k.
    const u32 k = (u32)(((r >> 32) * (u64)n) >> 32);
    const u64 occ = occupied(b);
    const u64 own = stm ? b.b0 : (occ & ~b.b0);
    const u32 np = (u32)__popcll(own);
    u32 lo = 0, clo = 0;
#pragma unroll
    for (u32 step = 8; step; step >>= 1) {
      const u32 mid = lo + step;
      const u64 real = mid < np ? ((1ull << select_bit_bf(own, mid)) - 1) : ~0ull;
      const u64 view = stm ? flip_rows(real) : real;
      const u32 c = (over || mid >= np) ? 0xFFFFFFFFu : ref_count_from_w(sw, pr, view);
      if (c <= k) {
        lo = mid;
        clo = c;
      }
    }
    const u32 f = over ? 0u : select_bit_bf(own, lo);
    const u64 tv = ref_piece_targets_w(w, (int)(f ^ flip));
    const u64 treal = stm ? flip_rows(tv) : tv;
    const u32 kth = (n && k - clo < (u32)__popcll(treal)) ? (f | (select_bit_bf(treal, k - clo) << 6)) : 0u;
    const u32 m = noise ? (u32)((r >> 8) & 0xFFF) : kth;
    *slot = over ? (uint16_t)0xFFFF : (uint16_t)m;
    const bool ok = !over && (!noise || ref_verdict(b, stm, m) == V_OK);
    if (ok) {
      ref_make(b, (int)(m & 63), (int)((m >> 6) & 63));
      stm ^= 1;
    }
  }
}
#endif  // DC_AB_KNOBS

// K5, round 3 (k_gen_games_ref).  The same games as round 2 (the k-th move in
// (from, to) order of real squares; C4's moves SHA-256 is the check), with
// the per-ply work restructured so that no source-restricted bulk count is
// repeated:
//   - pawns as four direction source sets (push, double push, two captures),
//     whose restricted counts are four masked popcounts;
//   - every other piece (at most 2 knights, 1 king, 3 diagonal and 3
//     orthogonal sliders from startpos: REF never adds a piece) as a slot
//     holding its real square and its move count, its targets from LDS tables
//     (knight, king, and per-direction rays whose first blocker is one
//     lsb/msb: r ^ ray[first blocker]);
//   - the source square of the k-th move by a 6-step binary search over real
//     squares on those slots and sets (round 2: four source-restricted bulk
//     counts with slider fills, 1,662 VALU per move);
//   - only the chosen piece's targets are built again.
struct GenTabs {
  u64 ray[8][64];  // 0 N, 1 S, 2 E, 3 W, 4 NE, 5 SW, 6 NW, 7 SE: squares beyond s to the edge
  u64 kn[64], kg[64];
};

__device__ __forceinline__ void gen_tabs_build(GenTabs& T) {
  constexpr int dx[8] = {1, -1, 0, 0, 1, -1, 1, -1}, dy[8] = {0, 0, 1, -1, 1, -1, -1, 1};
  for (u32 e = threadIdx.x; e < 8 * 64; e += blockDim.x) {
    const int d = (int)(e >> 6), sq = (int)(e & 63);
    u64 r = 0;
    int x = (sq >> 3) + dx[d], y = (sq & 7) + dy[d];
    while (x >= 0 && x < 8 && y >= 0 && y < 8) {
      r |= 1ull << (8 * x + y);
      x += dx[d];
      y += dy[d];
    }
    T.ray[d][sq] = r;
  }
  for (u32 sq = threadIdx.x; sq < 64; sq += blockDim.x) {
    const int x = (int)(sq >> 3), y = (int)(sq & 7);
    u64 kn = 0, kg = 0;
    for (int a = -2; a <= 2; ++a)
      for (int c = -2; c <= 2; ++c) {
        const int X = x + a, Y = y + c;
        if (X < 0 || X > 7 || Y < 0 || Y > 7) continue;
        const int aa = a < 0 ? -a : a, cc = c < 0 ? -c : c;
        if (aa * cc == 2) kn |= 1ull << (8 * X + Y);
        if (aa <= 1 && cc <= 1 && (aa | cc)) kg |= 1ull << (8 * X + Y);
      }
    T.kn[sq] = kn;
    T.kg[sq] = kg;
  }
}

// DC_GEN_LDS1 (round 6): every table read is its own ds_read_b64.  Reads of
// two rows at one square (NE and NW, N and E) sit 512 B apart, so the
// compiler merged them into ds_read2st64_b64, which serves a wave in 16-lane
// groups banked (a/4) mod 32: squares s and s + 16k of one group collide, and
// per-lane squares are random.  ds_read_b64 serves 32-lane groups banked
// (a/4) mod 64 (only s and s + 32 collide) at 2 LDS cycles against 8: the
// kernel had 2.10 conflict cycles per LDS cycle.  The row index goes through
// an empty asm so no two reads share a base register.  Measured (same box,
// alternating, profiles/r06/ab_gen_lds1.txt): conflicts 2.10 -> 0.74 per LDS
// cycle and wait fraction 0.67 -> 0.63, but 41 LDS reads per ply slot instead
// of 29 and 4.7 % more VALU (the addresses), and the kernel 18.27 -> 18.57 ms:
// the conflicts were not what it waits on.  Off (A/B knob).
#ifndef DC_GEN_LDS1
#define DC_GEN_LDS1 0
#endif
template <int D>
__device__ __forceinline__ u64 gen_tab_ray(const GenTabs& T, int s) {
#if DC_GEN_LDS1
  asm volatile("" : "+v"(s));
#endif
  return T.ray[D][s];
}

// Ray of direction D from s up to and including the first occupied square:
// the table ray minus the ray beyond that blocker (a sentinel blocker on the
// edge square whose ray is empty makes the unblocked case the same formula).
template <int D>
__device__ __forceinline__ u64 gen_ray(const GenTabs& T, int s, u64 occ) {
  const u64 r = gen_tab_ray<D>(T, s);
  const u64 bl = r & occ;
  const int b = (D & 1) == 0 ? lsb(bl | (1ull << 63)) : msb(bl | 1ull);
  return r ^ gen_tab_ray<D>(T, b);
}

// Ray of a direction D that runs to higher squares (N, E, NE, NW) up to and
// including the first occupied square, without a bit scan: bl ^ (bl - 1) is
// every square up to bl's lowest bit (all squares when bl = 0).  A south-going
// ray is the north-going one of the vertically flipped board (rows swapped by
// flip_rows, s ^ 56); a count does not care which board it was taken on.
template <int D>
__device__ __forceinline__ u64 gen_ray_up(const GenTabs& T, int s, u64 occ) {
  static_assert(D == 0 || D == 2 || D == 4 || D == 6, "a direction to higher squares");
  const u64 r = gen_tab_ray<D>(T, s);
  const u64 bl = r & occ;
  return r & (bl ^ (bl - 1));
}

#ifndef DC_GEN_MINW
#define DC_GEN_MINW 1
#endif
// DC_GEN_POSRAY (round 5): the slot counts take every ray but W through
// gen_ray_up (S, SW, SE on the flipped board); the round-4 form scanned each
// ray's first blocker with a 64-bit lsb / msb and read a second table entry,
// 33 % of the kernel's issue cycles in tools/bbprof.py's count.
#ifndef DC_GEN_POSRAY
#define DC_GEN_POSRAY 1
#endif
// DC_GEN_QSLOT (round 5): the queen (REF never adds a piece: at most one from
// startpos) is one slot counting both ray sets, beside two bishop and two rook
// slots -- 8 slots for the binary search to sum instead of 9 (2 B + Q, 2 R + Q).
#ifndef DC_GEN_QSLOT
#define DC_GEN_QSLOT 1
#endif
// DC_GEN_NOBR (round 6 A/B): the slider slots' ray reads without the per-slot
// wave-uniform skip (an empty slot reads square 0 and its count is masked).
// DC_GEN_BATCH (round 6 A/B): every table read of a ply (27 for the slot
// counts, 11 for the chosen piece) issued ahead of its use, held there by
// empty asms.  The kernel waits 0.67 of its wave cycles, with one
// lgkmcnt(0) after nearly every read, so the reads looked like the bound.
// Measured (profiles/r06/ab_gen_batch.txt, same box, alternating): 18.20 ->
// 19.29 ms.  The held reads take 117-122 VGPRs (4 waves/SIMD instead of 6),
// and with more reads in flight per wave the conflicts rose from 2.10 to
// 3.58 per LDS cycle: the waits were overlapped by other waves' issue all
// along.  Both off.
#ifndef DC_GEN_NOBR
#define DC_GEN_NOBR 0
#endif
#ifndef DC_GEN_BATCH
#define DC_GEN_BATCH 0
#endif
#if DC_GEN_BATCH && !(DC_GEN_POSRAY && DC_GEN_QSLOT)
#error "DC_GEN_BATCH needs DC_GEN_POSRAY and DC_GEN_QSLOT"
#endif
constexpr int kGenLine = DC_GEN_QSLOT ? 2 : 3;  // slots per slider line kind
constexpr int kGenSlots = 3 + 2 * kGenLine + (DC_GEN_QSLOT ? 1 : 0);
__global__ __launch_bounds__(256, DC_GEN_MINW) void k_gen_games_ref(u64 seed, u64 first_game, u32 n_games, u32 n_plies,
                                                       u32 noise_per_256, uint16_t* __restrict__ out) {
  __shared__ GenTabs T;
  gen_tabs_build(T);
  __syncthreads();
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_games) return;
  u64 s = seed ^ (first_game + g);
  Board b{0, 0, 0, 0};
  startpos_board(b);
  u32 stm = 0;
  bool over = false;
  for (u32 ply = 0; ply < n_plies; ++ply) {
    uint16_t* slot = out + (size_t)ply * n_games + g;
    const Board w = view_sel(b, stm);  // white to move (rows flipped for Black)
    const u32 flip = stm ? 56u : 0u;
    const Sides sw = sides<0>(w);
    const u64 E = sw.empty, no = sw.notown, occ = sw.occ;
#if DC_GEN_POSRAY
    const u64 occF = flip_rows(occ), noF = flip_rows(no);  // the board with its rows swapped
#endif
    // pawn sources per direction class (ref_count_from_w's pawn terms)
    const u64 S1 = sw.P & sh<-8>(E);
    const u64 S2 = S1 & kRow(1) & sh<-16>(E);
    const u64 SL = sw.P & sh<-7>(sw.enemy & kNotH);
    const u64 SR = sw.P & sh<-9>(sw.enemy & kNotA);
    u32 n = pc(S1) + pc(S2) + pc(SL) + pc(SR);
    // piece slots: (real square << 8) | move count; square 64 = empty slot
    u32 sl[kGenSlots];
    auto take = [](u64& rem, int& sv) {  // next piece of a set: its view square, or -1
      const bool any = rem != 0;
      sv = any ? lsb(rem) : 0;
      rem &= rem - 1;
      return any;
    };
#if DC_GEN_BATCH
    {
      // every slot's square first (view squares; 0 for an empty slot), then
      // every table read, then the counts: the reads issue together and
      // their latency overlaps (the slot-by-slot form waited on each read)
      u64 rem = sw.N;
      int n0, n1, k0, b0, b1, r0, r1, q0;
      const bool an0 = take(rem, n0), an1 = take(rem, n1);
      rem = sw.K;
      const bool ak = take(rem, k0);
      rem = sw.D & ~sw.O;
      const bool ab0 = take(rem, b0), ab1 = take(rem, b1);
      rem = sw.O & ~sw.D;
      const bool ar0 = take(rem, r0), ar1 = take(rem, r1);
      rem = sw.D & sw.O;
      const bool aq = take(rem, q0);
      u64 tn0 = T.kn[n0], tn1 = T.kn[n1], tk = T.kg[k0];
      u64 b0ne = T.ray[4][b0], b0nw = T.ray[6][b0], b0se = T.ray[4][b0 ^ 56], b0sw = T.ray[6][b0 ^ 56];
      u64 b1ne = T.ray[4][b1], b1nw = T.ray[6][b1], b1se = T.ray[4][b1 ^ 56], b1sw = T.ray[6][b1 ^ 56];
      u64 r0n = T.ray[0][r0], r0e = T.ray[2][r0], r0w = T.ray[3][r0], r0s = T.ray[0][r0 ^ 56];
      u64 r1n = T.ray[0][r1], r1e = T.ray[2][r1], r1w = T.ray[3][r1], r1s = T.ray[0][r1 ^ 56];
      u64 qn = T.ray[0][q0], qe = T.ray[2][q0], qw = T.ray[3][q0], qne = T.ray[4][q0], qnw = T.ray[6][q0];
      u64 qs = T.ray[0][q0 ^ 56], qse = T.ray[4][q0 ^ 56], qsw = T.ray[6][q0 ^ 56];
      // (the empty asms hold the reads ahead of the counts: the scheduler
      // otherwise sinks each read to its use, one wait per read)
      asm volatile("" : "+v"(tn0), "+v"(tn1), "+v"(tk), "+v"(b0ne), "+v"(b0nw), "+v"(b0se), "+v"(b0sw));
      asm volatile("" : "+v"(b1ne), "+v"(b1nw), "+v"(b1se), "+v"(b1sw), "+v"(r0n), "+v"(r0e), "+v"(r0w), "+v"(r0s));
      asm volatile("" : "+v"(r1n), "+v"(r1e), "+v"(r1w), "+v"(r1s), "+v"(qn), "+v"(qe), "+v"(qw), "+v"(qne));
      asm volatile("" : "+v"(qnw), "+v"(qs), "+v"(qse), "+v"(qsw));
      // W rays: the table ray minus the ray beyond its first blocker (gen_ray<3>)
      const u64 r0w2 = T.ray[3][msb((r0w & occ) | 1ull)], r1w2 = T.ray[3][msb((r1w & occ) | 1ull)];
      const u64 qw2 = T.ray[3][msb((qw & occ) | 1ull)];
      auto up = [](u64 r, u64 o) {  // gen_ray_up on a table ray already read
        const u64 bl = r & o;
        return r & (bl ^ (bl - 1));
      };
      auto put = [&](int j, bool any, int sv, u32 c) {
        c = any ? c : 0u;
        sl[j] = any ? (((u32)sv ^ flip) << 8) | c : 64u << 8;
        n += c;
      };
      put(0, an0, n0, pc(tn0 & no));
      put(1, an1, n1, pc(tn1 & no));
      put(2, ak, k0, pc(tk & no));
      put(3, ab0, b0, pc((up(b0ne, occ) | up(b0nw, occ)) & no) + pc((up(b0se, occF) | up(b0sw, occF)) & noF));
      put(4, ab1, b1, pc((up(b1ne, occ) | up(b1nw, occ)) & no) + pc((up(b1se, occF) | up(b1sw, occF)) & noF));
      put(5, ar0, r0, pc((up(r0n, occ) | up(r0e, occ) | (r0w ^ r0w2)) & no) + pc(up(r0s, occF) & noF));
      put(6, ar1, r1, pc((up(r1n, occ) | up(r1e, occ) | (r1w ^ r1w2)) & no) + pc(up(r1s, occF) & noF));
      put(7, aq, q0,
          pc((up(qn, occ) | up(qe, occ) | (qw ^ qw2) | up(qne, occ) | up(qnw, occ)) & no) +
              pc((up(qs, occF) | up(qse, occF) | up(qsw, occF)) & noF));
    }
#else
    {
      u64 rem = sw.N;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        int sv;
        const bool any = take(rem, sv);
        const u32 c = any ? pc(T.kn[sv] & no) : 0u;
        sl[j] = any ? (((u32)sv ^ flip) << 8) | c : 64u << 8;
        n += c;
      }
      rem = sw.K;
      int sv;
      const bool any = take(rem, sv);
      const u32 c = any ? pc(T.kg[sv] & no) : 0u;
      sl[2] = any ? (((u32)sv ^ flip) << 8) | c : 64u << 8;
      n += c;
    }
    {
      u64 rem = DC_GEN_QSLOT ? (sw.D & ~sw.O) : sw.D;
#pragma unroll
      for (int j = 0; j < kGenLine; ++j) {
        int sv;
        const bool any = take(rem, sv);
        u32 c = 0;
        if (DC_GEN_NOBR || any) {  // (DC_GEN_NOBR = 0: skipped by a wave none of whose games has a j-th such slider)
#if DC_GEN_POSRAY
          const int sf = sv ^ 56;  // SW / SE are NW / NE of the flipped board
          c = pc((gen_ray_up<4>(T, sv, occ) | gen_ray_up<6>(T, sv, occ)) & no) +
              pc((gen_ray_up<4>(T, sf, occF) | gen_ray_up<6>(T, sf, occF)) & noF);
#else
          const u64 t = gen_ray<4>(T, sv, occ) | gen_ray<5>(T, sv, occ) | gen_ray<6>(T, sv, occ) | gen_ray<7>(T, sv, occ);
          c = pc(t & no);
#endif
        }
        c = any ? c : 0u;
        sl[3 + j] = any ? (((u32)sv ^ flip) << 8) | c : 64u << 8;
        n += c;
      }
      rem = DC_GEN_QSLOT ? (sw.O & ~sw.D) : sw.O;
#pragma unroll
      for (int j = 0; j < kGenLine; ++j) {
        int sv;
        const bool any = take(rem, sv);
        u32 c = 0;
        if (DC_GEN_NOBR || any) {
#if DC_GEN_POSRAY
          c = pc((gen_ray_up<0>(T, sv, occ) | gen_ray_up<2>(T, sv, occ) | gen_ray<3>(T, sv, occ)) & no) +
              pc(gen_ray_up<0>(T, sv ^ 56, occF) & noF);  // S: N of the flipped board
#else
          const u64 t = gen_ray<0>(T, sv, occ) | gen_ray<1>(T, sv, occ) | gen_ray<2>(T, sv, occ) | gen_ray<3>(T, sv, occ);
          c = pc(t & no);
#endif
        }
        c = any ? c : 0u;
        sl[3 + kGenLine + j] = any ? (((u32)sv ^ flip) << 8) | c : 64u << 8;
        n += c;
      }
#if DC_GEN_QSLOT
      {
        rem = sw.D & sw.O;
        int sv;
        const bool any = take(rem, sv);
        u32 c = 0;
        if (DC_GEN_NOBR || any) {
          const int sf = sv ^ 56;
#if DC_GEN_POSRAY
          c = pc((gen_ray_up<0>(T, sv, occ) | gen_ray_up<2>(T, sv, occ) | gen_ray<3>(T, sv, occ) |
                  gen_ray_up<4>(T, sv, occ) | gen_ray_up<6>(T, sv, occ)) & no) +
              pc((gen_ray_up<0>(T, sf, occF) | gen_ray_up<4>(T, sf, occF) | gen_ray_up<6>(T, sf, occF)) & noF);
#else
          (void)sf;
          const u64 t = gen_ray<0>(T, sv, occ) | gen_ray<1>(T, sv, occ) | gen_ray<2>(T, sv, occ) | gen_ray<3>(T, sv, occ) |
                        gen_ray<4>(T, sv, occ) | gen_ray<5>(T, sv, occ) | gen_ray<6>(T, sv, occ) | gen_ray<7>(T, sv, occ);
          c = pc(t & no);
#endif
        }
        c = any ? c : 0u;
        sl[kGenSlots - 1] = any ? (((u32)sv ^ flip) << 8) | c : 64u << 8;
        n += c;
      }
#endif
    }
#endif
    if (over) n = 0;
    over = n == 0;
    u64 r = 0;
    if (!over) r = splitmix_next(s);
    const bool noise = (u32)(r & 0xFF) < noise_per_256;
    const u32 k = (u32)(((r >> 32) * (u64)n) >> 32);
    // the k-th move's real source square: the first x with D(x) > k, where
    // D(x) = moves whose real source square is <= x
    u32 lo = 0, dlo = 0;
#pragma unroll
    for (u32 step = 32; step; step >>= 1) {
      const u32 x = lo + step - 1;
      const u64 mr = (2ull << x) - 1;  // real squares <= x (x = 63: all)
      const u64 mv = stm ? flip_rows(mr) : mr;
      u32 d = pc(S1 & mv) + pc(S2 & mv) + pc(SL & mv) + pc(SR & mv);
#pragma unroll
      for (int j = 0; j < kGenSlots; ++j) d += (sl[j] >> 8) <= x ? (sl[j] & 0xFF) : 0u;
      if (d <= k) {
        lo = x + 1;
        dlo = d;
      }
    }
    // the piece whose targets are needed: the k-th move's source, or a noise
    // move's source (its verdict is then "t is one of that piece's targets":
    // ref_verdict's REF rules, chess.rs:82-125, restated set-wise -- the same
    // targets that give n; an empty or enemy square has none)
    const u32 mnoise = (u32)((r >> 8) & 0xFFF);
    const u32 f = noise ? (mnoise & 63) : lo;  // real
    const int fv = (int)(f ^ flip) & 63;
    const u64 bit = 1ull << fv;
    // targets of the piece on fv (view), every class masked by its kind
    u64 tv = (((S1 & bit) != 0) ? sh<8>(bit) : 0ull) | (((S2 & bit) != 0) ? sh<16>(bit) : 0ull) |
             (((SL & bit) != 0) ? sh<7>(bit) : 0ull) | (((SR & bit) != 0) ? sh<9>(bit) : 0ull);
#if DC_GEN_BATCH
    // every table row of fv read together (the piece's kind selects them after)
    u64 xn = T.kn[fv], xk = T.kg[fv], x4 = T.ray[4][fv], x6 = T.ray[6][fv], x4f = T.ray[4][fv ^ 56];
    u64 x6f = T.ray[6][fv ^ 56], x0 = T.ray[0][fv], x2 = T.ray[2][fv], x3 = T.ray[3][fv], x0f = T.ray[0][fv ^ 56];
    asm volatile("" : "+v"(xn), "+v"(xk), "+v"(x4), "+v"(x6), "+v"(x4f), "+v"(x6f), "+v"(x0), "+v"(x2), "+v"(x3), "+v"(x0f));
    const u64 x3b = T.ray[3][msb((x3 & occ) | 1ull)];
    auto upr = [](u64 r, u64 o) {
      const u64 bl = r & o;
      return r & (bl ^ (bl - 1));
    };
    const u64 md = (sw.D & bit) != 0 ? ~0ull : 0ull, mo = (sw.O & bit) != 0 ? ~0ull : 0ull;
    u64 tp = ((sw.N & bit) != 0 ? xn : 0ull) | ((sw.K & bit) != 0 ? xk : 0ull);
    tp |= md & (upr(x4, occ) | upr(x6, occ) | flip_rows(upr(x4f, occF) | upr(x6f, occF)));
    tp |= mo & (upr(x0, occ) | upr(x2, occ) | (x3 ^ x3b) | flip_rows(upr(x0f, occF)));
#else
    u64 tp = ((sw.N & bit) != 0 ? T.kn[fv] : 0ull) | ((sw.K & bit) != 0 ? T.kg[fv] : 0ull);
#endif
#if DC_GEN_BATCH
#elif DC_GEN_POSRAY
    if ((sw.D & bit) != 0)
      tp |= gen_ray_up<4>(T, fv, occ) | gen_ray_up<6>(T, fv, occ) |
            flip_rows(gen_ray_up<4>(T, fv ^ 56, occF) | gen_ray_up<6>(T, fv ^ 56, occF));
    if ((sw.O & bit) != 0)
      tp |= gen_ray_up<0>(T, fv, occ) | gen_ray_up<2>(T, fv, occ) | gen_ray<3>(T, fv, occ) |
            flip_rows(gen_ray_up<0>(T, fv ^ 56, occF));
#else
    if ((sw.D & bit) != 0)
      tp |= gen_ray<4>(T, fv, occ) | gen_ray<5>(T, fv, occ) | gen_ray<6>(T, fv, occ) | gen_ray<7>(T, fv, occ);
    if ((sw.O & bit) != 0)
      tp |= gen_ray<0>(T, fv, occ) | gen_ray<1>(T, fv, occ) | gen_ray<2>(T, fv, occ) | gen_ray<3>(T, fv, occ);
#endif
    tv |= tp & no;
    const u64 treal = stm ? flip_rows(tv) : tv;
    const u32 kk = k - dlo;
    const u32 kth = (n && kk < (u32)__popcll(treal)) ? (f | (select_bit_bf(treal, kk) << 6)) : 0u;
    const u32 m = noise ? mnoise : kth;
    *slot = over ? (uint16_t)0xFFFF : (uint16_t)m;
    const bool ok = !over && (!noise || ((treal >> (mnoise >> 6)) & 1) != 0);
    if (ok) {
      ref_make(b, (int)(m & 63), (int)((m >> 6) & 63));
      stm ^= 1;
    }
  }
}

#ifdef DC_AB_KNOBS  // round-1 generator, kept for A/B measurement only (DC_GEN=1)
__global__ __launch_bounds__(256) void k_gen_games_ref_v1(u64 seed, u64 first_game, u32 n_games, u32 n_plies,
                                                          u32 noise_per_256, uint16_t* __restrict__ out) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_games) return;
  u64 s = seed ^ (first_game + g);
  Board b{0, 0, 0, 0};
  startpos_board(b);
  u32 stm = 0;
  bool over = false;
  for (u32 ply = 0; ply < n_plies; ++ply) {
    uint16_t* slot = out + (size_t)ply * n_games + g;
    if (over) {
      *slot = 0xFFFF;
      continue;
    }
    const u32 n = ref_count_rt(b, stm);
    if (n == 0) {
      over = true;
      *slot = 0xFFFF;
      continue;
    }
    const u64 r = splitmix_next(s);
    u32 m;
    if ((u32)(r & 0xFF) < noise_per_256) m = (u32)((r >> 8) & 0xFFF);
    else m = ref_kth_move(b, stm, (u32)(((r >> 32) * (u64)n) >> 32));
    *slot = (uint16_t)m;
    if (ref_verdict(b, stm, m) == V_OK) {
      ref_make(b, (int)(m & 63), (int)((m >> 6) & 63));
      stm ^= 1;
    }
  }
}
#endif  // DC_AB_KNOBS

// ------------------------------------------------------------- FIDE (K1/K2/K5)
__global__ __launch_bounds__(256) void k_validate_fide(const DevPos* __restrict__ pos, const uint16_t* __restrict__ moves,
                                                       u32 n, uint8_t* __restrict__ out, u32* done, u32 seq) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const DevPos p = pos[i];
    const Board b{p.bb[0], p.bb[1], p.bb[2], p.bb[3]};
    out[i] = (uint8_t)fide_verdict(b, p.stm & 1, pack_meta(p.castle, p.ep), moves[i]);
  }
  publish_done(done, seq);
}

__device__ __forceinline__ void apply_fide_one(DevPos* __restrict__ pos, const uint16_t* __restrict__ moves, u32 i,
                                               uint8_t* __restrict__ verdicts, uint8_t* __restrict__ info) {
  DevPos p = pos[i];
  Board b{p.bb[0], p.bb[1], p.bb[2], p.bb[3]};
  const u32 m = moves[i];
  const u32 meta = pack_meta(p.castle, p.ep);
  const u32 v = fide_verdict(b, p.stm & 1, meta, m);
  verdicts[i] = (uint8_t)v;
  if (v != V_OK) {
    if (info) info[i] = 0xFF;
    return;
  }
  const int f = (int)(m & 63), t = (int)((m >> 6) & 63);
  if (info) {
    const u32 code = nibble(b, f) >> 1;
    const u32 cell_kind = (code == KC_P) ? 0 : (code == KC_N) ? 1 : (code == KC_B) ? 2 : (code == KC_R) ? 3
                        : (code == KC_Q) ? 4 : (code == KC_K) ? 5 : 6;
    info[i] = (uint8_t)(cell_kind | (((occupied(b) >> t) & 1) << 3));
  }
  const u32 nm = fide_make_rt(b, p.stm & 1, meta, f, t, (int)((m >> 12) & 7));
  p.bb[0] = b.b0;
  p.bb[1] = b.b1;
  p.bb[2] = b.b2;
  p.bb[3] = b.b3;
  p.stm ^= 1;
  p.castle = (uint8_t)(nm & 15);
  p.ep = (nm & META_EP_VALID) ? (int8_t)((nm >> 4) & 63) : (int8_t)-1;
  pos[i] = p;
}

__global__ __launch_bounds__(256) void k_apply_fide(DevPos* __restrict__ pos, const uint16_t* __restrict__ moves, u32 n,
                                                    uint8_t* __restrict__ verdicts, uint8_t* __restrict__ info, u32* done,
                                                    u32 seq) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) apply_fide_one(pos, moves, i, verdicts, info);
  publish_done(done, seq);
}

__global__ __launch_bounds__(256) void k_replay_fide(Board start, u32 stm0, u32 meta0, const uint16_t* __restrict__ moves,
                                                     u32 n_games, u32 n_plies, u64* __restrict__ bitmap,
                                                     u64* __restrict__ digests, u64* __restrict__ partial) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = g < n_games;
  const u32 words = (n_games + 63) >> 6;
  Board b = start;
  u32 stm = stm0, meta = meta0;
  u32 validated = 0, accepted = 0;
  for (u32 ply = 0; ply < n_plies; ++ply) {
    const u32 m = active ? moves[(size_t)ply * n_games + g] : 0xFFFFu;
    bool ok = false;
    if (m != 0xFFFFu) {
      ++validated;
      ok = fide_verdict(b, stm, meta, m) == V_OK;
      if (ok) {
        meta = fide_make_rt(b, stm, meta, (int)(m & 63), (int)((m >> 6) & 63), (int)((m >> 12) & 7));
        stm ^= 1;
        ++accepted;
      }
    }
    const u64 word = ballot(ok);
    if (bitmap && lane_id() == 0 && (g >> 6) < words) bitmap[(size_t)ply * words + (g >> 6)] = word;
  }
  u64 d = 0;
  if (active) {
    d = board_digest(b, stm);
    if (digests) digests[g] = d;
  }
  block_stats(validated, accepted, d, partial);
}

__global__ __launch_bounds__(256) void k_gen_games_fide(u64 seed, u64 first_game, u32 n_games, u32 n_plies,
                                                        u32 noise_per_256, uint16_t* __restrict__ out) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_games) return;
  u64 s = seed ^ (first_game + g);
  Board b{0, 0, 0, 0};
  startpos_board(b);
  u32 stm = 0, meta = CR_WK | CR_WQ | CR_BK | CR_BQ;
  bool over = false;
  for (u32 ply = 0; ply < n_plies; ++ply) {
    uint16_t* slot = out + (size_t)ply * n_games + g;
    if (over) {
      *slot = 0xFFFF;
      continue;
    }
    const u32 n = fide_count_rt(b, stm, meta);
    if (n == 0) {
      over = true;
      *slot = 0xFFFF;
      continue;
    }
    const u64 r = splitmix_next(s);
    u32 m;
    if ((u32)(r & 0xFF) < noise_per_256) m = (u32)((r >> 8) & 0xFFF);
    else m = fide_kth_move(b, stm, meta, (u32)(((r >> 32) * (u64)n) >> 32));
    *slot = (uint16_t)m;
    if (fide_verdict(b, stm, meta, m) == V_OK) {
      meta = fide_make_rt(b, stm, meta, (int)(m & 63), (int)((m >> 6) & 63), (int)((m >> 12) & 7));
      stm ^= 1;
    }
  }
}

// ------------------------------------------------------------- launchers

// ------------------------------------------------------- the live validator
// One wave resident on one CU, launched on its own stream (dc_api.hip): polls
// the request words of a pinned coherent LiveBox (dc_kernels.h) with
// system-scope loads, validates (and applies) up to 64 moves, one per lane,
// with the same per-move code as k_validate_ref / k_apply_ref (FIDE:
// k_validate_fide / k_apply_fide), and writes stamped response words.  It
// leaves when asked (ctl) or after lease_ticks without a request, always:
// every loop trip reads the clock, so the wave cannot outlive its lease even
// if the host never asks it to stop.
__device__ __forceinline__ u32 sys_load(const u32* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void sys_store(u32* p, u32 v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

#ifndef DC_LIVE_EXP
#define DC_LIVE_EXP 0  // (measurement only) 1: validate answers V_OK without computing
#endif
#ifndef DC_LIVE_GATHER
#define DC_LIVE_GATHER 1  // n = 1 REF validate from cross-lane ballots (0: the board assembled in one lane)
#endif
// One request: lane e < n validates (applies) entry e; `fld(k, e)` reads
// field k of entry e.  Writes the stamped response words.
template <class F>
__device__ __forceinline__ void live_serve(LiveBox* box, u32 stamp, u32 n, bool apply, bool fide, u32 lane, F&& fld) {
  if (lane >= n) return;
  DevPos p;
  for (int q = 0; q < 4; ++q)
    p.bb[q] = (u64)fld(4 * q) | ((u64)fld(4 * q + 1) << 16) | ((u64)fld(4 * q + 2) << 32) |
              ((u64)fld(4 * q + 3) << 48);
  const u32 f16 = fld(16);
  p.stm = (uint8_t)(f16 & 0xFF);
  p.castle = (uint8_t)(f16 >> 8);
  p.ep = (int8_t)(uint8_t)fld(17);
  p.r0 = 0;
  p.r1 = 0;
  const uint16_t mv = (uint16_t)fld(18);
  uint8_t v = 0, info = 0;
  if (apply) {
    if (fide) apply_fide_one(&p, &mv, 0, &v, &info);
    else apply_ref_one(&p, &mv, 0, &v, &info);
    const u32 sh = stamp << 16;
    for (int q = 0; q < 4; ++q)
      for (int h = 0; h < 4; ++h)
        sys_store(&box->resp[(1 + 4 * q + h) * n + lane], sh | (u32)((p.bb[q] >> (16 * h)) & 0xFFFF));
    sys_store(&box->resp[17 * n + lane], sh | p.stm | ((u32)p.castle << 8));
    sys_store(&box->resp[18 * n + lane], sh | (u32)(uint8_t)p.ep);
  } else {
    const Board b{p.bb[0], p.bb[1], p.bb[2], p.bb[3]};
#if DC_LIVE_EXP == 1
    v = 0;  // (measurement only) no verdict work: the mailbox round trip alone
    (void)b;
    (void)mv;
#else
    v = (uint8_t)(fide ? fide_verdict(b, p.stm & 1, pack_meta(p.castle, p.ep), mv) : ref_verdict(b, p.stm & 1, mv));
#endif
  }
  sys_store(&box->resp[lane], (stamp << 16) | v | ((u32)info << 8));
}

__global__ __launch_bounds__(64) void k_live(LiveBox* box, u32 seq, u64 lease_ticks) {
  __shared__ uint16_t fld[kLiveFields * kLiveMax];
  // a poll reads the request's first kPoll words (an n = 1 request is 20) and
  // the stop word: two 64-byte lines, not the 256 bytes of all 64 lanes
  constexpr u32 kPoll = 1 + kLiveFields + 3;
  const u32 lane = threadIdx.x;
  u64 t_last = wall_clock64();
  for (u32 spin = 1;; ++spin) {
    const u32 stamp = live_stamp(seq + 1);
    const u32 w0 = lane < kPoll ? sys_load(&box->req[lane]) : (lane == kPoll ? sys_load(&box->ctl) : 0u);
    const u32 hdr = lane_bcast(w0, 0);
    if ((hdr >> 16) == stamp) {
      const u32 n = min(max(hdr & 127u, 1u), kLiveMax);
      const bool apply = (hdr >> 7) & 1, fide = (hdr >> 8) & 1;
      const u32 words = 1 + kLiveFields * n;
      if (n == 1) {
        // the live consensus call: entry 0's fields are words 1..19, in the
        // lanes that polled them; lane 0 reads them across lanes (no LDS)
        if (__ballot(lane < words && (w0 >> 16) != stamp)) continue;  // still being written
        if (!apply && !fide && DC_LIVE_GATHER) {
          // REF validate: the board's facts gathered across the lanes that
          // polled its half-words (lane 1 + 4q + h: bits 16h.. of bb[q]), one
          // ballot per fact, instead of assembling the board in one lane
          // (3.16-3.19 -> 3.06-3.12 us median per call, same box, round 4)
          const u32 mv = lane_bcast(w0, 19) & 0xFFFFu, stm = lane_bcast(w0, 17) & 1u;
          const int f = (int)(mv & 63), t = (int)((mv >> 6) & 63), mid = (f + t) >> 1;
          const u32 k = lane - 1u, c = w0 & 0xFFFFu, h = k & 3u;
          const bool chunk = k < 16u;
          const u64 bf = ballot(chunk && (u32)(f >> 4) == h && ((c >> (f & 15)) & 1u));
          const u64 bt = ballot(chunk && (u32)(t >> 4) == h && ((c >> (t & 15)) & 1u));
          const u64 bm = ballot(chunk && (u32)(mid >> 4) == h && ((c >> (mid & 15)) & 1u));
          const u64 bb = ballot(chunk && k >= 4u && (c & ((u32)(between(f, t) >> (16 * h)) & 0xFFFFu)) != 0u);
          auto nib_at = [](u64 B, int s) -> u32 {  // bit q of the nibble: lane 1 + 4q + (s >> 4)
            const u64 x = B >> (1 + (s >> 4));
            return (u32)(x & 1) | ((u32)(x >> 3) & 2u) | ((u32)(x >> 6) & 4u) | ((u32)(x >> 9) & 8u);
          };
          const u32 nib = nib_at(bf, f), nt = nib_at(bt, t), nm = nib_at(bm, mid);
          const u32 t_occ = (nt >> 1) != 0u, mid_occ = (nm >> 1) != 0u;
          const u32 v = ref_verdict_core(stm, mv, nib, t_occ, t_occ & (u32)((nt & 1u) == stm), mid_occ, (u32)(bb == 0));
          if (lane == 0) sys_store(&box->resp[0], (stamp << 16) | v);
        } else {
          live_serve(box, stamp, 1, apply, fide, lane, [&](u32 k) { return lane_bcast(w0, 1 + k) & 0xFFFFu; });
        }
      } else {
        bool torn = false;
        for (u32 base = 0; base < words; base += 64) {
          const u32 j = base + lane;
          const u32 w = (base == 0 && lane < kPoll) ? w0 : (j < words ? sys_load(&box->req[j]) : 0u);
          if (j < words) {
            torn |= (w >> 16) != stamp;
            if (j >= 1) fld[j - 1] = (uint16_t)w;
          }
        }
        if (__ballot(torn)) continue;  // a request still being written: poll again
        __syncthreads();
        live_serve(box, stamp, n, apply, fide, lane, [&](u32 k) -> u32 { return fld[k * n + lane]; });
        __syncthreads();  // fld is rewritten by the next request
      }
      ++seq;
      t_last = wall_clock64();
      continue;
    }
    // the stop word, and the lease on the clock every 16th empty poll
    if (lane_bcast(w0, kPoll) == 1) break;
    if ((spin & 15) == 0 && wall_clock64() - t_last > lease_ticks) break;
  }
  if (lane == 0) __hip_atomic_store(&box->state, 2u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_live(hipStream_t st, LiveBox* box, u32 seq, u64 lease_ticks) {
  hipLaunchKernelGGL(k_live, dim3(1), dim3(64), 0, st, box, seq, lease_ticks);
  return hipGetLastError();
}

hipError_t launch_validate_ref(hipStream_t st, const DevPos* pos, const uint16_t* moves, u32 n, uint8_t* out, u32* done,
                               u32 seq) {
  if (n == 0) return hipSuccess;
  if (done && n > 256) return hipErrorInvalidValue;  // the flag is published by a single block
  hipLaunchKernelGGL(k_validate_ref, dim3(blocks_for(n, 256)), dim3(256), 0, st, pos, moves, n, out, done, seq);
  return hipGetLastError();
}

hipError_t launch_apply_ref(hipStream_t st, DevPos* pos, const uint16_t* moves, u32 n, uint8_t* verdicts,
                            uint8_t* info, u32* done, u32 seq) {
  if (n == 0) return hipSuccess;
  if (done && n > 256) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_apply_ref, dim3(blocks_for(n, 256)), dim3(256), 0, st, pos, moves, n, verdicts, info, done, seq);
  return hipGetLastError();
}

// Partials of either replay kernel: one record per block (k_replay_ref3's
// persistent grid is far smaller than k_replay_ref's).
u32 replay_partials(u32 n_games) { return blocks_for(n_games, 256); }

// DC_REPLAY=1 selects the arithmetic k_replay_ref (ref_verdict per ply, as the
// validate kernels) instead of the LDS-table k_replay_ref3, for A/B and parity.
static bool replay_arith() {
  static const bool v = [] {
    const char* e = ab_env("DC_REPLAY");
    return e && e[0] == '1';
  }();
  return v;
}

static u32 replay3_grid(u32 n_games) {
  static const u32 resident = [] {
    int per_cu = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_replay_ref3, (int)kR3Threads, 0) != hipSuccess ||
        per_cu < 1)
      per_cu = 1;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 1;
    return (u32)(per_cu * cus);
  }();
  const u32 chunks = blocks_for(n_games, 64);
  return std::max<u32>(1, std::min<u32>(resident, blocks_for(chunks, kR3Threads / 64)));
}

static Mailbox host_mailbox(const Board& b) {
  Mailbox r{};
  for (int s = 0; s < 64; ++s) {
    const u32 n = (u32)(((b.b0 >> s) & 1) | (((b.b1 >> s) & 1) << 1) | (((b.b2 >> s) & 1) << 2) |
                        (((b.b3 >> s) & 1) << 3));
    r.d[s >> 3] |= n << (4 * (s & 7));
  }
  return r;
}

hipError_t launch_replay_ref(hipStream_t st, const Board& start, u32 stm0, const uint16_t* moves, u32 n_games,
                             u32 n_plies, u64* bitmap, u64* digests, u64* stats, u64* partial, u64* stats_host,
                             bool* host_written, uint8_t* info, Board* boards) {
  *host_written = false;
  if (n_games == 0) return hipSuccess;
  if (info && n_plies > 0) {  // the resync path: k_replay_ref4<.., INFO> (one buffer descriptor: < 4 GiB of moves)
    if ((u64)n_games * n_plies * 2 > 0xFFFFFFFFull) return hipErrorInvalidValue;
    const u32 nb = replay3_grid(n_games);
    const bool dw = (n_games & 1) == 0;
    auto ki = dw ? k_replay_ref4<0, 4, true, true> : k_replay_ref4<0, 4, false, true>;
    hipLaunchKernelGGL(ki, dim3(nb), dim3(kR3Threads), 0, st, host_mailbox(start), start.b1 | start.b2 | start.b3,
                       stm0, moves, n_games, n_plies, bitmap, digests, partial, info, boards);
    hipLaunchKernelGGL(k_reduce_stats, dim3(1), dim3(256), 0, st, partial, nb, stats, stats_host);
    *host_written = stats_host != nullptr;
    return hipGetLastError();
  }
  // n_plies == 0 (no moves buffer to clamp loads into) takes k_replay_ref
  if (n_plies > 0 && !replay_arith()) {
    const u32 nb = replay3_grid(n_games);
    // k_replay_ref4 addresses the whole move array through one buffer
    // descriptor (32-bit offsets); larger batches, and DC_REPLAY=3 in the A/B
    // build, take k_replay_ref3's per-row descriptors
    static const bool force3 = [] {
      const char* e = ab_env("DC_REPLAY");
      return e && e[0] == '3';
    }();
    // A/B: DC_REPLAY=41 -> with the table lookahead, =42 -> u16 move loads,
    // =48 -> 8-ply move prefetch (round 2: 0.98 vs 0.88 ms for 4 plies)
    static const int v4 = [] {
      const char* e = ab_env("DC_REPLAY");
      return (e && e[0] == '4') ? atoi(e) : 0;
    }();
    const bool dw = (n_games & 1) == 0 && v4 != 42;
    auto k4 = dw ? k_replay_ref4<0, 4, true> : k_replay_ref4<0, 4, false>;
    if (v4 == 41) k4 = dw ? k_replay_ref4<1, 4, true> : k_replay_ref4<1, 4, false>;
    if (v4 == 48) k4 = dw ? k_replay_ref4<0, 8, true> : k_replay_ref4<0, 8, false>;
    const bool fits = (u64)n_games * n_plies * 2 <= 0xFFFFFFFFull;
    if (fits && !force3)
      hipLaunchKernelGGL(k4, dim3(nb), dim3(kR3Threads), 0, st, host_mailbox(start), start.b1 | start.b2 | start.b3,
                         stm0, moves, n_games, n_plies, bitmap, digests, partial, nullptr, nullptr);
    else
      hipLaunchKernelGGL(k_replay_ref3, dim3(nb), dim3(kR3Threads), 0, st, host_mailbox(start),
                         start.b1 | start.b2 | start.b3, stm0, moves, n_games, n_plies, bitmap, digests, partial);
    hipLaunchKernelGGL(k_reduce_stats, dim3(1), dim3(256), 0, st, partial, nb, stats, stats_host);
    *host_written = stats_host != nullptr;
    return hipGetLastError();
  }
  const u32 nb = blocks_for(n_games, 256);
  hipLaunchKernelGGL(k_replay_ref, dim3(nb), dim3(256), 0, st, start, stm0, moves, n_games, n_plies, bitmap, digests,
                     partial);
  hipLaunchKernelGGL(k_reduce_stats, dim3(1), dim3(256), 0, st, partial, nb, stats, stats_host);
  *host_written = stats_host != nullptr;
  return hipGetLastError();
}

hipError_t launch_gen_games_ref(hipStream_t st, u64 seed, u64 first_game, u32 n_games, u32 n_plies, u32 noise,
                                uint16_t* out) {
  if (n_games == 0) return hipSuccess;
#ifdef DC_AB_KNOBS
  // DC_GEN=1 / 2 (A/B build only): the round-1 / round-2 generators
  static const bool v1 = [] {
    const char* e = ab_env("DC_GEN");
    return e && e[0] == '1';
  }();
  static const bool v2 = [] {
    const char* e = ab_env("DC_GEN");
    return e && e[0] == '2';
  }();
  auto kg = v1 ? k_gen_games_ref_v1 : v2 ? k_gen_games_ref_v2 : k_gen_games_ref;
#else
  auto kg = k_gen_games_ref;
#endif
  hipLaunchKernelGGL(kg, dim3(blocks_for(n_games, 256)), dim3(256), 0, st, seed, first_game, n_games, n_plies, noise,
                     out);
  return hipGetLastError();
}

hipError_t launch_validate_fide(hipStream_t st, const DevPos* pos, const uint16_t* moves, u32 n, uint8_t* out, u32* done,
                                u32 seq) {
  if (n == 0) return hipSuccess;
  if (done && n > 256) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_validate_fide, dim3(blocks_for(n, 256)), dim3(256), 0, st, pos, moves, n, out, done, seq);
  return hipGetLastError();
}
hipError_t launch_apply_fide(hipStream_t st, DevPos* pos, const uint16_t* moves, u32 n, uint8_t* verdicts,
                             uint8_t* info, u32* done, u32 seq) {
  if (n == 0) return hipSuccess;
  if (done && n > 256) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_apply_fide, dim3(blocks_for(n, 256)), dim3(256), 0, st, pos, moves, n, verdicts, info, done, seq);
  return hipGetLastError();
}
hipError_t launch_replay_fide(hipStream_t st, const DevPos& start, const uint16_t* moves, u32 n_games, u32 n_plies,
                              u64* bitmap, u64* digests, u64* stats, u64* partial) {
  if (n_games == 0) return hipSuccess;
  const Board b{start.bb[0], start.bb[1], start.bb[2], start.bb[3]};
  const u32 nb = blocks_for(n_games, 256);
  hipLaunchKernelGGL(k_replay_fide, dim3(nb), dim3(256), 0, st, b, (u32)(start.stm & 1),
                     (u32)pack_meta(start.castle, start.ep), moves, n_games, n_plies, bitmap, digests, partial);
  hipLaunchKernelGGL(k_reduce_stats, dim3(1), dim3(256), 0, st, partial, nb, stats);
  return hipGetLastError();
}
hipError_t launch_gen_games_fide(hipStream_t st, u64 seed, u64 first_game, u32 n_games, u32 n_plies, u32 noise,
                                 uint16_t* out) {
  if (n_games == 0) return hipSuccess;
  hipLaunchKernelGGL(k_gen_games_fide, dim3(blocks_for(n_games, 256)), dim3(256), 0, st, seed, first_game, n_games,
                     n_plies, noise, out);
  return hipGetLastError();
}
}  // namespace dc
