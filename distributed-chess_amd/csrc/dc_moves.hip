// dc_moves.hip -- single-move kernels for gfx950, one lane per position or game.
//
//   k_validate_{ref,fide}   K2: one lane per (position, move)      -> verdict byte
//   k_apply_{ref,fide}      K2': validate + make in place           -> verdict, info
//   k_replay_{ref,fide}     K1: one lane per game, loop over plies  -> ply-major accept bitmap
//   k_gen_games_{ref,fide}  K5: one lane per game, seeded games     -> ply-major moves
#include <hip/hip_runtime.h>

#include "dc_common.h"

namespace dc {

// ------------------------------------------------------------- validation
__global__ __launch_bounds__(256) void k_validate_ref(const DevPos* __restrict__ pos, const uint16_t* __restrict__ moves,
                                                      u32 n, uint8_t* __restrict__ out) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const DevPos p = pos[i];
  const Board b{p.bb[0], p.bb[1], p.bb[2], p.bb[3]};
  out[i] = (uint8_t)ref_verdict(b, p.stm & 1, moves[i]);
}

__global__ __launch_bounds__(256) void k_apply_ref(DevPos* __restrict__ pos, const uint16_t* __restrict__ moves, u32 n,
                                                   uint8_t* __restrict__ verdicts, uint8_t* __restrict__ info) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
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

__global__ __launch_bounds__(256) void k_reduce_stats(const u64* __restrict__ partial, u32 n_blocks, u64* __restrict__ stats) {
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

__global__ __launch_bounds__(256) void k_gen_games_ref(u64 seed, u64 first_game, u32 n_games, u32 n_plies,
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

// ------------------------------------------------------------- FIDE (K1/K2/K5)
__global__ __launch_bounds__(256) void k_validate_fide(const DevPos* __restrict__ pos, const uint16_t* __restrict__ moves,
                                                       u32 n, uint8_t* __restrict__ out) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const DevPos p = pos[i];
  const Board b{p.bb[0], p.bb[1], p.bb[2], p.bb[3]};
  out[i] = (uint8_t)fide_verdict(b, p.stm & 1, pack_meta(p.castle, p.ep), moves[i]);
}

__global__ __launch_bounds__(256) void k_apply_fide(DevPos* __restrict__ pos, const uint16_t* __restrict__ moves, u32 n,
                                                    uint8_t* __restrict__ verdicts, uint8_t* __restrict__ info) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
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

hipError_t launch_validate_ref(hipStream_t st, const DevPos* pos, const uint16_t* moves, u32 n, uint8_t* out) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_validate_ref, dim3(blocks_for(n, 256)), dim3(256), 0, st, pos, moves, n, out);
  return hipGetLastError();
}

hipError_t launch_apply_ref(hipStream_t st, DevPos* pos, const uint16_t* moves, u32 n, uint8_t* verdicts,
                            uint8_t* info) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_apply_ref, dim3(blocks_for(n, 256)), dim3(256), 0, st, pos, moves, n, verdicts, info);
  return hipGetLastError();
}

u32 replay_partials(u32 n_games) { return blocks_for(n_games, 256); }

hipError_t launch_replay_ref(hipStream_t st, const Board& start, u32 stm0, const uint16_t* moves, u32 n_games,
                             u32 n_plies, u64* bitmap, u64* digests, u64* stats, u64* partial) {
  if (n_games == 0) return hipSuccess;
  const u32 nb = blocks_for(n_games, 256);
  hipLaunchKernelGGL(k_replay_ref, dim3(nb), dim3(256), 0, st, start, stm0, moves, n_games, n_plies, bitmap, digests,
                     partial);
  hipLaunchKernelGGL(k_reduce_stats, dim3(1), dim3(256), 0, st, partial, nb, stats);
  return hipGetLastError();
}

hipError_t launch_gen_games_ref(hipStream_t st, u64 seed, u64 first_game, u32 n_games, u32 n_plies, u32 noise,
                                uint16_t* out) {
  if (n_games == 0) return hipSuccess;
  hipLaunchKernelGGL(k_gen_games_ref, dim3(blocks_for(n_games, 256)), dim3(256), 0, st, seed, first_game, n_games,
                     n_plies, noise, out);
  return hipGetLastError();
}

hipError_t launch_validate_fide(hipStream_t st, const DevPos* pos, const uint16_t* moves, u32 n, uint8_t* out) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_validate_fide, dim3(blocks_for(n, 256)), dim3(256), 0, st, pos, moves, n, out);
  return hipGetLastError();
}
hipError_t launch_apply_fide(hipStream_t st, DevPos* pos, const uint16_t* moves, u32 n, uint8_t* verdicts,
                             uint8_t* info) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_apply_fide, dim3(blocks_for(n, 256)), dim3(256), 0, st, pos, moves, n, verdicts, info);
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
