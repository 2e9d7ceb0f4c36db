// dc_kernels.hip -- HIP kernels for gfx950 (RULES_REF and RULES_FIDE), one lane per position/game.
//
//   k_validate_ref   K2: one lane per (position, move)          -> verdict byte
//   k_apply_ref      K2': validate + make in place               -> verdict, info
//   k_replay_ref     K1: one lane per game, loop over plies      -> ply-major accept bitmap
//   k_gen_games_ref  K5: one lane per game, seeded legal games   -> ply-major moves
//   k_count_children K3a: children per frontier node (bulk count)
//   k_expand_write   K3b: deterministic frontier expansion at scanned offsets
//   k_count1         final level: bulk count per node, per-root accumulation
//   k_count2         final two levels fused: the wave's children are flattened
//                    into LDS (ballot/prefix-sum compaction) and every lane
//                    bulk-counts one child per round -> no trip-count divergence
//   k_scan_*         exclusive scan of child counts (u64 offsets)
#include <hip/hip_runtime.h>

#include "dc_fide.h"
#include "dc_fide_rules.h"
#include "dc_kernels.h"
#include "dc_ref.h"

namespace dc {

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ Board load_board(const Board* p, size_t i) {
  const ulonglong2* q = reinterpret_cast<const ulonglong2*>(p + i);
  const ulonglong2 a = q[0], c = q[1];
  return Board{a.x, a.y, c.x, c.y};
}
__device__ __forceinline__ void store_board(Board* p, size_t i, const Board& b) {
  ulonglong2* q = reinterpret_cast<ulonglong2*>(p + i);
  q[0] = ulonglong2{b.b0, b.b1};
  q[1] = ulonglong2{b.b2, b.b3};
}

// Wave-scope ordering of LDS traffic between lanes of one wave.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Adds `v` to divide[tag].  Nodes are ordered by root move, so a wave almost
// always holds one tag: reduce across the wave and issue one atomic.
__device__ __forceinline__ void accumulate_by_tag(u64* divide, u32 tag, u64 v, bool valid) {
  const u32 lane = lane_id();
  const u64 vmask = ballot(valid);
  if (vmask == 0) return;
  const int leader = lsb(vmask);
  const u32 tag0 = __shfl(tag, leader, 64);
  const bool same = !valid || tag == tag0;
  if (ballot(same) == ~0ull) {
    const u64 s = wave_sum64(valid ? v : 0);
    if ((int)lane == leader && s) atomicAdd(divide + tag0, s);
  } else if (valid && v) {
    atomicAdd(divide + tag, v);
  }
}

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

// ------------------------------------------------------------------ replay
// One lane per game; the wave's 64 verdicts of a ply are one ballot word, so
// bitmap stores are one u64 per wave per ply (ply-major, no transpose).
constexpr int kReplayPrefetch = 4;

__global__ __launch_bounds__(256) void k_replay_ref(Board start, u32 stm0, const uint16_t* __restrict__ moves,
                                                    u32 n_games, u32 n_plies, u64* __restrict__ bitmap,
                                                    u64* __restrict__ digests, u64* __restrict__ stats) {
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
  const u64 sv = wave_sum64(validated), sa = wave_sum64(accepted), sd = wave_sum64(d);
  u64 x = d;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x ^= __shfl_xor(x, o, 64);
  if (lane_id() == 0 && stats) {
    atomicAdd(stats + 0, sv);
    atomicAdd(stats + 1, sa);
    atomicAdd(stats + 2, sv - sa);
    atomicAdd(stats + 3, sd);
    atomicXor(stats + 4, x);
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
                                                     u64* __restrict__ digests, u64* __restrict__ stats) {
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
  const u64 sv = wave_sum64(validated), sa = wave_sum64(accepted), sd = wave_sum64(d);
  u64 x = d;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x ^= __shfl_xor(x, o, 64);
  if (lane_id() == 0 && stats) {
    atomicAdd(stats + 0, sv);
    atomicAdd(stats + 1, sa);
    atomicAdd(stats + 2, sv - sa);
    atomicAdd(stats + 3, sd);
    atomicXor(stats + 4, x);
  }
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

// -------------------------------------------------------------------- perft
// Rules policies: the perft kernels are shared by RULES_REF and RULES_FIDE.
struct RefRules {
  static constexpr bool kMeta = false;
  template <int STM>
  __device__ static __forceinline__ u32 count(const Board& b, u32) { return ref_count<STM>(b); }
  template <int STM, class V>
  __device__ static __forceinline__ void for_each(const Board& b, u32, V&& v) {
    ref_for_each_move<STM>(b, [&](int f, int t) { v(f, t, 0); });
  }
  template <int STM>
  __device__ static __forceinline__ u32 make(Board& b, u32, int f, int t, int) {
    ref_make(b, f, t);
    return 0;
  }
};

struct FideRules {
  static constexpr bool kMeta = true;
  template <int STM>
  __device__ static __forceinline__ u32 count(const Board& b, u32 meta) { return fide_count<STM>(b, meta); }
  template <int STM, class V>
  __device__ static __forceinline__ void for_each(const Board& b, u32 meta, V&& v) {
    fide_for_each_move<STM>(b, meta, v);
  }
  template <int STM>
  __device__ static __forceinline__ u32 make(Board& b, u32 meta, int f, int t, int promo) {
    return fide_make<STM>(b, meta, f, t, promo);
  }
};

template <class R>
__device__ __forceinline__ u32 load_meta(const uint16_t* meta, size_t i) {
  if constexpr (R::kMeta) return meta[i];
  else return 0;
}

template <class R, int STM>
__global__ __launch_bounds__(256) void k_count_children(const Board* __restrict__ nodes, const uint16_t* __restrict__ meta,
                                                        u32 n, u32* __restrict__ counts) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  counts[i] = R::template count<STM>(load_board(nodes, i), load_meta<R>(meta, i));
}

template <class R, int STM>
__global__ __launch_bounds__(256) void k_expand_write(const Board* __restrict__ nodes, const uint16_t* __restrict__ meta,
                                                      const uint16_t* __restrict__ tags, u32 n,
                                                      const u64* __restrict__ offsets, Board* __restrict__ out,
                                                      uint16_t* __restrict__ out_meta, uint16_t* __restrict__ out_tags,
                                                      uint16_t* __restrict__ out_moves, int root_level) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Board p = load_board(nodes, i);
  const u32 pm = load_meta<R>(meta, i);
  const uint16_t tag = tags[i];
  u64 o = offsets[i];
  u32 j = 0;
  R::template for_each<STM>(p, pm, [&](int f, int t, int promo) {
    Board c = p;
    const u32 cm = R::template make<STM>(c, pm, f, t, promo);
    store_board(out, o, c);
    if constexpr (R::kMeta) out_meta[o] = (uint16_t)cm;
    out_tags[o] = root_level ? (uint16_t)j : tag;
    if (out_moves) out_moves[o] = (uint16_t)(f | (t << 6) | (promo << 12));
    ++o;
    ++j;
  });
}

template <class R, int STM>
__global__ __launch_bounds__(256) void k_count1(const Board* __restrict__ nodes, const uint16_t* __restrict__ meta,
                                                const uint16_t* __restrict__ tags, u32 n, u64* __restrict__ divide) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = i < n;
  u32 c = 0, tag = 0;
  if (valid) {
    c = R::template count<STM>(load_board(nodes, i), load_meta<R>(meta, i));
    tag = tags[i];
  }
  accumulate_by_tag(divide, tag, c, valid);
}

// Fused last two plies.  Per wave: 64 parents -> their children's (from, to,
// promo, parent lane) are compacted into LDS at wave-prefix-sum offsets
// (ballot/scan compaction), then each round every lane takes one child, makes
// it and bulk-counts the grandchildren: no per-lane trip-count divergence.
constexpr int kC2Waves = 4;
constexpr int kC2Cap = 64 * 40;  // child slots per wave and window

struct C2Shared {
  Board parent[kC2Waves][64];
  u32 pmeta[kC2Waves][64];
  u32 slot[kC2Waves][kC2Cap];
};

template <class R, int STM>
__global__ __launch_bounds__(256) void k_count2(const Board* __restrict__ nodes, const uint16_t* __restrict__ meta,
                                                const uint16_t* __restrict__ tags, u32 n, u64* __restrict__ divide) {
  __shared__ C2Shared sh;
  const u32 w = threadIdx.x >> 6;
  const u32 lane = lane_id();
  Board* par = sh.parent[w];
  u32* pmeta = sh.pmeta[w];
  u32* slot = sh.slot[w];
  const u32 groups = (n + 63) >> 6;
  for (u32 g = blockIdx.x * kC2Waves + w; g < groups; g += gridDim.x * kC2Waves) {
    const u32 i = (g << 6) + lane;
    const bool valid = i < n;
    Board p{0, 0, 0, 0};
    u32 tag = 0, pm = 0;
    if (valid) {
      p = load_board(nodes, i);
      pm = load_meta<R>(meta, i);
      tag = tags[i];
    }
    const u32 cnt = valid ? R::template count<STM>(p, pm) : 0;
    const u32 incl = wave_incl_scan(cnt);
    const u32 excl = incl - cnt;
    const u32 total = __shfl(incl, 63, 64);
    const u64 vmask = ballot(valid);
    const u32 tag0 = __shfl(tag, lsb(vmask), 64);
    par[lane] = p;
    if constexpr (R::kMeta) pmeta[lane] = pm;
    u64 acc = 0;  // grandchildren under parents whose tag == tag0
    for (u32 base = 0; base < total; base += kC2Cap) {
      wave_lds_sync();
      u32 j = excl;
      if (valid) {
        R::template for_each<STM>(p, pm, [&](int f, int t, int promo) {
          if (j >= base && j - base < (u32)kC2Cap && j < excl + cnt)
            slot[j - base] = (u32)f | ((u32)t << 6) | ((u32)promo << 12) | (lane << 15);
          ++j;
        });
      }
      wave_lds_sync();
      const u32 nslots = min((u32)kC2Cap, total - base);
      for (u32 r = lane; r < ((nslots + 63) & ~63u); r += 64) {
        u32 k = 0, pl = 0;
        if (r < nslots) {
          const u32 e = slot[r];
          pl = e >> 15;
          Board c = par[pl];
          const u32 cm = R::template make<STM>(c, R::kMeta ? pmeta[pl] : 0u, (int)(e & 63), (int)((e >> 6) & 63),
                                               (int)((e >> 12) & 7));
          k = R::template count<1 - STM>(c, cm);
        }
        const u32 ptag = __shfl(tag, (int)pl, 64);
        if (ptag == tag0) acc += k;
        else if (k) atomicAdd(divide + ptag, (u64)k);
      }
    }
    const u64 s = wave_sum64(acc);
    if (lane == (u32)lsb(vmask) && s) atomicAdd(divide + tag0, s);
    wave_lds_sync();
  }
}

// --------------------------------------------------------------------- scan
// Exclusive scan of n counts into u64 offsets; block = 256 threads x 16 items.
constexpr int kScanItems = 16;
constexpr int kScanBlock = 256 * kScanItems;

template <class T>
__device__ __forceinline__ u64 block_excl_scan(u64 v, u64* total) {
  __shared__ u64 wsum[4];
  const u32 lane = lane_id(), w = threadIdx.x >> 6;
  u64 incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const u64 y = __shfl_up(incl, o, 64);
    if ((int)lane >= o) incl += y;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  u64 before = 0, all = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if ((u32)k < w) before += wsum[k];
    all += wsum[k];
  }
  __syncthreads();
  *total = all;
  return before + incl - v;
}

template <class T>
__global__ __launch_bounds__(256) void k_scan_reduce(const T* __restrict__ in, u64 n, u64* __restrict__ bsums) {
  const u64 base = (u64)blockIdx.x * kScanBlock + (u64)threadIdx.x * kScanItems;
  u64 s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k)
    if (base + k < n) s += in[base + k];
  u64 tot;
  block_excl_scan<T>(s, &tot);
  if (threadIdx.x == 0) bsums[blockIdx.x] = tot;
}

template <class T>
__global__ __launch_bounds__(256) void k_scan_apply(const T* __restrict__ in, u64 n, const u64* __restrict__ bexcl,
                                                    u64* __restrict__ out) {
  const u64 base = (u64)blockIdx.x * kScanBlock + (u64)threadIdx.x * kScanItems;
  T vals[kScanItems];
  u64 s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    vals[k] = (base + k < n) ? in[base + k] : (T)0;
    s += vals[k];
  }
  u64 tot;
  u64 run = block_excl_scan<T>(s, &tot) + (bexcl ? bexcl[blockIdx.x] : 0);
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    if (base + k < n) out[base + k] = run;
    run += vals[k];
  }
}

// ------------------------------------------------------------- launchers
static inline u32 blocks_for(u64 n, u32 per) { return (u32)((n + per - 1) / per); }

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

hipError_t launch_replay_ref(hipStream_t st, const Board& start, u32 stm0, const uint16_t* moves, u32 n_games,
                             u32 n_plies, u64* bitmap, u64* digests, u64* stats) {
  if (n_games == 0) return hipSuccess;
  hipLaunchKernelGGL(k_replay_ref, dim3(blocks_for(n_games, 256)), dim3(256), 0, st, start, stm0, moves, n_games,
                     n_plies, bitmap, digests, stats);
  return hipGetLastError();
}

hipError_t launch_gen_games_ref(hipStream_t st, u64 seed, u64 first_game, u32 n_games, u32 n_plies, u32 noise,
                                uint16_t* out) {
  if (n_games == 0) return hipSuccess;
  hipLaunchKernelGGL(k_gen_games_ref, dim3(blocks_for(n_games, 256)), dim3(256), 0, st, seed, first_game, n_games,
                     n_plies, noise, out);
  return hipGetLastError();
}

template <class R>
static hipError_t count_children_impl(hipStream_t st, int stm, const Board* nodes, const uint16_t* meta, u32 n,
                                      u32* counts) {
  if (n == 0) return hipSuccess;
  if (stm) hipLaunchKernelGGL((k_count_children<R, 1>), dim3(blocks_for(n, 256)), dim3(256), 0, st, nodes, meta, n, counts);
  else hipLaunchKernelGGL((k_count_children<R, 0>), dim3(blocks_for(n, 256)), dim3(256), 0, st, nodes, meta, n, counts);
  return hipGetLastError();
}

template <class R>
static hipError_t expand_write_impl(hipStream_t st, int stm, const Board* nodes, const uint16_t* meta,
                                    const uint16_t* tags, u32 n, const u64* offsets, Board* out, uint16_t* out_meta,
                                    uint16_t* out_tags, uint16_t* out_moves, int root_level) {
  if (n == 0) return hipSuccess;
  if (stm)
    hipLaunchKernelGGL((k_expand_write<R, 1>), dim3(blocks_for(n, 256)), dim3(256), 0, st, nodes, meta, tags, n, offsets,
                       out, out_meta, out_tags, out_moves, root_level);
  else
    hipLaunchKernelGGL((k_expand_write<R, 0>), dim3(blocks_for(n, 256)), dim3(256), 0, st, nodes, meta, tags, n, offsets,
                       out, out_meta, out_tags, out_moves, root_level);
  return hipGetLastError();
}

template <class R>
static hipError_t count1_impl(hipStream_t st, int stm, const Board* nodes, const uint16_t* meta, const uint16_t* tags,
                              u32 n, u64* divide) {
  if (n == 0) return hipSuccess;
  if (stm) hipLaunchKernelGGL((k_count1<R, 1>), dim3(blocks_for(n, 256)), dim3(256), 0, st, nodes, meta, tags, n, divide);
  else hipLaunchKernelGGL((k_count1<R, 0>), dim3(blocks_for(n, 256)), dim3(256), 0, st, nodes, meta, tags, n, divide);
  return hipGetLastError();
}

template <class R>
static hipError_t count2_impl(hipStream_t st, int stm, const Board* nodes, const uint16_t* meta, const uint16_t* tags,
                              u32 n, u64* divide, u32 max_blocks) {
  if (n == 0) return hipSuccess;
  const u32 groups = (n + 63) / 64;
  u32 blocks = (groups + kC2Waves - 1) / kC2Waves;
  if (max_blocks && blocks > max_blocks) blocks = max_blocks;
  if (stm) hipLaunchKernelGGL((k_count2<R, 1>), dim3(blocks), dim3(256), 0, st, nodes, meta, tags, n, divide);
  else hipLaunchKernelGGL((k_count2<R, 0>), dim3(blocks), dim3(256), 0, st, nodes, meta, tags, n, divide);
  return hipGetLastError();
}

hipError_t launch_count_children(hipStream_t st, int stm, const Board* nodes, u32 n, u32* counts) {
  return count_children_impl<RefRules>(st, stm, nodes, nullptr, n, counts);
}
hipError_t launch_expand_write(hipStream_t st, int stm, const Board* nodes, const uint16_t* tags, u32 n,
                               const u64* offsets, Board* out, uint16_t* out_tags, uint16_t* out_moves,
                               int root_level) {
  return expand_write_impl<RefRules>(st, stm, nodes, nullptr, tags, n, offsets, out, nullptr, out_tags, out_moves,
                                     root_level);
}
hipError_t launch_count1(hipStream_t st, int stm, const Board* nodes, const uint16_t* tags, u32 n, u64* divide) {
  return count1_impl<RefRules>(st, stm, nodes, nullptr, tags, n, divide);
}
hipError_t launch_count2(hipStream_t st, int stm, const Board* nodes, const uint16_t* tags, u32 n, u64* divide,
                         u32 max_blocks) {
  return count2_impl<RefRules>(st, stm, nodes, nullptr, tags, n, divide, max_blocks);
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
                              u64* bitmap, u64* digests, u64* stats) {
  if (n_games == 0) return hipSuccess;
  const Board b{start.bb[0], start.bb[1], start.bb[2], start.bb[3]};
  hipLaunchKernelGGL(k_replay_fide, dim3(blocks_for(n_games, 256)), dim3(256), 0, st, b, (u32)(start.stm & 1),
                     (u32)pack_meta(start.castle, start.ep), moves, n_games, n_plies, bitmap, digests, stats);
  return hipGetLastError();
}
hipError_t launch_gen_games_fide(hipStream_t st, u64 seed, u64 first_game, u32 n_games, u32 n_plies, u32 noise,
                                 uint16_t* out) {
  if (n_games == 0) return hipSuccess;
  hipLaunchKernelGGL(k_gen_games_fide, dim3(blocks_for(n_games, 256)), dim3(256), 0, st, seed, first_game, n_games,
                     n_plies, noise, out);
  return hipGetLastError();
}
hipError_t launch_count_children_fide(hipStream_t st, int stm, const Board* nodes, const uint16_t* meta, u32 n,
                                      u32* counts) {
  return count_children_impl<FideRules>(st, stm, nodes, meta, n, counts);
}
hipError_t launch_expand_write_fide(hipStream_t st, int stm, const Board* nodes, const uint16_t* meta,
                                    const uint16_t* tags, u32 n, const u64* offsets, Board* out, uint16_t* out_meta,
                                    uint16_t* out_tags, uint16_t* out_moves, int root_level) {
  return expand_write_impl<FideRules>(st, stm, nodes, meta, tags, n, offsets, out, out_meta, out_tags, out_moves,
                                      root_level);
}
hipError_t launch_count1_fide(hipStream_t st, int stm, const Board* nodes, const uint16_t* meta, const uint16_t* tags,
                              u32 n, u64* divide) {
  return count1_impl<FideRules>(st, stm, nodes, meta, tags, n, divide);
}
hipError_t launch_count2_fide(hipStream_t st, int stm, const Board* nodes, const uint16_t* meta, const uint16_t* tags,
                              u32 n, u64* divide, u32 max_blocks) {
  return count2_impl<FideRules>(st, stm, nodes, meta, tags, n, divide, max_blocks);
}

size_t scan_temp_elems(u64 n) {
  size_t tot = 0;
  while (n > 1) {
    n = (n + kScanBlock - 1) / kScanBlock;
    tot += 2 * n;
  }
  return tot + 2;
}

// Recursive exclusive scan: counts (u32) -> offsets (u64); temp sized by scan_temp_elems.
static hipError_t scan_u64(hipStream_t st, const u64* in, u64 n, u64* out, u64* temp);

hipError_t launch_scan_u32(hipStream_t st, const u32* in, u64 n, u64* out, u64* temp) {
  if (n == 0) return hipSuccess;
  const u32 nb = blocks_for(n, kScanBlock);
  if (nb == 1) {
    hipLaunchKernelGGL(k_scan_apply<u32>, dim3(1), dim3(256), 0, st, in, n, (const u64*)nullptr, out);
    return hipGetLastError();
  }
  u64* bsums = temp;
  u64* bexcl = temp + nb;
  hipLaunchKernelGGL(k_scan_reduce<u32>, dim3(nb), dim3(256), 0, st, in, n, bsums);
  hipError_t e = scan_u64(st, bsums, nb, bexcl, temp + 2 * (size_t)nb);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_scan_apply<u32>, dim3(nb), dim3(256), 0, st, in, n, bexcl, out);
  return hipGetLastError();
}

static hipError_t scan_u64(hipStream_t st, const u64* in, u64 n, u64* out, u64* temp) {
  const u32 nb = blocks_for(n, kScanBlock);
  if (nb == 1) {
    hipLaunchKernelGGL(k_scan_apply<u64>, dim3(1), dim3(256), 0, st, in, n, (const u64*)nullptr, out);
    return hipGetLastError();
  }
  u64* bsums = temp;
  u64* bexcl = temp + nb;
  hipLaunchKernelGGL(k_scan_reduce<u64>, dim3(nb), dim3(256), 0, st, in, n, bsums);
  hipError_t e = scan_u64(st, bsums, nb, bexcl, temp + 2 * (size_t)nb);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_scan_apply<u64>, dim3(nb), dim3(256), 0, st, in, n, bexcl, out);
  return hipGetLastError();
}

}  // namespace dc
