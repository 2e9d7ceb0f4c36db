// dc_kernels.hip -- HIP kernels for gfx950 (RULES_REF), one lane per position/game.
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

// -------------------------------------------------------------------- perft
template <int STM>
__global__ __launch_bounds__(256) void k_count_children(const Board* __restrict__ nodes, u32 n, u32* __restrict__ counts) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  counts[i] = ref_count<STM>(load_board(nodes, i));
}

template <int STM>
__global__ __launch_bounds__(256) void k_expand_write(const Board* __restrict__ nodes, const uint16_t* __restrict__ tags,
                                                      u32 n, const u64* __restrict__ offsets, Board* __restrict__ out,
                                                      uint16_t* __restrict__ out_tags, uint16_t* __restrict__ out_moves,
                                                      int root_level) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Board p = load_board(nodes, i);
  const uint16_t tag = tags[i];
  u64 o = offsets[i];
  u32 j = 0;
  ref_for_each_move<STM>(p, [&](int f, int t) {
    Board c = p;
    ref_make(c, f, t);
    store_board(out, o, c);
    out_tags[o] = root_level ? (uint16_t)j : tag;
    if (out_moves) out_moves[o] = (uint16_t)(f | (t << 6));
    ++o;
    ++j;
  });
}

template <int STM>
__global__ __launch_bounds__(256) void k_count1(const Board* __restrict__ nodes, const uint16_t* __restrict__ tags, u32 n,
                                                u64* __restrict__ divide) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = i < n;
  u32 c = 0, tag = 0;
  if (valid) {
    c = ref_count<STM>(load_board(nodes, i));
    tag = tags[i];
  }
  accumulate_by_tag(divide, tag, c, valid);
}

// Fused last two plies.  Per wave: 64 parents -> their children's (from,to,
// parent lane) are compacted into LDS at wave-prefix-sum offsets, then each
// round every lane takes one child, makes it and bulk-counts the grandchildren.
constexpr int kC2Waves = 4;
constexpr int kC2Cap = 64 * 40;  // child slots per wave and window

struct C2Shared {
  Board parent[kC2Waves][64];
  u32 slot[kC2Waves][kC2Cap];
};

template <int STM>
__global__ __launch_bounds__(256) void k_count2(const Board* __restrict__ nodes, const uint16_t* __restrict__ tags, u32 n,
                                                u64* __restrict__ divide) {
  __shared__ C2Shared sh;
  const u32 w = threadIdx.x >> 6;
  const u32 lane = lane_id();
  Board* par = sh.parent[w];
  u32* slot = sh.slot[w];
  const u32 groups = (n + 63) >> 6;
  for (u32 g = blockIdx.x * kC2Waves + w; g < groups; g += gridDim.x * kC2Waves) {
    const u32 i = (g << 6) + lane;
    const bool valid = i < n;
    Board p{0, 0, 0, 0};
    u32 tag = 0;
    if (valid) {
      p = load_board(nodes, i);
      tag = tags[i];
    }
    const u32 cnt = valid ? ref_count<STM>(p) : 0;
    const u32 incl = wave_incl_scan(cnt);
    const u32 excl = incl - cnt;
    const u32 total = __shfl(incl, 63, 64);
    const u64 vmask = ballot(valid);
    const u32 tag0 = __shfl(tag, lsb(vmask), 64);
    par[lane] = p;
    u64 acc = 0;  // grandchildren under parents whose tag == tag0
    for (u32 base = 0; base < total; base += kC2Cap) {
      wave_lds_sync();
      u32 j = excl;
      if (valid) {
        ref_for_each_move<STM>(p, [&](int f, int t) {
          if (j >= base && j - base < (u32)kC2Cap) slot[j - base] = (u32)f | ((u32)t << 6) | (lane << 12);
          ++j;
        });
      }
      wave_lds_sync();
      const u32 nslots = min((u32)kC2Cap, total - base);
      for (u32 r = lane; r < ((nslots + 63) & ~63u); r += 64) {
        u32 k = 0, pl = 0;
        if (r < nslots) {
          const u32 e = slot[r];
          pl = e >> 12;
          Board c = par[pl];
          ref_make(c, (int)(e & 63), (int)((e >> 6) & 63));
          k = ref_count<1 - STM>(c);
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

hipError_t launch_count_children(hipStream_t st, int stm, const Board* nodes, u32 n, u32* counts) {
  if (n == 0) return hipSuccess;
  if (stm) hipLaunchKernelGGL(k_count_children<1>, dim3(blocks_for(n, 256)), dim3(256), 0, st, nodes, n, counts);
  else hipLaunchKernelGGL(k_count_children<0>, dim3(blocks_for(n, 256)), dim3(256), 0, st, nodes, n, counts);
  return hipGetLastError();
}

hipError_t launch_expand_write(hipStream_t st, int stm, const Board* nodes, const uint16_t* tags, u32 n,
                               const u64* offsets, Board* out, uint16_t* out_tags, uint16_t* out_moves,
                               int root_level) {
  if (n == 0) return hipSuccess;
  if (stm)
    hipLaunchKernelGGL(k_expand_write<1>, dim3(blocks_for(n, 256)), dim3(256), 0, st, nodes, tags, n, offsets, out,
                       out_tags, out_moves, root_level);
  else
    hipLaunchKernelGGL(k_expand_write<0>, dim3(blocks_for(n, 256)), dim3(256), 0, st, nodes, tags, n, offsets, out,
                       out_tags, out_moves, root_level);
  return hipGetLastError();
}

hipError_t launch_count1(hipStream_t st, int stm, const Board* nodes, const uint16_t* tags, u32 n, u64* divide) {
  if (n == 0) return hipSuccess;
  if (stm) hipLaunchKernelGGL(k_count1<1>, dim3(blocks_for(n, 256)), dim3(256), 0, st, nodes, tags, n, divide);
  else hipLaunchKernelGGL(k_count1<0>, dim3(blocks_for(n, 256)), dim3(256), 0, st, nodes, tags, n, divide);
  return hipGetLastError();
}

hipError_t launch_count2(hipStream_t st, int stm, const Board* nodes, const uint16_t* tags, u32 n, u64* divide,
                         u32 max_blocks) {
  if (n == 0) return hipSuccess;
  const u32 groups = (n + 63) / 64;
  u32 blocks = (groups + kC2Waves - 1) / kC2Waves;
  if (max_blocks && blocks > max_blocks) blocks = max_blocks;
  if (stm) hipLaunchKernelGGL(k_count2<1>, dim3(blocks), dim3(256), 0, st, nodes, tags, n, divide);
  else hipLaunchKernelGGL(k_count2<0>, dim3(blocks), dim3(256), 0, st, nodes, tags, n, divide);
  return hipGetLastError();
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
