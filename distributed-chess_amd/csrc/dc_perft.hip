// dc_perft.hip -- device-driven perft pipeline for gfx950 (RULES_REF and RULES_FIDE).
//
// A perft(d) run is one fixed launch sequence with the level sizes kept on the
// device (Range descriptors), so the host synchronises once per run:
//
//   k_expand_top      one workgroup expands the root to ply T (<= 2) in LDS-
//                     scanned, deterministic (parent, class, target) order and
//                     records the root moves (the divide keys)
//   k_count_children  K3a  children per frontier node (bulk count)         \  per level,
//   k_scan_*          exclusive scan -> u64 offsets + next level's Range   |  grid-stride,
//   k_expand_write    K3b  children written at their offsets (<= cap)      /  n read on device
//   k_slice           contiguous shard of a level for data-parallel runs
//   k_count2          the last two plies fused: per wave, 64 parents' children
//                     are compacted into LDS (wave prefix sum) and each lane
//                     makes one child and bulk-counts its moves per round
//   k_count1          the last ply alone (depth 2)
// Writes beyond a level's capacity are dropped and flagged; the host then
// reruns the exact (host-sized) path.  Divide counts accumulate per root move
// with one atomic per wave.
#include <hip/hip_runtime.h>

#include "dc_common.h"
#include "dc_perft.h"

namespace dc {

// ------------------------------------------------------------ rules policies
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
__device__ __forceinline__ u32 load_meta(const uint16_t* meta, u64 i) {
  if constexpr (R::kMeta) return meta[i];
  else return 0;
}

template <class R>
__device__ __forceinline__ u32 count_rt(const Board& b, u32 meta, u32 stm) {
  return stm ? R::template count<1>(b, meta) : R::template count<0>(b, meta);
}

// ------------------------------------------------------------- block scan
// Exclusive scan over a 1024-thread (16-wave) or 256-thread block.
template <int NW>
__device__ __forceinline__ u64 block_excl_scan64(u64 v, u64* wsum /*LDS[NW]*/, u64* total) {
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
  for (int k = 0; k < NW; ++k) {
    const u64 x = wsum[k];
    before += ((u32)k < w) ? x : 0;
    all += x;
  }
  __syncthreads();
  *total = all;
  return before + incl - v;
}

// ------------------------------------------------------------- k_expand_top
constexpr int kTopThreads = 1024;

template <class R, int STM>
__device__ __forceinline__ void top_level(const Board* cur, const uint16_t* cur_meta, const uint16_t* cur_tags, u64 n,
                                          Board* nxt, uint16_t* nxt_meta, uint16_t* nxt_tags, u64 cap, bool root,
                                          PerftResult* res, u64* wsum, u64* s_total) {
  const u32 t = threadIdx.x;
  const u64 k = (n + kTopThreads - 1) / kTopThreads;
  const u64 lo = min(n, (u64)t * k), hi = min(n, lo + k);
  u64 mine = 0;
  for (u64 i = lo; i < hi; ++i) mine += R::template count<STM>(cur[i], load_meta<R>(cur_meta, i));
  u64 total;
  u64 o = block_excl_scan64<kTopThreads / 64>(mine, wsum, &total);
  if (t == 0) *s_total = total;
  if (total > cap) return;  // caller flags overflow
  for (u64 i = lo; i < hi; ++i) {
    const Board p = cur[i];
    const u32 pm = load_meta<R>(cur_meta, i);
    const uint16_t tag = cur_tags[i];
    R::template for_each<STM>(p, pm, [&](int f, int to, int promo) {
      Board c = p;
      const u32 cm = R::template make<STM>(c, pm, f, to, promo);
      nxt[o] = c;
      if constexpr (R::kMeta) nxt_meta[o] = (uint16_t)cm;
      if (root) {
        nxt_tags[o] = (uint16_t)o;
        if (o < 256) res->root_moves[o] = (uint16_t)(f | (to << 6) | (promo << 12));
      } else {
        nxt_tags[o] = tag;
      }
      ++o;
    });
  }
}

// One workgroup: root (level 0) -> level `target` (1 or 2).  Level 1 lives in
// scratch; the target level goes to `out` (capacity cap_out) with Range out_rng.
template <class R>
__global__ __launch_bounds__(kTopThreads) void k_expand_top(const Board* __restrict__ root, const uint16_t* __restrict__ root_meta,
                                                             u32 stm0, u32 target, Board* __restrict__ s_nodes,
                                                             uint16_t* __restrict__ s_meta, uint16_t* __restrict__ s_tags,
                                                             u64 cap_s, Board* __restrict__ out, uint16_t* __restrict__ out_meta,
                                                             uint16_t* __restrict__ out_tags, u64 cap_out,
                                                             PerftResult* __restrict__ res, Range* __restrict__ out_rng) {
  __shared__ u64 wsum[kTopThreads / 64];
  __shared__ u64 s_total;
  __shared__ uint16_t s_root_tag;
  if (threadIdx.x == 0) s_root_tag = 0;
  __syncthreads();
  const Board rb = root[0];
  const uint16_t rmeta = R::kMeta ? root_meta[0] : (uint16_t)0;
  // level 0 -> 1
  {
    Board* dst = target == 1 ? out : s_nodes;
    uint16_t* dm = target == 1 ? out_meta : s_meta;
    uint16_t* dt = target == 1 ? out_tags : s_tags;
    const u64 cap = target == 1 ? cap_out : cap_s;
    if (stm0) top_level<R, 1>(&rb, &rmeta, &s_root_tag, 1, dst, dm, dt, cap, true, res, wsum, &s_total);
    else top_level<R, 0>(&rb, &rmeta, &s_root_tag, 1, dst, dm, dt, cap, true, res, wsum, &s_total);
    __syncthreads();
    const u64 n1 = s_total;
    if (threadIdx.x == 0) {
      res->n_root = (u32)min(n1, (u64)0xFFFFFFFFu);
      res->level_n[1] = n1;
      if (n1 > cap || n1 > 256) res->overflow = 1;
    }
    if (n1 > cap || n1 > 256) {
      if (threadIdx.x == 0) *out_rng = Range{0, 0};
      return;
    }
    if (target == 1) {
      if (threadIdx.x == 0) *out_rng = Range{0, n1};
      return;
    }
  }
  // level 1 -> 2
  __syncthreads();
  const u64 n1 = s_total;
  __syncthreads();
  if (stm0) top_level<R, 0>(s_nodes, s_meta, s_tags, n1, out, out_meta, out_tags, cap_out, false, res, wsum, &s_total);
  else top_level<R, 1>(s_nodes, s_meta, s_tags, n1, out, out_meta, out_tags, cap_out, false, res, wsum, &s_total);
  __syncthreads();
  if (threadIdx.x == 0) {
    const u64 n2 = s_total;
    res->level_n[2] = n2;
    if (n2 > cap_out) {
      res->overflow = 1;
      *out_rng = Range{0, 0};
    } else {
      *out_rng = Range{0, n2};
    }
  }
}

// ---------------------------------------------------------- level kernels
template <class R, int STM>
__global__ __launch_bounds__(256) void k_count_children(const Board* __restrict__ nodes, const uint16_t* __restrict__ meta,
                                                        const Range* __restrict__ rng, u32* __restrict__ counts) {
  const u64 lo = rng->lo, hi = rng->hi;
  for (u64 i = lo + (u64)blockIdx.x * blockDim.x + threadIdx.x; i < hi; i += (u64)gridDim.x * blockDim.x)
    counts[i - lo] = R::template count<STM>(load_board(nodes, i), load_meta<R>(meta, i));
}

template <class R, int STM>
__global__ __launch_bounds__(256) void k_expand_write(const Board* __restrict__ nodes, const uint16_t* __restrict__ meta,
                                                      const uint16_t* __restrict__ tags, const Range* __restrict__ rng,
                                                      const u64* __restrict__ offsets, Board* __restrict__ out,
                                                      uint16_t* __restrict__ out_meta, uint16_t* __restrict__ out_tags,
                                                      u64 cap) {
  const u64 lo = rng->lo, hi = rng->hi;
  for (u64 i = lo + (u64)blockIdx.x * blockDim.x + threadIdx.x; i < hi; i += (u64)gridDim.x * blockDim.x) {
    const Board p = load_board(nodes, i);
    const u32 pm = load_meta<R>(meta, i);
    const uint16_t tag = tags[i];
    u64 o = offsets[i - lo];
    R::template for_each<STM>(p, pm, [&](int f, int t, int promo) {
      if (o < cap) {
        Board c = p;
        const u32 cm = R::template make<STM>(c, pm, f, t, promo);
        store_board(out, o, c);
        if constexpr (R::kMeta) out_meta[o] = (uint16_t)cm;
        out_tags[o] = tag;
      }
      ++o;
    });
  }
}

__global__ void k_slice(Range* rng, u32 shard, u32 n_shards) {
  const u64 lo = rng->lo, n = rng->hi - rng->lo;
  *rng = Range{lo + n * shard / n_shards, lo + n * (shard + 1) / n_shards};
}

template <class R, int STM>
__global__ __launch_bounds__(256) void k_count1(const Board* __restrict__ nodes, const uint16_t* __restrict__ meta,
                                                const uint16_t* __restrict__ tags, const Range* __restrict__ rng,
                                                u64* __restrict__ divide) {
  __shared__ u64 hist[256];
  tag_hist_init(hist);
  const u64 lo = rng->lo, hi = rng->hi;
  for (u64 base = lo + (u64)blockIdx.x * blockDim.x; base < hi; base += (u64)gridDim.x * blockDim.x) {
    const u64 i = base + threadIdx.x;
    const bool valid = i < hi;
    u32 c = 0, tag = 0;
    if (valid) {
      c = R::template count<STM>(load_board(nodes, i), load_meta<R>(meta, i));
      tag = tags[i];
    }
    tag_hist_add(hist, tag, c, valid);
  }
  tag_hist_flush(hist, divide);
}

constexpr int kC2Waves = 4;
constexpr int kC2Cap = 64 * 28;  // child slots per wave and window (4 blocks of 4 waves per CU)

struct C2Shared {
  Board parent[kC2Waves][64];
  u32 pmeta[kC2Waves][64];
  u32 slot[kC2Waves][kC2Cap];
  u64 hist[256];
};

template <class R, int STM>
__global__ __launch_bounds__(256, 4) void k_count2(const Board* __restrict__ nodes, const uint16_t* __restrict__ meta,
                                                const uint16_t* __restrict__ tags, const Range* __restrict__ rng,
                                                u64* __restrict__ divide) {
  __shared__ C2Shared sh;
  tag_hist_init(sh.hist);
  const u32 w = threadIdx.x >> 6;
  const u32 lane = lane_id();
  Board* par = sh.parent[w];
  u32* pmeta = sh.pmeta[w];
  u32* slot = sh.slot[w];
  const u64 lo = rng->lo, hi = rng->hi;
  const u64 groups = (hi - lo + 63) >> 6;
  for (u64 g = (u64)blockIdx.x * kC2Waves + w; g < groups; g += (u64)gridDim.x * kC2Waves) {
    const u64 i = lo + (g << 6) + lane;
    const bool valid = i < hi;
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
        else if (k) atomicAdd((unsigned long long*)&sh.hist[ptag], (unsigned long long)k);
      }
    }
    tag_hist_add(sh.hist, tag0, acc, true);
    wave_lds_sync();
  }
  tag_hist_flush(sh.hist, divide);
}

// ------------------------------------------------- descriptor path (small final levels)
// k_emit_desc: the parents' children become 8-byte descriptors {parent index,
// move} at scanned offsets (k_count_children + scan, no atomics).  k_count_desc
// then gives every child its own lane, so the last ply is balanced over the
// whole GPU even when the parent level is too small to fill it in wave-sized
// groups.
template <class R, int STM>
__global__ __launch_bounds__(256) void k_emit_desc(const Board* __restrict__ nodes, const uint16_t* __restrict__ meta,
                                                   const Range* __restrict__ rng, const u64* __restrict__ offsets,
                                                   u64* __restrict__ desc, u64 cap) {
  const u64 lo = rng->lo, hi = rng->hi;
  for (u64 i = lo + (u64)blockIdx.x * blockDim.x + threadIdx.x; i < hi; i += (u64)gridDim.x * blockDim.x) {
    const Board p = load_board(nodes, i);
    const u32 pm = load_meta<R>(meta, i);
    u64 o = offsets[i - lo];
    R::template for_each<STM>(p, pm, [&](int f, int t, int promo) {
      if (o < cap) desc[o] = i | ((u64)((u32)f | ((u32)t << 6) | ((u32)promo << 12)) << 32);
      ++o;
    });
  }
}

template <class R, int STM>
__global__ __launch_bounds__(256) void k_count_desc(const Board* __restrict__ nodes, const uint16_t* __restrict__ meta,
                                                    const uint16_t* __restrict__ tags, const u64* __restrict__ desc,
                                                    const Range* __restrict__ drng, u64* __restrict__ divide) {
  __shared__ u64 hist[256];
  tag_hist_init(hist);
  const u64 n = drng->hi;
  for (u64 base = (u64)blockIdx.x * blockDim.x; base < n; base += (u64)gridDim.x * blockDim.x) {
    const u64 j = base + threadIdx.x;
    const bool valid = j < n;
    u32 k = 0, tag = 0;
    if (valid) {
      const u64 d = desc[j];
      const u64 pi = d & 0xFFFFFFFFull;
      const u32 m = (u32)(d >> 32);
      Board c = load_board(nodes, pi);
      const u32 cm = R::template make<STM>(c, load_meta<R>(meta, pi), (int)(m & 63), (int)((m >> 6) & 63),
                                           (int)((m >> 12) & 7));
      k = R::template count<1 - STM>(c, cm);
      tag = tags[pi];
    }
    tag_hist_add(hist, tag, k, valid);
  }
  tag_hist_flush(hist, divide);
}

// -------------------------------------------------------------------- scan
constexpr int kScanItems = 16;
constexpr int kScanBlock = 256 * kScanItems;

// n: explicit (n_dev == nullptr) or rng->hi - rng->lo.
template <class T>
__global__ __launch_bounds__(256) void k_scan_reduce(const T* __restrict__ in, u64 n_static, const Range* __restrict__ rng,
                                                     u64* __restrict__ bsums) {
  __shared__ u64 wsum[4];
  const u64 n = rng ? rng->hi - rng->lo : n_static;
  const u64 base = (u64)blockIdx.x * kScanBlock + (u64)threadIdx.x * kScanItems;
  u64 s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k)
    if (base + k < n) s += in[base + k];
  u64 tot;
  block_excl_scan64<4>(s, wsum, &tot);
  if (threadIdx.x == 0) bsums[blockIdx.x] = tot;
}

// Writes exclusive offsets; with `next` set, the thread holding the last
// element publishes the next level's Range and flags overflow beyond `cap`.
template <class T>
__global__ __launch_bounds__(256) void k_scan_apply(const T* __restrict__ in, u64 n_static, const Range* __restrict__ rng,
                                                    const u64* __restrict__ bexcl, u64* __restrict__ out,
                                                    Range* __restrict__ next, u64 cap, PerftResult* __restrict__ res) {
  __shared__ u64 wsum[4];
  const u64 n = rng ? rng->hi - rng->lo : n_static;
  const u64 base = (u64)blockIdx.x * kScanBlock + (u64)threadIdx.x * kScanItems;
  T vals[kScanItems];
  u64 s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    vals[k] = (base + k < n) ? in[base + k] : (T)0;
    s += vals[k];
  }
  u64 tot;
  u64 run = block_excl_scan64<4>(s, wsum, &tot) + (bexcl ? bexcl[blockIdx.x] : 0);
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    if (base + k < n) {
      out[base + k] = run;
      if (next && base + k == n - 1) {
        const u64 total = run + vals[k];
        if (total > cap) {  // the level did not fit: flag it and leave the rest of the run empty
          res->overflow = 1;
          *next = Range{0, 0};
        } else {
          *next = Range{0, total};
        }
      }
    }
    run += vals[k];
  }
  if (next && n == 0 && blockIdx.x == 0 && threadIdx.x == 0) *next = Range{0, 0};
}

// ------------------------------------------------------------- launchers
static constexpr u32 kMaxGrid = 2048;  // 8 blocks of 256 per CU; grid-stride beyond

static inline u32 grid_for(u64 n, u32 per) {
  const u64 b = (n + per - 1) / per;
  return (u32)std::max<u64>(1, std::min<u64>(b, kMaxGrid));
}

#define DC_LAUNCH_STM(KERNEL, R, grid, block, st, ...)                                           \
  do {                                                                                           \
    if (stm) hipLaunchKernelGGL((KERNEL<R, 1>), dim3(grid), dim3(block), 0, st, __VA_ARGS__);   \
    else hipLaunchKernelGGL((KERNEL<R, 0>), dim3(grid), dim3(block), 0, st, __VA_ARGS__);       \
  } while (0)

hipError_t launch_expand_top(hipStream_t st, u32 rules, const Board* root, const uint16_t* root_meta, u32 stm0,
                             u32 target, Board* s_nodes, uint16_t* s_meta, uint16_t* s_tags, u64 cap_s, Board* out,
                             uint16_t* out_meta, uint16_t* out_tags, u64 cap_out, PerftResult* res, Range* out_rng) {
  if (rules == 0)
    hipLaunchKernelGGL(k_expand_top<RefRules>, dim3(1), dim3(kTopThreads), 0, st, root, root_meta, stm0, target, s_nodes,
                       s_meta, s_tags, cap_s, out, out_meta, out_tags, cap_out, res, out_rng);
  else
    hipLaunchKernelGGL(k_expand_top<FideRules>, dim3(1), dim3(kTopThreads), 0, st, root, root_meta, stm0, target,
                       s_nodes, s_meta, s_tags, cap_s, out, out_meta, out_tags, cap_out, res, out_rng);
  return hipGetLastError();
}

hipError_t launch_count_children(hipStream_t st, u32 rules, int stm, const Board* nodes, const uint16_t* meta,
                                 const Range* rng, u64 n_bound, u32* counts) {
  const u32 g = grid_for(n_bound, 256);
  if (rules == 0) DC_LAUNCH_STM(k_count_children, RefRules, g, 256, st, nodes, meta, rng, counts);
  else DC_LAUNCH_STM(k_count_children, FideRules, g, 256, st, nodes, meta, rng, counts);
  return hipGetLastError();
}

hipError_t launch_expand_write(hipStream_t st, u32 rules, int stm, const Board* nodes, const uint16_t* meta,
                               const uint16_t* tags, const Range* rng, u64 n_bound, const u64* offsets, Board* out,
                               uint16_t* out_meta, uint16_t* out_tags, u64 cap) {
  const u32 g = grid_for(n_bound, 256);
  if (rules == 0) DC_LAUNCH_STM(k_expand_write, RefRules, g, 256, st, nodes, meta, tags, rng, offsets, out, out_meta, out_tags, cap);
  else DC_LAUNCH_STM(k_expand_write, FideRules, g, 256, st, nodes, meta, tags, rng, offsets, out, out_meta, out_tags, cap);
  return hipGetLastError();
}

hipError_t launch_slice(hipStream_t st, Range* rng, u32 shard, u32 n_shards) {
  hipLaunchKernelGGL(k_slice, dim3(1), dim3(1), 0, st, rng, shard, n_shards);
  return hipGetLastError();
}

hipError_t launch_final(hipStream_t st, u32 rules, int stm, int plies, const Board* nodes, const uint16_t* meta,
                        const uint16_t* tags, const Range* rng, u64 n_bound, u64* divide) {
  if (plies == 1) {
    const u32 g = grid_for(n_bound, 256);
    if (rules == 0) DC_LAUNCH_STM(k_count1, RefRules, g, 256, st, nodes, meta, tags, rng, divide);
    else DC_LAUNCH_STM(k_count1, FideRules, g, 256, st, nodes, meta, tags, rng, divide);
  } else {
    const u32 g = grid_for(n_bound, 64 * kC2Waves);
    if (rules == 0) DC_LAUNCH_STM(k_count2, RefRules, g, 256, st, nodes, meta, tags, rng, divide);
    else DC_LAUNCH_STM(k_count2, FideRules, g, 256, st, nodes, meta, tags, rng, divide);
  }
  return hipGetLastError();
}

hipError_t launch_emit_desc(hipStream_t st, u32 rules, int stm, const Board* nodes, const uint16_t* meta,
                            const Range* rng, u64 n_bound, const u64* offsets, u64* desc, u64 cap) {
  const u32 g = grid_for(n_bound, 256);
  if (rules == 0) DC_LAUNCH_STM(k_emit_desc, RefRules, g, 256, st, nodes, meta, rng, offsets, desc, cap);
  else DC_LAUNCH_STM(k_emit_desc, FideRules, g, 256, st, nodes, meta, rng, offsets, desc, cap);
  return hipGetLastError();
}

hipError_t launch_count_desc(hipStream_t st, u32 rules, int stm, const Board* nodes, const uint16_t* meta,
                             const uint16_t* tags, const u64* desc, const Range* drng, u64 n_bound, u64* divide) {
  const u32 g = grid_for(n_bound, 256);
  if (rules == 0) DC_LAUNCH_STM(k_count_desc, RefRules, g, 256, st, nodes, meta, tags, desc, drng, divide);
  else DC_LAUNCH_STM(k_count_desc, FideRules, g, 256, st, nodes, meta, tags, desc, drng, divide);
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

// Recursive scan of static-size u64 block sums.
static hipError_t scan_static(hipStream_t st, const u64* in, u64 n, u64* out, u64* temp) {
  const u32 nb = (u32)((n + kScanBlock - 1) / kScanBlock);
  if (nb <= 1) {
    hipLaunchKernelGGL(k_scan_apply<u64>, dim3(1), dim3(256), 0, st, in, n, (const Range*)nullptr, (const u64*)nullptr,
                       out, (Range*)nullptr, (u64)0, (PerftResult*)nullptr);
    return hipGetLastError();
  }
  u64* bsums = temp;
  u64* bexcl = temp + nb;
  hipLaunchKernelGGL(k_scan_reduce<u64>, dim3(nb), dim3(256), 0, st, in, n, (const Range*)nullptr, bsums);
  hipError_t e = scan_static(st, bsums, nb, bexcl, temp + 2 * (size_t)nb);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_scan_apply<u64>, dim3(nb), dim3(256), 0, st, in, n, (const Range*)nullptr, bexcl, out,
                     (Range*)nullptr, (u64)0, (PerftResult*)nullptr);
  return hipGetLastError();
}

hipError_t launch_scan_level(hipStream_t st, const u32* counts, const Range* rng, u64 n_bound, u64* offsets, u64* temp,
                             Range* next, u64 cap_next, PerftResult* res) {
  const u32 nb = (u32)std::max<u64>(1, (n_bound + kScanBlock - 1) / kScanBlock);
  if (nb == 1) {
    hipLaunchKernelGGL(k_scan_apply<u32>, dim3(1), dim3(256), 0, st, counts, (u64)0, rng, (const u64*)nullptr, offsets,
                       next, cap_next, res);
    return hipGetLastError();
  }
  u64* bsums = temp;
  u64* bexcl = temp + nb;
  hipLaunchKernelGGL(k_scan_reduce<u32>, dim3(nb), dim3(256), 0, st, counts, (u64)0, rng, bsums);
  hipError_t e = scan_static(st, bsums, nb, bexcl, temp + 2 * (size_t)nb);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_scan_apply<u32>, dim3(nb), dim3(256), 0, st, counts, (u64)0, rng, bexcl, offsets, next, cap_next,
                     res);
  return hipGetLastError();
}

}  // namespace dc
