// dc_perft.hip -- device-driven perft pipeline for gfx950 (RULES_REF and RULES_FIDE).
//
// A perft(d) run is one fixed launch sequence with the level sizes kept on the
// device (Range descriptors), so the host synchronises once per run:
//
//   k_expand_top      one workgroup expands the root to ply T (<= 3) in block-
//                     scanned, deterministic (parent, class, target) order and
//                     records the root moves (the divide keys)
//   k_level_count     K3a  children per frontier node (bulk count) + per-chunk  \  3 launches
//                          sums (a chunk = 256 consecutive nodes = one block)   |  per level,
//   k_chunk_scan      one workgroup scans the chunk sums -> chunk bases and   |  grid-stride,
//                     the next level's Range (overflow flagged beyond cap)    |  n read on
//   k_level_write     K3b  block scan of the chunk + base -> children written   /  the device
//   k_slice           contiguous shard of a level for data-parallel runs
//   k_count2          the last two plies fused: per wave, 64 parents' children
//                     are compacted into LDS (wave prefix sum) and each lane
//                     makes one child and bulk-counts its moves per round
//   k_emit_desc +     the last two plies for small parent levels: children as
//   k_count_desc      8-byte descriptors, then one lane per child (balanced)
//   k_count1          the last ply alone (depth 2)
// Writes beyond a level's capacity are dropped and flagged; the host then
// reruns the exact (host-sized) path.  Divide counts accumulate per root move
// with one atomic per wave.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstddef>
#include <cstring>
#include <map>
#include <mutex>

#include "dc_common.h"
#include "dc_perft.h"

DC_BBPROF_DEFINE(perft)  // measurement builds only (tools/bbprof.py)

namespace dc {

// ------------------------------------------------------------ rules policies
struct RefRules {
  static constexpr bool kMeta = false;
  static constexpr bool kSplit = false;  // k_count2b: REF's final stage split is k_count2c / k_count3c
  // blocks of 256 per CU the level / final-stage kernels are built for
  // (FIDE's legal-move analysis needs the registers of 2: spill-free)
  static constexpr int kMinBlocks = 4;
  static constexpr int kFinalMinBlocks = 4;  // k_count2b
  static constexpr int kTopThreads = 1024;    // k_expand_top's one workgroup
  template <int STM>
  __device__ static __forceinline__ u32 count(const Board& b, u32) { return ref_count<STM>(b); }
  template <int STM>
  __device__ static __forceinline__ u32 count_final(const Board& b, u32) { return ref_count<STM>(b); }
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

#ifndef DC_FIDE_TAB
#define DC_FIDE_TAB 0  // 1: k_count2b<FideRules> leaf counts with kAtt king/knight sets -- WRONG counts, see DESIGN.md §3.6
#endif
#ifndef DC_FIDE_MINB
#define DC_FIDE_MINB 2  // (A/B: 4 = the round-3 budget, 128 VGPRs with spills)
#endif
#ifndef DC_FIDE_SPLIT
#define DC_FIDE_SPLIT 2  // k_count2b<FideRules>: simple children counted as c0 (fide_sens); 0: every child
                         // made; 1: the counting pass enumerates; 2: it counts set-wise (fide_count_split)
#endif
struct FideRules {
  static constexpr bool kMeta = true;
  static constexpr bool kSplit = DC_FIDE_SPLIT != 0;
  static constexpr int kMinBlocks = DC_FIDE_MINB;
  // k_count2b: 3 blocks/CU (148 VGPRs, 0 B) since the parent is re-read from
  // LDS for the enumeration (its registers are free across the child loop)
  static constexpr int kFinalMinBlocks = DC_FIDE_MINB > 3 ? DC_FIDE_MINB : 3;
  // k_expand_top: 512 threads (2 waves/SIMD, 256 VGPRs): the legal-move
  // analysis fits without scratch (1024 threads: 128 VGPRs, 180 B/lane)
  static constexpr int kTopThreads = 512;
  template <int STM>
  __device__ static __forceinline__ u32 count(const Board& b, u32 meta) { return fide_count<STM>(b, meta); }
  // the final stage's leaf counts: king/knight attack sets from kAtt
  template <int STM>
  __device__ static __forceinline__ u32 count_final(const Board& b, u32 meta) {
    return fide_count<STM, DC_FIDE_TAB != 0>(b, meta);
  }
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
// threadIdx.x rebuilt at the point of use from the lane's mbcnt and the
// wave's index (an SGPR): an opaque statement the compiler cannot hoist or
// merge, so no thread-index-derived address stays live (and spills) across
// the final stage's register-heavy code (round 3: k_count3c spill-free).
// DC_C2C_LIVE_TID=1 (A/B only) restores the round-2 code generation: the
// plain thread index, kept live by the compiler and spilled at 4 waves/SIMD
// (with -DDC_C2C_REC=0 -DDC_C2C_SOA=1: a layout of the round-2 failing kind;
// tools/c2c_variants.sh soa_r2 rebuilds the exact failing source).
#ifndef DC_C2C_LIVE_TID
#define DC_C2C_LIVE_TID 0
#endif
__device__ __forceinline__ u32 otid(u32 wave) {
#if DC_C2C_LIVE_TID
  (void)wave;
  return threadIdx.x;
#endif
  u32 t;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0\n\tv_lshl_add_u32 %0, %1, 6, %0"
               : "=&v"(t)
               : "s"(wave));
  return t;
}

// 32-bit counts whose block total fits 32 bits (the final stage's special
// moves per parent): one DPP add per scan step (round 4: the 64-bit scan was
// 1.6 % of k_count3c's VALU issue cycles)
template <int NW>
__device__ __forceinline__ u32 block_excl_scan32(u32 v, u32* wsum /*LDS[NW]*/, u32* total, u32 w = threadIdx.x >> 6) {
  const u32 incl = wave_incl_scan(v);
  if (lane_id() == 63) wsum[w] = incl;
  __syncthreads();
  u32 before = 0, all = 0;
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    const u32 x = wsum[k];
    before += ((u32)k < w) ? x : 0u;
    all += x;
  }
  __syncthreads();
  *total = all;
  return before + incl - v;
}

template <int NW>
__device__ __forceinline__ u64 block_excl_scan64(u64 v, u64* wsum /*LDS[NW]*/, u64* total,
                                                 u32 w = threadIdx.x >> 6) {
  const u32 lane = lane_id();
  const u64 incl = wave_incl_scan64(v);
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

// Move slots of one top-level window in LDS: parent index << 15 | f | t << 6 | promo << 12.
constexpr u32 kTopSlots = 9216;  // 36 KB: startpos ply 3 (8,902 children) in one window

#ifdef DC_AB_KNOBS
// A/B build: k_expand_top's timeline (wall clock, 100 MHz): per ply the ticks
// at entry, after the counts, after the scan, after the enumeration, at exit.
__device__ u64 g_top_trace[4 * 5];
#define DC_TOP_STAMP(ply, k) \
  do {                       \
    if (threadIdx.x == 0 && (ply) < 4) g_top_trace[(ply) * 5 + (k)] = wall_clock64(); \
  } while (0)
#else
#define DC_TOP_STAMP(ply, k) \
  do {                       \
  } while (0)
#endif

// Nodes of a top-level ply staged in LDS (parents read per child without a
// global round trip) when the ply holds at most this many (startpos ply 2: 400).
constexpr u32 kTopStage = 512;

// One ply of the top expansion: counts per node, block scan, then in windows
// of kTopSlots children: every thread writes its nodes' move words into LDS
// at its scan offset, and all 1024 threads make and store one child per slot
// (coalesced).  Making the children in the enumeration loop itself left ply
// 3 to 400 threads making ~22 children each, one after another.  A ply of at
// most kTopStage nodes is staged in LDS (spar/smeta/stags) as it is counted,
// so the enumeration and the children read their parents from LDS: reading
// them from the previous ply's global output cost a dependent L2 round trip
// per child (9 per thread at ply 3).
// Class groups [g0, g0 + ng) of ref_group_moves, in order (g0, ng wave- or
// lane-varying: a switch per group).
template <int STM, class V>
__device__ __forceinline__ void ref_groups_moves(const Board& b, u32 g0, u32 ng, V&& visit) {
  for (u32 g = g0; g < g0 + ng; ++g) {
    switch (g) {
      case 0: ref_group_moves<STM, 0>(b, visit); break;
      case 1: ref_group_moves<STM, 1>(b, visit); break;
      case 2: ref_group_moves<STM, 2>(b, visit); break;
      default: ref_group_moves<STM, 3>(b, visit); break;
    }
  }
}
template <int STM>
__device__ __forceinline__ u32 ref_groups_count(const Board& b, u32 g0, u32 ng) {
  u32 c = 0;
  for (u32 g = g0; g < g0 + ng; ++g) {
    switch (g) {
      case 0: c += ref_group_count<STM, 0>(b); break;
      case 1: c += ref_group_count<STM, 1>(b); break;
      case 2: c += ref_group_count<STM, 2>(b); break;
      default: c += ref_group_count<STM, 3>(b); break;
    }
  }
  return c;
}

// REF plies of at most kTopGroupNodes nodes split each node's moves over the
// four class groups of ref_group_moves: thread t takes groups
// [g0, g0 + ng) of node t % NB, with NB = 256 nodes per group (ng = 1) when
// n <= 256, else NB = 512 (ng = 2), so every wave runs one group's code (no
// divergence between groups).  A node's offset comes from a block scan of the
// node totals (the group counts summed in LDS) and a group's from the counts
// of the node's earlier groups: the children keep ref_for_each_move's
// class-major order.  One lane walking all of a node's moves took 3.5 / 4.2 /
// 5.6 us to enumerate plies 1 / 2 / 3 of startpos (tools/top_trace.py, round 2;
// splitting a node's groups over adjacent lanes of one wave was slower still).
constexpr u32 kTopGroupNodes = 512;


template <class R, int STM>
__device__ __forceinline__ void top_level(const Board* cur, const uint16_t* cur_meta, const uint16_t* cur_tags, u64 n,
                                          Board* nxt, uint16_t* nxt_meta, uint16_t* nxt_tags, u64 cap, bool root,
                                          PerftResult* res, u64* wsum, u64* s_total, u32* slots, Board* spar,
                                          uint16_t* smeta, uint16_t* stags, u32 ply, u32* gcnt, u32* node_off,
                                          u32* words = nullptr) {
  constexpr int kTopThreads = R::kTopThreads;  // (shadows the file-wide 1024)
  const u32 t = threadIdx.x;
  DC_TOP_STAMP(ply, 0);
  const bool stage = n <= kTopStage;
  const bool grp = !R::kMeta && n <= kTopGroupNodes;  // (kTopGroupNodes <= kTopStage: grouped plies are staged)
  const u32 NB = n <= 256 ? 256u : 512u, ng = NB / 256u;
  const u32 gnode = t % NB, g0 = (t / NB) * ng;
  const u64 k = (n + kTopThreads - 1) / kTopThreads;
  const u64 lo = grp ? min(n, (u64)gnode) : min(n, (u64)t * k);
  const u64 hi = grp ? min(n, (u64)gnode + 1) : min(n, lo + k);
  u64 mine = 0;
  for (u64 i = lo; i < hi; ++i) {
    const Board bi = cur[i];
    const u32 mi = load_meta<R>(cur_meta, i);
    if (stage && (!grp || g0 == 0)) {
      spar[i] = bi;
      if constexpr (R::kMeta) smeta[i] = (uint16_t)mi;
      stags[i] = root ? (uint16_t)0 : cur_tags[i];
    }
    if constexpr (!R::kMeta) {
      if (grp) mine += ref_groups_count<STM>(bi, g0, ng);
      else mine += R::template count<STM>(bi, mi);
    } else {
      mine += R::template count<STM>(bi, mi);
    }
  }
  DC_TOP_STAMP(ply, 1);
  u64 total, o;
  if (grp) {
    // group counts -> LDS (gcnt[g * NB + node]), node totals scanned in node
    // order (by wave 0 alone up to 64 nodes), then each lane's offset within
    // its node
    gcnt[t] = (u32)mine;
    __syncthreads();
    if (n <= 64) {
      if (t < 64) {
        u64 ntot = 0;
        if (t < n)
          for (u32 g = 0; g < 4 / ng; ++g) ntot += gcnt[g * NB + t];
        const u64 incl = wave_incl_scan64(ntot);
        node_off[t] = (u32)(incl - ntot);
        if (t == 63) wsum[0] = incl;
      }
      __syncthreads();
      total = wsum[0];
    } else {
      u64 ntot = 0;
      if (t < n)
        for (u32 g = 0; g < 4 / ng; ++g) ntot += gcnt[g * NB + t];
      const u64 nodeoff = block_excl_scan64<kTopThreads / 64>(ntot, wsum, &total);
      if (t < n) node_off[t] = (u32)nodeoff;
      __syncthreads();
    }
    o = 0;
    if (lo < hi) {
      o = node_off[gnode];
      for (u32 g = 0; g < t / NB; ++g) o += gcnt[g * NB + gnode];
    }
  } else {
    o = block_excl_scan64<kTopThreads / 64>(mine, wsum, &total);  // its barriers publish the staging
  }
  DC_TOP_STAMP(ply, 2);
  if (t == 0) *s_total = total;
  if (total > cap) return;  // caller flags overflow
  const Board* par = stage ? spar : cur;
  auto pmeta = [&](u64 i) -> u32 {
    if constexpr (R::kMeta) return stage ? smeta[i] : cur_meta[i];
    else return 0;
  };
  for (u64 wb = 0; wb < total; wb += kTopSlots) {
    if (wb) __syncthreads();  // the previous window's slots are consumed
    if (o < wb + kTopSlots && o + mine > wb) {
      u64 j = o;
      for (u64 i = lo; i < hi; ++i) {
        auto put = [&](int f, int to, int promo) {
          if (j >= wb && j < wb + kTopSlots) slots[j - wb] = ((u32)i << 15) | (u32)f | ((u32)to << 6) | ((u32)promo << 12);
          ++j;
        };
        if constexpr (!R::kMeta) {
          if (grp) {
            ref_groups_moves<STM>(par[i], g0, ng, [&](int f, int to) { put(f, to, 0); });
            continue;
          }
        }
        R::template for_each<STM>(par[i], pmeta(i), put);
      }
    }
    __syncthreads();
    DC_TOP_STAMP(ply, 3);
    const u32 ns = (u32)min((u64)kTopSlots, total - wb);
    if (words) {  // the children are made and counted by k_make_count, on many CUs
      for (u32 r = t; r < ns; r += kTopThreads) words[wb + r] = slots[r];
      continue;
    }
    for (u32 r = t; r < ns; r += kTopThreads) {
      const u32 e = slots[r];
      const u32 pl = e >> 15;
      const int f = (int)(e & 63), to = (int)((e >> 6) & 63), promo = (int)((e >> 12) & 7);
      Board c = par[pl];
      const u32 cm = R::template make<STM>(c, pmeta(pl), f, to, promo);
      const u64 oo = wb + r;
      nxt[oo] = c;
      if constexpr (R::kMeta) nxt_meta[oo] = (uint16_t)cm;
      if (root) {
        nxt_tags[oo] = (uint16_t)oo;
        if (oo < 256) {
          res->root_moves[oo] = (uint16_t)(f | (to << 6) | (promo << 12));
          res->root_parent[oo] = (uint8_t)pl;
        }
      } else {
        nxt_tags[oo] = stage ? stags[pl] : cur_tags[pl];
      }
    }
  }
}

struct TopBufs {
  Board* nodes[2];  // scratch for plies 1 and 2 (capacities cap[0], cap[1])
  uint16_t* meta[2];
  uint16_t* tags[2];
  u64 cap[2];
};

// One workgroup: root (ply 0) -> ply `target` (1..3).  Intermediate plies go
// to scratch; the target ply goes to `out` (capacity cap_out), Range out_rng.
template <class R>
__global__ __launch_bounds__(R::kTopThreads) void k_expand_top(const Board* __restrict__ root,
                                                             const uint16_t* __restrict__ root_meta, u32 stm0,
                                                             u32 target, TopBufs sb, Board* __restrict__ out,
                                                             uint16_t* __restrict__ out_meta,
                                                             uint16_t* __restrict__ out_tags, u64 cap_out,
                                                             PerftResult* __restrict__ res, Range* __restrict__ out_rng,
                                                             u32* __restrict__ words, u32 n_root) {
  constexpr int kTopThreads = R::kTopThreads;  // (shadows the file-wide 1024)
  __shared__ u64 wsum[kTopThreads / 64];
  __shared__ u64 s_total;
  __shared__ u32 slots[kTopSlots];
  __shared__ u32 gcnt[kTopThreads];         // grouped plies: per-thread group counts
  __shared__ u32 node_off[kTopGroupNodes];  // ... and node offsets
  __shared__ Board spar[kTopStage];
  __shared__ uint16_t smeta[R::kMeta ? kTopStage : 1];
  __shared__ uint16_t stags[kTopStage];
  __shared__ uint16_t s_root_tag;
  __shared__ Board s_root[kMaxPerftRoots];  // one position, or a batch's (dc_perft_batch)
  __shared__ uint16_t s_root_meta[kMaxPerftRoots];
  // the run's result block is cleared here, not by a separate memset launch
  // (one ~5 us graph node less per perft)
  static_assert(sizeof(PerftResult) % 8 == 0, "PerftResult is cleared in u64 words");
  for (u32 k = threadIdx.x; k < sizeof(PerftResult) / 8; k += kTopThreads) reinterpret_cast<u64*>(res)[k] = 0;
  n_root = min(max(n_root, 1u), kMaxPerftRoots);  // (the host checks the count)
  if (threadIdx.x == 0) s_root_tag = 0;
  if (threadIdx.x < n_root) {
    s_root[threadIdx.x] = root[threadIdx.x];
    s_root_meta[threadIdx.x] = R::kMeta ? root_meta[threadIdx.x] : (uint16_t)0;
  }
  __syncthreads();
  const Board* cur = s_root;
  const uint16_t* cur_meta = s_root_meta;
  const uint16_t* cur_tags = &s_root_tag;  // (ply 1 tags each child by its index: roots need none)
  u64 n = n_root;
  for (u32 ply = 1; ply <= target; ++ply) {
    const bool last = ply == target;
    Board* dst = last ? out : sb.nodes[ply - 1];
    uint16_t* dm = last ? out_meta : sb.meta[ply - 1];
    uint16_t* dt = last ? out_tags : sb.tags[ply - 1];
    const u64 cap = last ? cap_out : sb.cap[ply - 1];
    u32* wd = last && ply >= 2 ? words : nullptr;  // target ply as move words (k_make_count makes it)
    if ((stm0 ^ (ply - 1)) & 1)
      top_level<R, 1>(cur, cur_meta, cur_tags, n, dst, dm, dt, cap, ply == 1, res, wsum, &s_total, slots, spar, smeta,
                      stags, ply, gcnt, node_off, wd);
    else
      top_level<R, 0>(cur, cur_meta, cur_tags, n, dst, dm, dt, cap, ply == 1, res, wsum, &s_total, slots, spar, smeta,
                      stags, ply, gcnt, node_off, wd);
    __syncthreads();
    DC_TOP_STAMP(ply, 4);
    n = s_total;
    __syncthreads();
    bool bad = n > cap;
    if (ply == 1) {
      bad = bad || n > 256;
      if (threadIdx.x == 0) res->n_root = (u32)min(n, (u64)0xFFFFFFFFu);
    }
    if (threadIdx.x == 0) res->level_n[ply] = n;
    if (bad) {
      if (threadIdx.x == 0) {
        res->overflow = 1;
        *out_rng = Range{0, 0};
      }
      return;
    }
    cur = dst;
    cur_meta = dm;
    cur_tags = dt;
  }
  if (threadIdx.x == 0) *out_rng = Range{0, n};
}

// ---------------------------------------------------------- level kernels
// A chunk is 256 consecutive nodes of the level's range, processed by one
// block; chunk sums are scanned by one workgroup; no global atomics.
constexpr u32 kChunk = 256;

template <class R, int STM>
__global__ __launch_bounds__(256) void k_level_count(const Board* __restrict__ nodes, const uint16_t* __restrict__ meta,
                                                     const Range* __restrict__ rng, u32* __restrict__ counts,
                                                     u64* __restrict__ chunk_sum) {
  __shared__ u64 wsum[4];
  const u64 lo = rng->lo, hi = rng->hi;
  const u64 nch = (hi - lo + kChunk - 1) / kChunk;
  for (u64 c = blockIdx.x; c < nch; c += gridDim.x) {
    const u64 i = lo + c * kChunk + threadIdx.x;
    u32 cnt = 0;
    if (i < hi) {
      cnt = R::template count<STM>(load_board(nodes, i), load_meta<R>(meta, i));
      counts[i - lo] = cnt;
    }
    u64 tot;
    block_excl_scan64<4>(cnt, wsum, &tot);
    if (threadIdx.x == 0) chunk_sum[c] = tot;
  }
}

// k_level_count for a level k_expand_top left as move words (words != nullptr
// there): each child is made from its parent (the previous top ply, still in
// the top scratch) and stored with its tag before it is counted.  Making the
// 8,902 ply-3 children of startpos inside the one-workgroup k_expand_top took
// 7.1 us (tools/top_trace.py); here they spread over 35 blocks.
// STM = side to move at the parents.
template <class R, int STM>
__global__ __launch_bounds__(256) void k_make_count(const Board* __restrict__ par, const uint16_t* __restrict__ par_meta,
                                                    const uint16_t* __restrict__ par_tags, const u32* __restrict__ words,
                                                    const Range* __restrict__ rng, Board* __restrict__ out,
                                                    uint16_t* __restrict__ out_meta, uint16_t* __restrict__ out_tags,
                                                    u32* __restrict__ counts, u64* __restrict__ chunk_sum, u32 wsh,
                                                    u32 wstride) {
  __shared__ u64 wsum[4];
  const u64 lo = rng->lo, hi = rng->hi;
  const u64 nch = (hi - lo + kChunk - 1) / kChunk;
  for (u64 c = blockIdx.x; c < nch; c += gridDim.x) {
    const u64 i = lo + c * kChunk + threadIdx.x;
    u32 cnt = 0;
    if (i < hi) {
      const u32 e = words[wsh + i * wstride];  // (a strided shard of the word level: wstride > 1)
      const u32 pl = e >> 15;
      Board ch = par[pl];
      const u32 cm = R::template make<STM>(ch, load_meta<R>(par_meta, pl), (int)(e & 63), (int)((e >> 6) & 63),
                                           (int)((e >> 12) & 7));
      store_board(out, i, ch);
      if constexpr (R::kMeta) out_meta[i] = (uint16_t)cm;
      out_tags[i] = par_tags[pl];
      cnt = R::template count<1 - STM>(ch, cm);
      counts[i - lo] = cnt;
    }
    u64 tot;
    block_excl_scan64<4>(cnt, wsum, &tot);
    if (threadIdx.x == 0) chunk_sum[c] = tot;
  }
}

// Exclusive scan of the chunk sums of `rng` (one 1024-thread workgroup); writes
// the next level's Range and flags overflow beyond cap.
// select_path != 0: instead of flagging overflow, a total beyond cap -- or a
// parent level larger than select_path nodes -- selects the LDS count2 path
// (res->path = 1) and leaves the descriptor range empty.
__global__ __launch_bounds__(kTopThreads) void k_chunk_scan(const u64* __restrict__ chunk_sum, const Range* __restrict__ rng,
                                                             u64* __restrict__ chunk_base, Range* __restrict__ next,
                                                             u64 cap, PerftResult* __restrict__ res, int select_path,
                                                             u64 guard, u64* __restrict__ zero, u64 zero_max) {
  __shared__ u64 wsum[kTopThreads / 64];
  const u64 nch = (rng->hi - rng->lo + kChunk - 1) / kChunk;
  const u64 per = (nch + kTopThreads - 1) / kTopThreads;
  const u64 a = min(nch, (u64)threadIdx.x * per), b = min(nch, a + per);
  u64 s = 0;
  for (u64 c = a; c < b; ++c) s += chunk_sum[c];
  u64 total;
  u64 run = block_excl_scan64<kTopThreads / 64>(s, wsum, &total);
  for (u64 c = a; c < b; ++c) {
    const u64 v = chunk_sum[c];
    chunk_base[c] = run;
    run += v;
  }
  // zero != nullptr: the next level's chunk sums are accumulated by the
  // k_level_write that makes it (ncounts/nsum): clear its chunks first
  if (zero) {
    const u64 nz = min((total + kChunk - 1) / kChunk, zero_max);
    for (u64 c = threadIdx.x; c < nz; c += kTopThreads) zero[c] = 0;
  }
  if (threadIdx.x == 0) {
    // large parent levels keep count2 busy on their own: no descriptor round trip
    if (select_path && rng->hi - rng->lo > (u64)select_path) total = cap + 1;
    const bool guard_hit = guard && rng->hi - rng->lo > guard;
    if (total > cap || guard_hit) {  // the level would not fit: flag it (or pick count2) and leave the range empty
      if (select_path && !guard_hit) res->path = 1;
      else res->overflow = 1;
      *next = Range{0, 0};
    } else {
      *next = Range{0, total};
    }
  }
}

// Children of one 256-parent chunk, flattened: the parents' moves are
// compacted into LDS slots at block-scan offsets, then every lane makes one
// child per round and stores it at chunk_base + slot -- consecutive lanes write
// consecutive nodes (coalesced), and a ~200k-node ply keeps all lanes busy.
constexpr u32 kWriteCap = 256 * 30;
constexpr u32 kWriteSplit = 16;  // at most this many blocks share one chunk  // ply-5 chunks of perft(7) average 24.8 children per parent: one window

struct WriteShared {
  Board par[256];
  u32 pmeta[256];
  u32 slot[kWriteCap];
  u64 wsum[4];
  uint16_t ptag[256];
};

template <class R, int STM>
__global__ __launch_bounds__(256, R::kMinBlocks) void k_level_write(const Board* __restrict__ nodes, const uint16_t* __restrict__ meta,
                                                        const uint16_t* __restrict__ tags, const Range* __restrict__ rng,
                                                        const u32* __restrict__ counts, const u64* __restrict__ chunk_base,
                                                        Board* __restrict__ out, uint16_t* __restrict__ out_meta,
                                                        uint16_t* __restrict__ out_tags, u64 cap,
                                                        u32* __restrict__ ncounts = nullptr, u64* __restrict__ nsum = nullptr) {
  __shared__ WriteShared sh;
  const u32 tid = threadIdx.x;
  const u64 lo = rng->lo, hi = rng->hi;
  const u64 nch = (hi - lo + kChunk - 1) / kChunk;
  // A level of few chunks (startpos ply 4: 35) would leave most of the
  // resident grid idle with each block making ~5,600 children in ~22 rounds:
  // then S blocks share a chunk, each enumerating its moves but making only
  // its S-th of every window's children.
  const u32 S = (u32)max<u64>(1, min<u64>(kWriteSplit, gridDim.x / max<u64>(nch, 1)));
  for (u64 item = blockIdx.x; item < nch * S; item += gridDim.x) {
    const u64 c = item / S;
    const u32 part = (u32)(item % S);
    const u64 i = lo + c * kChunk + tid;
    const bool valid = i < hi;
    const u32 cnt = valid ? counts[i - lo] : 0;
    u64 total64;
    const u32 excl = (u32)block_excl_scan64<4>(cnt, sh.wsum, &total64);
    const u32 total = (u32)total64;
    const u64 base_out = chunk_base[c];
    Board p{0, 0, 0, 0};
    u32 pm = 0;
    if (valid) {
      p = load_board(nodes, i);
      pm = load_meta<R>(meta, i);
      sh.par[tid] = p;
      if constexpr (R::kMeta) sh.pmeta[tid] = pm;
      sh.ptag[tid] = tags[i];
    }
    for (u32 wb = 0; wb < total; wb += kWriteCap) {
      if (wb) __syncthreads();  // previous window fully consumed
      // this block's part of the window: children [base, base + nslots)
      const u32 nw = min(kWriteCap, total - wb);
      const u32 base = wb + (u32)((u64)nw * part / S);
      const u32 nslots = wb + (u32)((u64)nw * (part + 1) / S) - base;
      u32 j = excl;
      if (valid && j < base + nslots && j + cnt > base) {
        R::template for_each<STM>(p, pm, [&](int f, int t, int promo) {
          if (j >= base && j - base < nslots) sh.slot[j - base] = (u32)f | ((u32)t << 6) | ((u32)promo << 12) | (tid << 15);
          ++j;
        });
      }
      __syncthreads();
      // wave-uniform rounds (the children's counts are wave-reduced)
      for (u32 r0 = 0; r0 < nslots; r0 += 256) {
        const u32 r = r0 + tid;
        const u64 o = base_out + base + r;
        const bool live = r < nslots && o < cap;
        u32 cnt = 0;
        if (live) {
          const u32 e = sh.slot[r];
          const u32 pl = e >> 15;
          Board ch = sh.par[pl];
          const u32 cm = R::template make<STM>(ch, R::kMeta ? sh.pmeta[pl] : 0u, (int)(e & 63), (int)((e >> 6) & 63),
                                               (int)((e >> 12) & 7));
          store_board(out, o, ch);
          if constexpr (R::kMeta) out_meta[o] = (uint16_t)cm;
          out_tags[o] = sh.ptag[pl];
          // ncounts (the next level is counted here, not by k_level_count):
          // the child's own move count, added into its 256-node chunk's sum
          if (ncounts) {
            cnt = R::template count<1 - STM>(ch, cm);
            ncounts[o] = cnt;
          }
        }
        if (ncounts) {  // a wave's 64 consecutive children span at most two chunks
          const u64 k0 = (base_out + base + r0 + (tid & ~63u)) / kChunk;
          const bool in0 = live && o / kChunk == k0;
          const u64 s0 = wave_sum64(in0 ? cnt : 0u), s1 = wave_sum64(live && !in0 ? cnt : 0u);
          if (lane_id() == 0) {
            if (s0) atomicAdd((unsigned long long*)&nsum[k0], (unsigned long long)s0);
            if (s1) atomicAdd((unsigned long long*)&nsum[k0 + 1], (unsigned long long)s1);
          }
        }
      }
    }
    __syncthreads();  // par/slot reused by the next chunk
  }
}

// k_count3c's input (REF): every child of the level `rng` as one u32 move word
// {parent index relative to the level << 12 | f | t << 6} at its scan offset
// (4 instead of 34 bytes per child).  A block takes a quarter of a 256-parent
// chunk (64 parents) and its four waves take the four class groups of
// ref_group_moves (pawns, knights, king + orthogonal rays, diagonal rays), one
// lane per parent: a lane walks about a quarter of its position's moves.
// (Round 2's first version, k_level_write<MW>, had one lane walk all of a
// parent's ~25 moves: 7.4 us of a median block's 10.9 us, the slowest block
// 21.5 us -- tools/lw_trace.py.)  Words go through LDS slots so the global
// stores stay coalesced.
constexpr u32 kMwParents = 64;
constexpr u32 kMwCap = kMwParents * 48;  // word slots per window (a quarter averages ~25 per parent)

struct MwShared {
  u32 slot[kMwCap];
  u32 gcnt[4][kMwParents];
  u32 sexcl[kChunk];
  u64 wsum[4];
};

// W: u32 words (grandparent index < 2^20) or u64 words (perft(8): the ply-5
// grandparents of startpos are 4.9M).
template <int STM, class W = u32>
__global__ __launch_bounds__(256) void k_level_moves(const Board* __restrict__ nodes, const Range* __restrict__ rng,
                                                     const u32* __restrict__ counts, const u64* __restrict__ chunk_base,
                                                     W* __restrict__ mw, u64 cap) {
  __shared__ MwShared sh;
  const u32 tid = threadIdx.x, g = tid >> 6, lane = lane_id();
  const u64 lo = rng->lo, hi = rng->hi;
  const u64 nch = (hi - lo + kChunk - 1) / kChunk;
  for (u64 item = blockIdx.x; item < nch * 4; item += gridDim.x) {
    const u64 c = item >> 2;
    const u32 q = (u32)(item & 3);
    // every global load of the item issues before the scan's barriers
    const u64 ic = lo + c * kChunk + tid;
    const u32 cnt = ic < hi ? counts[ic - lo] : 0u;
    const u32 pl = q * kMwParents + lane;  // this lane's parent within the chunk
    const u64 i = lo + c * kChunk + pl;
    const bool valid = i < hi;
    Board p{0, 0, 0, 0};
    if (valid) p = load_board(nodes, i);
    // (relative to chunk_base[0]: 0 for a whole level, the slice's first word
    // for a slice of one, perft_enqueue's sliced final stage)
    const u64 cbase = chunk_base[c] - chunk_base[0];
    // the chunk's exclusive move offsets (each quarter's block scans the chunk)
    u64 tot64;
    sh.sexcl[tid] = (u32)block_excl_scan64<4>(cnt, sh.wsum, &tot64);
    u32 gc = 0;  // moves of this wave's class group
    if (valid) {
      switch (g) {  // wave-uniform
        case 0: gc = ref_group_count<STM, 0>(p); break;
        case 1: gc = ref_group_count<STM, 1>(p); break;
        case 2: gc = ref_group_count<STM, 2>(p); break;
        default: gc = ref_group_count<STM, 3>(p); break;
      }
    }
    sh.gcnt[g][lane] = gc;
    __syncthreads();
    const u32 qbase = sh.sexcl[q * kMwParents];
    const u32 qend = q == 3 ? (u32)tot64 : sh.sexcl[(q + 1) * kMwParents];
    u32 goff = sh.sexcl[pl] - qbase;
    for (u32 k = 0; k < g; ++k) goff += sh.gcnt[k][lane];
    const u32 qtotal = qend - qbase;
    const u64 base_out = cbase + qbase;
    for (u32 wb = 0; wb < qtotal; wb += kMwCap) {
      if (wb) __syncthreads();  // the previous window is written out
      u32 j = goff;
      if (valid && gc && j < wb + kMwCap && j + gc > wb) {
        auto put = [&](int f, int t) {
          if (j >= wb && j - wb < kMwCap) sh.slot[j - wb] = (u32)f | ((u32)t << 6) | (pl << 12);
          ++j;
        };
        switch (g) {
          case 0: ref_group_moves<STM, 0>(p, put); break;
          case 1: ref_group_moves<STM, 1>(p, put); break;
          case 2: ref_group_moves<STM, 2>(p, put); break;
          default: ref_group_moves<STM, 3>(p, put); break;
        }
      }
      __syncthreads();
      const u32 ns = min(kMwCap, qtotal - wb);
      for (u32 r = tid; r < ns; r += 256) {
        const u64 o = base_out + wb + r;
        if (o < cap) {  // words beyond cap are dropped (the level is flagged)
          const u32 e = sh.slot[r];
          mw[o] = ((W)(c * kChunk + (e >> 12)) << 12) | (W)(e & 0xFFFu);
        }
      }
    }
    __syncthreads();  // sexcl, gcnt and slot are reused by the next item
  }
}

// ------------------------------------------------- k_front (REF, round 6)
// The whole front end of REF perft(6) / perft(7) in one launch: root -> the
// final stage's grandparents (ply 3 + E) as boards and their children as u32
// move words for k_count3c, replacing k_expand_top (one workgroup), k_make_count,
// k_chunk_scan, k_level_write, k_chunk_scan and k_level_moves (~67 us of
// dependent, latency-bound launches per run, round 5).
//
//  * One 1024-thread block per CU.  Every block rebuilds plies 1 and 2 and
//    the ply-3 move counts of the ply-2 nodes in LDS (a few hundred nodes:
//    cheaper than a launch and a global round trip), so every block knows the
//    canonical ply-3 order -- ply-1 parents in order, ref_for_each_move's
//    class-major order within a parent -- that the strided shards of
//    dc_perft_shard are cut from.  (Four 256-thread blocks per CU rebuilt the
//    top four times per CU, and the fourth, whose waves lose the SIMDs'
//    oldest-first arbitration, finished last: tools/front_trace.py.)
//  * Items of P3 consecutive ply-3 nodes of this rank's shard (P3 sized so one
//    pass of the grid covers the shard) are expanded E plies (0: perft(6),
//    1: perft(7)); the boards and their move words are counted first, and the
//    item's offsets come from a decoupled look-back over the earlier items'
//    published (boards, words) -- no same-address atomics (a first version
//    took both from two global cursors: 768 blocks queued on them for up to
//    ~15 us) -- so both levels come out in the canonical order of the legacy
//    chain.  The item's words are walked into an LDS window (board index
//    relative to the item) before the look-back and rebased when stored.
//  * Every serial walk is split over the four class groups of
//    ref_group_moves (a lane walks a quarter of a position's moves).  Group g
//    is taken by waves 4g .. 4g + 3, which sit on the four SIMDs, so each SIMD
//    holds one wave of each group: pawn moves are ~60 % of the words, and a
//    group-per-SIMD mapping (group = wave % 4) left three SIMDs mostly idle.
//  * The block holding the last item publishes the two Ranges (or, when a
//    level is past its capacity or the top past the LDS bounds, flags
//    overflow + front_declined: the host reruns on the legacy chain).  Block
//    0 clears the run's result block and records the root moves.
constexpr u32 kFrontThreads = 1024, kFrontWaves = kFrontThreads / 64;
constexpr u32 kFrontPly1Max = 128;     // root moves (more: the legacy chain)
constexpr u32 kFrontPly2Max = 2048;    // ply-2 nodes (more: the legacy chain)
constexpr u32 kFrontP3Max = 128;       // ply-3 nodes per item
constexpr u32 kFrontBoardsMax = 2048;  // boards per item (more: declined)
constexpr u32 kFrontWin = 28672;       // move words of one LDS window (112 KB: startpos perft(7) items
                                       // hold 12k-32k words)
constexpr u32 kFrontSpillItems = 1024; // items with a spill row for a second window
constexpr u32 kFrontChunk = 5;         // consecutive ply-3 nodes per chunk of an item

#ifdef DC_AB_KNOBS
// A/B build: k_front's timeline (wall clock, 100 MHz) per block:
// kFrontTraceWords stamps each, read back by dc_ab_front_trace
// (tools/front_trace.py).
constexpr u32 kFrontTraceBlocks = 2048, kFrontTraceWords = 16;
__device__ u64 g_front_trace[kFrontTraceBlocks * kFrontTraceWords];
#define DC_FRONT_STAMP(k)                                                                     \
  do {                                                                                        \
    if (threadIdx.x == 0 && blockIdx.x < kFrontTraceBlocks)                                   \
      g_front_trace[blockIdx.x * kFrontTraceWords + (k)] = wall_clock64();                    \
  } while (0)
#else
#define DC_FRONT_STAMP(k) \
  do {                    \
  } while (0)
#endif

struct FrontTop {            // the top, rebuilt by every block (front_top)
  Board p1[kFrontPly1Max];
  u32 w2[kFrontPly2Max];     // ply-2 nodes: ply-1 index << 12 | f | t << 6
  u32 off3[kFrontPly2Max];   // their ply-3 move counts, then exclusive offsets
};
static_assert(sizeof(FrontTop) <= kFrontWin * sizeof(u32), "the window covers the top");

struct FrontShared {
  // The word window overlays the top: it is dead once an item's ply-3 nodes
  // are selected, and a block holding a further item rebuilds it.
  union {
    FrontTop top;
    u32 slotw[kFrontWin];
  };
  union {
    Board b2[kFrontP3Max];           // an item's ply-3 nodes' parents (selection)
    uint16_t gw[4][kFrontBoardsMax]; // per-(group, board) word counts (from pass 1 on)
  };
  Board b3[kFrontP3Max];     // an item's ply-3 nodes
  u32 r3[kFrontP3Max];       // ... their rank among the parent's moves
  uint16_t t3[kFrontP3Max];  // ... their tags (root move index)
  uint16_t m1[kFrontPly1Max];
  u32 gc[4][kFrontP3Max];    // per-group move counts (ply 2, selection, ply 4)
  u32 noff[kFrontP3Max];     // per-node move offsets (ply 2, ply 4)
  u32 slot4[kFrontBoardsMax];      // E = 1: an item's ply-4 moves (ply-3 node << 12 | f | t << 6)
  u32 woff[kFrontBoardsMax];       // per-board word offsets
  u64 red[kFrontWaves][3];
  u64 tot[3];
  u32 g1[4];
  u32 wsum[kFrontWaves];
  u32 jm;
};

// Per item: the published aggregate and inclusive prefix (FrontState, dc_perft.h),
// each one u64 {ready:1 | bad:1 | boards:22 | words:40}.  The slots are zero
// when a run starts: the k_count3c after each k_front zeroes the run's n_items.
__device__ __forceinline__ u64 front_pack(u64 bad, u64 nb, u64 nw) {
  bad |= (nb >> 22) | (nw >> 40) ? 1ull : 0ull;  // (a prefix past the fields is flagged, never wrapped)
  return (1ull << 63) | (bad << 62) | ((nb & 0x3FFFFFull) << 40) | (nw & 0xFFFFFFFFFFull);
}

template <int S, class V>
__device__ __forceinline__ void front_group_moves(u32 g, const Board& b, V&& visit) {
  switch (g) {  // wave-uniform (g = wave % 4)
    case 0: ref_group_moves<S, 0>(b, visit); break;
    case 1: ref_group_moves<S, 1>(b, visit); break;
    case 2: ref_group_moves<S, 2>(b, visit); break;
    default: ref_group_moves<S, 3>(b, visit); break;
  }
}
template <int S>
__device__ __forceinline__ u32 front_group_count(u32 g, const Board& b) {
  switch (g) {
    case 0: return ref_group_count<S, 0>(b);
    case 1: return ref_group_count<S, 1>(b);
    case 2: return ref_group_count<S, 2>(b);
    default: return ref_group_count<S, 3>(b);
  }
}

// Sum of the (bad, boards, words) of every thread of the block: per wave,
// then the wave sums by wave 0.
__device__ __forceinline__ void front_block_sum(FrontShared& sh, u64& bad, u64& nb, u64& nw) {
  bad = wave_sum64(bad);
  nb = wave_sum64(nb);
  nw = wave_sum64(nw);
  const u32 w = threadIdx.x >> 6, l = lane_id();
  if (l == 0) {
    sh.red[w][0] = bad;
    sh.red[w][1] = nb;
    sh.red[w][2] = nw;
  }
  __syncthreads();
  if (w == 0) {
    const u64 x0 = wave_sum64(l < kFrontWaves ? sh.red[l][0] : 0ull);
    const u64 x1 = wave_sum64(l < kFrontWaves ? sh.red[l][1] : 0ull);
    const u64 x2 = wave_sum64(l < kFrontWaves ? sh.red[l][2] : 0ull);
    if (l == 0) {
      sh.tot[0] = x0;
      sh.tot[1] = x1;
      sh.tot[2] = x2;
    }
  }
  __syncthreads();
  bad = sh.tot[0];
  nb = sh.tot[1];
  nw = sh.tot[2];
}

// Decoupled look-back: the (bad, boards, words) of items [0, it), read
// backwards in windows of 1,024 items (one per thread); a window holding an
// inclusive prefix ends the walk.  Every earlier item is held by a resident
// block that takes its items in increasing order, so every slot waited on is
// written.  The slots carry all the data exchanged, so the loads and stores
// are relaxed device-scope atomics: acquire / release forms add a cache
// invalidate or write-back per access (a spinning first version spent ~30 us
// here).
__device__ __forceinline__ void front_lookback(FrontShared& sh, FrontState* st, u32 it, u64& bad, u64& nb, u64& nw) {
  const u32 t = threadIdx.x;
  bad = nb = nw = 0;
  u32 hi = it;
  while (hi > 0) {  // block-uniform
    const u32 lo = hi > kFrontThreads ? hi - kFrontThreads : 0u;
    const u32 j = lo + t;
    u64 a = 0, inc = 0;
    if (j < hi) {
      for (;;) {
        a = __hip_atomic_load(&st->agg[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a >> 63) break;
        __builtin_amdgcn_s_sleep(2);  // (backoff: ~128 cycles between polls of a slot not yet written)
      }
      inc = __hip_atomic_load(&st->incl[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (t == 0) sh.jm = 0;
    __syncthreads();
    if (j < hi && (inc >> 63)) atomicMax(&sh.jm, j + 1);  // the window's last inclusive prefix (+1)
    __syncthreads();
    const u32 jm = sh.jm;  // 0: none in this window
    u64 v = 0;
    if (jm && j == jm - 1) v = inc;
    else if (j < hi && (!jm || j >= jm)) v = a;
    u64 b1 = (v >> 62) & 1, n1 = (v >> 40) & 0x3FFFFFull, w1 = v & 0xFFFFFFFFFFull;
    front_block_sum(sh, b1, n1, w1);
    bad |= b1 ? 1ull : 0ull;
    nb += n1;
    nw += w1;
    if (jm) break;
    hi = lo;
  }
}

// S0 = side to move at the root; E = plies between ply 3 and the boards written
// (0: perft(6), boards = ply 3; 1: perft(7), boards = ply 4).  rng_out[0] = the
// boards' Range, rng_out[1] = the words' (k_count3c's rng / rng_ch).
// spill (kFrontSpillItems x kFrontWin words): an item of up to two windows
// puts the words past the first in its spill row during the one walk and
// copies them to their place after the look-back (a second walk of the item
// made the ~3 % of startpos perft(7) items past one window the last blocks).
template <int S0, int E>
__global__ __launch_bounds__(kFrontThreads) void k_front(const Board* __restrict__ root_p, u32 shard, u32 n_shards,
                                                         Board* __restrict__ out, uint16_t* __restrict__ out_tags,
                                                         u32 cap_b, u32* __restrict__ mw, u64 cap_w,
                                                         PerftResult* __restrict__ res, Range* __restrict__ rng_out,
                                                         FrontState* __restrict__ st, u32* __restrict__ spill) {
  constexpr int S1 = S0 ^ 1;       // side to move at ply 1 (and ply 3)
  constexpr int SF = E ? S0 : S1;  // side to move at the boards written
  constexpr u32 NT = kFrontThreads, NW = kFrontWaves;
  __shared__ FrontShared sh;
  const u32 t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const u32 grp = wave >> 2;                   // class group of the wave (waves 4g .. 4g + 3: one per SIMD)
  const u32 qlane = lane + 64 * (wave & 3);    // the thread's index within its group (0 .. 255)
  DC_FRONT_STAMP(0);
  if (blockIdx.x == 0) {
    static_assert(sizeof(PerftResult) % 8 == 0, "PerftResult is cleared in u64 words");
    for (u32 k = t; k < sizeof(PerftResult) / 8; k += NT) reinterpret_cast<u64*>(res)[k] = 0;
  }
  const Board root = root_p[0];
  u32 n1 = 0, n2 = 0, n3 = 0;
  // The top: plies 1 and 2 and the ply-3 offsets of the ply-2 nodes in LDS.
  // Returns false when it does not fit (block-uniform).  Block 0 records the
  // root moves (after the clear: barriers between).
  auto front_top = [&](bool record) -> bool {
    // ply 1: wave g < 4 counts and walks class group g of the root
    if (wave < 4 && lane == 0) sh.g1[wave] = front_group_count<S0>(wave, root);
    __syncthreads();
    n1 = sh.g1[0] + sh.g1[1] + sh.g1[2] + sh.g1[3];
    if (n1 > kFrontPly1Max) return false;
    if (wave < 4 && lane == 0) {
      u32 j = 0;
      for (u32 g = 0; g < wave; ++g) j += sh.g1[g];
      front_group_moves<S0>(wave, root, [&](int f, int to) { sh.m1[j++] = (uint16_t)(f | (to << 6)); });
    }
    __syncthreads();
    if (t < n1) {
      const u32 m = sh.m1[t];
      Board b = root;
      ref_make(b, (int)(m & 63), (int)(m >> 6));
      sh.top.p1[t] = b;
      if (record) res->root_moves[t] = (uint16_t)m;
    }
    __syncthreads();
    DC_FRONT_STAMP(1);
    // ply 2: group grp of node qlane
    if (qlane < kFrontPly1Max) sh.gc[grp][qlane] = qlane < n1 ? front_group_count<S1>(grp, sh.top.p1[qlane]) : 0u;
    __syncthreads();
    const u32 tot = t < kFrontPly1Max ? sh.gc[0][t] + sh.gc[1][t] + sh.gc[2][t] + sh.gc[3][t] : 0u;
    const u32 ex = block_excl_scan32<NW>(tot, sh.wsum, &n2);
    if (t < kFrontPly1Max) sh.noff[t] = ex;
    __syncthreads();
    DC_FRONT_STAMP(2);
    if (n2 > kFrontPly2Max) return false;
    if (qlane < n1) {
      u32 j = sh.noff[qlane];
      for (u32 g = 0; g < grp; ++g) j += sh.gc[g][qlane];
      front_group_moves<S1>(grp, sh.top.p1[qlane],
                            [&](int f, int to) { sh.top.w2[j++] = (qlane << 12) | (u32)f | ((u32)to << 6); });
    }
    __syncthreads();
    DC_FRONT_STAMP(3);
    // ply-3 counts of the ply-2 nodes, scanned in place into offsets
    for (u32 j = t; j < n2; j += NT) {
      const u32 e = sh.top.w2[j];
      Board b = sh.top.p1[e >> 12];
      ref_make(b, (int)(e & 63), (int)((e >> 6) & 63));
      sh.top.off3[j] = ref_count<S0>(b);
    }
    __syncthreads();
    DC_FRONT_STAMP(4);
    const u32 seg = (n2 + NT - 1) / NT, a = min(n2, t * seg), z = min(n2, a + seg);
    u32 s = 0;
    for (u32 j = a; j < z; ++j) s += sh.top.off3[j];
    u32 run = block_excl_scan32<NW>(s, sh.wsum, &n3);
    for (u32 j = a; j < z; ++j) {
      const u32 v = sh.top.off3[j];
      sh.top.off3[j] = run;
      run += v;
    }
    __syncthreads();
    DC_FRONT_STAMP(5);
    return true;
  };
  const bool ok = front_top(blockIdx.x == 0);
  if (blockIdx.x == 0 && t == 0) {
    res->n_root = n1;
    res->level_n[1] = n1;
    res->level_n[2] = n2;
    res->level_n[3] = n3;
  }
  // ---- this rank's ply-3 nodes (shard, shard + n_shards, ...): local index
  //      k in [0, m3), cut into chunks of kFrontChunk consecutive nodes; item
  //      i takes chunks i, i + n_items, i + 2 n_items, ... (one item per block
  //      while its chunks fit kFrontP3Max).  Contiguous items of 35 nodes held
  //      12k-32k words at perft(7), and the largest set the kernel's end.
  //      (E = 0: one chunk per item -- contiguous items: their few words
  //      vary little, and k_count3c's per-wave root tags stay uniform)
  const u32 m3 = ok && n3 > shard ? (n3 - shard + n_shards - 1) / n_shards : 0u;
  const u32 C = E ? kFrontChunk : min(kFrontP3Max, max(1u, (m3 + gridDim.x - 1) / gridDim.x));
  const u32 NC = (m3 + C - 1) / C;
  u32 n_items = min(gridDim.x, NC);
  n_items = max(n_items, (NC + kFrontP3Max / C - 1) / (kFrontP3Max / C));
  n_items = min(n_items, kFrontItemsMax);  // (more chunks than that per item: declined below)
  const u32 cpi = n_items ? (NC + n_items - 1) / n_items : 0u;  // chunks per item
  if (blockIdx.x == 0 && t == 0) st->n_items = n_items;  // (k_count3c clears that many slots)
  if (!ok || n_items == 0) {  // nothing to expand: block 0 publishes the result
    if (blockIdx.x == 0 && t == 0) {
      if (!ok) {
        res->overflow = 1;
        res->front_declined = 1;
      }
      rng_out[0] = Range{0, 0};
      rng_out[1] = Range{0, 0};
    }
    return;
  }
  for (u32 it = blockIdx.x; it < n_items; it += gridDim.x) {
    if (it != blockIdx.x) (void)front_top(false);  // the previous item's words overwrote it
    // the item's nodes: lane t -> chunk it + n_items (t / C), node t % C in
    // it; the valid lanes are a prefix (only chunk NC - 1 can be short)
    const u32 cj = it < NC ? (NC - 1 - it) / n_items + 1 : 0u;  // chunks of this item
    const u32 last_c = it + n_items * (cj - 1);
    const u32 np3 = cpi * C > kFrontP3Max ? 0u : (cj - 1) * C + min(C, m3 - last_c * C);
    const bool too_big = cpi * C > kFrontP3Max;  // block-uniform (flagged below)
    // -- select the item's ply-3 nodes: parent by binary search, the rank's
    //    class group by one group count per (node, group), the move by one walk
    if (t < np3) {
      const u32 k = (it + n_items * (t / C)) * C + t % C;
      const u32 q = shard + k * n_shards;
      u32 lo = 0, hi = n2;  // the last ply-2 node whose offset is <= q (it has q's move)
      while (hi - lo > 1) {
        const u32 mid = (lo + hi) >> 1;
        if (sh.top.off3[mid] <= q) lo = mid;
        else hi = mid;
      }
      const u32 e = sh.top.w2[lo];
      Board b2 = sh.top.p1[e >> 12];
      ref_make(b2, (int)(e & 63), (int)((e >> 6) & 63));
      sh.b2[t] = b2;
      sh.r3[t] = q - sh.top.off3[lo];
      sh.t3[t] = (uint16_t)(e >> 12);
    }
    __syncthreads();
    if (qlane < np3) sh.gc[grp][qlane] = front_group_count<S0>(grp, sh.b2[qlane]);
    __syncthreads();
    if (qlane < np3) {
      u32 r = sh.r3[qlane];
      for (u32 g = 0; g < grp; ++g) r -= sh.gc[g][qlane];  // (wraps when the move is in an earlier group)
      if (r < sh.gc[grp][qlane]) {
        int f = 0, to = 0;
        u32 k = 0;
        const Board b2 = sh.b2[qlane];
        front_group_moves<S0>(grp, b2, [&](int ff, int tt) {
          if (k == r) {
            f = ff;
            to = tt;
          }
          ++k;
        });
        Board b3 = b2;
        ref_make(b3, f, to);
        sh.b3[qlane] = b3;
      }
    }
    __syncthreads();
    if (it == blockIdx.x) DC_FRONT_STAMP(6);
    // -- the item's boards: E = 0 the ply-3 nodes, E = 1 their children
    u32 nbd = np3;
    bool bad = too_big;
    if constexpr (E == 1) {
      if (qlane < np3) sh.gc[grp][qlane] = front_group_count<S1>(grp, sh.b3[qlane]);
      __syncthreads();
      const u32 tot = t < np3 ? sh.gc[0][t] + sh.gc[1][t] + sh.gc[2][t] + sh.gc[3][t] : 0u;
      const u32 ex = block_excl_scan32<NW>(tot, sh.wsum, &nbd);
      if (t < kFrontP3Max) sh.noff[t] = ex;
      __syncthreads();
      bad = nbd > kFrontBoardsMax;  // block-uniform
      if (!bad && qlane < np3) {
        u32 j = sh.noff[qlane];
        for (u32 g = 0; g < grp; ++g) j += sh.gc[g][qlane];
        front_group_moves<S1>(grp, sh.b3[qlane],
                              [&](int f, int to) { sh.slot4[j++] = (qlane << 12) | (u32)f | ((u32)to << 6); });
      }
      __syncthreads();
      if (it == blockIdx.x) DC_FRONT_STAMP(7);
    }
    if (bad) nbd = 0;
    auto board_at = [&](u32 k) -> Board {
      if constexpr (E == 1) {
        const u32 e = sh.slot4[k];
        Board b = sh.b3[e >> 12];
        ref_make(b, (int)(e & 63), (int)((e >> 6) & 63));
        return b;
      } else {
        return sh.b3[k];
      }
    };
    // -- pass 1: word counts per (group, board)
    for (u32 k = qlane; k < nbd; k += 256) sh.gw[grp][k] = (uint16_t)front_group_count<SF>(grp, board_at(k));
    __syncthreads();
    const u32 seg = (nbd + NT - 1) / NT, a = min(nbd, t * seg), z = min(nbd, a + seg);
    auto wcount = [&](u32 k) -> u32 { return (u32)sh.gw[0][k] + sh.gw[1][k] + sh.gw[2][k] + sh.gw[3][k]; };
    u32 s = 0;
    for (u32 k = a; k < z; ++k) s += wcount(k);
    u32 nw;
    u32 run = block_excl_scan32<NW>(s, sh.wsum, &nw);
    for (u32 k = a; k < z; ++k) {
      sh.woff[k] = run;
      run += wcount(k);
    }
    // -- publish the item's counts, walk its words into the first LDS window
    //    (board index relative to the item, rebased when stored), then look
    //    back: a block waiting on a slower predecessor has its walk done
    if (t == 0)
      __hip_atomic_store(&st->agg[it], front_pack(bad, nbd, nw), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifdef DC_AB_KNOBS
    if (it == blockIdx.x) DC_FRONT_STAMP(12);
#endif
    __syncthreads();  // woff / wc
    // the words [wb, wb + kFrontWin) into slotw; the first walk also puts
    // [kFrontWin, 2 kFrontWin) into the item's spill row when it has one
    u32* srow = spill && it < kFrontSpillItems && nw <= 2 * kFrontWin ? spill + (size_t)it * kFrontWin : nullptr;
    auto walk = [&](u32 wb) {
      const u32 we = wb + (wb == 0 && srow ? 2 * kFrontWin : kFrontWin);
      for (u32 k = qlane; k < nbd; k += 256) {
        u32 j = sh.woff[k];
        for (u32 g = 0; g < grp; ++g) j += sh.gw[g][k];
        const u32 c = sh.gw[grp][k];
        if (c && j < we && j + c > wb)
          front_group_moves<SF>(grp, board_at(k), [&](int f, int to) {
            const u32 w = (k << 12) | (u32)f | ((u32)to << 6);
            if (j >= wb && j - wb < kFrontWin) sh.slotw[j - wb] = w;
            else if (j >= wb + kFrontWin && j < we) srow[j - wb - kFrontWin] = w;
            ++j;
          });
      }
      __syncthreads();
    };
    if (nw) walk(0);
#ifdef DC_AB_KNOBS
    if (it == blockIdx.x) DC_FRONT_STAMP(11);
#endif
    u64 pbad, pb, pw;
    front_lookback(sh, st, it, pbad, pb, pw);
    if (t == 0)
      __hip_atomic_store(&st->incl[it], front_pack(pbad | bad, pb + nbd, pw + nw), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    if (it == blockIdx.x) DC_FRONT_STAMP(8);
    const u64 base_b = pb, base_w = pw;
    const bool fits = !pbad && !bad && base_b + nbd <= cap_b;  // (else flagged below: no store)
    // -- the boards, then the words window by window
    if (fits)
      for (u32 k = t; k < nbd; k += NT) {
        store_board(out, base_b + k, board_at(k));
        out_tags[base_b + k] = E == 1 ? sh.t3[sh.slot4[k] >> 12] : sh.t3[k];
      }
#ifdef DC_AB_KNOBS
    if (it == blockIdx.x && t == 0 && blockIdx.x < kFrontTraceBlocks) {
      g_front_trace[blockIdx.x * kFrontTraceWords + 13] = nw;
      g_front_trace[blockIdx.x * kFrontTraceWords + 14] = nbd;
    }
    if (it == blockIdx.x) DC_FRONT_STAMP(10);
#endif
    const u32 rebase = (u32)base_b << 12;
    for (u32 wb = 0; fits && wb < nw; wb += kFrontWin) {  // block-uniform
      const u32 ns = min(kFrontWin, nw - wb);
      if (wb && srow) {  // the spilled second window (written by this block's walk)
        for (u32 r = t; r < ns; r += NT) {
          const u64 o = base_w + wb + r;
          if (o < cap_w) mw[o] = srow[r] + rebase;
        }
        continue;
      }
      if (wb) {
        __syncthreads();  // the previous window is stored
        walk(wb);
      }
      for (u32 r = t; r < ns; r += NT) {
        const u64 o = base_w + wb + r;
        if (o < cap_w) mw[o] = sh.slotw[r] + rebase;
      }
    }
    if (it == blockIdx.x) DC_FRONT_STAMP(9);
    // -- the last item publishes the Ranges
    if (it == n_items - 1 && t == 0) {
      const u64 tb = base_b + nbd, tw = base_w + nw;
      if (pbad || bad || tb > cap_b || tw > cap_w) {
        res->overflow = 1;
        res->front_declined = 1;
        rng_out[0] = Range{0, 0};
        rng_out[1] = Range{0, 0};
      } else {
        rng_out[0] = Range{0, tb};
        rng_out[1] = Range{0, tw};
      }
    }
    __syncthreads();  // the item's LDS (and the windows over the top) is reused by the next item
  }
}

// Children of the final level as 8-byte descriptors {parent index, move}.
template <class R, int STM>
__global__ __launch_bounds__(256) void k_emit_desc(const Board* __restrict__ nodes, const uint16_t* __restrict__ meta,
                                                   const Range* __restrict__ rng, const u32* __restrict__ counts,
                                                   const u64* __restrict__ chunk_base, u64* __restrict__ desc, u64 cap,
                                                   const PerftResult* __restrict__ res) {
  __shared__ u64 wsum[4];
  if (res->path != 0) return;  // count2 was selected
  const u64 lo = rng->lo, hi = rng->hi;
  const u64 nch = (hi - lo + kChunk - 1) / kChunk;
  for (u64 c = blockIdx.x; c < nch; c += gridDim.x) {
    const u64 i = lo + c * kChunk + threadIdx.x;
    const bool valid = i < hi;
    const u32 cnt = valid ? counts[i - lo] : 0;
    u64 tot;
    u64 o = block_excl_scan64<4>(cnt, wsum, &tot) + chunk_base[c];
    if (!valid) continue;
    const Board p = load_board(nodes, i);
    const u32 pm = load_meta<R>(meta, i);
    R::template for_each<STM>(p, pm, [&](int f, int t, int promo) {
      if (o < cap) desc[o] = i | ((u64)((u32)f | ((u32)t << 6) | ((u32)promo << 12)) << 32);
      ++o;
    });
  }
}

// One slice [s0, s0 + len) of the grandparent level `lvl` (lo = 0) for the
// sliced fused final stage: out[0] = its nodes {0, n}, out[1] = its children's
// move words {0, w} (from the level's chunk offsets; words_total = the level's
// child Range), the slice's group counter zeroed.  A slice past `cap` words is
// flagged (overflow: exact rerun) and emptied.
__global__ void k_wide_slice(const Range* __restrict__ lvl, const u64* __restrict__ chunk_base,
                             const Range* __restrict__ words_total, u64 s0, u64 len, Range* __restrict__ out,
                             u32* __restrict__ counter, PerftResult* __restrict__ res, u64 cap) {
  const u64 n = lvl->hi - lvl->lo;
  const u64 gn = s0 < n ? min(len, n - s0) : 0ull;
  u64 w = 0;
  if (gn) {
    const u64 wbeg = chunk_base[s0 / kChunk];
    const u64 wend = s0 + gn >= n ? words_total->hi - words_total->lo : chunk_base[(s0 + gn) / kChunk];
    w = wend - wbeg;
  }
  if (w > cap) {
    res->overflow = 1;
    w = 0;
  }
  out[0] = Range{0, w ? gn : 0ull};
  out[1] = Range{0, w};
  *counter = 0;
}

__global__ void k_slice(Range* rng, u32 shard, u32 n_shards) {
  const u64 lo = rng->lo, n = rng->hi - rng->lo;
  *rng = Range{lo + n * shard / n_shards, lo + n * (shard + 1) / n_shards};
}

// Strided shard of a level: nodes lo + shard, lo + shard + n_shards, ... are
// gathered to the front of `out` and the level's Range becomes [0, count).
// Subtree sizes vary along the frontier (a contiguous eighth of ply 3 held
// 1.5x the leaves of another); every n-th node evens them out.  One block:
// all threads read the Range before thread 0 rewrites it.
__global__ __launch_bounds__(1024) void k_gather_shard(const Board* __restrict__ in, const uint16_t* __restrict__ in_meta,
                                                       const uint16_t* __restrict__ in_tags, Range* rng, u32 shard,
                                                       u32 n_shards, Board* __restrict__ out,
                                                       uint16_t* __restrict__ out_meta, uint16_t* __restrict__ out_tags) {
  const u64 lo = rng->lo, hi = rng->hi;
  const u64 n = hi > lo + shard ? (hi - lo - shard + n_shards - 1) / n_shards : 0;
  for (u64 k = threadIdx.x; k < n; k += blockDim.x) {
    const u64 i = lo + shard + k * n_shards;
    store_board(out, k, load_board(in, i));
    if (in_meta) out_meta[k] = in_meta[i];
    out_tags[k] = in_tags[i];
  }
  __syncthreads();
  if (threadIdx.x == 0) *rng = Range{0, n};
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

#ifdef DC_AB_KNOBS  // round-1 final stage, kept for A/B measurement only
template <class R, int STM>
__global__ __launch_bounds__(256, 4) void k_count2(const Board* __restrict__ nodes, const uint16_t* __restrict__ meta,
                                                const uint16_t* __restrict__ tags, const Range* __restrict__ rng,
                                                u64* __restrict__ divide, const PerftResult* __restrict__ res) {
  if (res && res->path == 0) return;  // the descriptor path was selected
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
#endif  // DC_AB_KNOBS

// ---------------------------------------------------- k_count2b (final stage)
// The last two plies, one block = 256 parents (one per lane).  Their children
// (from, to, promo, parent) are compacted into LDS at block-scan offsets, then
// all 256 lanes take one child per round: make it, bulk-count its moves.  The
// work unit is a 256-parent chunk, so even a ~200k-node final level (perft 6)
// spreads evenly over the GPU, and no child ever round-trips through HBM.
// FIDE (kSplit): the parents' simple children (fide_sens, dc_fide_rules.h)
// are never made: each adds c0, the opponent's count in the parent; only the
// others take slots, whose area shrinks to make room for the per-parent
// sensitivity sets (three blocks per CU either way).
template <bool SPLIT>
struct C2bCfg {
  static constexpr u32 kCap = SPLIT ? 256 * 22 : 256 * 28;  // child slots per window
};

// The per-parent sensitivity sets exist in the split instantiation only (the
// REF-shaped one carries no 2 KB of dead LDS).
template <bool SPLIT>
struct C2bSens {
  u64 sens[SN_COUNT][256];  // sens_masks, [set][parent]
};
template <>
struct C2bSens<false> {};

template <bool SPLIT>
struct C2bShared : C2bSens<SPLIT> {
  Board par[256];
  u32 pmeta[256];
  u32 slot[C2bCfg<SPLIT>::kCap];
  u64 hist[256];
  u64 wsum[4];
  uint16_t ptag[256];
  u32 next;  // the chunk this block takes next (dynamic scheduling)
};
static_assert(sizeof(C2bShared<false>) + sizeof(u64) * SN_COUNT * 256 == sizeof(C2bShared<true>) +
                  sizeof(u32) * (C2bCfg<false>::kCap - C2bCfg<true>::kCap),
              "only the split instantiation carries the sensitivity sets");

// DC_DIAG_CHILD (diagnostic builds only, never the product):
// every child k_count2b counts is written as one 64-byte record at a position
// fixed by (block, chunk, slot) -- no atomics, so the kernel's timing changes
// only by the stores -- for tools/fide_child_diag.py to recount on the host.
// DC_DIAG_CHILD == 2 also counts each child a second time (same code, an
// opaque copy of the board in between) and records both counts; == 3 writes
// the count alone (one dword per child at the same position).
#ifdef DC_DIAG_CHILD
struct DiagRec {
  u64 b[4];
  u32 cm, k, k2, e;  // e: the slot word | STM << 31
  u32 pidx, hwid, xcc, misc;  // misc: active lanes | lane << 8 | wave << 16 | (window > 0) << 24
};
static_assert(sizeof(DiagRec) == 64, "diag record");
__device__ DiagRec* g_diag_rec;
__device__ u64 g_diag_cap;
extern "C" __attribute__((visibility("default"))) int dc_diag_child_set(void* dev_recs, u64 cap) {
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_diag_rec), &dev_recs, sizeof(dev_recs)) != hipSuccess) return -1;
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_diag_cap), &cap, sizeof(cap)) != hipSuccess) return -1;
  return 0;
}
#endif

// DC_C2B_DYN (round 5): blocks take 256-parent chunks from a counter (the run's
// PerftResult.next_chunk, zeroed by k_expand_top) instead of an equal static
// share: a parent's cost varies several-fold, and with a handful of chunks per
// block (the FIDE suite's one batched final stage: 938 chunks over 768 blocks)
// the static split left most CUs idle behind the slowest blocks.
#ifndef DC_C2B_DYN
#define DC_C2B_DYN 1
#endif
#ifndef DC_C2B_EVEN
#define DC_C2B_EVEN 0
#endif
#ifndef DC_C2B_GUIDED
#define DC_C2B_GUIDED 0
#endif
template <class R, int STM>
__global__ __launch_bounds__(256, R::kFinalMinBlocks) void k_count2b(const Board* __restrict__ nodes, const uint16_t* __restrict__ meta,
                                                    const uint16_t* __restrict__ tags, const Range* __restrict__ rng,
                                                    u64* __restrict__ divide, u32* __restrict__ next_chunk) {
  constexpr bool SPLIT = R::kSplit;
  constexpr u32 kC2bCap = C2bCfg<SPLIT>::kCap;
  __shared__ C2bShared<SPLIT> sh;
  tag_hist_init(sh.hist);
  const u32 tid = threadIdx.x;
  const u32 wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // Equal contiguous share of the level per resident block (the grid is one
  // resident wave of blocks, so every CU carries the same number of parents).
  const u64 lo = rng->lo, hi = rng->hi;
#if DC_C2B_DYN && !defined(DC_DIAG_CHILD)
  // chunks of min(256, the block's equal share): a level of < 256 parents a
  // block (the suite's single positions) one chunk per block, as the static
  // split had it.  Each block's first chunk is its own index (no atomic round
  // trip at the start: that alone cost the single suite positions 4-9 %); the
  // counter hands out the rest from gridDim.x on.  (Chunks of a quarter share
  // for mid-size levels measured slower on the suite batch: 0.426 vs 0.418 ms,
  // profiles/r05/ab_z2.jsonl.)
  const u64 share = max<u64>(1, (hi - lo + gridDim.x - 1) / gridDim.x);
#if DC_C2B_EVEN
  // DC_C2B_EVEN (round 6 A/B): a level of r < share / 256 <= r + 1 rounds of
  // full chunks (the suite batch: 1.22 rounds, 938 chunks over 768 blocks)
  // in ceil(share / 256) rounds of equal chunks instead.  Measured slower
  // (profiles/r06/ab_c2b_even.txt): the suite's final stage 0.355 -> 0.366 ms.
  const u64 cs = (share + (share + kChunk - 1) / kChunk - 1) / ((share + kChunk - 1) / kChunk);
#else
  const u64 cs = min<u64>(kChunk, share);
#endif
#if DC_C2B_GUIDED
  // DC_C2B_GUIDED (round 6): a level of more than one round of chunks ends in
  // 64-parent chunks (its last 2 x grid x 64 parents).  A chunk's parent phase
  // runs one thread per parent, and a wave none of whose threads holds a
  // parent skips it, so a 64-parent chunk costs one wave's parent phase, not
  // four; the small chunks let the blocks that finish early take the tail.
  // Measured slower (profiles/r06/ab_c2b_guided.txt, same box, alternating):
  // the suite step 0.329-0.333 -> 0.345-0.347 ms.  Off (A/B knob).
  constexpr u64 kTail = 64;
  const u64 nlev = hi - lo;
  const u64 tail = share > kChunk ? min<u64>(nlev, 2ull * gridDim.x * kTail) : 0ull;
  const u64 nbig = (nlev - tail) / cs, tstart = nbig * cs;
  const u64 nch = nbig + (nlev - tstart + kTail - 1) / kTail * (tail ? 1 : 0) + (tail ? 0 : (nlev - tstart + cs - 1) / cs);
  for (u64 c = blockIdx.x; c < nch;) {  // block-uniform
    const bool big = c < nbig || !tail;
    const u64 s = lo + (big ? c * cs : tstart + (c - nbig) * kTail);
    const u64 bhi = min(hi, s + (big ? cs : kTail));
#else
  const u64 nch = (hi - lo + cs - 1) / cs;
  for (u64 c = blockIdx.x; c < nch;) {  // block-uniform
    const u64 s = lo + c * cs;
    const u64 bhi = min(hi, s + cs);
#endif
#else
  (void)next_chunk;
  const u64 per = (hi - lo + gridDim.x - 1) / gridDim.x;  // (DC_C2B_DYN=0, and the diagnostic builds)
  const u64 blo = min(hi, lo + (u64)blockIdx.x * per), bhi = min(hi, blo + per);
#ifdef DC_DIAG_CHILD
  u64 diag_off = (u64)blockIdx.x * per * 218;  // 218: the most legal moves of any position
#endif
  for (u64 s = blo; s < bhi; s += kChunk) {
#endif
    const u64 i = s + tid;
    const bool valid = i < bhi;
    Board p{0, 0, 0, 0};
    u32 pm = 0, tag = 0;
    if (valid) {
      p = load_board(nodes, i);
      pm = load_meta<R>(meta, i);
      tag = tags[i];
    }
    u32 cnt = 0;
    u64 simple_leaves = 0;  // simple children x c0 (SPLIT)
    // the lane's sensitivity sets, read from LDS where the enumeration uses
    // them (the thread index rebuilt at each use, otid: no address kept live)
    auto sens_at = [&](int k) -> u64 {
      if constexpr (SPLIT) return sh.sens[k][otid(wave)];  // (the sets exist in the split only)
      else return 0ull;
    };
    if constexpr (SPLIT) {
      if (valid) {
        u64 m[SN_COUNT];
        sens_masks(fide_sens<STM>(p, pm), m);
#pragma unroll
        for (int k = 0; k < SN_COUNT; ++k) sh.sens[k][tid] = m[k];
#if DC_FIDE_SPLIT == 2
        u32 ns;
        cnt = fide_count_split<STM>(p, pm, sens_at, ns);
#else
        const u32 ns = fide_for_each_split<STM>(p, pm, sens_at, [&](int, int, int) { ++cnt; });
#endif
        if (ns) simple_leaves = (u64)ns * fide_count<1 - STM>(p, pm & 15u);  // THEM to move, no en passant
      }
    } else {
      cnt = valid ? R::template count<STM>(p, pm) : 0;
    }
    u64 total64;
    const u32 excl = (u32)block_excl_scan64<4>(cnt, sh.wsum, &total64);
    const u32 total = (u32)total64;
    sh.par[tid] = p;
    if constexpr (R::kMeta) sh.pmeta[tid] = pm;
    sh.ptag[tid] = (uint16_t)tag;
    __syncthreads();
    const u32 tag0 = sh.ptag[0];
    u64 acc = 0;  // grandchildren under parents whose tag == tag0 (the norm: nodes stay ordered by root)
    if constexpr (SPLIT) {
      if (tag == tag0) acc = simple_leaves;
      else if (simple_leaves) atomicAdd((unsigned long long*)&sh.hist[tag], (unsigned long long)simple_leaves);
    }
    for (u32 base = 0; base < total; base += kC2bCap) {
      if (base) __syncthreads();  // previous window fully read
      u32 j = excl;
      if (valid && j < base + kC2bCap && j + cnt > base) {
        // the parent read back from LDS: p and pm are not live across the
        // child loop (FIDE fits 4 blocks/CU only with every such VGPR freed)
        const Board pp = sh.par[tid];
        const u32 ppm = R::kMeta ? sh.pmeta[tid] : 0u;
        j -= base;  // slot index in this window (wraps below 0 for earlier windows)
        auto put = [&](int f, int t, int promo) {
          if (j < kC2bCap) sh.slot[j] = (u32)f | ((u32)t << 6) | ((u32)promo << 12) | ((SPLIT ? otid(wave) : tid) << 15);
          ++j;
        };
        if constexpr (SPLIT) {
          (void)fide_for_each_split<STM>(pp, ppm, sens_at, put);
        } else {
          R::template for_each<STM>(pp, ppm, put);
        }
      }
      __syncthreads();
      const u32 nslots = min(kC2bCap, total - base);
      for (u32 r0 = 0; r0 < nslots; r0 += 256) {
        const u32 r = r0 + tid;
        if (r < nslots) {
          const u32 e = sh.slot[r];
          const u32 pl = e >> 15;
          Board ch = sh.par[pl];
          const u32 cm = R::template make<STM>(ch, R::kMeta ? sh.pmeta[pl] : 0u, (int)(e & 63), (int)((e >> 6) & 63),
                                               (int)((e >> 12) & 7));
          const u32 k = R::template count_final<1 - STM>(ch, cm);
          const u32 ptag = sh.ptag[pl];
          if (ptag == tag0) acc += k;
          else if (k) atomicAdd((unsigned long long*)&sh.hist[ptag], (unsigned long long)k);
#ifdef DC_DIAG_CHILD
          {
            DiagRec* rec = g_diag_rec;
            const u64 at = diag_off + base + r;
#if DC_DIAG_CHILD == 3
            // the count alone, one dword at the record's position (the least
            // perturbing form; the children are identified by a full-record run)
            if (rec && at < g_diag_cap) reinterpret_cast<u32*>(rec)[at] = k;
            if (false) {
#else
            if (rec && at < g_diag_cap) {
#endif
              u32 k2 = k;
#if DC_DIAG_CHILD == 2
              Board c2 = ch;
              u32 cm2 = cm;
              asm volatile("" : "+v"(c2.b0), "+v"(c2.b1), "+v"(c2.b2), "+v"(c2.b3), "+v"(cm2));
              k2 = R::template count_final<1 - STM>(c2, cm2);
#endif
              u32 hwid, xcc;
              asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
              asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
              const u64 ex = __builtin_amdgcn_read_exec();
              DiagRec d;
              d.b[0] = ch.b0;
              d.b[1] = ch.b1;
              d.b[2] = ch.b2;
              d.b[3] = ch.b3;
              d.cm = cm;
              d.k = k;
              d.k2 = k2;
              d.e = (e & 0x7FFFFFFFu) | ((u32)STM << 31);
              d.pidx = (u32)(s + pl);
              d.hwid = hwid;
              d.xcc = xcc;
              d.misc = (u32)__popcll(ex) | ((tid & 63) << 8) | ((tid >> 6) << 16) | ((base ? 1u : 0u) << 24);
              rec[at] = d;
            }
          }
#endif
        }
      }
    }
#ifdef DC_DIAG_CHILD
    diag_off += total;
#endif
    tag_hist_add(sh.hist, tag0, acc, true);
    __syncthreads();  // par/ptag/slot reused by the next chunk
#if DC_C2B_DYN && !defined(DC_DIAG_CHILD)
    if (tid == 0) sh.next = gridDim.x + atomicAdd(next_chunk, 1u);
    __syncthreads();
    c = sh.next;
#endif
  }
  tag_hist_flush(sh.hist, divide);
}

// ---------------------------------------------------- k_count2c (REF final stage)
// The last two plies under RULES_REF with the quiet-move shortcut of
// ref_count_nonpawn: per parent P (side S to move, opponent O) the block first
// computes base = O's knight/king/slider moves in P and att = O's slider rays.
// A child reached by a quiet move f -> t with f, t outside att then has
//     count_O(child) = base + O's pawn moves in the child      (~40 VALU ops)
// and every other child (captures, moves touching a ray) is recounted in full.
// Those are compacted per wave into an LDS queue and recounted 64 at a time,
// so the full count never runs with idle lanes.  At plies 6-7 of startpos
// about 88 % of the children take the short path.
constexpr int kC2cQueue = 128;

#ifndef DC_C2C_SOA
#define DC_C2C_SOA 0
#endif
#ifndef DC_C2C_PAIR
#define DC_C2C_PAIR 1
#endif
#ifndef DC_C3C_STATIC
#define DC_C3C_STATIC 0
#endif
// Parents' boards: array of structs (two ds_read_b128 per fetch, shipped);
// DC_C2C_SOA=1 (A/B experiments only) keeps each bitboard in its own array.
struct C2cParents {
#if DC_C2C_SOA
  u64 b[4][256];
  __device__ __forceinline__ Board get(u32 i) const { return Board{b[0][i], b[1][i], b[2][i], b[3][i]}; }
  __device__ __forceinline__ void set(u32 i, const Board& p) {
    b[0][i] = p.b0;
    b[1][i] = p.b1;
    b[2][i] = p.b2;
    b[3][i] = p.b3;
  }
#else
  Board p[256];
  __device__ __forceinline__ Board get(u32 i) const { return p[i]; }
  __device__ __forceinline__ void set(u32 i, const Board& x) { p[i] = x; }
#endif
};

#ifndef DC_C2C_REC
#define DC_C2C_REC 1
#endif
// DC_C2C_REC = 1 (shipped since round 3): each parent's board, rays, base
// count and tag in one 48-byte record -- one per-thread LDS address instead of
// four differently scaled ones, and one record read per candidate child
// (perft(7) final stage 0.482 -> 0.477 ms, same-box).  0: the round-2 arrays.
// DC_C2C_DIAGQ = 1 (shipped since round 3, needs the records): full-recount
// children whose move leaves the opponent's orthogonal group unchanged (about
// 83 % of them at perft(7): profiles/r03/c2c_stats_d7.txt) go to a second
// per-wave queue and are counted group-wise (ref_count_child_diag: the
// diagonal group and the pawns recomputed, the leapers corrected at t);
// the rest keep the full recount.
#ifndef DC_C2C_DIAGQ
#define DC_C2C_DIAGQ DC_C2C_REC
#endif
#if DC_C2C_DIAGQ && !DC_C2C_REC
#error "DC_C2C_DIAGQ needs DC_C2C_REC"
#endif
// DC_C2C_REUSE = 1: the parent split keeps the side to move's eight slider
// target sets (its own fills) for the first window's enumeration of the
// special moves, which otherwise runs the same eight fills again.
#ifndef DC_C2C_REUSE
#define DC_C2C_REUSE 1
#endif
#if DC_C2C_DIAGQ
struct alignas(8) C2cRec {
  u64 b0, b1, b2, b3, att, orth;
  u32 base;
  uint16_t tag, diag;
};
#else
struct alignas(16) C2cRec {
  u64 b0, b1, b2, b3, att;
  u32 base;
  uint16_t tag, pad;
};
#endif
// Special-child slots per group of 256 parents: 24 per parent, trimmed with
// the 48-byte records so that four blocks' LDS (<= 40,960 B each) fit a CU;
// 19.9 with the 56-byte records and the second queue (the mean at perft(7) is
// 7.6: 0.306 of 24.7 children).
// DC_C2C_QQ (round 5, with the group-wise queue): the quiet special children
// (after the target-side pawn correction: 1.7 % of perft(7)'s children, 11 %
// of the enumerated ones) go to a third per-wave queue and get their pawn
// recount 64 at a time, instead of the whole wave running it in nearly every
// consume round; their 512 queue slots come out of the slot area (19.9 -> 17.9
// per parent; 3.9 special children per parent on average since the correction).
#ifndef DC_C2C_QQ
#define DC_C2C_QQ DC_C2C_DIAGQ
#endif
constexpr u32 kC2cCap = DC_C2C_REC ? (DC_C2C_DIAGQ ? (DC_C2C_QQ ? 5104 - 4 * kC2cQueue : 5104) : 6128) : 256 * 24;

template <u32 CAP>
struct C2cShared {
#if DC_C2C_REC
  C2cRec rec[256];
#else
  C2cParents par;
  u64 att[256];
  u32 base[256];
#endif
  u32 slot[CAP];
  u32 queue[4][kC2cQueue];
#if DC_C2C_DIAGQ
  u32 queue_d[4][kC2cQueue];
#endif
#if DC_C2C_QQ
  u32 queue_q[4][kC2cQueue];
#endif
  u64 hist[256];
  u64 wsum[6];  // scans; the pooled final drains' per-wave leftovers (12 u32)
  u32 next;
#if !DC_C2C_REC
  uint16_t ptag[256];
#endif
  __device__ __forceinline__ void put(u32 i, const Board& p, u64 a, u32 bs, u32 tg, u64 orth = 0, u32 diag = 0) {
#if DC_C2C_DIAGQ
    (void)tg;  // written by put_tag before the parent split (fewer live VGPRs there)
    C2cRec& r = rec[i];
    r.b0 = p.b0;
    r.b1 = p.b1;
    r.b2 = p.b2;
    r.b3 = p.b3;
    r.att = a;
    r.orth = orth;
    r.base = bs;
    r.diag = (uint16_t)diag;
#elif DC_C2C_REC
    (void)orth;
    (void)diag;
    rec[i] = C2cRec{p.b0, p.b1, p.b2, p.b3, a, bs, (uint16_t)tg, 0};
#else
    par.set(i, p);
    att[i] = a;
    base[i] = bs;
    ptag[i] = (uint16_t)tg;
#endif
  }
  __device__ __forceinline__ void put_tag(u32 i, u32 tg) {
#if DC_C2C_DIAGQ
    rec[i].tag = (uint16_t)tg;
#else
    (void)i;
    (void)tg;
#endif
  }
#if DC_C2C_REC
  __device__ __forceinline__ Board board(u32 i) const { return Board{rec[i].b0, rec[i].b1, rec[i].b2, rec[i].b3}; }
  __device__ __forceinline__ u64 rays(u32 i) const { return rec[i].att; }
  __device__ __forceinline__ u32 basec(u32 i) const { return rec[i].base; }
  __device__ __forceinline__ u32 tag(u32 i) const { return rec[i].tag; }
#if DC_C2C_DIAGQ
  __device__ __forceinline__ u64 orth(u32 i) const { return rec[i].orth; }
  __device__ __forceinline__ u32 diagc(u32 i) const { return rec[i].diag; }
#endif
#else
  __device__ __forceinline__ Board board(u32 i) const { return par.get(i); }
  __device__ __forceinline__ u64 rays(u32 i) const { return att[i]; }
  __device__ __forceinline__ u32 basec(u32 i) const { return base[i]; }
  __device__ __forceinline__ u32 tag(u32 i) const { return ptag[i]; }
#endif
};

template <int STM, u32 CAP>
__device__ __forceinline__ u32 c2c_full(const C2cShared<CAP>& sh, u32 e) {
  const u32 pl = e >> 15;
  Board ch = sh.board(pl);
  ref_make(ch, (int)(e & 63), (int)((e >> 6) & 63));
  return ref_count<1 - STM>(ch);
}

#if DC_C2C_DIAGQ
template <int STM, u32 CAP>
__device__ __forceinline__ u32 c2c_diag(const C2cShared<CAP>& sh, u32 e) {
  const u32 pl = e >> 15;
  return ref_count_child_diag<1 - STM>(sh.board(pl), (int)(e & 63), (int)((e >> 6) & 63), sh.basec(pl) - sh.diagc(pl));
}
#endif

// BULK: children reached by "simple" moves -- quiet, f and t off the
// opponent's slider rays and off its pawn-sensitive squares G
// (ref_pawn_sensitive) -- all have count_O = base + pawn_O(parent), so they are
// counted per parent as n_simple x (base + pawn_O) and never enumerated; only
// the other ("special") children go through the LDS slots.
// PHASE (timing experiments only; wrong counts unless 0): 1 skips the children,
// 2 also skips the enumeration, leaving the per-parent counts; 5 skips the
// full recounts (queued children still drained), 6 also the quiet children's
// pawn counts; 7 replaces the counts by statistics (tools/c2c_stats.py);
// 8 is 0 plus a per-block timeline (tools/c2c_trace.py).  Phases other
// than 0 are instantiated only in the A/B build (-DDC_AB_KNOBS, libdchess_ab.so).
#ifndef DC_C2C_POOL
#define DC_C2C_POOL 1  // pooled final queue drains (0: one partial drain per wave, A/B)
#endif
// One group of 256 parents (one per thread; `valid` false for an empty slot):
// the last two plies below each, added into the block's divide histogram.
// Called by k_count2c (parents read from a level in HBM) and k_perft_dfs
// (parents produced by each lane's DFS stack).  Block-uniform call; ends with
// a block barrier (par/att/ptag/slot are reused by the next group).
template <int STM, u32 CAP, int PHASE = 0, bool BULK = true>
__device__ __forceinline__ void c2c_group(C2cShared<CAP>& sh, bool valid, const Board& p, u32 tag,
                                          u64* __restrict__ divide, u32 wave) {
  // wave: this wave's index in the block (an SGPR, readfirstlane at kernel
  // entry); the thread index is rebuilt where it is used (otid)
  const u32 w = wave, lane = lane_id();
  // GQ: the group-wise recount queue (DC_C2C_DIAGQ) in the bulk split
  constexpr bool GQ = DC_C2C_DIAGQ && BULK;
  u32* q = sh.queue[w];
#if DC_C2C_DIAGQ
  static_assert(offsetof(C2cShared<CAP>, queue_d) == offsetof(C2cShared<CAP>, queue) + sizeof(sh.queue),
                "queue_d must follow queue");
  u32* qd = sh.queue_d[w];
#else
  u32* qd = q;
#endif
  // QQ: the quiet special children's queue (their pawn recount, 64 at a time)
  constexpr bool QQ = DC_C2C_QQ && GQ;
#if DC_C2C_QQ
  u32* qq = sh.queue_q[w];
#else
  u32* qq = q;
#endif
  u32 qnq = 0;
  u32 cnt = 0, base = 0, diag = 0;
  u64 att = 0, orth = 0, Fs = 0, Ts = 0, simple_leaves = 0;
  u32 nsim = 0;
  constexpr bool REUSE = GQ && DC_C2C_REUSE;
  u64 tgt[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // (REUSE) slider target sets, compile-time indexed
  sh.put_tag(otid(w), tag);  // (the previous group ended with a barrier)
  if (valid) {
    if constexpr (BULK) {
      ParentSplit ps;
      ref_parent_split<STM, GQ, REUSE>(p, ps, tgt);
      base = ps.base;
      att = ps.att;
      if constexpr (GQ) {
        orth = ps.orth;
        diag = ps.diag;
      }
      Fs = ps.Fs;
      Ts = ps.Ts;
      cnt = ps.n_total - ps.n_simple;  // enumerated (special) children only
      simple_leaves = (u32)(ps.n_simple * (ps.base + ps.pawn_o) + ps.gcorr);  // (>= 0: a sum of child counts)
      nsim = ps.n_simple;
    } else {
      cnt = ref_count<STM>(p);
      base = ref_count_nonpawn<1 - STM>(p, att);
    }
  }
  u32 total;  // (at most 256 parents x 218 moves)
  const u32 excl = block_excl_scan32<4>(cnt, reinterpret_cast<u32*>(sh.wsum), &total, w);
  sh.put(otid(w), p, att, base, tag, orth, diag);
  __syncthreads();
  const u32 tag0 = sh.tag(0);
  u64 acc = 0;  // grandchildren under parents whose tag == tag0
  // k leaves under the root move `ptag` (read with the record, so no LDS
  // round trip of its own)
  auto add_tag = [&](u32 ptag, u32 k, bool live) {
    if constexpr (PHASE == 7) return;
    if (!live) return;
    if (ptag == tag0) acc += k;
    else if (k) atomicAdd((unsigned long long*)&sh.hist[ptag], (unsigned long long)k);
  };
  auto add = [&](u32 pl, u32 k, bool live) { add_tag(sh.tag(pl), k, live); };
  u32 qn = 0, qnd = 0;  // queue lengths: wave-uniform (kept scalar via readfirstlane)
  // One candidate child: its parent's LDS record is loaded first (so two
  // candidates' loads can be in flight together), then the short path if the
  // move is quiet, else the child is appended to a queue: the group-wise one
  // (GQ) if the move is off the opponent's orthogonal group, else the full one.
  struct Cand {
    u32 e, base, tag;
    Board pb;
    u64 a, o;
  };
  auto fetch = [&](u32 e) {
    const u32 pl = e >> 15;
#if DC_C2C_DIAGQ
    // the whole 56-byte record: board, rays, orthogonal group, base/tag/diag
    return Cand{e, sh.basec(pl), sh.tag(pl), sh.board(pl), sh.rays(pl), GQ ? sh.orth(pl) : 0ull};
#else
    return Cand{e, sh.basec(pl), sh.tag(pl), sh.board(pl), sh.rays(pl), 0ull};
#endif
  };
  auto consume = [&](const Cand& c, bool live) {
    const int f = (int)(c.e & 63), t = (int)((c.e >> 6) & 63);
    const u64 occ = occupied(c.pb);
    const bool quiet = ((((occ | c.a) >> t) | (c.a >> f)) & 1) == 0;
    if constexpr (QQ) {
      const u64 qmask = ballot(live && quiet);
      if (live && quiet) qq[qnq + mask_rank(qmask)] = c.e;
      qnq = __builtin_amdgcn_readfirstlane(qnq + (u32)__popcll(qmask));
    } else {
      if (live && quiet) add_tag(c.tag, c.base + (PHASE == 6 ? (u32)t : ref_pawn_count_child<1 - STM>(c.pb, f, t)), true);
    }
    const bool full = live && !quiet;
    const u64 em = ballot(full);
    if constexpr (PHASE == 7) {  // statistics: divide[0] quiet special children, [1] full-recount children
      const u64 qm = ballot(live && quiet);
      if (lane == 0) {
        atomicAdd((unsigned long long*)divide, (unsigned long long)__popcll(qm));
        atomicAdd((unsigned long long*)(divide + 1), (unsigned long long)__popcll(em));
      }
      // full children by the opponent O's slider group whose rays the move
      // changes: [4] captures, [5] orthogonal only, [6] diagonal only, [7] both, [8] neither
      const Sides so = sides<1 - STM>(c.pb);
      const u64 e = so.empty;
      const u64 ao = ray_attacks<8, kAll>(so.O, e) | ray_attacks<-8, kAll>(so.O, e) | ray_attacks<1, kNotA>(so.O, e) |
                     ray_attacks<-1, kNotH>(so.O, e);
      const u64 ad = ray_attacks<9, kNotA>(so.D, e) | ray_attacks<-9, kNotH>(so.D, e) | ray_attacks<7, kNotH>(so.D, e) |
                     ray_attacks<-7, kNotA>(so.D, e);
      const u64 ft = (1ull << f) | (1ull << t);
      const bool capt = (occ >> t) & 1;
      const bool go = (ao & ft) || ((so.O >> t) & 1), gd = (ad & ft) || ((so.D >> t) & 1);
      const u64 m4 = ballot(full && capt), m5 = ballot(full && go && !gd), m6 = ballot(full && gd && !go);
      const u64 m7 = ballot(full && go && gd), m8 = ballot(full && !go && !gd);
      if (lane == 0) {
        atomicAdd((unsigned long long*)(divide + 4), (unsigned long long)__popcll(m4));
        atomicAdd((unsigned long long*)(divide + 5), (unsigned long long)__popcll(m5));
        atomicAdd((unsigned long long*)(divide + 6), (unsigned long long)__popcll(m6));
        atomicAdd((unsigned long long*)(divide + 7), (unsigned long long)__popcll(m7));
        atomicAdd((unsigned long long*)(divide + 8), (unsigned long long)__popcll(m8));
      }
    }
    if constexpr (GQ) {
      const bool go = ((((c.o >> t) | (c.o >> f)) & 1) != 0);
      const u64 ef = ballot(full && go), ed = em ^ ef;
      if (full) {
        // one store through a selected address; the ranks from v_mbcnt on the
        // SGPR masks (round 4: 20 -> 8 VALU per candidate, tools/bbprof.py)
        // (qd = q + kQd: sh.queue_d follows sh.queue, so one base address)
        constexpr u32 kQd = sizeof(sh.queue) / sizeof(u32);
        u32 rf = mask_rank(ef), rd = mask_rank(ed);
        asm("" : "+v"(rf), "+v"(rd));  // both ranks, then one select (not a select of the masks)
        q[go ? qn + rf : kQd + qnd + rd] = c.e;
      }
      qn = __builtin_amdgcn_readfirstlane(qn + (u32)__popcll(ef));
      qnd = __builtin_amdgcn_readfirstlane(qnd + (u32)__popcll(ed));
    } else {
      if (full) q[qn + mask_rank(em)] = c.e;
      qn = __builtin_amdgcn_readfirstlane(qn + (u32)__popcll(em));
    }
  };
  auto drain64 = [&]() {  // qn >= 64: recount 64 queued children in full
    wave_lds_sync();
    const u32 e2 = q[lane];
    const u32 tg = sh.tag(e2 >> 15);  // issued with the record reads
    add_tag(tg, PHASE == 5 || PHASE == 6 ? e2 & 1 : c2c_full<STM>(sh, e2), true);
    wave_lds_sync();
    if (lane + 64 < qn) q[lane] = q[lane + 64];
    qn = __builtin_amdgcn_readfirstlane(qn - 64);
  };
  auto drain64d = [&]() {  // qnd >= 64: count 64 queued children group-wise
#if DC_C2C_DIAGQ
    wave_lds_sync();
    const u32 e2 = qd[lane];
    const u32 tg = sh.tag(e2 >> 15);
    add_tag(tg, PHASE == 5 || PHASE == 6 ? e2 & 1 : c2c_diag<STM>(sh, e2), true);
    wave_lds_sync();
    if (lane + 64 < qnd) qd[lane] = qd[lane + 64];
    qnd = __builtin_amdgcn_readfirstlane(qnd - 64);
#endif
  };
  // one quiet child: base + O's pawn moves in the child (the record's board)
  auto quiet_count = [&](u32 e2) -> u32 {
    const u32 pl = e2 >> 15;
    const int f = (int)(e2 & 63), t = (int)((e2 >> 6) & 63);
    return sh.basec(pl) + (PHASE == 6 ? (u32)t : ref_pawn_count_child<1 - STM>(sh.board(pl), f, t));
  };
  auto drain64q = [&]() {  // qnq >= 64: 64 queued quiet children
    wave_lds_sync();
    const u32 e2 = qq[lane];
    const u32 tg = sh.tag(e2 >> 15);
    add_tag(tg, quiet_count(e2), true);
    wave_lds_sync();
    if (lane + 64 < qnq) qq[lane] = qq[lane + 64];
    qnq = __builtin_amdgcn_readfirstlane(qnq - 64);
  };
  auto drain = [&]() {
    if (qn >= 64) drain64();
    if constexpr (GQ) if (qnd >= 64) drain64d();
    if constexpr (QQ) if (qnq >= 64) drain64q();
  };
  if constexpr (BULK && PHASE != 7) add(otid(w), (u32)simple_leaves, valid);
  if constexpr (PHASE == 7) {  // [2] simple children, [3] parents
    const u64 ns = wave_sum64(nsim), np = __popcll(ballot(valid));
    if (lane == 0) {
      atomicAdd((unsigned long long*)(divide + 2), (unsigned long long)ns);
      atomicAdd((unsigned long long*)(divide + 3), (unsigned long long)np);
    }
  }
  if constexpr (PHASE == 1 || PHASE == 2) acc += cnt + base + (u32)att;
  for (u32 wbase = 0; wbase < (PHASE == 2 ? 0u : total); wbase += CAP) {
    if (wbase) __syncthreads();  // previous window fully read
    // each (f, t) of this parent's enumerated (BULK: special) moves -> visit(f, t)
    // the parent is read back from its record (after the barrier: a fresh
    // LDS read), so its board is not live across the consume/drain loop
    // (GQ) and the simple-move masks rebuilt from it and its rays
    // (ref_parent_split's keep), so neither is live across the loop
    auto each_move = [&](auto&& visit) {
      if constexpr (REUSE) {
        if (wbase == 0) {  // the norm: the split's masks and fills are still live
          ref_for_each_special_pre<STM>(sh.board(otid(w)), Fs, Ts, tgt, visit);
          return;
        }
      }
      if constexpr (GQ) {
        const Board pp = sh.board(otid(w));
        u32 unused;
        const u64 rays = sh.rays(otid(w));
        const u64 occ = occupied(pp), own = STM ? pp.b0 : (occ & ~pp.b0);
#if DC_C2C_GCORR
        u64 p1, n1, big;
        const u64 g = ref_pawn_planes<1 - STM>(pp, unused, p1, n1, big);
        ref_for_each_special<STM>(pp, own & ~(rays | g), ~(occ | rays | big), visit);
#else
        const u64 keep = ~(rays | ref_pawn_sensitive<1 - STM>(pp, unused));
        ref_for_each_special<STM>(pp, own & keep, ~occ & keep, visit);
#endif
      } else if constexpr (BULK) {
        ref_for_each_special<STM>(p, Fs, Ts, visit);
      } else {
        ref_for_each_move<STM>(p, visit);
      }
    };
    const u32 pl15 = otid(w) << 15;
    if (total <= CAP) {  // the norm: one window, no range checks
      u32 j = excl;
      if (valid) each_move([&](int f, int t) { sh.slot[j++] = (u32)f | ((u32)t << 6) | pl15; });
    } else {
      u32 j = excl;
      if (valid && j < wbase + CAP && j + cnt > wbase) {
        each_move([&](int f, int t) {
          if (j >= wbase && j - wbase < CAP) sh.slot[j - wbase] = (u32)f | ((u32)t << 6) | pl15;
          ++j;
        });
      }
    }
    __syncthreads();
    const u32 nslots = min(CAP, total - wbase);
    // two slots per lane per step, loaded together, so the LDS round trips overlap
    u32 r0 = (PHASE == 1 || PHASE == 2) ? nslots : w * 64;
    for (; DC_C2C_PAIR && r0 + 256 < nslots; r0 += 512) {
      const u32 ra = r0 + lane, rb = r0 + 256 + lane;
      const bool lb = rb < nslots;
      const Cand ca = fetch(sh.slot[ra]);
      const Cand cb = fetch(lb ? sh.slot[rb] : 0u);
      consume(ca, true);
      drain();
      consume(cb, lb);
      drain();
    }
    for (; r0 < nslots; r0 += 256) {  // (DC_C2C_PAIR: at most one round left)
      const u32 ra = r0 + lane;
      const bool la = ra < nslots;
      consume(fetch(la ? sh.slot[ra] : 0u), la);
      drain();
    }
  }
#if DC_C2C_POOL
  // Pooled final drains (round 4): the waves' leftover queue entries (fewer
  // than 64 of each kind per wave) are gathered into one block list in the
  // slot area and drained 64 at a time, the chunks dealt to the waves in turn:
  // ceil(total / 64) drains per kind instead of one partial drain per wave
  // (the partial final drains were 15 % of k_count3c's VALU issue cycles,
  // tools/bbprof_inline.py).  The parents' records are still in LDS.
  {
    // [0..3] full, [4..7] group-wise, [8..11] quiet (the scan is done)
    u32* cnt = reinterpret_cast<u32*>(sh.wsum);
    __syncthreads();  // every wave is past its last slot read: the slot area is free
    if (lane == 0) {
      cnt[w] = qn;
      cnt[4 + w] = GQ ? qnd : 0u;
      cnt[8 + w] = QQ ? qnq : 0u;
    }
    __syncthreads();
    u32 of = 0, od = 0, oq = 0, nf = 0, nd = 0, nq = 0;
#pragma unroll
    for (u32 v = 0; v < 4; ++v) {
      const u32 a = cnt[v], b = cnt[4 + v], x = cnt[8 + v];
      of += v < w ? a : 0u;
      od += v < w ? b : 0u;
      oq += v < w ? x : 0u;
      nf += a;
      nd += b;
      nq += x;
    }
    nf = __builtin_amdgcn_readfirstlane(nf);
    nd = __builtin_amdgcn_readfirstlane(nd);
    nq = __builtin_amdgcn_readfirstlane(nq);
    if (lane < qn) sh.slot[of + lane] = q[lane];
    if (GQ && lane < qnd) sh.slot[nf + od + lane] = qd[lane];
    if (QQ && lane < qnq) sh.slot[nf + nd + oq + lane] = qq[lane];
    __syncthreads();
    const u32 cf = (nf + 63) / 64, cd = (nd + 63) / 64, cq = (nq + 63) / 64;
    for (u32 c = w; c < cf + cd + cq; c += 4) {
      const u32 kind = c < cf ? 0u : c < cf + cd ? 1u : 2u;  // wave-uniform
      const u32 k = (kind == 0 ? c * 64 : kind == 1 ? nf + (c - cf) * 64 : nf + nd + (c - cf - cd) * 64) + lane;
      const bool live = k < (kind == 0 ? nf : kind == 1 ? nf + nd : nf + nd + nq);
      const u32 e2 = live ? sh.slot[k] : 0u;
      u32 r = 0;
      if (kind == 0) r = live ? (PHASE == 5 || PHASE == 6 ? e2 & 1 : c2c_full<STM>(sh, e2)) : 0u;
#if DC_C2C_DIAGQ
      else if (kind == 1) r = live ? (PHASE == 5 || PHASE == 6 ? e2 & 1 : c2c_diag<STM>(sh, e2)) : 0u;
#endif
      else if (QQ) r = live ? quiet_count(e2) : 0u;
      add(e2 >> 15, r, live);
    }
  }
#else
  // drain this wave's queue (par/att of the chunk are still in LDS)
  if (qn) {
    wave_lds_sync();
    const bool live = lane < qn;
    const u32 e2 = live ? q[lane] : 0u;
    const u32 k = live ? (PHASE == 5 || PHASE == 6 ? e2 & 1 : c2c_full<STM>(sh, e2)) : 0u;
    add(e2 >> 15, k, live);
  }
#if DC_C2C_DIAGQ
  if (GQ && qnd) {
    wave_lds_sync();
    const bool live = lane < qnd;
    const u32 e2 = live ? qd[lane] : 0u;
    const u32 k = live ? (PHASE == 5 || PHASE == 6 ? e2 & 1 : c2c_diag<STM>(sh, e2)) : 0u;
    add(e2 >> 15, k, live);
  }
#endif
  if (QQ && qnq) {
    wave_lds_sync();
    const bool live = lane < qnq;
    const u32 e2 = live ? qq[lane] : 0u;
    add(e2 >> 15, live ? quiet_count(e2) : 0u, live);
  }
#endif
  tag_hist_add(sh.hist, tag0, acc, true);
  __syncthreads();  // par/att/ptag/slot reused by the next group
}

#ifdef DC_AB_KNOBS
// PHASE 8 (A/B build): PHASE 0 plus a per-block timeline (wall clock, 100 MHz)
// in g_c2c_trace, read back by dc_ab_c2c_trace (tools/c2c_trace.py).
constexpr int kTraceWords = 8;
constexpr int kTraceBlocks = 4096;
__device__ u64 g_c2c_trace[kTraceBlocks * kTraceWords];
#endif

template <int STM, u32 CAP, int PHASE = 0, bool BULK = true, int MINW = 4>
__global__ __launch_bounds__(256, MINW) void k_count2c(const Board* __restrict__ nodes, const uint16_t* __restrict__ tags,
                                                 const Range* __restrict__ rng, u64* __restrict__ divide,
                                                 u32* __restrict__ next_chunk) {
  __shared__ C2cShared<CAP> sh;
  constexpr int GP = PHASE == 8 ? 0 : PHASE;
  [[maybe_unused]] u64 t_entry = 0, t_wait = 0, t_last = 0, n_chunks = 0;
  if constexpr (PHASE == 8) t_entry = wall_clock64();
  tag_hist_init(sh.hist);
  const u32 wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool t0 = wave == 0 && lane_id() == 0;
  const u64 lo = rng->lo, hi = rng->hi;
  // Blocks take 256-parent chunks from a counter: the cost of a chunk varies
  // with its positions, and static ranges left the slowest block behind (a
  // sharded launch has only ~3 chunks per block).  The counter's round trips
  // are 2.7 % of a block's lifetime at perft(7) (tools/c2c_trace.py).  Each
  // block's first chunk is its own index (round 5, as k_count3c): the counter
  // hands out the rest from gridDim.x on.
  for (bool first = true;; first = false) {
    [[maybe_unused]] u64 ta = 0;
    if constexpr (PHASE == 8) ta = wall_clock64();
    if (t0) sh.next = first ? blockIdx.x : gridDim.x + atomicAdd(next_chunk, 1u);
    __syncthreads();
    if constexpr (PHASE == 8) {
      t_last = wall_clock64();
      t_wait += t_last - ta;
    }
    const u64 s = lo + (u64)sh.next * kChunk;
    if (s >= hi) break;  // block-uniform
    if constexpr (PHASE == 8) ++n_chunks;
    const u64 i = s + otid(wave);
    const bool valid = i < hi;
    Board p{0, 0, 0, 0};
    u32 tag = 0;
    if (valid) {
      p = load_board(nodes, i);
      tag = tags[i];
    }
    c2c_group<STM, CAP, GP, BULK>(sh, valid, p, tag, divide, wave);
  }
  tag_hist_flush(sh.hist, divide, otid(wave));
#ifdef DC_AB_KNOBS
  if constexpr (PHASE == 8) {
    if (t0 && blockIdx.x < kTraceBlocks) {
      u32 xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      u64* r = g_c2c_trace + blockIdx.x * kTraceWords;
      r[0] = t_entry;
      r[1] = wall_clock64();
      r[2] = n_chunks;
      r[3] = t_wait;
      r[4] = xcc & 15;
      r[5] = t_last;
      r[6] = gridDim.x;
      r[7] = 0;
    }
  }
#endif
}

// ---------------------------------------- k_count3c (REF: the last three plies)
// k_count2c fed by its parents' parents: the level above the final stage's
// parents (perft(7): ply 4, 197k nodes) is counted and scanned as before
// (k_level_count, k_chunk_scan), but its children (ply 5, 4.9M nodes) are
// never written as boards.  k_level_moves writes each child as one 32-bit
// word {grandparent index << 12 | f | t << 6} at its scan offset (20 MB
// instead of k_level_write's 167 MB of boards and tags), and k_count3c takes
// groups of 256 consecutive words from a counter: each lane loads its word
// and its grandparent (a handful of distinct boards per group, L2 hits),
// makes the child and hands the 256 children to c2c_group.  Every child is
// counted exactly once and carries its grandparent's root tag.
// (Round 2: expanding the grandparents inside k_count3c instead -- one lane
// per grandparent enumerating into LDS while the block waited -- made the
// final stage 0.56 vs 0.49 + 0.04 ms.)
constexpr u32 kGroup = 256;
#ifndef DC_C3C_EVEN
#define DC_C3C_EVEN 0
#endif
#ifndef DC_C3C_TAIL
#define DC_C3C_TAIL 0
#endif
#ifndef DC_C3C_LOG
#define DC_C3C_LOG 0
#endif
#if DC_C3C_LOG
constexpr u32 kC3cLogGroups = 20480, kC3cLogWords = 258;
__device__ u64 g_c3c_log[kC3cLogGroups * kC3cLogWords];
extern "C" __attribute__((visibility("default"))) int dc_ab_c3c_log(u64* out, u64 n_words) {
  const u64 n = n_words < (u64)kC3cLogGroups * kC3cLogWords ? n_words : (u64)kC3cLogGroups * kC3cLogWords;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_c3c_log), n * sizeof(u64), 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
constexpr u32 kMoveWordNodes = 1u << 20;  // grandparent index field of a move word

// A level of more than kMoveWordNodes grandparents (possible only past a
// speculative bound) is flagged by the scan that sizes its children
// (k_chunk_scan's guard): the children's Range is empty and
// the host reruns in exact mode, which takes the k_level_write path.
template <int STM_G, u32 CAP, int MINW = 4, class W = u32>
__global__ __launch_bounds__(256, MINW) void k_count3c(const Board* __restrict__ nodes, const uint16_t* __restrict__ tags,
                                                 const Range* __restrict__ rng, const Range* __restrict__ rng_ch,
                                                 const W* __restrict__ mw, u64* __restrict__ divide,
                                                 u32* __restrict__ next_group, FrontState* __restrict__ fst) {
  __shared__ C2cShared<CAP> sh;
  if (fst) {  // after k_front: its look-back slots are cleared for the next run
    const u32 n = fst->n_items;
    for (u32 k = blockIdx.x * 256 + threadIdx.x; k < n; k += gridDim.x * 256) {
      fst->agg[k] = 0;
      fst->incl[k] = 0;
    }
  }
  tag_hist_init(sh.hist);
  const u32 wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool t0 = wave == 0 && lane_id() == 0;
  const u64 lo = rng->lo;
  const u32 total = (u32)(rng_ch->hi - rng_ch->lo);  // children (< 2^32: launcher)
#if DC_C3C_STATIC
  u32 k_static = 0;  // A/B diagnostics: block b takes groups b, b + grid, ... (no counter)
#endif
  // Each block's first group is its own index (round 5: no atomic round trip
  // before the first load, as in k_count2b); the counter hands out the rest
  // from gridDim.x on.
#if DC_C3C_EVEN
  // DC_C3C_EVEN (round 6): groups of gsz <= 256 words, gsz chosen so that the
  // level is a whole number of rounds of the grid.  With 256-word groups a
  // strided shard of perft(7) (613k words: 2.34 rounds of 1,024 blocks) ran
  // its last third of a round on a third of the blocks, one group's latency
  // at low occupancy: its k_count3c took 57 us for 41 us of work.  Measured
  // slower (profiles/r06/ab_c3even.jsonl, same box, alternating): shard 0 of 8
  // 0.084 -> 0.091 ms, perft(6) 0.047 -> 0.049 ms, perft(7) unchanged: more
  // groups means more per-group parent splits, whose issue cost does not
  // shrink with the group.  Off (A/B knob).
  const u32 rounds = (total + kGroup * gridDim.x - 1) / (kGroup * gridDim.x);
  const u32 gsz = rounds ? (total + rounds * gridDim.x - 1) / (rounds * gridDim.x) : kGroup;
#else
  constexpr u32 gsz = kGroup;
#endif
#if DC_C3C_TAIL
  // DC_C3C_TAIL (round 6 A/B): a level of more than one round of groups ends
  // in 64-word groups (its last 2 x grid x 64 words).  A wave none of whose
  // lanes holds a word skips the parent split, so a 64-word group pays one
  // wave's split, not four (DC_C3C_EVEN's partial waves paid them all).
  // Measured slower (profiles/r06/ab_c3tail.jsonl): shard 0 of 8 0.084 ->
  // 0.099 ms, perft(7) 0.375 -> 0.390 ms on one context; each small group
  // still pays the block's scans, barriers and pooled queue drains.
  constexpr u32 kTail = 64;
  const u32 tail = (total + gridDim.x - 1) / gridDim.x > kGroup ? min(total, 2u * gridDim.x * kTail) : 0u;
  const u32 nbig = (total - tail) / gsz, tstart = nbig * gsz;
#endif
  u32 grp = blockIdx.x;
  for (;;) {
    // (fetching the next group's index one group ahead, to take its round
    // trip off the load chain, made the kernel 0.495 -> 0.519 ms at perft(7):
    // a block then holds a group it cannot start, which lengthens the tail)
#if DC_C3C_TAIL
    const bool big = grp < nbig || !tail;
    const u64 s = big ? (u64)grp * gsz : (u64)tstart + (u64)(grp - nbig) * kTail;
    const u32 gn = big ? gsz : kTail;
#else
    const u64 s = (u64)grp * gsz;
    const u32 gn = gsz;
#endif
    if (s >= total) break;  // block-uniform
    const u32 ot = otid(wave);
    const u64 i = s + ot;
    const bool valid = ot < gn && i < total;
    Board ch{0, 0, 0, 0};
    u32 tag = 0;
    if (valid) {
      const W e = mw[i];
      const u64 g = lo + (u64)(e >> 12);
      ch = load_board(nodes, g);
      tag = tags[g];
      const u32 mv = (u32)e;
      ref_make(ch, (int)(mv & 63), (int)((mv >> 6) & 63));
    }
    c2c_group<1 - STM_G, CAP>(sh, valid, ch, tag, divide, wave);
#if DC_C3C_LOG
    // diagnostics: the block's cumulative histogram after each group
    // (read back by dc_ab_c3c_log; tools/c2c_groups.py takes differences)
    if (grp < kC3cLogGroups) {
      u64* rec = g_c3c_log + (u64)grp * kC3cLogWords;
      const u32 tid = otid(wave);
      rec[tid] = sh.hist[tid];
      if (tid == 0) {
        rec[256] = blockIdx.x;
        rec[257] = wall_clock64();
      }
    }
    __syncthreads();
#endif
    // (c2c_group ended with a barrier: every thread is past its read of grp's state)
#if DC_C3C_STATIC
    if (t0) sh.next = blockIdx.x + (++k_static) * gridDim.x;
#else
    if (t0) sh.next = gridDim.x + atomicAdd(next_group, 1u);
#endif
    __syncthreads();
    grp = sh.next;
  }
  tag_hist_flush(sh.hist, divide, otid(wave));
}

// ------------------------------------------------- K4: per-lane DFS (REF)
// perft below a frontier level without materialising the deeper levels: every
// lane walks the subtree of one frontier node depth first with an explicit
// stack, and each node it reaches at L plies below the frontier is handed to
// the block's c2c_group as a parent (the last two plies, bulk-counted as in
// k_count2c).  Memory stays at the frontier level plus L - 1 stack frames per
// lane, so perft(8), perft(9), ... need no level beyond ply 5 (a BFS level of
// ply 7 of startpos alone is 3.3e9 nodes, ~112 GB).
//
// A lane's state is its top frame in registers -- the board being expanded,
// the own pieces whose moves are still to come (srcs), the remaining targets
// of the current piece f (tgts) -- with the frames above it in `stack`, SoA
// [frame][field][lane] in HBM (coalesced; touched only on push and pop).
// Moves are generated per piece (ref_piece_targets, chess.rs:199-360), so a
// frame needs no move list.  Lanes take frontier nodes from one counter in
// the run's result block (one atomic per wave per refill).
struct DfsStack {
  u64* frames;  // (L - 1) frames x 7 u64 (b0..b3, srcs, tgts, f) x lanes; null when L == 1
  u64 lanes;    // grid x 256
};

template <int STM_P, u32 CAP, int L>
__global__ __launch_bounds__(256, 3) void k_perft_dfs(const Board* __restrict__ nodes, const uint16_t* __restrict__ tags,
                                                      const Range* __restrict__ rng, u64* __restrict__ divide,
                                                      u32* __restrict__ cursor, DfsStack stack) {
  static_assert(L >= 1, "L = 0 is k_count2c");
  constexpr u32 kStmF = (u32)(STM_P ^ (L & 1));  // side to move at the frontier ply
  __shared__ C2cShared<CAP> sh;
  tag_hist_init(sh.hist);
  const u32 lane = lane_id();
  const u64 gid = (u64)blockIdx.x * 256 + threadIdx.x;
  const u64 lo = rng->lo, n_front = rng->hi - rng->lo;
  int lvl = -1;  // frame of the board being expanded; -1: take a frontier node
  bool done = false;
  Board cb{0, 0, 0, 0};
  u64 srcs = 0, tgts = 0;
  int cf = 0;
  u32 tag = 0;
  auto own_of = [](const Board& b, u32 stm) { const u64 occ = occupied(b); return stm ? b.b0 : (occ & ~b.b0); };
  auto frame = [&](int k, int field) -> u64& { return stack.frames[((u64)k * 7 + field) * stack.lanes + gid]; };
  for (;;) {
    Board p{0, 0, 0, 0};
    bool valid = false;
    while (!done && !valid) {
      if (lvl < 0) {  // refill from the frontier: one atomic per wave
        const u64 need = ballot(true);
        const int leader = lsb(need);
        u32 base = 0;
        if ((int)lane == leader) base = atomicAdd(cursor, (u32)__popcll(need));
        base = __shfl(base, leader, 64);
        const u64 idx = (u64)base + (u64)__popcll(need & ((1ull << lane) - 1));
        if (idx >= n_front) {
          done = true;
          break;
        }
        cb = load_board(nodes, lo + idx);
        tag = tags[lo + idx];
        srcs = own_of(cb, kStmF);
        tgts = 0;
        lvl = 0;
        continue;
      }
      const u32 stm = kStmF ^ ((u32)lvl & 1);
      if (tgts == 0) {
        if (srcs == 0) {  // frame exhausted: pop
          if (--lvl >= 0) {
            cb = Board{frame(lvl, 0), frame(lvl, 1), frame(lvl, 2), frame(lvl, 3)};
            srcs = frame(lvl, 4);
            tgts = frame(lvl, 5);
            cf = (int)frame(lvl, 6);
          }
          continue;
        }
        cf = lsb(srcs);
        srcs &= srcs - 1;
        tgts = ref_piece_targets(cb, cf, stm, nibble(cb, cf) >> 1);
        continue;
      }
      const int t = lsb(tgts);
      tgts &= tgts - 1;
      Board child = cb;
      ref_make(child, cf, t);
      if (lvl + 1 == L) {
        p = child;
        valid = true;
        break;
      }
      if constexpr (L > 1) {  // push: the frame below the new top keeps its iterator
        frame(lvl, 0) = cb.b0;
        frame(lvl, 1) = cb.b1;
        frame(lvl, 2) = cb.b2;
        frame(lvl, 3) = cb.b3;
        frame(lvl, 4) = srcs;
        frame(lvl, 5) = tgts;
        frame(lvl, 6) = (u64)cf;
        ++lvl;
        cb = child;
        srcs = own_of(cb, stm ^ 1);
        tgts = 0;
      }
    }
    if (__syncthreads_or(valid) == 0) break;  // every lane of the block is done
    c2c_group<STM_P, CAP>(sh, valid, p, tag, divide, __builtin_amdgcn_readfirstlane(threadIdx.x >> 6));
  }
  tag_hist_flush(sh.hist, divide);
}

// ------------------------------------------------------------- launchers
static constexpr u32 kMaxGrid = 1u << 20;

static inline u32 grid_for(u64 n, u32 per) {
  const u64 b = (n + per - 1) / per;
  return (u32)std::max<u64>(1, std::min<u64>(b, kMaxGrid));
}

// Grid-stride kernels get at most one resident wave of blocks (occupancy x CUs):
// a second, partial round of statically assigned blocks is pure tail.
template <class K>
static u32 resident_grid(K kernel, u32 block, u32 want) {
  static std::mutex mu;
  static std::map<const void*, u32> cache;
  const void* key = reinterpret_cast<const void*>(kernel);
  u32 cap;
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find(key);
    if (it == cache.end()) {
      int per_cu = 0, dev = 0, cus = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, (int)block, 0) != hipSuccess || per_cu < 1)
        per_cu = 1;
      (void)hipGetDevice(&dev);
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
      it = cache.emplace(key, (u32)(per_cu * cus)).first;
    }
    cap = it->second;
  }
  return std::max<u32>(1, std::min(want, cap));
}

#define DC_LAUNCH_STM(KERNEL, R, grid, block, st, ...)                                                     \
  do {                                                                                                     \
    if (stm) {                                                                                             \
      auto k_ = KERNEL<R, 1>;                                                                              \
      hipLaunchKernelGGL(k_, dim3(resident_grid(k_, block, grid)), dim3(block), 0, st, __VA_ARGS__);      \
    } else {                                                                                               \
      auto k_ = KERNEL<R, 0>;                                                                              \
      hipLaunchKernelGGL(k_, dim3(resident_grid(k_, block, grid)), dim3(block), 0, st, __VA_ARGS__);      \
    }                                                                                                      \
  } while (0)

#define DC_LAUNCH_RULES_STM(KERNEL, grid, block, st, ...)                                        \
  do {                                                                                           \
    if (rules == 0) DC_LAUNCH_STM(KERNEL, RefRules, grid, block, st, __VA_ARGS__);              \
    else DC_LAUNCH_STM(KERNEL, FideRules, grid, block, st, __VA_ARGS__);                        \
  } while (0)

hipError_t launch_expand_top(hipStream_t st, u32 rules, const Board* root, const uint16_t* root_meta, u32 stm0,
                             u32 target, const TopScratch& s, Board* out, uint16_t* out_meta, uint16_t* out_tags,
                             u64 cap_out, PerftResult* res, Range* out_rng, u32* words, u32 n_root) {
  TopBufs b;
  for (int k = 0; k < 2; ++k) {
    b.nodes[k] = s.nodes[k];
    b.meta[k] = s.meta[k];
    b.tags[k] = s.tags[k];
    b.cap[k] = s.cap[k];
  }
  if (rules == 0)
    hipLaunchKernelGGL(k_expand_top<RefRules>, dim3(1), dim3(RefRules::kTopThreads), 0, st, root, root_meta, stm0, target, b, out,
                       out_meta, out_tags, cap_out, res, out_rng, words, n_root);
  else
    hipLaunchKernelGGL(k_expand_top<FideRules>, dim3(1), dim3(FideRules::kTopThreads), 0, st, root, root_meta, stm0, target, b,
                       out, out_meta, out_tags, cap_out, res, out_rng, words, n_root);
  return hipGetLastError();
}

u64 chunks_for(u64 n) { return (n + kChunk - 1) / kChunk; }

hipError_t launch_level_count(hipStream_t st, u32 rules, int stm, const Board* nodes, const uint16_t* meta,
                              const Range* rng, u64 n_bound, u32* counts, u64* chunk_sum) {
  DC_LAUNCH_RULES_STM(k_level_count, grid_for(n_bound, kChunk), 256, st, nodes, meta, rng, counts, chunk_sum);
  return hipGetLastError();
}

hipError_t launch_make_count(hipStream_t st, u32 rules, int stm_par, const Board* par, const uint16_t* par_meta,
                             const uint16_t* par_tags, const u32* words, const Range* rng, u64 n_bound, Board* out,
                             uint16_t* out_meta, uint16_t* out_tags, u32* counts, u64* chunk_sum, u32 wsh,
                             u32 wstride) {
  const int stm = stm_par;
  DC_LAUNCH_RULES_STM(k_make_count, grid_for(n_bound, kChunk), 256, st, par, par_meta, par_tags, words, rng, out,
                      out_meta, out_tags, counts, chunk_sum, wsh, wstride);
  return hipGetLastError();
}

__global__ void k_shard_range(Range* rng, u32 shard, u32 n_shards) {
  const u64 lo = rng->lo, hi = rng->hi;
  const u64 n = hi > lo + shard ? (hi - lo - shard + n_shards - 1) / n_shards : 0;  // as k_gather_shard
  *rng = Range{0, n};
}

hipError_t launch_shard_range(hipStream_t st, Range* rng, u32 shard, u32 n_shards) {
  hipLaunchKernelGGL(k_shard_range, dim3(1), dim3(1), 0, st, rng, shard, n_shards);
  return hipGetLastError();
}

hipError_t launch_chunk_scan(hipStream_t st, const u64* chunk_sum, const Range* rng, u64* chunk_base, Range* next,
                             u64 cap, PerftResult* res, int select_path, u64 guard, u64* zero_next, u64 zero_max) {
  hipLaunchKernelGGL(k_chunk_scan, dim3(1), dim3(kTopThreads), 0, st, chunk_sum, rng, chunk_base, next, cap, res,
                     select_path, guard, zero_next, zero_max);
  return hipGetLastError();
}

hipError_t launch_level_write(hipStream_t st, u32 rules, int stm, const Board* nodes, const uint16_t* meta,
                              const uint16_t* tags, const Range* rng, u64 n_bound, const u32* counts,
                              const u64* chunk_base, Board* out, uint16_t* out_meta, uint16_t* out_tags, u64 cap,
                              u32* next_counts, u64* next_sum) {
  DC_LAUNCH_RULES_STM(k_level_write, grid_for(n_bound, kChunk), 256, st, nodes, meta, tags, rng, counts, chunk_base,
                      out, out_meta, out_tags, cap, next_counts, next_sum);
  return hipGetLastError();
}

hipError_t launch_gather_shard(hipStream_t st, const Board* in, const uint16_t* in_meta, const uint16_t* in_tags,
                               Range* rng, u32 shard, u32 n_shards, Board* out, uint16_t* out_meta,
                               uint16_t* out_tags) {
  hipLaunchKernelGGL(k_gather_shard, dim3(1), dim3(1024), 0, st, in, in_meta, in_tags, rng, shard, n_shards, out,
                     out_meta, out_tags);
  return hipGetLastError();
}

__global__ void k_set_result_cursor(ResultCursor* cur, u64* base, u32 idx0, u32 stride) {
  *cur = ResultCursor{base, idx0, stride};
}

hipError_t launch_set_result_cursor(hipStream_t st, ResultCursor* cur, u64* base, u32 idx0, u32 stride) {
  hipLaunchKernelGGL(k_set_result_cursor, dim3(1), dim3(1), 0, st, cur, base, idx0, stride);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_copy_result(const PerftResult* __restrict__ r, ResultCursor* __restrict__ cur) {
  __shared__ u64 ws[4];
  const ResultCursor rc = *cur;  // every thread reads it before thread 0 advances it
  u64* __restrict__ out = rc.base + 258 * (u64)rc.idx;
  const u32 i = threadIdx.x, nr = r->n_root;
  const u64 v = i < nr ? r->divide[i] : 0;
  out[i] = v;
  const u64 s = wave_sum64(v);
  if (lane_id() == 0) ws[i >> 6] = s;
  __syncthreads();
  if (i == 0) {
    out[256] = (u64)nr | ((u64)r->overflow << 32);
    out[257] = ws[0] + ws[1] + ws[2] + ws[3];
    cur->idx = rc.idx + rc.stride;  // after the barrier: all threads hold rc
  }
}

hipError_t launch_copy_result(hipStream_t st, const PerftResult* res, ResultCursor* cur) {
  hipLaunchKernelGGL(k_copy_result, dim3(1), dim3(256), 0, st, res, cur);
  return hipGetLastError();
}

hipError_t launch_wide_slice(hipStream_t st, const Range* lvl, const u64* chunk_base, const Range* words_total,
                             u64 s0, u64 len, Range* out, u32* counter, PerftResult* res, u64 cap) {
  hipLaunchKernelGGL(k_wide_slice, dim3(1), dim3(1), 0, st, lvl, chunk_base, words_total, s0, len, out, counter, res,
                     cap);
  return hipGetLastError();
}

hipError_t launch_slice(hipStream_t st, Range* rng, u32 shard, u32 n_shards) {
  hipLaunchKernelGGL(k_slice, dim3(1), dim3(1), 0, st, rng, shard, n_shards);
  return hipGetLastError();
}

#ifdef DC_AB_KNOBS
// Final-stage selection (for A/B measurement): DC_FINAL=2b forces k_count2b
// under REF (k_count2c: 24 child slots per parent, the best of 20/24/28).
static int final_variant() {
  static const int v = [] {
    const char* e = ab_env("DC_FINAL");
    return (e && std::strcmp(e, "2b") == 0) ? 0 : 1;
  }();
  return v;
}
#endif

template <u32 CAP, int PHASE, bool BULK, int MINW = 4>
static void launch_count2c_cap(hipStream_t st, int stm, const Board* nodes, const uint16_t* tags, const Range* rng,
                               u64* divide) {
  // divide is the first member of the run's PerftResult (perft_enqueue): its
  // next_chunk field, zeroed with the block at the start of the run, is the
  // chunk counter
  static_assert(offsetof(PerftResult, divide) == 0, "divide heads PerftResult");
  u32* next = &reinterpret_cast<PerftResult*>(divide)->next_chunk;
  if (stm) {
    auto k = k_count2c<1, CAP, PHASE, BULK, MINW>;
    hipLaunchKernelGGL(k, dim3(resident_grid(k, 256, kMaxGrid)), dim3(256), 0, st, nodes, tags, rng, divide, next);
  } else {
    auto k = k_count2c<0, CAP, PHASE, BULK, MINW>;
    hipLaunchKernelGGL(k, dim3(resident_grid(k, 256, kMaxGrid)), dim3(256), 0, st, nodes, tags, rng, divide, next);
  }
}

static void launch_count2c(hipStream_t st, int stm, const Board* nodes, const uint16_t* tags, const Range* rng,
                           u64* divide) {
  // DC_C2C_PHASE (A/B and timing only): 3 = no bulk split; 1, 2 = partial phases
  static const int phase = [] {
    const char* e = ab_env("DC_C2C_PHASE");
    return e ? std::atoi(e) : 0;
  }();
  // DC_C2C_WAVES (A/B): minimum waves per SIMD of the launch bounds, i.e. the
  // VGPR budget.  4 (default since round 2): 128 VGPRs with 52 B/lane of
  // spills; 3: 140 VGPRs, no scratch.  perft(7) count2: 0.498-0.505 vs
  // 0.523-0.532 ms (tools/ab_phase.sh, round 2; round 1's body measured equal).
  // Two round-2 dead ends: 16 instead of 24 slots per parent (LDS for 4
  // blocks per CU) measured the same, and a chunk prefetch pipeline (next
  // chunk's parents in registers across the group, next index fetched a group
  // ahead) was slower at either budget (0.542 / 0.574 ms).
  static const int waves = [] {
    const char* e = ab_env("DC_C2C_WAVES");
    return e ? std::atoi(e) : 4;
  }();
#ifdef DC_AB_KNOBS
  if (phase == 1) launch_count2c_cap<kC2cCap, 1, true>(st, stm, nodes, tags, rng, divide);
  else if (phase == 2) launch_count2c_cap<kC2cCap, 2, true>(st, stm, nodes, tags, rng, divide);
  else if (phase == 3) launch_count2c_cap<kC2cCap, 0, false>(st, stm, nodes, tags, rng, divide);
  else if (phase == 5) launch_count2c_cap<kC2cCap, 5, true>(st, stm, nodes, tags, rng, divide);
  else if (phase == 6) launch_count2c_cap<kC2cCap, 6, true>(st, stm, nodes, tags, rng, divide);
  else if (phase == 7) launch_count2c_cap<kC2cCap, 7, true>(st, stm, nodes, tags, rng, divide);
  else if (phase == 8) launch_count2c_cap<kC2cCap, 8, true>(st, stm, nodes, tags, rng, divide);
  else if (waves == 4) launch_count2c_cap<kC2cCap, 0, true, 4>(st, stm, nodes, tags, rng, divide);
  else launch_count2c_cap<kC2cCap, 0, true, 3>(st, stm, nodes, tags, rng, divide);
#else
  (void)phase;
  (void)waves;
  launch_count2c_cap<kC2cCap, 0, true, 4>(st, stm, nodes, tags, rng, divide);
#endif
}

#ifdef DC_AB_KNOBS
// A/B build only: the last PHASE 8 launch's per-block timeline
// (kTraceWords u64 per block: entry, exit, chunks, counter-wait ticks, XCC id,
// last counter return, grid size).
extern "C" __attribute__((visibility("default"))) int dc_ab_c2c_trace(u64* out, u64 n_words) {
  const u64 n = std::min<u64>(n_words, (u64)kTraceBlocks * kTraceWords);
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_c2c_trace), n * sizeof(u64), 0, hipMemcpyDeviceToHost) == hipSuccess
             ? 0
             : -1;
}
#endif

#ifdef DC_AB_KNOBS
extern "C" __attribute__((visibility("default"))) int dc_ab_top_trace(u64* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_top_trace), sizeof(g_top_trace), 0, hipMemcpyDeviceToHost) == hipSuccess
             ? 0
             : -1;
}
#endif

u64 dfs_lanes() {
  return (u64)resident_grid(k_perft_dfs<0, kC2cCap, 1>, 256, kMaxGrid) * 256;
}

hipError_t launch_perft_dfs(hipStream_t st, int stm_parent, u32 L, const Board* nodes, const uint16_t* tags,
                            const Range* rng, PerftResult* res, u64* stack_frames, u64 lanes) {
  const DfsStack ds{stack_frames, lanes};
  const u32 grid = (u32)(lanes / 256);
#define DC_DFS(S, LL)                                                                                        \
  hipLaunchKernelGGL((k_perft_dfs<S, kC2cCap, LL>), dim3(grid), dim3(256), 0, st, nodes, tags, rng, res->divide, \
                     &res->dfs_next, ds)
  if (L == 1) {
    if (stm_parent) DC_DFS(1, 1);
    else DC_DFS(0, 1);
  } else if (L == 2) {
    if (stm_parent) DC_DFS(1, 2);
    else DC_DFS(0, 2);
  } else if (L == 3) {
    if (stm_parent) DC_DFS(1, 3);
    else DC_DFS(0, 3);
  } else {
    return hipErrorNotSupported;
  }
#undef DC_DFS
  return hipGetLastError();
}

template <class W>
static hipError_t level_moves_w(hipStream_t st, int stm, const Board* nodes, const Range* rng, u64 n_bound,
                                const u32* counts, const u64* chunk_base, W* mw, u64 mw_cap) {
  // words beyond mw_cap are dropped (a flagged level is never read)
  auto k = stm ? k_level_moves<1, W> : k_level_moves<0, W>;
  hipLaunchKernelGGL(k, dim3(resident_grid(k, 256, grid_for(std::min<u64>(n_bound, kMoveWordNodes) * 4, kChunk))),
                     dim3(256), 0, st, nodes, rng, counts, chunk_base, mw, mw_cap);
  return hipGetLastError();
}
hipError_t launch_level_moves(hipStream_t st, int stm, const Board* nodes, const Range* rng, u64 n_bound,
                              const u32* counts, const u64* chunk_base, u32* mw, u64 mw_cap) {
  return level_moves_w(st, stm, nodes, rng, n_bound, counts, chunk_base, mw, mw_cap);
}
hipError_t launch_level_moves(hipStream_t st, int stm, const Board* nodes, const Range* rng, u64 n_bound,
                              const u32* counts, const u64* chunk_base, u64* mw, u64 mw_cap) {
  return level_moves_w(st, stm, nodes, rng, n_bound, counts, chunk_base, mw, mw_cap);
}

// k_count3c's special-child slots per parent and waves per SIMD (VGPR budget);
// compile-time only (tools/ab_perft_libs.sh builds variants with -D).
#ifdef DC_C3C_SLOTS
constexpr u32 kC3cCap = 256 * DC_C3C_SLOTS;
#else
constexpr u32 kC3cCap = kC2cCap;
#endif
#ifndef DC_C3C_MINW
#define DC_C3C_MINW 4
#endif
template <class W>
static hipError_t count3c_w(hipStream_t st, int stm_g, const Board* nodes, const uint16_t* tags, const Range* rng,
                            const Range* rng_ch, const W* mw, PerftResult* res, u32* counter, FrontState* fst = nullptr) {
  u32* next = counter ? counter : &res->next_chunk;
  if (stm_g) {
    auto k = k_count3c<1, kC3cCap, DC_C3C_MINW, W>;
    hipLaunchKernelGGL(k, dim3(resident_grid(k, 256, kMaxGrid)), dim3(256), 0, st, nodes, tags, rng, rng_ch, mw,
                       res->divide, next, fst);
  } else {
    auto k = k_count3c<0, kC3cCap, DC_C3C_MINW, W>;
    hipLaunchKernelGGL(k, dim3(resident_grid(k, 256, kMaxGrid)), dim3(256), 0, st, nodes, tags, rng, rng_ch, mw,
                       res->divide, next, fst);
  }
  return hipGetLastError();
}
hipError_t launch_count3c(hipStream_t st, int stm_g, const Board* nodes, const uint16_t* tags, const Range* rng,
                          const Range* rng_ch, const u32* mw, PerftResult* res, u32* counter, FrontState* fst) {
  return count3c_w(st, stm_g, nodes, tags, rng, rng_ch, mw, res, counter, fst);
}
hipError_t launch_count3c(hipStream_t st, int stm_g, const Board* nodes, const uint16_t* tags, const Range* rng,
                          const Range* rng_ch, const u64* mw, PerftResult* res, u32* counter) {
  return count3c_w(st, stm_g, nodes, tags, rng, rng_ch, mw, res, counter);
}

#ifdef DC_AB_KNOBS
extern "C" __attribute__((visibility("default"))) int dc_ab_front_trace(u64* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_front_trace), sizeof(g_front_trace), 0, hipMemcpyDeviceToHost) ==
                 hipSuccess
             ? 0
             : -1;
}
#endif

u64 front_spill_words() { return (u64)kFrontSpillItems * kFrontWin; }

hipError_t launch_front(hipStream_t st, int stm0, u32 depth, const Board* root, u32 shard, u32 n_shards, Board* out,
                        uint16_t* out_tags, u32 cap_b, u32* mw, u64 cap_w, PerftResult* res, Range* rng_out,
                        FrontState* fst, u32* spill) {
  if (depth != 6 && depth != 7) return hipErrorInvalidValue;
  // one pass of the resident grid: every block does the top once
#define DC_FRONT(S, E)                                                                                        \
  do {                                                                                                        \
    auto k_ = k_front<S, E>;                                                                                  \
    hipLaunchKernelGGL(k_, dim3(resident_grid(k_, kFrontThreads, kMaxGrid)), dim3(kFrontThreads), 0, st, root,    \
                       shard, n_shards,                                                                       \
                       out, out_tags, cap_b, mw, cap_w, res, rng_out, fst, spill);                            \
  } while (0)
  if (depth == 7) {
    if (stm0) DC_FRONT(1, 1);
    else DC_FRONT(0, 1);
  } else {
    if (stm0) DC_FRONT(1, 0);
    else DC_FRONT(0, 0);
  }
#undef DC_FRONT
  return hipGetLastError();
}

// Product: REF -> k_count2c (the bulk split), FIDE -> k_count2b<FideRules>.
// k_count2 and k_count2b<RefRules> are compiled only into the A/B build.
hipError_t launch_final(hipStream_t st, u32 rules, int stm, int plies, const Board* nodes, const uint16_t* meta,
                        const uint16_t* tags, const Range* rng, u64 n_bound, u64* divide, const PerftResult* res) {
  // divide is the run's PerftResult.divide (its first member): k_count2b's chunk counter sits in the same block
  static_assert(offsetof(PerftResult, divide) == 0, "divide heads the result block");
  u32* next_chunk = &reinterpret_cast<PerftResult*>(divide)->next_chunk;
  if (plies == 1) {
    DC_LAUNCH_RULES_STM(k_count1, grid_for(n_bound, 256), 256, st, nodes, meta, tags, rng, divide);
    return hipGetLastError();
  }
#ifdef DC_AB_KNOBS
  if (res != nullptr) {
    DC_LAUNCH_RULES_STM(k_count2, grid_for(n_bound, 64 * kC2Waves), 256, st, nodes, meta, tags, rng, divide, res);
    return hipGetLastError();
  }
  if (rules == 0 && final_variant() == 0) {
    DC_LAUNCH_STM(k_count2b, RefRules, kMaxGrid, 256, st, nodes, meta, tags, rng, divide, next_chunk);
    return hipGetLastError();
  }
#else
  (void)res;
#endif
  if (rules == 0) launch_count2c(st, stm, nodes, tags, rng, divide);
  else DC_LAUNCH_STM(k_count2b, FideRules, kMaxGrid, 256, st, nodes, meta, tags, rng, divide, next_chunk);
  return hipGetLastError();
}

}  // namespace dc
