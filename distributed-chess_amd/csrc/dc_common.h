// dc_common.h -- device helpers shared by the move and perft kernels.
#pragma once
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
  const u32 tag0 = lane_bcast(tag, (u32)leader);
  const bool same = !valid || tag == tag0;
  if (ballot(same) == ~0ull) {
    const u64 s = wave_sum64(valid ? v : 0);
    if ((int)lane == leader && s) atomicAdd(divide + tag0, s);
  } else if (valid && v) {
    atomicAdd(divide + tag, v);
  }
}


// Per-block accumulation of divide counts: waves add into an LDS histogram
// (one LDS atomic per wave when its lanes share a root tag, which is the norm
// because nodes stay ordered by root move) and the block flushes each non-zero
// bin with one global atomic.  Global same-address atomics from every wave
// serialise at the memory side and were the limiter (rocprofv3, round 1).
__device__ __forceinline__ void tag_hist_init(u64* hist) {
  for (u32 t = threadIdx.x; t < 256; t += blockDim.x) hist[t] = 0;
  __syncthreads();
}
__device__ __forceinline__ void tag_hist_add(u64* hist, u32 tag, u64 v, bool valid) {
  const bool live = valid && v != 0;
  const u64 lmask = ballot(live);
  if (lmask == 0) return;
  const int leader = lsb(lmask);
  const u32 tag0 = lane_bcast(tag, (u32)leader);
  if (ballot(live && tag != tag0) == 0) {
    const u64 s = ballot(live && (v >> 26) != 0) ? wave_sum64(live ? v : 0) : (u64)wave_sum32(live ? (u32)v : 0u);
    if ((int)lane_id() == leader) atomicAdd((unsigned long long*)&hist[tag0], (unsigned long long)s);
  } else if (live) {
    atomicAdd((unsigned long long*)&hist[tag], (unsigned long long)v);
  }
}
__device__ __forceinline__ void tag_hist_flush(const u64* hist, u64* divide, u32 tid = threadIdx.x) {
  __syncthreads();
  for (u32 t = tid; t < 256; t += blockDim.x)
    if (hist[t]) atomicAdd((unsigned long long*)(divide + t), (unsigned long long)hist[t]);
}

static inline u32 blocks_for(u64 n, u32 per) { return (u32)((n + per - 1) / per); }

}  // namespace dc
