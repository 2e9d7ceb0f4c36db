// Test-only probe of the FIDE final stage's split (k_count2b<FideRules> with
// kSplit, dc_perft.hip): for each position it runs the three device functions
// the kernel pairs -- fide_count_split (the counting pass: visits and simple
// children, set-wise), fide_for_each_split (the enumeration that writes child
// slots at offsets the counting pass handed out) and fide_for_each_move (every
// legal move) -- and writes what each returned.  tests/test_gpu_fide_split.py
// checks that the two split passes agree exactly (a mismatch would make child
// slots overlap or leave gaps with no error) and that the moves the enumeration
// leaves out are the simple moves of tools/fide_simple_proto.py.
//   hipcc --offload-arch=gfx950 -O3 -fPIC -shared -I distributed-chess_amd/csrc \
//         -o tests/kern/libsplitprobe.so tests/kern/split_probe.hip
#include <hip/hip_runtime.h>

#include "dc_common.h"
#include "dc_fide_rules.h"

using namespace dc;

namespace {

constexpr int kMaxMoves = 256;

struct ProbeOut {
  u32 count_c, ns_c;  // fide_count_split: visits, simple children
  u32 count_e, ns_e;  // fide_for_each_split: visits, its return value
  u32 n_all;          // fide_for_each_move visits
  u32 pad[3];
};

template <int STM>
__device__ void probe_one(const Board& b, u32 meta, ProbeOut& o, u32* split_mv, u32* all_mv) {
  u64 m[SN_COUNT];
  sens_masks(fide_sens<STM>(b, meta), m);
  auto sn = [&](int k) -> u64 { return m[k]; };
  u32 ns_c = 0;
  o.count_c = fide_count_split<STM>(b, meta, sn, ns_c);
  o.ns_c = ns_c;
  u32 ce = 0;
  o.ns_e = fide_for_each_split<STM>(b, meta, sn, [&](int f, int t, int promo) {
    if (ce < kMaxMoves) split_mv[ce] = (u32)f | ((u32)t << 6) | ((u32)promo << 12);
    ++ce;
  });
  o.count_e = ce;
  u32 ca = 0;
  fide_for_each_move<STM>(b, meta, [&](int f, int t, int promo) {
    if (ca < kMaxMoves) all_mv[ca] = (u32)f | ((u32)t << 6) | ((u32)promo << 12);
    ++ca;
  });
  o.n_all = ca;
}

__global__ void k_split_probe(const Board* __restrict__ b, const uint8_t* __restrict__ stm, const uint16_t* __restrict__ meta,
                              u32 n, ProbeOut* __restrict__ out, u32* __restrict__ split_mv, u32* __restrict__ all_mv) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  ProbeOut o{};
  const Board p = b[i];
  if (stm[i]) probe_one<1>(p, meta[i], o, split_mv + (size_t)i * kMaxMoves, all_mv + (size_t)i * kMaxMoves);
  else probe_one<0>(p, meta[i], o, split_mv + (size_t)i * kMaxMoves, all_mv + (size_t)i * kMaxMoves);
  out[i] = o;
}

}  // namespace

// host buffers in, host buffers out (n positions; moves: n x 256 words each)
extern "C" int split_probe(const void* boards, const uint8_t* stm, const uint16_t* meta, uint32_t n, void* out,
                           uint32_t* split_mv, uint32_t* all_mv) {
  if (n == 0) return 0;
  Board* db = nullptr;
  uint8_t* ds = nullptr;
  uint16_t* dm = nullptr;
  ProbeOut* dout = nullptr;
  u32 *dsm = nullptr, *dam = nullptr;
  const size_t mv_bytes = (size_t)n * kMaxMoves * sizeof(u32);
  int rc = -1;
  if (hipMalloc(&db, n * sizeof(Board)) == hipSuccess && hipMalloc(&ds, n) == hipSuccess &&
      hipMalloc(&dm, n * 2) == hipSuccess && hipMalloc(&dout, n * sizeof(ProbeOut)) == hipSuccess &&
      hipMalloc(&dsm, mv_bytes) == hipSuccess && hipMalloc(&dam, mv_bytes) == hipSuccess &&
      hipMemcpy(db, boards, n * sizeof(Board), hipMemcpyHostToDevice) == hipSuccess &&
      hipMemcpy(ds, stm, n, hipMemcpyHostToDevice) == hipSuccess &&
      hipMemcpy(dm, meta, n * 2, hipMemcpyHostToDevice) == hipSuccess) {
    hipLaunchKernelGGL(k_split_probe, dim3((n + 63) / 64), dim3(64), 0, 0, db, ds, dm, n, dout, dsm, dam);
    if (hipGetLastError() == hipSuccess && hipDeviceSynchronize() == hipSuccess &&
        hipMemcpy(out, dout, n * sizeof(ProbeOut), hipMemcpyDeviceToHost) == hipSuccess &&
        hipMemcpy(split_mv, dsm, mv_bytes, hipMemcpyDeviceToHost) == hipSuccess &&
        hipMemcpy(all_mv, dam, mv_bytes, hipMemcpyDeviceToHost) == hipSuccess)
      rc = 0;
  }
  (void)hipFree(db);
  (void)hipFree(ds);
  (void)hipFree(dm);
  (void)hipFree(dout);
  (void)hipFree(dsm);
  (void)hipFree(dam);
  return rc;
}
