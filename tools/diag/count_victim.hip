// A minimal victim for the DESIGN.md §3.6 fault study: the FIDE leaf count
// (fide_count<STM, TAB>, dc_fide_rules.h) alone, one lane per board in a
// grid-stride loop, each board counted `reps` times -- no LDS protocol, no
// enumeration, no histogram.  Built against a chosen revision's headers
// (tools/diag/count_victim.sh); run beside co-resident noise waves
// (tools/diag/noise.hip) by tools/diag/count_victim.py.
#include <hip/hip_runtime.h>

#include "dc_fide_rules.h"

using namespace dc;

template <int STM, bool TAB>
__global__ __launch_bounds__(256) void k_cv(const Board* __restrict__ b, const uint32_t* __restrict__ meta, uint32_t n,
                                            uint32_t* __restrict__ out, uint32_t reps) {
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    uint32_t c = 0;
    for (uint32_t r = 0; r < reps; ++r) {
      Board x = b[i];
      uint32_t m = meta[i];
      asm volatile("" : "+v"(x.b0), "+v"(x.b1), "+v"(x.b2), "+v"(x.b3), "+v"(m));
      c += fide_count<STM, TAB>(x, m);
    }
    out[i] = c;
  }
}

extern "C" int cv_run(int stm, int tab, const void* boards, const void* meta, uint32_t n, void* out, uint32_t reps,
                      int blocks) {
  const Board* b = (const Board*)boards;
  const uint32_t* m = (const uint32_t*)meta;
  uint32_t* o = (uint32_t*)out;
  if (stm == 0 && tab) hipLaunchKernelGGL((k_cv<0, true>), dim3(blocks), dim3(256), 0, 0, b, m, n, o, reps);
  else if (stm == 0) hipLaunchKernelGGL((k_cv<0, false>), dim3(blocks), dim3(256), 0, 0, b, m, n, o, reps);
  else if (tab) hipLaunchKernelGGL((k_cv<1, true>), dim3(blocks), dim3(256), 0, 0, b, m, n, o, reps);
  else hipLaunchKernelGGL((k_cv<1, false>), dim3(blocks), dim3(256), 0, 0, b, m, n, o, reps);
  if (hipGetLastError() != hipSuccess) return -1;
  return hipDeviceSynchronize() == hipSuccess ? 0 : -2;
}
