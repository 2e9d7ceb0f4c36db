// Which XCD / SE / CU each block of a grid runs on (diagnostics, DESIGN.md
// §3.6): under a HIP CU mask (ROC_GLOBAL_CU_MASK) prints the distinct
// (xcc, se, sh, cu) slots the blocks landed on.
//   hipcc --offload-arch=gfx950 -O2 -o tools/diag/cu_probe tools/diag/cu_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <set>
#include <tuple>
#include <vector>

__global__ void k_probe(unsigned* out) {
  if (threadIdx.x == 0) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
  }
  // stay resident a while so the blocks spread out
  long long t0 = clock64();
  while (clock64() - t0 < 200000) {
  }
}

int main(int argc, char** argv) {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int n = argc > 1 ? atoi(argv[1]) : 3 * cus;
  unsigned* d;
  if (hipMalloc(&d, sizeof(unsigned) * 2 * n) != hipSuccess) return 1;
  hipLaunchKernelGGL(k_probe, dim3(n), dim3(256), 0, 0, d);
  std::vector<unsigned> h(2 * n);
  if (hipMemcpy(h.data(), d, sizeof(unsigned) * 2 * n, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  std::set<std::tuple<unsigned, unsigned, unsigned, unsigned>> slots;
  for (int b = 0; b < n; ++b) {
    const unsigned hw = h[2 * b], xcc = h[2 * b + 1] & 0xF;
    slots.insert({xcc, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 15});
  }
  std::set<unsigned> xccs;
  for (auto& s : slots) xccs.insert(std::get<0>(s));
  printf("{\"cus_reported\": %d, \"blocks\": %d, \"distinct_cu_slots\": %zu, \"xccs\": [", cus, n, slots.size());
  bool first = true;
  for (unsigned x : xccs) { printf("%s%u", first ? "" : ", ", x); first = false; }
  printf("], \"slots\": [");
  first = true;
  for (auto& s : slots) {
    printf("%s[%u,%u,%u,%u]", first ? "" : ",", std::get<0>(s), std::get<1>(s), std::get<2>(s), std::get<3>(s));
    first = false;
  }
  printf("]}\n");
  hipFree(d);
  return 0;
}
