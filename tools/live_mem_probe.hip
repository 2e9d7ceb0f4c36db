// live_mem_probe.hip -- measurement only: host<->GPU ping-pong latency of a
// resident wave.  Request words in pinned host memory (the live validator's
// mailbox, polled over PCIe) unless noted; the response word is pinned host
// memory.  Modes:
//   A  lane 0 polls one dword
//   B  fine-grained device memory written by the host through its mapping
//      (round 4: stalls -- a host store was not seen -- so not usable)
//   C  23 lanes poll words 0..22 and one lane a word on a third line (the
//      live validator's poll), answer at once
//   D  20 lanes poll words 0..19 (two lines), answer at once
//   E  D, then 19 readlanes and ~150 dependent VALU ops before answering
//   build: hipcc --offload-arch=gfx950 -O2 tools/live_mem_probe.hip -o tools/live_mem_probe
//   run:   tools/live_mem_probe A|B [calls]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::printf("{\"error\": \"%s: %s\"}\n", #x, hipGetErrorString(e_));          \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

__global__ void k_pong(unsigned* req, unsigned* resp, unsigned n, int mode) {
  // the wave leaves after answering request n (or on 0xFFFFFFFF, or after 5 s)
  const unsigned lane = threadIdx.x;
  const unsigned nl = mode == 'C' ? 24u : (mode == 'D' || mode == 'E') ? 20u : 1u;
  if (lane >= nl) return;
  const unsigned idx = (mode == 'C' && lane == 23) ? 40u : lane;  // word 40: a third line
  unsigned want = 1;
  const unsigned long long t_end = wall_clock64() + 100ull * 1000 * 1000 * 5;  // 5 s at 100 MHz
  while (want <= n) {
    const unsigned w = __hip_atomic_load(req + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned v = __builtin_amdgcn_readfirstlane(w);
    if (v == 0xFFFFFFFFu) break;
    if (v == want) {
      unsigned out = v;
      if (mode == 'E') {
        unsigned acc = 0;
        for (int k = 1; k < 20; ++k) acc += (unsigned)__builtin_amdgcn_readlane((int)w, k);
        for (int k = 0; k < 150; ++k) acc = (acc << 1) ^ (acc >> 3) ^ (unsigned)k;  // a dependent chain
        out = v | (acc & 0u);
        asm volatile("" ::"v"(acc));
      }
      if (lane == 0) __hip_atomic_store(resp, out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      ++want;
    }
    if (wall_clock64() > t_end) break;
  }
}

int main(int argc, char** argv) {
  const char mode = argc > 1 ? argv[1][0] : 'A';
  const unsigned n = argc > 2 ? (unsigned)std::atoi(argv[2]) : 5000;
  unsigned *req = nullptr, *resp = nullptr;
  CHECK(hipHostMalloc((void**)&resp, 64, hipHostMallocCoherent));
  if (mode != 'B') {
    CHECK(hipHostMalloc((void**)&req, 256, hipHostMallocCoherent));
    for (int k = 0; k < 64; ++k) req[k] = 0;
  } else {
    CHECK(hipExtMallocWithFlags((void**)&req, 256, hipDeviceMallocFinegrained));
  }
  *resp = 0;
  // the host writes the request word through the pointer itself (B: device
  // memory through the host mapping -- a fault here means no such mapping)
  __atomic_store_n(req, 0u, __ATOMIC_RELEASE);
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipLaunchKernelGGL(k_pong, dim3(1), dim3(64), 0, st, req, resp, n, (int)mode);
  CHECK(hipGetLastError());
  std::vector<double> us(n);
  for (unsigned i = 1; i <= n; ++i) {
    const auto t0 = std::chrono::steady_clock::now();
    if (mode == 'D' || mode == 'E' || mode == 'C')
      for (int k = 1; k < 20; ++k) __atomic_store_n(req + k, i, __ATOMIC_RELAXED);  // the request's fields
    __atomic_store_n(req, i, __ATOMIC_RELEASE);
    unsigned long long spins = 0;
    while (__atomic_load_n(resp, __ATOMIC_ACQUIRE) != i) {
      if (++spins > 2000000000ull) {
        std::printf("{\"mode\": \"%c\", \"error\": \"no answer to request %u\"}\n", mode, i);
        __atomic_store_n(req, 0xFFFFFFFFu, __ATOMIC_RELEASE);
        (void)hipStreamSynchronize(st);
        return 2;
      }
    }
    us[i - 1] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  }
  CHECK(hipStreamSynchronize(st));
  std::sort(us.begin(), us.end());
  std::printf("{\"mode\": \"%c\", \"calls\": %u, \"median_us\": %.3f, \"p99_us\": %.3f, \"min_us\": %.3f}\n", mode, n,
              us[n / 2], us[(size_t)(n * 0.99)], us[0]);
  return 0;
}
