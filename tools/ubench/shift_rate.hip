// Micro-benchmark: issue cost of 64-bit shifts vs 32-bit ops on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned long long u64;
template <int MODE>
__global__ __launch_bounds__(256) void k(u64* out, u64 seed, int iters) {
  u64 a = seed ^ threadIdx.x, b = seed * 3 + blockIdx.x, c = a ^ 0x5555, d = b ^ 0x3333;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if constexpr (MODE == 0) {  // 64-bit shifts (4 independent chains)
        asm volatile("v_lshlrev_b64 %0, 7, %0" : "+v"(a));
        asm volatile("v_lshlrev_b64 %0, 9, %0" : "+v"(b));
        asm volatile("v_lshrrev_b64 %0, 7, %0" : "+v"(c));
        asm volatile("v_lshrrev_b64 %0, 9, %0" : "+v"(d));
      } else if constexpr (MODE == 1) {  // 32-bit ands on both halves (8 ops)
        unsigned al = (unsigned)a, ah = (unsigned)(a >> 32);
        asm volatile("v_and_b32 %0, 7, %0\n v_and_b32 %1, 9, %1" : "+v"(al), "+v"(ah));
        unsigned bl = (unsigned)b, bh = (unsigned)(b >> 32);
        asm volatile("v_and_b32 %0, 7, %0\n v_and_b32 %1, 9, %1" : "+v"(bl), "+v"(bh));
        unsigned cl = (unsigned)c, ch = (unsigned)(c >> 32);
        asm volatile("v_or_b32 %0, 7, %0\n v_or_b32 %1, 9, %1" : "+v"(cl), "+v"(ch));
        unsigned dl = (unsigned)d, dh = (unsigned)(d >> 32);
        asm volatile("v_or_b32 %0, 7, %0\n v_or_b32 %1, 9, %1" : "+v"(dl), "+v"(dh));
        a = ((u64)ah << 32) | al; b = ((u64)bh << 32) | bl; c = ((u64)ch << 32) | cl; d = ((u64)dh << 32) | dl;
      } else if constexpr (MODE == 2) {  // alignbit (funnel shift, 4 ops)
        unsigned al = (unsigned)a, ah = (unsigned)(a >> 32);
        asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(ah) : "v"(al));
        unsigned bl = (unsigned)b, bh = (unsigned)(b >> 32);
        asm volatile("v_alignbit_b32 %0, %0, %1, 9" : "+v"(bh) : "v"(bl));
        unsigned cl = (unsigned)c, ch = (unsigned)(c >> 32);
        asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(ch) : "v"(cl));
        unsigned dl = (unsigned)d, dh = (unsigned)(d >> 32);
        asm volatile("v_alignbit_b32 %0, %0, %1, 9" : "+v"(dh) : "v"(dl));
        a = ((u64)ah << 32) | al; b = ((u64)bh << 32) | bl; c = ((u64)ch << 32) | cl; d = ((u64)dh << 32) | dl;
      } else if constexpr (MODE == 3) {  // bitop3 (4 ops)
        unsigned al = (unsigned)a, bl = (unsigned)b, cl = (unsigned)c, dl = (unsigned)d;
        asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xf8" : "+v"(al) : "v"(bl), "v"(cl));
        asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xf8" : "+v"(bl) : "v"(cl), "v"(dl));
        asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xf8" : "+v"(cl) : "v"(dl), "v"(al));
        asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xf8" : "+v"(dl) : "v"(al), "v"(bl));
        a = al; b = bl; c = cl; d = dl;
      } else {  // popcount accumulate (4 ops)
        unsigned al = (unsigned)a, bl = (unsigned)b, cl = (unsigned)c, dl = (unsigned)d;
        asm volatile("v_bcnt_u32_b32 %0, %1, %0" : "+v"(al) : "v"(bl));
        asm volatile("v_bcnt_u32_b32 %0, %1, %0" : "+v"(bl) : "v"(cl));
        asm volatile("v_bcnt_u32_b32 %0, %1, %0" : "+v"(cl) : "v"(dl));
        asm volatile("v_bcnt_u32_b32 %0, %1, %0" : "+v"(dl) : "v"(al));
        a = al; b = bl; c = cl; d = dl;
      }
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = a ^ b ^ c ^ d;
}

template <int M>
static double run(u64* out, int iters, const char* name, int ops_per_iter) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int blocks = 256 * 8;
  hipLaunchKernelGGL(k<M>, dim3(blocks), dim3(256), 0, 0, out, 1ull, iters);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k<M>, dim3(blocks), dim3(256), 0, 0, out, 1ull, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double wave_instr = (double)blocks * 4 * iters * 16 * ops_per_iter;
  const double rate = wave_instr / (ms * 1e-3);
  printf("%-28s %8.3f ms  %.3e wave-instr/s  (%.2f of 1.229e12 = 256CU*4SIMD*2.4GHz/2)\n", name, ms, rate, rate / 1.2288e12);
  return rate;
}

int main() {
  u64* out;
  (void)hipMalloc(&out, 256 * 8 * 256 * 8);
  const int it = 4000;
  run<0>(out, it, "v_lshl/lshrrev_b64", 4);
  run<1>(out, it, "v_and/or_b32", 8);
  run<2>(out, it, "v_alignbit_b32", 4);
  run<3>(out, it, "v_bitop3_b32", 4);
  run<4>(out, it, "v_bcnt_u32_b32", 4);
  return 0;
}
