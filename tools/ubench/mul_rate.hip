// Micro-benchmark 3: issue rate of the integer multiply forms a 256-bit field
// multiplication can be built from (dc_secp.h), 4 independent chains per lane.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned long long u64;
template <int MODE>
__global__ __launch_bounds__(256) void k(unsigned* out, unsigned seed, int iters) {
  unsigned e = seed ^ threadIdx.x, f = seed * 3 + blockIdx.x;
  u64 A = e, B = f, C = e ^ 0x5555, D = f ^ 0x3333;
  unsigned a = e, b = f, c = e + 1, d = f + 1;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if constexpr (MODE == 0)
        asm volatile("v_mad_u64_u32 %0, vcc, %4, %5, %0\nv_mad_u64_u32 %1, vcc, %5, %4, %1\nv_mad_u64_u32 %2, vcc, %4, %5, %2\nv_mad_u64_u32 %3, vcc, %5, %4, %3"
                     : "+v"(A), "+v"(B), "+v"(C), "+v"(D) : "v"(e), "v"(f) : "vcc");
      if constexpr (MODE == 1)
        asm volatile("v_mul_lo_u32 %0, %4, %0\nv_mul_lo_u32 %1, %5, %1\nv_mul_lo_u32 %2, %4, %2\nv_mul_lo_u32 %3, %5, %3" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(e), "v"(f));
      if constexpr (MODE == 2)
        asm volatile("v_mul_hi_u32 %0, %4, %0\nv_mul_hi_u32 %1, %5, %1\nv_mul_hi_u32 %2, %4, %2\nv_mul_hi_u32 %3, %5, %3" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(e), "v"(f));
      if constexpr (MODE == 3)
        asm volatile("v_mad_u32_u24 %0, %4, %0, %5\nv_mad_u32_u24 %1, %5, %1, %4\nv_mad_u32_u24 %2, %4, %2, %5\nv_mad_u32_u24 %3, %5, %3, %4" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(e), "v"(f));
      if constexpr (MODE == 4)
        asm volatile("v_mul_hi_u32_u24_e32 %0, %4, %0\nv_mul_hi_u32_u24_e32 %1, %5, %1\nv_mul_hi_u32_u24_e32 %2, %4, %2\nv_mul_hi_u32_u24_e32 %3, %5, %3" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(e), "v"(f));
      if constexpr (MODE == 5)
        asm volatile("v_lshl_add_u64 %0, %0, 0, %1\nv_lshl_add_u64 %1, %1, 0, %2\nv_lshl_add_u64 %2, %2, 0, %3\nv_lshl_add_u64 %3, %3, 0, %0" : "+v"(A), "+v"(B), "+v"(C), "+v"(D));
      if constexpr (MODE == 6)
        asm volatile("v_add_co_u32_e32 %0, vcc, %4, %0\nv_addc_co_u32_e32 %1, vcc, %5, %1, vcc\nv_add_co_u32_e32 %2, vcc, %4, %2\nv_addc_co_u32_e32 %3, vcc, %5, %3, vcc" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(e), "v"(f) : "vcc");
      if constexpr (MODE == 7)
        asm volatile("v_mov_b32_e32 %0, %4\nv_mov_b32_e32 %1, %5\nv_mov_b32_e32 %2, %4\nv_mov_b32_e32 %3, %5" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(e), "v"(f));
      if constexpr (MODE == 8)
        asm volatile("v_add3_u32 %0, %4, %5, %0\nv_add3_u32 %1, %5, %4, %1\nv_add3_u32 %2, %4, %5, %2\nv_add3_u32 %3, %5, %4, %3" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(e), "v"(f));
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = a ^ b ^ c ^ d ^ (unsigned)(A ^ B ^ C ^ D);
}
template <int M>
static void run(unsigned* out, const char* name) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int blocks = 256 * 8, iters = 2000;
  hipLaunchKernelGGL(k<M>, dim3(blocks), dim3(256), 0, 0, out, 1u, iters);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k<M>, dim3(blocks), dim3(256), 0, 0, out, 1u, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double rate = (double)blocks * 4 * iters * 16 * 4 / (ms * 1e-3);
  printf("%-34s %7.3f ms  %.3e wave-instr/s  %.2f of full rate\n", name, ms, rate, rate / 1.2288e12);
}
int main() {
  unsigned* out;
  (void)hipMalloc(&out, 256 * 8 * 256 * 4);
  run<0>(out, "v_mad_u64_u32 (VOP3b)");
  run<1>(out, "v_mul_lo_u32");
  run<2>(out, "v_mul_hi_u32");
  run<3>(out, "v_mad_u32_u24");
  run<4>(out, "v_mul_hi_u32_u24");
  run<5>(out, "v_lshl_add_u64");
  run<6>(out, "v_add_co/addc_co_u32 (VOP2)");
  run<7>(out, "v_mov_b32");
  run<8>(out, "v_add3_u32");
  return 0;
}
