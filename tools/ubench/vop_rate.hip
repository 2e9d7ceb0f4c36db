// Micro-benchmark 2: VOP2 vs VOP3 encodings of the same op, and operand counts.
#include <hip/hip_runtime.h>
#include <cstdio>
#define OP4(A, B, C, D) asm volatile(A "\n" B "\n" C "\n" D : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(e), "v"(f))
template <int MODE>
__global__ __launch_bounds__(256) void k(unsigned* out, unsigned seed, int iters) {
  unsigned a = seed ^ threadIdx.x, b = seed * 3 + blockIdx.x, c = a ^ 0x5555, d = b ^ 0x3333, e = a + 7, f = b + 9;
  unsigned long long A = a, B = b, C = c, D = d;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if constexpr (MODE == 0) OP4("v_and_b32_e32 %0, %4, %0", "v_and_b32_e32 %1, %5, %1", "v_or_b32_e32 %2, %4, %2", "v_or_b32_e32 %3, %5, %3");
      if constexpr (MODE == 1) OP4("v_and_b32_e64 %0, %4, %0", "v_and_b32_e64 %1, %5, %1", "v_or_b32_e64 %2, %4, %2", "v_or_b32_e64 %3, %5, %3");
      if constexpr (MODE == 2) OP4("v_bcnt_u32_b32 %0, %4, %0", "v_bcnt_u32_b32 %1, %5, %1", "v_bcnt_u32_b32 %2, %4, %2", "v_bcnt_u32_b32 %3, %5, %3");
      if constexpr (MODE == 3) OP4("v_add3_u32 %0, %4, %5, %0", "v_add3_u32 %1, %5, %4, %1", "v_add3_u32 %2, %4, %5, %2", "v_add3_u32 %3, %5, %4, %3");
      if constexpr (MODE == 4) OP4("v_lshlrev_b32_e32 %0, 3, %0", "v_lshlrev_b32_e32 %1, 5, %1", "v_lshrrev_b32_e32 %2, 3, %2", "v_lshrrev_b32_e32 %3, 5, %3");
      if constexpr (MODE == 5) OP4("v_bitop3_b32 %0, %4, %5, %0 bitop3:0xf8", "v_bitop3_b32 %1, %5, %4, %1 bitop3:0xf8", "v_bitop3_b32 %2, %4, %5, %2 bitop3:0x80", "v_bitop3_b32 %3, %5, %4, %3 bitop3:0x80");
      if constexpr (MODE == 6) OP4("v_add_u32_e32 %0, %4, %0", "v_add_u32_e32 %1, %5, %1", "v_sub_u32_e32 %2, %4, %2", "v_xor_b32_e32 %3, %5, %3");
      if constexpr (MODE == 7) OP4("v_ffbl_b32_e32 %0, %0", "v_ffbh_u32_e32 %1, %1", "v_ffbl_b32_e32 %2, %2", "v_not_b32_e32 %3, %3");
      if constexpr (MODE == 8) OP4("v_and_or_b32 %0, %4, %5, %0", "v_and_or_b32 %1, %5, %4, %1", "v_and_or_b32 %2, %4, %5, %2", "v_and_or_b32 %3, %5, %4, %3");
      if constexpr (MODE == 9) OP4("v_bfe_u32 %0, %0, %4, 4", "v_bfe_u32 %1, %1, %5, 4", "v_bfe_u32 %2, %2, %4, 4", "v_bfe_u32 %3, %3, %5, 4");
      if constexpr (MODE == 10) OP4("v_lshl_or_b32 %0, %0, 4, %4", "v_lshl_or_b32 %1, %1, 4, %5", "v_lshl_or_b32 %2, %2, 4, %4", "v_lshl_or_b32 %3, %3, 4, %5");
      if constexpr (MODE == 11)
        asm volatile("v_lshlrev_b64 %0, %4, %0\nv_lshlrev_b64 %1, %5, %1\nv_lshlrev_b64 %2, %4, %2\nv_lshlrev_b64 %3, %5, %3"
                     : "+v"(A), "+v"(B), "+v"(C), "+v"(D) : "v"(e), "v"(f));
      if constexpr (MODE == 12) OP4("v_cndmask_b32_e64 %0, %0, %4, s[0:1]", "v_cndmask_b32_e64 %1, %1, %5, s[0:1]", "v_cndmask_b32_e64 %2, %2, %4, s[0:1]", "v_cndmask_b32_e64 %3, %3, %5, s[0:1]");
      if constexpr (MODE == 13) OP4("v_perm_b32 %0, %0, %4, %5", "v_perm_b32 %1, %1, %5, %4", "v_perm_b32 %2, %2, %4, %5", "v_perm_b32 %3, %3, %5, %4");
      if constexpr (MODE == 14) OP4("v_lshl_add_u32 %0, %0, 2, %4", "v_lshl_add_u32 %1, %1, 2, %5", "v_lshl_add_u32 %2, %2, 2, %4", "v_lshl_add_u32 %3, %3, 2, %5");
      if constexpr (MODE == 15) OP4("v_pk_add_u16 %0, %0, %4", "v_pk_add_u16 %1, %1, %5", "v_pk_add_u16 %2, %2, %4", "v_pk_add_u16 %3, %3, %5");
      if constexpr (MODE == 16) OP4("v_mad_u32_u24 %0, %0, %4, %5", "v_mad_u32_u24 %1, %1, %5, %4", "v_mad_u32_u24 %2, %2, %4, %5", "v_mad_u32_u24 %3, %3, %5, %4");
      if constexpr (MODE == 17) OP4("v_xor_b32_e64 %0, %4, %0", "v_lshlrev_b32_e64 %1, 3, %1", "v_xor_b32_e64 %2, %4, %2", "v_lshlrev_b32_e64 %3, 5, %3");
      if constexpr (MODE == 18) OP4("v_alignbit_b32 %0, %0, %4, %5", "v_alignbit_b32 %1, %1, %5, %4", "v_alignbit_b32 %2, %2, %4, %5", "v_alignbit_b32 %3, %3, %5, %4");
      if constexpr (MODE == 19) OP4("v_mov_b32_e32 %0, %4", "v_mov_b32_e32 %1, %5", "v_mov_b32_e32 %2, %4", "v_mov_b32_e32 %3, %5");
      if constexpr (MODE == 20) OP4("v_mul_lo_u32 %0, %0, %4", "v_mul_lo_u32 %1, %1, %5", "v_mul_lo_u32 %2, %2, %4", "v_mul_lo_u32 %3, %3, %5");
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = a ^ b ^ c ^ d ^ (unsigned)(A ^ B ^ C ^ D);
}
template <int M>
static void run(unsigned* out, const char* name) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int blocks = 256 * 8, iters = 4000;
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
  run<0>(out, "v_and/or_b32_e32 (VOP2)");
  run<1>(out, "v_and/or_b32_e64 (VOP3 encoding)");
  run<2>(out, "v_bcnt_u32_b32 (VOP3)");
  run<3>(out, "v_add3_u32 (VOP3, 3 src)");
  run<4>(out, "v_lshl/lshrrev_b32_e32 (VOP2)");
  run<5>(out, "v_bitop3_b32 (VOP3, 3 src)");
  run<6>(out, "v_add/sub/xor_e32 (VOP2)");
  run<7>(out, "v_ffbl/ffbh/not_e32 (VOP1)");
  run<8>(out, "v_and_or_b32 (VOP3, 3 src)");
  run<9>(out, "v_bfe_u32 (VOP3)");
  run<10>(out, "v_lshl_or_b32 (VOP3, 3 src)");
  run<11>(out, "v_lshlrev_b64 (64-bit, counted x1)");
  run<12>(out, "v_cndmask_b32_e64 (SGPR mask)");
  run<13>(out, "v_perm_b32");
  run<14>(out, "v_lshl_add_u32");
  run<15>(out, "v_pk_add_u16");
  run<16>(out, "v_mad_u32_u24");
  run<17>(out, "xor / lshlrev mix (VOP3)");
  run<18>(out, "v_alignbit_b32");
  run<19>(out, "v_mov_b32");
  run<20>(out, "v_mul_lo_u32");
  return 0;
}
