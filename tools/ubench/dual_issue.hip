// dual_issue.hip -- gfx950 VALU issue cost per instruction class, by waves per SIMD.
//
// Each wave runs 4 (or 8) independent dependency chains of ONE opcode (or a
// fixed pair of opcodes) for `iters` x 16 x 4 instructions and reads the shader
// clock (s_memtime, a scalar READ) around the loop.  Blocks of 256 threads are
// one wave per SIMD; the grid is 256 x W blocks with the LDS allocation sized
// so that at most W blocks fit a CU, so every SIMD holds W waves.  Printed per
// class and W:  SIMD cycles per wave64 instruction = wave cycles / (W x n).
// rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 over this binary gives,
// per kernel, how many quad-cycles issued two VALU instructions (dual issue).
// These costs price the instruction-mix model of tools/isa_mix.py.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define OP4(A, B, C, D) asm volatile(A "\n" B "\n" C "\n" D : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(e), "v"(f))
#define OP4C(A, B, C, D, ...) \
  asm volatile(A "\n" B "\n" C "\n" D : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(e), "v"(f) : __VA_ARGS__)
#define OP4_64(A, B, C, D) \
  asm volatile(A "\n" B "\n" C "\n" D : "+v"(A64), "+v"(B64), "+v"(C64), "+v"(D64) : "v"(e), "v"(f))

template <int MODE>
__global__ __launch_bounds__(256) void k(unsigned long long* cyc, unsigned* out, unsigned seed, int iters) {
  extern __shared__ unsigned lds[];  // only sizes the blocks per CU
  unsigned a = seed ^ threadIdx.x, b = seed * 3 + blockIdx.x, c = a ^ 0x5555, d = b ^ 0x3333, e = a + 7, f = b + 9;
  unsigned long long A64 = a, B64 = b, C64 = c, D64 = d;
  if (iters < 0) lds[threadIdx.x] = a;  // never true: keeps the allocation
  unsigned long long t0, t1;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0));
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if constexpr (MODE == 0) OP4("v_add_u32_e32 %0, %4, %0", "v_add_u32_e32 %1, %5, %1", "v_add_u32_e32 %2, %4, %2", "v_add_u32_e32 %3, %5, %3");
      if constexpr (MODE == 1) OP4("v_xor_b32_e32 %0, %4, %0", "v_and_b32_e32 %1, %5, %1", "v_or_b32_e32 %2, %4, %2", "v_xor_b32_e32 %3, %5, %3");
      if constexpr (MODE == 2) OP4("v_and_b32_e64 %0, %4, %0", "v_or_b32_e64 %1, %5, %1", "v_and_b32_e64 %2, %4, %2", "v_or_b32_e64 %3, %5, %3");
      if constexpr (MODE == 3) OP4("v_bitop3_b32 %0, %4, %5, %0 bitop3:0xf8", "v_bitop3_b32 %1, %5, %4, %1 bitop3:0xf8", "v_bitop3_b32 %2, %4, %5, %2 bitop3:0x80", "v_bitop3_b32 %3, %5, %4, %3 bitop3:0x80");
      if constexpr (MODE == 4) OP4("v_bcnt_u32_b32 %0, %4, %0", "v_bcnt_u32_b32 %1, %5, %1", "v_bcnt_u32_b32 %2, %4, %2", "v_bcnt_u32_b32 %3, %5, %3");
      if constexpr (MODE == 5) OP4_64("v_lshlrev_b64 %0, 7, %0", "v_lshlrev_b64 %1, 9, %1", "v_lshrrev_b64 %2, 7, %2", "v_lshrrev_b64 %3, 9, %3");
      if constexpr (MODE == 6) OP4("v_lshlrev_b32_e32 %0, 3, %0", "v_lshlrev_b32_e32 %1, 5, %1", "v_lshrrev_b32_e32 %2, 3, %2", "v_lshrrev_b32_e32 %3, 5, %3");
      if constexpr (MODE == 7) OP4("v_cndmask_b32_e32 %0, %0, %4, vcc", "v_cndmask_b32_e32 %1, %1, %5, vcc", "v_cndmask_b32_e32 %2, %2, %4, vcc", "v_cndmask_b32_e32 %3, %3, %5, vcc");
      if constexpr (MODE == 8) OP4("v_cndmask_b32_e64 %0, %0, %4, s[0:1]", "v_cndmask_b32_e64 %1, %1, %5, s[0:1]", "v_cndmask_b32_e64 %2, %2, %4, s[0:1]", "v_cndmask_b32_e64 %3, %3, %5, s[0:1]");
      if constexpr (MODE == 9) OP4("v_add3_u32 %0, %4, %5, %0", "v_add3_u32 %1, %5, %4, %1", "v_add3_u32 %2, %4, %5, %2", "v_add3_u32 %3, %5, %4, %3");
      if constexpr (MODE == 10) OP4("v_alignbit_b32 %0, %0, %4, 7", "v_alignbit_b32 %1, %1, %5, 9", "v_alignbit_b32 %2, %2, %4, 7", "v_alignbit_b32 %3, %3, %5, 9");
      if constexpr (MODE == 11) OP4("v_bfe_u32 %0, %0, %4, 4", "v_bfe_u32 %1, %1, %5, 4", "v_bfe_u32 %2, %2, %4, 4", "v_bfe_u32 %3, %3, %5, 4");
      if constexpr (MODE == 12) OP4("v_mov_b32_e32 %0, %4", "v_mov_b32_e32 %1, %5", "v_mov_b32_e32 %2, %4", "v_mov_b32_e32 %3, %5");
      if constexpr (MODE == 13) OP4("v_ffbl_b32_e32 %0, %0", "v_ffbh_u32_e32 %1, %1", "v_ffbl_b32_e32 %2, %2", "v_ffbh_u32_e32 %3, %3");
      if constexpr (MODE == 14) OP4("v_not_b32_e32 %0, %0", "v_not_b32_e32 %1, %1", "v_not_b32_e32 %2, %2", "v_not_b32_e32 %3, %3");
      if constexpr (MODE == 15) OP4("v_or3_b32 %0, %4, %5, %0", "v_or3_b32 %1, %5, %4, %1", "v_or3_b32 %2, %4, %5, %2", "v_or3_b32 %3, %5, %4, %3");
      if constexpr (MODE == 16) OP4("v_lshl_or_b32 %0, %0, 4, %4", "v_lshl_or_b32 %1, %1, 4, %5", "v_lshl_or_b32 %2, %2, 4, %4", "v_lshl_or_b32 %3, %3, 4, %5");
      if constexpr (MODE == 17) OP4C("v_cmp_eq_u32_e32 vcc, %0, %4", "v_add_u32_e32 %1, %5, %1", "v_cmp_lt_u32_e32 vcc, %2, %4", "v_add_u32_e32 %3, %5, %3", "vcc");
      if constexpr (MODE == 18) OP4("v_sub_u32_e32 %0, %4, %0", "v_subrev_u32_e32 %1, %5, %1", "v_sub_u32_e32 %2, %4, %2", "v_subrev_u32_e32 %3, %5, %3");
      if constexpr (MODE == 19) OP4("v_max_u32_e32 %0, %4, %0", "v_min_u32_e32 %1, %5, %1", "v_max_u32_e32 %2, %4, %2", "v_min_u32_e32 %3, %5, %3");
      // mixes within one wave: a slow op next to a fast one
      if constexpr (MODE == 20) OP4("v_bcnt_u32_b32 %0, %4, %0", "v_and_b32_e32 %1, %5, %1", "v_bcnt_u32_b32 %2, %4, %2", "v_or_b32_e32 %3, %5, %3");
      if constexpr (MODE == 21)
        asm volatile("v_lshlrev_b64 %0, 7, %0\n v_bitop3_b32 %2, %4, %5, %2 bitop3:0xf8\n v_lshrrev_b64 %1, 9, %1\n v_bitop3_b32 %3, %5, %4, %3 bitop3:0x80"
                     : "+v"(A64), "+v"(B64), "+v"(c), "+v"(d) : "v"(e), "v"(f));
      if constexpr (MODE == 22) OP4("v_mbcnt_lo_u32_b32 %0, %4, %0", "v_mbcnt_hi_u32_b32 %1, %5, %1", "v_mbcnt_lo_u32_b32 %2, %4, %2", "v_mbcnt_hi_u32_b32 %3, %5, %3");
      if constexpr (MODE == 23) OP4C("v_add_co_u32_e32 %0, vcc, %4, %0", "v_addc_co_u32_e32 %1, vcc, %5, %1, vcc", "v_add_co_u32_e32 %2, vcc, %4, %2", "v_addc_co_u32_e32 %3, vcc, %5, %3, vcc", "vcc");
      if constexpr (MODE == 24) OP4("v_lshl_add_u32 %0, %0, 2, %4", "v_lshl_add_u32 %1, %1, 2, %5", "v_lshl_add_u32 %2, %2, 2, %4", "v_lshl_add_u32 %3, %3, 2, %5");
      if constexpr (MODE == 25) OP4("v_and_or_b32 %0, %4, %5, %0", "v_and_or_b32 %1, %5, %4, %1", "v_and_or_b32 %2, %4, %5, %2", "v_and_or_b32 %3, %5, %4, %3");
      if constexpr (MODE == 26) OP4("v_perm_b32 %0, %0, %4, %5", "v_perm_b32 %1, %1, %5, %4", "v_perm_b32 %2, %2, %4, %5", "v_perm_b32 %3, %3, %5, %4");
      if constexpr (MODE == 27) OP4("v_mul_lo_u32 %0, %0, %4", "v_mul_lo_u32 %1, %1, %5", "v_mul_lo_u32 %2, %2, %4", "v_mul_lo_u32 %3, %3, %5");
      if constexpr (MODE == 28) OP4("v_xad_u32 %0, %0, %4, %5", "v_xad_u32 %1, %1, %5, %4", "v_xad_u32 %2, %2, %4, %5", "v_xad_u32 %3, %3, %5, %4");
      // selects in their real context: the mask written by a compare just before
      if constexpr (MODE == 30) OP4C("v_cmp_gt_u32_e32 vcc, %0, %4", "v_cndmask_b32_e32 %1, %1, %5, vcc", "v_cmp_gt_u32_e32 vcc, %2, %4", "v_cndmask_b32_e32 %3, %3, %5, vcc", "vcc");
      if constexpr (MODE == 31) OP4C("v_cmp_gt_u32_e64 s[2:3], %0, %4", "v_cndmask_b32_e64 %1, %1, %5, s[2:3]", "v_cmp_gt_u32_e64 s[4:5], %2, %4", "v_cndmask_b32_e64 %3, %3, %5, s[4:5]", "s2", "s3", "s4", "s5");
      if constexpr (MODE == 32) OP4C("s_mov_b64 vcc, -1", "v_cndmask_b32_e32 %1, %1, %5, vcc", "v_cndmask_b32_e32 %2, %2, %4, vcc", "v_cndmask_b32_e32 %3, %3, %5, vcc", "vcc");
      if constexpr (MODE == 29) OP4C("v_readfirstlane_b32 s2, %0", "v_add_u32_e32 %1, %5, %1", "v_readfirstlane_b32 s3, %2", "v_add_u32_e32 %3, %5, %3", "s2", "s3");
    }
  }
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1));
  const unsigned wave = (blockIdx.x * 256 + threadIdx.x) >> 6;
  if ((threadIdx.x & 63) == 0) cyc[wave] = t1 - t0;
  out[blockIdx.x * 256 + threadIdx.x] = a ^ b ^ c ^ d ^ (unsigned)(A64 ^ B64 ^ C64 ^ D64);
}

static const char* kName[] = {
    "v_add_u32_e32 (VOP2)", "v_xor/and/or_b32_e32 (VOP2)", "v_and/or_b32_e64 (VOP3 enc)", "v_bitop3_b32",
    "v_bcnt_u32_b32", "v_lshl/lshrrev_b64 (const)", "v_lshl/lshrrev_b32_e32", "v_cndmask_b32_e32 (vcc)",
    "v_cndmask_b32_e64 (sgpr)", "v_add3_u32", "v_alignbit_b32", "v_bfe_u32", "v_mov_b32_e32", "v_ffbl/ffbh_b32",
    "v_not_b32_e32", "v_or3_b32", "v_lshl_or_b32", "v_cmp_e32 + v_add_e32", "v_sub/subrev_u32_e32",
    "v_max/min_u32_e32", "v_bcnt + v_and/or (mix)", "v_lshl_b64 + v_bitop3 (mix)", "v_mbcnt_lo/hi",
    "v_add_co/addc_co_e32", "v_lshl_add_u32", "v_and_or_b32", "v_perm_b32", "v_mul_lo_u32", "v_xad_u32",
    "v_readfirstlane + v_add (mix)", "v_cmp_e32 -> v_cndmask_b32_e32 (vcc)", "v_cmp_e64 -> v_cndmask_b32_e64 (sgpr)",
    "s_mov vcc -> 3x v_cndmask_b32_e32"};
constexpr int kModes = 33;

template <int M>
static void run(int W, unsigned long long* d_cyc, unsigned* out, unsigned long long* h_cyc, int lds_bytes) {
  const int blocks = 256 * W, iters = 2000;
  (void)hipFuncSetAttribute((const void*)k<M>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
  hipLaunchKernelGGL(k<M>, dim3(blocks), dim3(256), lds_bytes, 0, d_cyc, out, 1u, iters);
  (void)hipDeviceSynchronize();
  (void)hipMemcpy(h_cyc, d_cyc, sizeof(unsigned long long) * blocks * 4, hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < blocks * 4; ++i) s += (double)h_cyc[i];
  const double wave_cyc = s / (blocks * 4);
  const double n = (double)iters * 16 * 4;
  printf("%-32s W=%d  %6.2f SIMD cycles/instr  (wave: %6.2f cycles/instr)\n", kName[M], W, wave_cyc / (W * n),
         wave_cyc / n);
}

template <int M>
static void run_all(unsigned long long* d_cyc, unsigned* out, unsigned long long* h_cyc) {
  // LDS per block so that at most W blocks fit a CU's 160 KB
  for (int W : {1, 2, 4, 8}) run<M>(W, d_cyc, out, h_cyc, 160 * 1024 / W - 1024);
  if constexpr (M + 1 < kModes) run_all<M + 1>(d_cyc, out, h_cyc);
}

int main() {
  unsigned long long *d_cyc, *h_cyc;
  unsigned* out;
  (void)hipMalloc(&d_cyc, sizeof(unsigned long long) * 256 * 8 * 4);
  (void)hipMalloc(&out, 256 * 8 * 256 * 4);
  h_cyc = (unsigned long long*)malloc(sizeof(unsigned long long) * 256 * 8 * 4);
  run_all<0>(d_cyc, out, h_cyc);
  return 0;
}
