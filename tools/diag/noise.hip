// Co-resident "noise" waves for the DESIGN.md §3.6 fault study: a kernel that
// keeps waves busy on every CU for a fixed wall time, on its own stream, while
// another kernel (the victim) runs beside it.  Each kind exercises one part of
// the CU, so a victim whose result changes only beside one kind points at the
// resource the two waves share.
//   hipcc --offload-arch=gfx950 -O3 -fPIC -shared -o tools/diag/libnoise.so tools/diag/noise.hip
//   kinds: 0 VALU pairable (v_xor/v_add)   1 VALU single-issue (64-bit shifts, v_bcnt)
//          2 LDS reads/writes              3 idle waves (s_sleep)
//          4 global loads (L2-resident)    5 SALU only
//   single opcodes (inline asm, four independent chains):
//          6 v_lshlrev_b64/v_lshrrev_b64   7 v_bcnt_u32_b32   8 v_mov_b64
//          9 v_cmp_ne_u64_e64 (to SGPRs)   10 v_cndmask_b32_e64   11 v_add3_u32
//          12 v_lshlrev_b32   13 v_mad_u64_u32   14 v_lshl_add_u64   15 v_alignbit_b32
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memrealtime(); }  // 100 MHz

template <int KIND>
__global__ __launch_bounds__(256) void k_noise(uint64_t ticks, uint32_t* sink, const uint32_t* src) {
  __shared__ uint32_t lds[4096];
  const uint64_t t0 = now();
  uint32_t a = threadIdx.x * 2654435761u, b = blockIdx.x + 1, c = a ^ 0x9E3779B9u, d = b * 7u;
  uint64_t x = ((uint64_t)a << 32) | b;
  if (KIND == 2)
    for (int i = threadIdx.x; i < 4096; i += 256) lds[i] = i * 17u;
  __syncthreads();
  while (now() - t0 < ticks) {
#pragma unroll 1
    for (int it = 0; it < 64; ++it) {
      if constexpr (KIND == 0) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          a ^= b; b += c; c ^= d; d += a;
        }
      } else if constexpr (KIND == 1) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          x = (x << 7) ^ (x >> 9) ^ (uint64_t)__popcll(x);
        }
      } else if constexpr (KIND == 2) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint32_t j = (a + k * 257u) & 4095u;
          a += lds[j];
          lds[(j + 64) & 4095u] = a;
        }
      } else if constexpr (KIND == 3) {
        __builtin_amdgcn_s_sleep(8);
      } else if constexpr (KIND == 4) {
#pragma unroll
        for (int k = 0; k < 4; ++k) a += src[(a + threadIdx.x + k * 4096u) & ((1u << 20) - 1)];
      } else if constexpr (KIND >= 6) {
        uint64_t y = x ^ 0x5555, z = x + 77, w = x * 3;
        uint32_t e = a, f = b, g = c, h = d;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if constexpr (KIND == 6) {
            asm volatile("v_lshlrev_b64 %0, 7, %0\n\tv_lshrrev_b64 %1, 9, %1\n\tv_lshlrev_b64 %2, 3, %2\n\tv_lshrrev_b64 %3, 5, %3"
                         : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
          } else if constexpr (KIND == 7) {
            asm volatile("v_bcnt_u32_b32 %0, %0, %1\n\tv_bcnt_u32_b32 %1, %1, %2\n\tv_bcnt_u32_b32 %2, %2, %3\n\tv_bcnt_u32_b32 %3, %3, %0"
                         : "+v"(e), "+v"(f), "+v"(g), "+v"(h));
          } else if constexpr (KIND == 8) {
            asm volatile("v_mov_b64 %0, %1\n\tv_mov_b64 %1, %2\n\tv_mov_b64 %2, %3\n\tv_mov_b64 %3, %0"
                         : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
          } else if constexpr (KIND == 9) {
            uint64_t m0, m1, m2, m3;
            asm volatile("v_cmp_ne_u64_e64 %0, 0, %4\n\tv_cmp_ne_u64_e64 %1, 0, %5\n\tv_cmp_ne_u64_e64 %2, 0, %6\n\tv_cmp_ne_u64_e64 %3, 0, %7"
                         : "=s"(m0), "=s"(m1), "=s"(m2), "=s"(m3) : "v"(x), "v"(y), "v"(z), "v"(w));
            x += m0 ^ m1 ^ m2 ^ m3;
          } else if constexpr (KIND == 10) {
            const uint64_t m = __builtin_amdgcn_read_exec() ^ (uint64_t)b;
            asm volatile("v_cndmask_b32_e64 %0, %0, %1, %4\n\tv_cndmask_b32_e64 %1, %1, %2, %4\n\tv_cndmask_b32_e64 %2, %2, %3, %4\n\tv_cndmask_b32_e64 %3, %3, %0, %4"
                         : "+v"(e), "+v"(f), "+v"(g), "+v"(h) : "s"(m));
          } else if constexpr (KIND == 11) {
            asm volatile("v_add3_u32 %0, %0, %1, %2\n\tv_add3_u32 %1, %1, %2, %3\n\tv_add3_u32 %2, %2, %3, %0\n\tv_add3_u32 %3, %3, %0, %1"
                         : "+v"(e), "+v"(f), "+v"(g), "+v"(h));
          } else if constexpr (KIND == 12) {
            asm volatile("v_lshlrev_b32 %0, 7, %0\n\tv_lshlrev_b32 %1, 9, %1\n\tv_lshlrev_b32 %2, 3, %2\n\tv_lshlrev_b32 %3, 5, %3"
                         : "+v"(e), "+v"(f), "+v"(g), "+v"(h));
          } else if constexpr (KIND == 13) {
            uint64_t c0;
            asm volatile("v_mad_u64_u32 %0, %4, %5, %6, %0\n\tv_mad_u64_u32 %1, %4, %6, %7, %1\n\tv_mad_u64_u32 %2, %4, %7, %8, %2\n\tv_mad_u64_u32 %3, %4, %8, %5, %3"
                         : "+v"(x), "+v"(y), "+v"(z), "+v"(w), "=s"(c0) : "v"(e), "v"(f), "v"(g), "v"(h));
          } else if constexpr (KIND == 14) {
            asm volatile("v_lshl_add_u64 %0, %0, 1, %1\n\tv_lshl_add_u64 %1, %1, 2, %2\n\tv_lshl_add_u64 %2, %2, 3, %3\n\tv_lshl_add_u64 %3, %3, 1, %0"
                         : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
          } else {
            asm volatile("v_alignbit_b32 %0, %0, %1, 7\n\tv_alignbit_b32 %1, %1, %2, 9\n\tv_alignbit_b32 %2, %2, %3, 3\n\tv_alignbit_b32 %3, %3, %0, 5"
                         : "+v"(e), "+v"(f), "+v"(g), "+v"(h));
          }
        }
        x ^= y ^ z ^ w;
        a ^= e ^ f ^ g ^ h;
      } else {
        // SALU only: a scalar loop the compiler cannot fold
        uint32_t s = __builtin_amdgcn_readfirstlane(b);
#pragma unroll
        for (int k = 0; k < 16; ++k) s = s * 1664525u + 1013904223u;
        b = __builtin_amdgcn_readfirstlane(s) | 1u;
      }
    }
  }
  if ((a ^ b ^ c ^ d ^ (uint32_t)x) == 0x12345678u) sink[blockIdx.x] = a;  // keeps the work live
}

hipStream_t g_stream = nullptr;
uint32_t* g_sink = nullptr;
uint32_t* g_src = nullptr;

}  // namespace

extern "C" int noise_start(int kind, int blocks, double ms) {
  if (!g_stream && hipStreamCreateWithFlags(&g_stream, hipStreamNonBlocking) != hipSuccess) return -1;
  if (!g_sink && hipMalloc(&g_sink, 4u << 20) != hipSuccess) return -2;
  if (!g_src && hipMalloc(&g_src, 4u << 20) != hipSuccess) return -3;
  const uint64_t ticks = (uint64_t)(ms * 1e5);
  switch (kind) {
    case 0: hipLaunchKernelGGL(k_noise<0>, dim3(blocks), dim3(256), 0, g_stream, ticks, g_sink, g_src); break;
    case 1: hipLaunchKernelGGL(k_noise<1>, dim3(blocks), dim3(256), 0, g_stream, ticks, g_sink, g_src); break;
    case 2: hipLaunchKernelGGL(k_noise<2>, dim3(blocks), dim3(256), 0, g_stream, ticks, g_sink, g_src); break;
    case 3: hipLaunchKernelGGL(k_noise<3>, dim3(blocks), dim3(256), 0, g_stream, ticks, g_sink, g_src); break;
    case 4: hipLaunchKernelGGL(k_noise<4>, dim3(blocks), dim3(256), 0, g_stream, ticks, g_sink, g_src); break;
    case 5: hipLaunchKernelGGL(k_noise<5>, dim3(blocks), dim3(256), 0, g_stream, ticks, g_sink, g_src); break;
#define DC_NOISE_CASE(K) \
    case K: hipLaunchKernelGGL(k_noise<K>, dim3(blocks), dim3(256), 0, g_stream, ticks, g_sink, g_src); break;
    DC_NOISE_CASE(6) DC_NOISE_CASE(7) DC_NOISE_CASE(8) DC_NOISE_CASE(9) DC_NOISE_CASE(10)
    DC_NOISE_CASE(11) DC_NOISE_CASE(12) DC_NOISE_CASE(13) DC_NOISE_CASE(14) DC_NOISE_CASE(15)
    default: return -4;
  }
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" int noise_wait() { return g_stream && hipStreamSynchronize(g_stream) == hipSuccess ? 0 : -1; }
