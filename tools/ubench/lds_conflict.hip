// LDS access-pattern microbenchmark for gfx950: one kernel per pattern, each
// wave issuing ITER accesses of that shape.  Run under rocprofv3 --pmc
// SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS to read the conflict
// cycles per LDS instruction of each shape (the shapes k_count2c and
// k_replay_ref3 use).  Build: hipcc --offload-arch=gfx950 -O3 -o lds_conflict lds_conflict.hip
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int ITER = 4096;
typedef unsigned long long u64;
typedef unsigned v4u __attribute__((ext_vector_type(4)));

struct B32x8 {
  u64 a, b, c, d;
};

#define KERNEL(NAME, BODY)                                                      \
  __global__ __launch_bounds__(256) void NAME(unsigned* out, unsigned seed) {   \
    __shared__ __attribute__((aligned(16))) unsigned char sm[64 * 1024];        \
    const unsigned tid = threadIdx.x, lane = tid & 63;                          \
    for (unsigned i = tid; i < 64 * 1024 / 4; i += 256) ((unsigned*)sm)[i] = i; \
    __syncthreads();                                                            \
    unsigned acc = 0, x = seed ^ (tid * 0x9E3779B9u);                           \
    for (int it = 0; it < ITER; ++it) {                                         \
      BODY;                                                                     \
    }                                                                           \
    out[blockIdx.x * 256 + tid] = acc;                                          \
  }

// 1. b32 read, consecutive lanes
KERNEL(k_b32_consec, acc += ((unsigned*)sm)[(lane + it) & 16383])
// 2. b32 read, random index (table gather, replay's geo[])
KERNEL(k_b32_random, x = x * 1664525u + 1013904223u; acc += ((unsigned*)sm)[(x >> 18) & 4095])
// 3. b64 read, random index (replay's btw[])
KERNEL(k_b64_random, x = x * 1664525u + 1013904223u; acc += (unsigned)((u64*)sm)[(x >> 19) & 4095])
// 4. b128 read, 32-B records, 8 distinct records per wave (consecutive) (count2c fetch of par[pl])
KERNEL(k_b128_rec8, {
  const v4u v = ((const v4u*)sm)[2 * (((lane >> 3) + it) & 255)];
  acc += v.x + v.w;
})
// 5. b128 read, 32-B records, one per lane (stride 32 B)
KERNEL(k_b128_stride32, {
  const v4u v = ((const v4u*)sm)[2 * ((lane + it) & 255)];
  acc += v.x + v.w;
})
// 6. b128 read, consecutive 16 B per lane
KERNEL(k_b128_consec, {
  const v4u v = ((const v4u*)sm)[(lane + it) & 1023];
  acc += v.x + v.w;
})
// 7. b32 write, lanes 8 dwords apart (count2c slot writes at excl + k)
KERNEL(k_b32_write_stride8, ((unsigned*)sm)[(lane * 8 + it) & 16383] = it)
// 8. b32 write, lanes ~7.5 dwords apart (irregular)
KERNEL(k_b32_write_irreg, ((unsigned*)sm)[(((lane * 15) >> 1) + it) & 16383] = it)
// 9. b16 write consecutive (ptag[tid])
KERNEL(k_b16_write, ((unsigned short*)sm)[(lane + it) & 32767] = (unsigned short)it)
// 10. b64 read random within 256 records (count2c att[pl] for random pl, queue drains)
KERNEL(k_b64_rand256, x = x * 1664525u + 1013904223u; acc += (unsigned)((u64*)sm)[(x >> 24) & 255])
// 11. b128 read of 32-B records, random among 256 (drain: par[pl] for queued children)
KERNEL(k_b128_rand256, {
  x = x * 1664525u + 1013904223u;
  const v4u v = ((const v4u*)sm)[2 * ((x >> 24) & 255)];
  acc += v.x + v.w;
})
// 12. ds_xor b32 in the lane's own column (replay mailbox)
KERNEL(k_xor_own, atomicXor(((unsigned*)sm) + ((it & 7) * 256 + tid), 1u))

int main() {
  unsigned* out;
  hipMalloc(&out, 1024 * 256 * 4);
  void (*ks[])(unsigned*, unsigned) = {k_b32_consec, k_b32_random, k_b64_random, k_b128_rec8,  k_b128_stride32, k_b128_consec,
                                       k_b32_write_stride8, k_b32_write_irreg, k_b16_write, k_b64_rand256, k_b128_rand256, k_xor_own};
  for (auto k : ks) hipLaunchKernelGGL(k, dim3(1024), dim3(256), 0, 0, out, 7u);
  hipDeviceSynchronize();
  printf("done\n");
  return 0;
}
