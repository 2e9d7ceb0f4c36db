// fetch_calib.hip -- what FETCH_SIZE reports for k_verify_tx's access pattern.
//
// MI355X_MICROARCH.md calibrates FETCH_SIZE only for wide coalesced streaming
// reads (16 B per lane: it reports half the bytes) and says other widths are
// uncalibrated.  k_verify_tx reads its transaction strings one byte at a time
// per lane, each lane in its own 326-byte record, so one load instruction of a
// wave touches 64 different lines.  Both kernels below read the same buffer of
// n records of R bytes once:
//   k_lane_bytes   lane i sums the bytes of record i, one byte load at a time
//                  (the transaction kernel's pattern)
//   k_stream16     a grid-stride 16-B-per-lane coalesced read (the guide's
//                  calibrated pattern)
// Run under `rocprofv3 --pmc FETCH_SIZE` and compare each kernel's FETCH_SIZE
// with the buffer's byte count (printed).
//   hipcc --offload-arch=gfx950 -O3 -o build/fetch_calib tools/ubench/fetch_calib.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32;

__global__ __launch_bounds__(128) void k_lane_bytes(const unsigned char* __restrict__ buf, u32 n, u32 rec,
                                                    u32* __restrict__ out) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned char* p = buf + (size_t)i * rec;
  u32 s = 0;
  for (u32 k = 0; k < rec; ++k) s = s * 31u + p[k];
  out[i] = s;
}

__global__ __launch_bounds__(256) void k_stream16(const uint4* __restrict__ buf, size_t n16, u32* __restrict__ out) {
  u32 s = 0;
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < n16; k += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = buf[k];
    s ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));     \
      return 1;                                                        \
    }                                                                  \
  } while (0)

int main(int argc, char** argv) {
  const u32 n = argc > 1 ? (u32)std::atoi(argv[1]) : 262144u;
  const u32 rec = argc > 2 ? (u32)std::atoi(argv[2]) : 326u;
  const size_t bytes = (size_t)n * rec, padded = (bytes + 15) & ~(size_t)15;
  std::vector<unsigned char> h(padded);
  for (size_t k = 0; k < padded; ++k) h[k] = (unsigned char)(k * 2654435761u >> 13);
  unsigned char* d = nullptr;
  u32* o = nullptr;
  CK(hipMalloc(&d, padded));
  CK(hipMalloc(&o, (size_t)(n > 1024 * 256 ? n : 1024 * 256) * sizeof(u32)));
  CK(hipMemcpy(d, h.data(), padded, hipMemcpyHostToDevice));
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(k_lane_bytes, dim3((n + 127) / 128), dim3(128), 0, 0, d, n, rec, o);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k_stream16, dim3(1024), dim3(256), 0, 0, reinterpret_cast<const uint4*>(d), padded / 16, o);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
  }
  std::printf("{\"records\": %u, \"record_bytes\": %u, \"buffer_bytes\": %zu, \"buffer_kb\": %.1f}\n", n, rec, padded,
              padded / 1024.0);
  CK(hipFree(d));
  CK(hipFree(o));
  return 0;
}
