// dc_txsig.hip -- batched transaction-signature check on gfx950.
//
//   k_secp_gtab   one lane per G-table entry: j 2^(8 i) G in affine form
//                 (built once per context, 512 KB)
//   k_verify_tx   one lane per Transaction: serde_json message -> SHA-256 ->
//                 hex/parse of signature and public key -> ECDSA verify
//                 (libsecp256k1 0.7.1 semantics) -> optional owner check
//
// What every replica runs per transaction besides the move check
// (App::validate_signature, core/src/consensus/hotstuff.rs:168-208, called by
// is_valid_tx at :139); SURVEY §8f row 2.  The per-lane body is
// dc::secp::check_tx (dc_txsig.h), shared with the host unit test.
//
// Cost model: ~2.7k field multiplications per transaction (GLV: 128 doublings
// and 66 Jacobian additions for u2 Q, 32 mixed additions from the G table for
// u1 G, the sliding-window s^-1 mod n and, for compressed keys, a square
// root); all integer VALU work (Comba v_mad_u64_u32 chains, dc_secp.h), no MFMA.
#include <hip/hip_runtime.h>

#include "dc_kernels.h"
#include "dc_txsig.h"
#include "dc_txsig_k.h"

namespace dc {

constexpr u32 kTxThreads = 128;
#ifndef DC_TX_MINW
#define DC_TX_MINW 2  // waves per SIMD: 2 (248 VGPRs) is spill-free; 3 (168) spilled 452 B/lane
#endif

__global__ __launch_bounds__(256) void k_secp_gtab(secp::Ge* __restrict__ gtab) {
  const int k = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (k >= secp::kGTabEntries) return;
  secp::Ge e;
  secp::gtab_entry(e, k >> 8, k & 255);
  gtab[k] = e;
}

__global__ __launch_bounds__(kTxThreads, DC_TX_MINW) void k_verify_tx(const char* __restrict__ strings, const u32* __restrict__ off,
                                                          const u32* __restrict__ actions,
                                                          const int8_t* __restrict__ turns, u32 n,
                                                          const secp::Ge* __restrict__ gtab,
                                                          uint8_t* __restrict__ verdicts) {
  __shared__ __attribute__((aligned(16))) uint8_t blk[16][kTxThreads][4];  // SHA-256 blocks, dword-major (BlkRef)
  const u32 i = blockIdx.x * kTxThreads + threadIdx.x;
  if (i >= n) return;
  const size_t b = (size_t)4 * i;
  const u32 o0 = off[b], o1 = off[b + 1], o2 = off[b + 2], o3 = off[b + 3], o4 = off[b + 4];
  const u32 act[4] = {actions[b], actions[b + 1], actions[b + 2], actions[b + 3]};
  const int turn = turns ? (int)turns[i] : -1;
  // The owner comparison (is_valid_tx, hotstuff.rs:141-148) is made here,
  // before the message hash, and applied after check_tx (which then skips
  // it): check_tx made it after the ~2.7k-multiplication verify, by which time
  // the key's and the name's lines had left the caches, so both strings were
  // fetched from HBM twice.  A bad signature still outranks a wrong owner.
  // The bit waits in LDS (a VGPR live across the verify spills at the 248-VGPR
  // budget).
  __shared__ uint8_t own_bit[kTxThreads];
  {
    const char* pk = strings + o3;
    const u32 pl = o4 - o3;
    own_bit[threadIdx.x] =
        turn < 0 ? 1 : (turn == 0 ? secp::str_eq(pk, pl, strings + o0, o1 - o0) : secp::str_eq(pk, pl, strings + o1, o2 - o1));
  }
  int skip = -1;  // check_tx's own owner branch, kept but never taken: with a
  asm volatile("" : "+v"(skip));  // constant -1 folded in, its body spilled 344 B
  u32 v = secp::check_tx(strings + o0, o1 - o0, strings + o1, o2 - o1, act, strings + o2, o3 - o2, strings + o3, o4 - o3,
                         skip, gtab, secp::BlkRef{&blk[0][threadIdx.x][0], kTxThreads * 4});
  if (v == secp::SIG_OK && !*(volatile uint8_t*)&own_bit[threadIdx.x]) v = secp::SIG_WRONG_OWNER;
  verdicts[i] = (uint8_t)v;
}

hipError_t launch_secp_gtab(hipStream_t st, secp::Ge* gtab) {
  hipLaunchKernelGGL(k_secp_gtab, dim3((secp::kGTabEntries + 255) / 256), dim3(256), 0, st, gtab);
  return hipGetLastError();
}

hipError_t launch_verify_tx(hipStream_t st, const char* strings, const u32* off, const u32* actions,
                            const int8_t* turns, u32 n, const secp::Ge* gtab, uint8_t* verdicts) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_verify_tx, dim3((n + kTxThreads - 1) / kTxThreads), dim3(kTxThreads), 0, st, strings, off,
                     actions, turns, n, gtab, verdicts);
  return hipGetLastError();
}

}  // namespace dc
