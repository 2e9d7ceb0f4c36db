// dc_fide.h -- launch wrappers of the RULES_FIDE kernels (defined in dc_moves.hip).
#pragma once
#include "dc_kernels.h"

namespace dc {

// Per-node FIDE state beside the quad-bitboard: castle rights (bits 0-3) and
// en-passant target (bits 4-9 square, bit 10 valid).
__host__ __device__ inline uint16_t pack_meta(uint8_t castle, int8_t ep) {
  return (uint16_t)((castle & 15) | (ep >= 0 && ep < 64 ? (((unsigned)ep << 4) | 0x400u) : 0u));
}

hipError_t launch_validate_fide(hipStream_t st, const DevPos* pos, const uint16_t* moves, u32 n, uint8_t* out, u32* done = nullptr, u32 seq = 0);
hipError_t launch_apply_fide(hipStream_t st, DevPos* pos, const uint16_t* moves, u32 n, uint8_t* verdicts,
                             uint8_t* info, u32* done = nullptr, u32 seq = 0);
hipError_t launch_replay_fide(hipStream_t st, const DevPos& start, const uint16_t* moves, u32 n_games, u32 n_plies,
                              u64* bitmap, u64* digests, u64* stats, u64* partial);
hipError_t launch_gen_games_fide(hipStream_t st, u64 seed, u64 first_game, u32 n_games, u32 n_plies, u32 noise,
                                 uint16_t* out);
}  // namespace dc
