// dc_hash.h -- launch wrapper of dc_hash.hip (consensus state hash of replayed games).
#pragma once
#include "dc_kernels.h"

namespace dc {
// hashes[32 g] = keccak256(serde_json(final GameState of game g)); names and the
// start history JSON-escaped, names_off[2 n_games + 1] (white_g, black_g pairs).
hipError_t launch_state_hash_ref(hipStream_t st, const Board& start, u32 stm0, const uint16_t* moves, u32 n_games,
                                 u32 n_plies, const char* hist, u32 hist_len, u32 hist_tokens, const char* names,
                                 const u32* names_off, uint8_t* out);
}  // namespace dc
