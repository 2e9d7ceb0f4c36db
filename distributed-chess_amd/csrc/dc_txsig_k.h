// dc_txsig_k.h -- launch wrappers of dc_txsig.hip (batched transaction-signature check).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dc_secp.h"

namespace dc {
// gtab[256 i + j] = j 2^(8 i) G, secp::kGTabEntries entries
hipError_t launch_secp_gtab(hipStream_t st, secp::Ge* gtab);
// Per transaction i: strings[off[4i] .. off[4i+4]) = white, black, signature
// hex, pub_key hex; actions[4i .. 4i+4) = from.x, from.y, to.x, to.y;
// turns[i] (optional) = the game's turn for the owner check, -1 to skip.
hipError_t launch_verify_tx(hipStream_t st, const char* strings, const uint32_t* off, const uint32_t* actions,
                            const int8_t* turns, uint32_t n, const secp::Ge* gtab, uint8_t* verdicts);
}  // namespace dc
