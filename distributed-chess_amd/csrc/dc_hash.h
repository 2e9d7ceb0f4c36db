// dc_hash.h -- launch wrapper of dc_hash.hip (consensus state hash of replayed games).
#pragma once
#include "dc_kernels.h"

namespace dc {
// hashes[32 g] = keccak256(serde_json(final GameState of game g)); names and the
// start history JSON-escaped, names_off[2 n_games + 1] (white_g, black_g pairs).
hipError_t launch_state_hash_ref(hipStream_t st, const Board& start, u32 stm0, const uint16_t* moves, u32 n_games,
                                 u32 n_plies, const char* hist, u32 hist_len, u32 hist_tokens, const char* names,
                                 const u32* names_off, const uint8_t* info, uint8_t* out,
                                 const Board* final_boards = nullptr, u32 bcd_max = 10000000u);
// (final_boards, with info: every game's final board from the replay kernel's
// info pass, so the hash kernel makes no move itself; bcd_max <= 10^7: move
// numbers below it are kept as 32-bit BCD, else divided)
// serde_json escaping of n_str raw UTF-8 strings names[off[i] .. off[i+1]) on
// the device, in two steps so the host can size the output in between:
//   len_scan: esc64[i] = base + escaped length of strings 0..i-1 (i <= n_str;
//             esc64[n_str] = the end); lens[n_str + 1] and tmp
//             (escape_scan_tmp_bytes) are scratch
//   write:    out + esc64[i] <- string i escaped; out_off[i] = (u32)esc64[i]
size_t escape_scan_tmp_bytes(u32 n_str);
// *flag = 1 if any name byte needs an escape or an offset decreases (else the
// raw names and offsets serve as the escaped ones)
hipError_t launch_names_plain(hipStream_t st, const char* names, const u32* off, u32 n_str, u32* flag);
hipError_t launch_escape_len_scan(hipStream_t st, const char* names, const u32* off, u32 n_str, u64 base, u32* lens,
                                  void* tmp, size_t tmp_bytes, u64* esc64);
hipError_t launch_escape_write(hipStream_t st, const char* names, const u32* off, u32 n_str, const u64* esc64,
                               u32* out_off, char* out);
}  // namespace dc
