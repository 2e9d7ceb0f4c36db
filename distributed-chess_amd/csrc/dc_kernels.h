// dc_kernels.h -- launch wrappers of dc_kernels.hip (host side of the engine).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

namespace dc {

// A/B knobs (kernel-variant and timing experiments) are compiled only into
// the A/B build (`make ab` -> libdchess_ab.so, -DDC_AB_KNOBS): the shipped
// libdchess.so reads no environment variable that selects a kernel or
// changes a result, so a replica's environment cannot alter its verdicts.
inline const char* ab_env(const char* name) {
#ifdef DC_AB_KNOBS
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

typedef unsigned long long u64;
typedef uint32_t u32;

}  // namespace dc

// Basic-block execution counts (tools/bbprof.py, measurement builds only:
// -DDC_BBPROF).  The counter array is written only by instrumentation that
// tools/bbprof.py inserts into one kernel's assembly; the product never
// defines DC_BBPROF.
#ifdef DC_BBPROF
#define DC_BBPROF_DEFINE(NAME)                                                                            \
  __device__ unsigned long long dc_bbprof_##NAME[8192];                                                 \
  extern "C" __attribute__((visibility("default"))) int dc_ab_bbprof_##NAME(unsigned long long* out,    \
                                                                           int reset) {                 \
    if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(dc_bbprof_##NAME), sizeof(dc_bbprof_##NAME), 0,       \
                                   hipMemcpyDeviceToHost) != hipSuccess)                                  \
      return -1;                                                                                          \
    if (reset) {                                                                                          \
      static unsigned long long zero[8192];                                                               \
      if (hipMemcpyToSymbol(HIP_SYMBOL(dc_bbprof_##NAME), zero, sizeof(zero), 0, hipMemcpyHostToDevice) !=  \
          hipSuccess)                                                                                     \
        return -1;                                                                                        \
    }                                                                                                     \
    return 0;                                                                                             \
  }
#else
#define DC_BBPROF_DEFINE(NAME)
#endif

namespace dc {

// One position: quad-bitboard of include/dchess.h (b0 black, b1..b3 kind bits).
struct Board {
  u64 b0, b1, b2, b3;
};

// Device image of dc_pos (include/dchess.h), 40 bytes.
struct DevPos {
  u64 bb[4];
  uint8_t stm, castle;
  int8_t ep;
  uint8_t r0;
  uint32_t r1;
};
static_assert(sizeof(DevPos) == 40, "dc_pos layout");

// Startpos quad-bitboard (chess.rs:383-434): b0 black, b1..b3 kind bits.
constexpr u64 kStartB0 = 0xFFFF000000000000ull;
constexpr u64 kStartB1 = 0x3CFF00000000FF3Cull;
constexpr u64 kStartB2 = 0xDB000000000000DBull;
constexpr u64 kStartB3 = 0xAD000000000000ADull;

template <class B>
__host__ __device__ inline void startpos_board(B& b) {
  b.b0 = kStartB0;
  b.b1 = kStartB1;
  b.b2 = kStartB2;
  b.b3 = kStartB3;
}

hipError_t launch_validate_ref(hipStream_t st, const DevPos* pos, const uint16_t* moves, u32 n, uint8_t* out, u32* done = nullptr, u32 seq = 0);

// ---- the live validator (dc_live_validator): one resident wave that serves
// small validate / apply calls from a pinned, coherent mailbox, so the live
// n = 1 call of a voting replica costs a host store and a poll, not a launch.
// Every mailbox dword is stamp << 16 | payload: a dword is written and read
// whole, so a reader accepts a request (or a response) only when every dword
// it needs carries the current stamp -- no fence orders one against another.
// Stamps run 1..65535 (stamp(seq) = seq % 65535 + 1); the host zeroes the
// request area every kLiveClearEvery requests and the response words before
// each request, so a stale dword never carries the current stamp.
// Request: word 0 = stamp | n (1..64) | apply << 7 | fide << 8; then
// kLiveFields fields field-major (word 1 + k * n + e): 16 bitboard half-words,
// stm | castle << 8, (u8)ep, the move.  Response: word k * n + e; k = 0 the
// verdict | info << 8, k = 1..18 (apply) the position's fields.
constexpr u32 kLiveMax = 64, kLiveFields = 19;
constexpr u32 kLiveReqWords = 1 + kLiveFields * kLiveMax;
constexpr u32 kLiveClearEvery = 16384;
struct alignas(64) LiveBox {
  u32 req[kLiveReqWords];
  alignas(64) u32 resp[kLiveFields * kLiveMax];
  alignas(64) u32 state;  // device -> host: 2 once the wave takes no more requests
  alignas(64) u32 ctl;    // host -> device: 1 asks the wave to stop
};
__host__ __device__ inline u32 live_stamp(u32 seq) { return seq % 65535u + 1u; }
// lease_ticks: the wave stops after that many wall-clock ticks (100 MHz) with
// no request; `seq` = requests already served (the first one it takes is seq + 1)
hipError_t launch_live(hipStream_t st, LiveBox* box, u32 seq, u64 lease_ticks);
hipError_t launch_apply_ref(hipStream_t st, DevPos* pos, const uint16_t* moves, u32 n, uint8_t* verdicts,
                            uint8_t* info, u32* done = nullptr, u32 seq = 0);
// stats[5] = validated, accepted, rejected, digest sum, digest xor; partial has
// replay_partials(n_games) x 5 u64 of scratch.  *host_written: the five
// counters were also stored into pinned `stats_host` (valid once the stream is
// synchronised; no copy needed).
u32 replay_partials(u32 n_games);
hipError_t launch_replay_ref(hipStream_t st, const Board& start, u32 stm0, const uint16_t* moves, u32 n_games,
                             u32 n_plies, u64* bitmap, u64* digests, u64* stats, u64* partial, u64* stats_host,
                             bool* host_written, uint8_t* info = nullptr, Board* boards = nullptr);
// (info != nullptr: the per-ply info form; boards != nullptr then also
// receives every game's final board, the state hash's board JSON)
hipError_t launch_gen_games_ref(hipStream_t st, u64 seed, u64 first_game, u32 n_games, u32 n_plies, u32 noise,
                                uint16_t* out);
}  // namespace dc
