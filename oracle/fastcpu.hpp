// oracle/fastcpu.hpp -- TEST INFRASTRUCTURE ONLY (second, faster oracle).
//
// A mailbox (8x8 array, direction walks) chess engine with two rule sets:
//   RULES_REF  -- the reference validator's geometry-only rules
//                 (/root/reference/core/src/chess.rs:199-360);
//   RULES_FIDE -- standard chess (castling, en passant, promotion, no self-check),
//                 pinned by the published perft tables.
// It is deliberately a different algorithm from the HIP kernels (which are
// set-wise bitboard code) so the two cross-check each other.  RULES_REF is
// checked for equivalence against refcpu (the literal restatement) over all
// 4096 (from,to) pairs of random positions in tests/test_oracle.py.
// Used only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline.
#pragma once
#include <cstdint>
#include <vector>

namespace fastcpu {

enum Rules : uint8_t { RULES_REF = 0, RULES_FIDE = 1 };
enum Kind : int8_t { P = 0, N = 1, B = 2, R = 3, Q = 4, K = 5, X = 6 };
enum Verdict : uint8_t { V_OK = 0, V_NO_PIECE = 1, V_WRONG_TURN = 2, V_ILLEGAL = 3, V_OOR = 4 };

// Castling bits (FIDE only).
enum : uint8_t { CW_K = 1, CW_Q = 2, CB_K = 4, CB_Q = 8 };

struct Pos {
  int8_t sq[64];  // -1 empty, else color*8 + kind; square = 8*row + col (a1 = 0)
  uint8_t stm;    // 0 white, 1 black
  uint8_t castle; // FIDE castling rights
  int8_t ep;      // FIDE en-passant target square or -1
};

struct Move {
  uint8_t from, to, promo;  // promo: 0 none, 1 N, 2 B, 3 R, 4 Q
};

// 16-bit move word of the ABI: from | to<<6 | promo<<12; bit 15 = coordinate out of range.
inline uint16_t encode(const Move& m) {
  return static_cast<uint16_t>(m.from | (m.to << 6) | (m.promo << 12));
}
constexpr uint16_t kSentinel = 0xFFFF;
constexpr uint16_t kOorFlag = 0x8000;

void startpos(Pos& p);
bool from_fen(const char* fen, Pos& p);
void to_quad(const Pos& p, uint64_t bb[4]);
uint64_t digest(const Pos& p);

// Moves in canonical order: from ascending, then to ascending, then promo (N,B,R,Q).
int gen_moves(const Pos& p, Rules r, Move* out /*>= 256*/);
uint8_t validate(const Pos& p, Rules r, uint16_t move);
void make(Pos& p, Rules r, const Move& m);
// Returns {moved kind, captured?} for history notation: (kind | capture<<3).
uint8_t apply_info(const Pos& p, const Move& m);

uint64_t perft(const Pos& p, Rules r, unsigned depth, unsigned threads,
               std::vector<uint64_t>* divide /* per canonical root move */);

// SURVEY §8d C4 generator: splitmix64(seed ^ game_id); per ply one draw r:
// (r & 0xFF) < noise_per_256 -> move = (r >> 8) & 0xFFF, else the
// ((r>>32)*n >> 32)-th legal move in canonical order.  No legal move ->
// 0xFFFF for the remaining plies.  Accepted moves are applied.
void gen_games(uint64_t seed, uint64_t first_game, uint32_t n_games, uint32_t n_plies,
               uint32_t noise_per_256, Rules r, uint16_t* out /* ply-major [n_plies][n_games] */,
               unsigned threads);

struct ReplayStats {
  uint64_t validated, accepted, rejected, digest_sum, digest_xor;
};
// Replays ply-major moves from startpos (or *start).  bitmap is ply-major
// [n_plies][ceil(n_games/64)]; digests[g] = final-state digest.
void replay(const Pos* start, const uint16_t* moves, uint32_t n_games, uint32_t n_plies, Rules r,
            uint64_t* bitmap, uint64_t* digests, ReplayStats* stats, unsigned threads);

}  // namespace fastcpu
