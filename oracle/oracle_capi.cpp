// oracle/oracle_capi.cpp -- TEST INFRASTRUCTURE ONLY.
// extern "C" surface over refcpu and fastcpu so that tests/ and bench.py can
// drive the oracle through ctypes.  Never linked into the product library.
#include <atomic>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "fastcpu.hpp"
#include "refcpu.hpp"

namespace {

refcpu::GameState ref_state(const int8_t* cells, int32_t turn) {
  refcpu::GameState g = refcpu::GameState::create("white", "black");
  if (cells) refcpu::board_from_cells(cells, *g.board);
  g.turn = turn;
  return g;
}

fastcpu::Pos fast_pos(const int8_t* cells, uint8_t stm, uint8_t castle, int8_t ep) {
  fastcpu::Pos p;
  if (cells) {
    std::memcpy(p.sq, cells, 64);
    p.stm = stm;
    p.castle = castle;
    p.ep = ep;
  } else {
    fastcpu::startpos(p);
  }
  return p;
}

template <class F>
void par(size_t n, unsigned threads, F&& fn) {
  if (threads <= 1) {
    for (size_t i = 0; i < n; ++i) fn(i);
    return;
  }
  std::atomic<size_t> next{0};
  std::vector<std::thread> pool;
  for (unsigned t = 0; t < threads; ++t)
    pool.emplace_back([&] {
      for (size_t i; (i = next.fetch_add(1)) < n;) fn(i);
    });
  for (auto& th : pool) th.join();
}

}  // namespace

extern "C" {

// ----------------------------------------------------------------- refcpu
void or_startpos_cells(int8_t* cells) {
  refcpu::Board b = refcpu::Board::initial();
  refcpu::board_to_cells(b, cells);
}

int or_ref_validate(const int8_t* cells, int32_t turn, uint32_t fx, uint32_t fy, uint32_t tx, uint32_t ty) {
  const refcpu::GameState g = ref_state(cells, turn);
  return g.validate_move({fx, fy}, {tx, ty});
}

const char* or_ref_message(int v) { return refcpu::verdict_message(static_cast<uint8_t>(v)); }

// Applies one move in place.  history: in/out NUL-terminated buffer of cap bytes.
int or_ref_apply(int8_t* cells, int32_t* turn, char* history, size_t cap, uint32_t fx, uint32_t fy,
                 uint32_t tx, uint32_t ty) {
  refcpu::GameState g = ref_state(cells, *turn);
  g.history = std::string(history ? history : "");
  const uint8_t v = g.apply_move({fx, fy}, {tx, ty});
  refcpu::board_to_cells(*g.board, cells);
  *turn = g.turn;
  if (history && cap) {
    std::strncpy(history, g.history->c_str(), cap - 1);
    history[cap - 1] = 0;
  }
  return v;
}

// All 4096 (from,to) verdicts of one position, out[64*from + to].
void or_ref_verdicts_all(const int8_t* cells, int32_t turn, uint8_t* out) {
  const refcpu::GameState g = ref_state(cells, turn);
  for (uint32_t f = 0; f < 64; ++f)
    for (uint32_t t = 0; t < 64; ++t) out[f * 64 + t] = g.validate_move({f >> 3, f & 7}, {t >> 3, t & 7});
}

// Brute-force REF perft through validate_move; divide[4096] indexed 64*from+to (may be null).
// Threads split the root pairs.
uint64_t or_ref_perft(const int8_t* cells, int32_t turn, unsigned depth, unsigned threads, uint64_t* divide) {
  const refcpu::GameState g = ref_state(cells, turn);
  if (depth == 0) return 1;
  std::vector<uint64_t> per(4096, 0);
  par(4096, threads, [&](size_t i) {
    const uint32_t f = static_cast<uint32_t>(i >> 6), t = static_cast<uint32_t>(i & 63);
    const refcpu::Position pf{f >> 3, f & 7}, pt{t >> 3, t & 7};
    if (g.validate_move(pf, pt) != refcpu::V_OK) return;
    refcpu::GameState c = g;
    c.apply_move(pf, pt, false);
    per[i] = refcpu::perft(c, depth - 1, nullptr);
  });
  uint64_t tot = 0;
  for (int i = 0; i < 4096; ++i) tot += per[i];
  if (divide) std::memcpy(divide, per.data(), sizeof(uint64_t) * 4096);
  return tot;
}

// Replay ply-major moves from startpos with the literal restatement.
// stats[5] = validated, accepted, rejected, digest_sum, digest_xor.
void or_ref_replay(const uint16_t* moves, uint32_t n_games, uint32_t n_plies, unsigned threads,
                   uint64_t* bitmap, uint64_t* digests, uint64_t* stats) {
  const uint32_t words = (n_games + 63) / 64;
  if (bitmap) std::memset(bitmap, 0, sizeof(uint64_t) * words * n_plies);
  std::vector<uint64_t> part(static_cast<size_t>(words) * 5, 0);
  par(words, threads, [&](size_t w) {
    uint64_t* st = &part[w * 5];
    for (uint32_t g = static_cast<uint32_t>(w * 64); g < n_games && g < (w + 1) * 64; ++g) {
      refcpu::GameState s = refcpu::GameState::create("white", "black");
      for (uint32_t ply = 0; ply < n_plies; ++ply) {
        const uint16_t m = moves[static_cast<size_t>(ply) * n_games + g];
        if (m == 0xFFFF) continue;
        ++st[0];
        refcpu::Position pf{8, 0}, pt{8, 0};  // OOR flag: any coordinate >= 8
        if (!(m & 0x8000)) {
          pf = {static_cast<uint32_t>((m & 63) >> 3), static_cast<uint32_t>(m & 7)};
          pt = {static_cast<uint32_t>(((m >> 6) & 63) >> 3), static_cast<uint32_t>((m >> 6) & 7)};
        }
        if (s.apply_move(pf, pt) == refcpu::V_OK) {
          ++st[1];
          if (bitmap) bitmap[static_cast<size_t>(ply) * words + w] |= 1ull << (g & 63);
        } else {
          ++st[2];
        }
      }
      const uint64_t d = refcpu::state_digest(s);
      if (digests) digests[g] = d;
      st[3] += d;
      st[4] ^= d;
    }
  });
  uint64_t tot[5] = {0, 0, 0, 0, 0};
  for (uint32_t w = 0; w < words; ++w) {
    for (int k = 0; k < 4; ++k) tot[k] += part[w * 5 + k];
    tot[4] ^= part[w * 5 + 4];
  }
  if (stats) std::memcpy(stats, tot, sizeof tot);
}

// ----------------------------------------------------------------- fastcpu
int or_fast_from_fen(const char* fen, int8_t* cells, uint8_t* stm, uint8_t* castle, int8_t* ep) {
  fastcpu::Pos p;
  if (!fastcpu::from_fen(fen, p)) return -1;
  std::memcpy(cells, p.sq, 64);
  *stm = p.stm;
  *castle = p.castle;
  *ep = p.ep;
  return 0;
}

void or_fast_verdicts_all(const int8_t* cells, uint8_t stm, uint8_t castle, int8_t ep, int rules, uint8_t* out) {
  const fastcpu::Pos p = fast_pos(cells, stm, castle, ep);
  for (uint32_t f = 0; f < 64; ++f)
    for (uint32_t t = 0; t < 64; ++t)
      out[f * 64 + t] = fastcpu::validate(p, static_cast<fastcpu::Rules>(rules), static_cast<uint16_t>(f | (t << 6)));
}

int or_fast_validate(const int8_t* cells, uint8_t stm, uint8_t castle, int8_t ep, int rules, uint16_t move) {
  const fastcpu::Pos p = fast_pos(cells, stm, castle, ep);
  return fastcpu::validate(p, static_cast<fastcpu::Rules>(rules), move);
}

int or_fast_gen_moves(const int8_t* cells, uint8_t stm, uint8_t castle, int8_t ep, int rules, uint16_t* out) {
  const fastcpu::Pos p = fast_pos(cells, stm, castle, ep);
  fastcpu::Move ms[256];
  const int n = fastcpu::gen_moves(p, static_cast<fastcpu::Rules>(rules), ms);
  for (int i = 0; i < n; ++i) out[i] = fastcpu::encode(ms[i]);
  return n;
}

// Makes `move` (assumed accepted) on the position in place.
void or_fast_make(int8_t* cells, uint8_t* stm, uint8_t* castle, int8_t* ep, int rules, uint16_t move) {
  fastcpu::Pos p = fast_pos(cells, *stm, *castle, *ep);
  fastcpu::make(p, static_cast<fastcpu::Rules>(rules),
                fastcpu::Move{static_cast<uint8_t>(move & 63), static_cast<uint8_t>((move >> 6) & 63),
                              static_cast<uint8_t>((move >> 12) & 7)});
  std::memcpy(cells, p.sq, 64);
  *stm = p.stm;
  *castle = p.castle;
  *ep = p.ep;
}

// Perft; divide/root_moves sized >= 256 (canonical root-move order).
uint64_t or_fast_perft(const int8_t* cells, uint8_t stm, uint8_t castle, int8_t ep, int rules, unsigned depth,
                       unsigned threads, uint64_t* divide, uint16_t* root_moves, uint32_t* n_root) {
  const fastcpu::Pos p = fast_pos(cells, stm, castle, ep);
  std::vector<uint64_t> div;
  const uint64_t tot = fastcpu::perft(p, static_cast<fastcpu::Rules>(rules), depth, threads, &div);
  fastcpu::Move ms[256];
  const int n = fastcpu::gen_moves(p, static_cast<fastcpu::Rules>(rules), ms);
  if (n_root) *n_root = static_cast<uint32_t>(n);
  for (int i = 0; i < n; ++i) {
    if (root_moves) root_moves[i] = fastcpu::encode(ms[i]);
    if (divide) divide[i] = depth ? div[i] : 0;
  }
  return tot;
}

void or_fast_gen_games(uint64_t seed, uint64_t first_game, uint32_t n_games, uint32_t n_plies,
                       uint32_t noise_per_256, int rules, uint16_t* out, unsigned threads) {
  fastcpu::gen_games(seed, first_game, n_games, n_plies, noise_per_256, static_cast<fastcpu::Rules>(rules), out,
                     threads);
}

void or_fast_replay(const uint16_t* moves, uint32_t n_games, uint32_t n_plies, int rules, unsigned threads,
                    uint64_t* bitmap, uint64_t* digests, uint64_t* stats) {
  fastcpu::ReplayStats st;
  fastcpu::replay(nullptr, moves, n_games, n_plies, static_cast<fastcpu::Rules>(rules), bitmap, digests, &st,
                  threads);
  if (stats) {
    stats[0] = st.validated;
    stats[1] = st.accepted;
    stats[2] = st.rejected;
    stats[3] = st.digest_sum;
    stats[4] = st.digest_xor;
  }
}

void or_fast_quad(const int8_t* cells, uint64_t* bb) {
  fastcpu::Pos p = fast_pos(cells, 0, 0, -1);
  fastcpu::to_quad(p, bb);
}

uint64_t or_fast_digest(const int8_t* cells, uint8_t stm) {
  fastcpu::Pos p = fast_pos(cells, stm, 0, -1);
  return fastcpu::digest(p);
}

// Legal-move counts of n quad-bitboard positions (bb[4*i..4*i+3], the device
// Board layout; meta: castle rights | ep square << 4 | 0x400 when valid) --
// the per-child recount of tools/fide_child_diag.py.
void or_fast_count_quad(const uint64_t* bb, const uint8_t* stm, const uint16_t* meta, uint32_t n, int rules,
                        unsigned threads, uint32_t* out) {
  static const int8_t kind_of_code[8] = {-1, fastcpu::P, fastcpu::N, fastcpu::K, fastcpu::X,
                                         fastcpu::B, fastcpu::R, fastcpu::Q};
  par(n, threads, [&](size_t i) {
    const uint64_t* q = bb + 4 * i;
    fastcpu::Pos p;
    for (int s = 0; s < 64; ++s) {
      const int code = static_cast<int>(((q[1] >> s) & 1) | (((q[2] >> s) & 1) << 1) | (((q[3] >> s) & 1) << 2));
      p.sq[s] = code ? static_cast<int8_t>(((q[0] >> s) & 1) * 8 + kind_of_code[code]) : int8_t(-1);
    }
    p.stm = stm[i];
    const uint16_t m = meta ? meta[i] : 0;
    p.castle = static_cast<uint8_t>(m & 15);
    p.ep = (m & 0x400) ? static_cast<int8_t>((m >> 4) & 63) : int8_t(-1);
    fastcpu::Move ms[256];
    out[i] = static_cast<uint32_t>(fastcpu::gen_moves(p, static_cast<fastcpu::Rules>(rules), ms));
  });
}

}  // extern "C"
