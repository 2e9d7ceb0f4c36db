// oracle/fastcpu.cpp -- TEST INFRASTRUCTURE ONLY.  See fastcpu.hpp.
#include "fastcpu.hpp"

#include <atomic>
#include <cstring>
#include <string>
#include <thread>

namespace fastcpu {

static inline int color_of(int8_t c) { return c >> 3; }
static inline int kind_of(int8_t c) { return c & 7; }
static inline bool on_board(int r, int c) { return r >= 0 && r < 8 && c >= 0 && c < 8; }

static const int kKnight[8][2] = {{1, 2}, {2, 1}, {2, -1}, {1, -2}, {-1, -2}, {-2, -1}, {-2, 1}, {-1, 2}};
static const int kKing[8][2] = {{1, 0}, {1, 1}, {0, 1}, {-1, 1}, {-1, 0}, {-1, -1}, {0, -1}, {1, -1}};
static const int kOrth[4][2] = {{1, 0}, {-1, 0}, {0, 1}, {0, -1}};
static const int kDiag[4][2] = {{1, 1}, {1, -1}, {-1, 1}, {-1, -1}};

void startpos(Pos& p) {
  static const int8_t back[8] = {R, N, B, Q, K, B, N, R};
  std::memset(p.sq, -1, sizeof p.sq);
  for (int c = 0; c < 8; ++c) {
    p.sq[c] = back[c];
    p.sq[8 + c] = P;
    p.sq[48 + c] = 8 + P;
    p.sq[56 + c] = static_cast<int8_t>(8 + back[c]);
  }
  p.stm = 0;
  p.castle = CW_K | CW_Q | CB_K | CB_Q;
  p.ep = -1;
}

bool from_fen(const char* fen, Pos& p) {
  std::memset(p.sq, -1, sizeof p.sq);
  p.stm = 0;
  p.castle = 0;
  p.ep = -1;
  int row = 7, col = 0;
  const char* s = fen;
  for (; *s && *s != ' '; ++s) {
    const char ch = *s;
    if (ch == '/') {
      --row;
      col = 0;
      continue;
    }
    if (ch >= '1' && ch <= '8') {
      col += ch - '0';
      continue;
    }
    int kind;
    switch (ch | 0x20) {
      case 'p': kind = P; break;
      case 'n': kind = N; break;
      case 'b': kind = B; break;
      case 'r': kind = R; break;
      case 'q': kind = Q; break;
      case 'k': kind = K; break;
      default: return false;
    }
    if (row < 0 || col > 7) return false;
    const int color = (ch >= 'a') ? 1 : 0;
    p.sq[8 * row + col] = static_cast<int8_t>(color * 8 + kind);
    ++col;
  }
  if (*s == ' ') ++s;
  if (*s == 'b') p.stm = 1;
  while (*s && *s != ' ') ++s;
  if (*s == ' ') ++s;
  for (; *s && *s != ' '; ++s) {
    if (*s == 'K') p.castle |= CW_K;
    if (*s == 'Q') p.castle |= CW_Q;
    if (*s == 'k') p.castle |= CB_K;
    if (*s == 'q') p.castle |= CB_Q;
  }
  if (*s == ' ') ++s;
  if (*s >= 'a' && *s <= 'h' && s[1] >= '1' && s[1] <= '8') p.ep = static_cast<int8_t>((s[1] - '1') * 8 + (s[0] - 'a'));
  return true;
}

// ABI quad-bitboard: bb[0] black, bb[1..3] kind-code bits, P=1 N=2 K=3 X=4 B=5 R=6 Q=7.
void to_quad(const Pos& p, uint64_t bb[4]) {
  static const int code[7] = {1, 2, 5, 6, 7, 3, 4};
  bb[0] = bb[1] = bb[2] = bb[3] = 0;
  for (int s = 0; s < 64; ++s) {
    if (p.sq[s] < 0) continue;
    const uint64_t m = 1ull << s;
    const int k = code[kind_of(p.sq[s])];
    if (color_of(p.sq[s])) bb[0] |= m;
    if (k & 1) bb[1] |= m;
    if (k & 2) bb[2] |= m;
    if (k & 4) bb[3] |= m;
  }
}

static inline uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

uint64_t digest(const Pos& p) {
  uint64_t bb[4];
  to_quad(p, bb);
  uint64_t h = 0x6A09E667F3BCC909ull ^ static_cast<uint64_t>(p.stm & 1);
  h = fmix64(h ^ bb[3]);
  h = fmix64(h ^ bb[2]);
  h = fmix64(h ^ bb[1]);
  h = fmix64(h ^ bb[0]);
  return h;
}

static inline bool empty_or_enemy(const Pos& p, int s, int color) {
  return p.sq[s] < 0 || color_of(p.sq[s]) != color;
}

static uint64_t ray_targets(const Pos& p, int f, int color, const int (*dirs)[2], int ndirs) {
  uint64_t t = 0;
  const int r0 = f >> 3, c0 = f & 7;
  for (int d = 0; d < ndirs; ++d) {
    int r = r0 + dirs[d][0], c = c0 + dirs[d][1];
    while (on_board(r, c)) {
      const int s = 8 * r + c;
      if (p.sq[s] < 0) {
        t |= 1ull << s;
      } else {
        if (color_of(p.sq[s]) != color) t |= 1ull << s;
        break;
      }
      r += dirs[d][0];
      c += dirs[d][1];
    }
  }
  return t;
}

static uint64_t step_targets(const Pos& p, int f, int color, const int (*offs)[2]) {
  uint64_t t = 0;
  const int r0 = f >> 3, c0 = f & 7;
  for (int d = 0; d < 8; ++d) {
    const int r = r0 + offs[d][0], c = c0 + offs[d][1];
    if (on_board(r, c) && empty_or_enemy(p, 8 * r + c, color)) t |= 1ull << (8 * r + c);
  }
  return t;
}

// Pseudo targets of the piece on f (rules common to REF and FIDE, minus pawn
// specials, castling and promotion).  REF: this is exactly can_move_to.
static uint64_t piece_targets(const Pos& p, int f, bool fide) {
  const int8_t pc = p.sq[f];
  const int color = color_of(pc);
  const int r0 = f >> 3, c0 = f & 7;
  switch (kind_of(pc)) {
    case P: {
      uint64_t t = 0;
      const int dir = color == 0 ? 1 : -1;
      const int start = color == 0 ? 1 : 6;
      const int r1 = r0 + dir;
      if (r1 >= 0 && r1 < 8) {
        if (p.sq[8 * r1 + c0] < 0) {
          t |= 1ull << (8 * r1 + c0);
          const int r2 = r0 + 2 * dir;
          if (r0 == start && p.sq[8 * r2 + c0] < 0) t |= 1ull << (8 * r2 + c0);
        }
        for (int dc = -1; dc <= 1; dc += 2) {
          const int c1 = c0 + dc;
          if (c1 < 0 || c1 > 7) continue;
          const int s = 8 * r1 + c1;
          if (p.sq[s] >= 0 && color_of(p.sq[s]) != color) t |= 1ull << s;
          if (fide && s == p.ep) t |= 1ull << s;
        }
      }
      return t;
    }
    case N: return step_targets(p, f, color, kKnight);
    case K: return step_targets(p, f, color, kKing);
    case B: return ray_targets(p, f, color, kDiag, 4);
    case R: return ray_targets(p, f, color, kOrth, 4);
    case Q: return ray_targets(p, f, color, kOrth, 4) | ray_targets(p, f, color, kDiag, 4);
    default: return 0;  // unknown kind: immovable (chess.rs:210)
  }
}

static bool attacked(const Pos& p, int s, int by) {
  const int r0 = s >> 3, c0 = s & 7;
  // pawns of `by` attack forward-diagonally
  const int pr = r0 - (by == 0 ? 1 : -1);
  for (int dc = -1; dc <= 1; dc += 2) {
    const int pc = c0 + dc;
    if (on_board(pr, pc) && p.sq[8 * pr + pc] == by * 8 + P) return true;
  }
  for (int d = 0; d < 8; ++d) {
    int r = r0 + kKnight[d][0], c = c0 + kKnight[d][1];
    if (on_board(r, c) && p.sq[8 * r + c] == by * 8 + N) return true;
    r = r0 + kKing[d][0];
    c = c0 + kKing[d][1];
    if (on_board(r, c) && p.sq[8 * r + c] == by * 8 + K) return true;
  }
  for (int pass = 0; pass < 2; ++pass) {
    const int (*dirs)[2] = pass ? kDiag : kOrth;
    const int8_t slider = static_cast<int8_t>(by * 8 + (pass ? B : R));
    for (int d = 0; d < 4; ++d) {
      int r = r0 + dirs[d][0], c = c0 + dirs[d][1];
      while (on_board(r, c)) {
        const int8_t q = p.sq[8 * r + c];
        if (q >= 0) {
          if (q == slider || q == by * 8 + Q) return true;
          break;
        }
        r += dirs[d][0];
        c += dirs[d][1];
      }
    }
  }
  return false;
}

static int king_square(const Pos& p, int color) {
  for (int s = 0; s < 64; ++s)
    if (p.sq[s] == color * 8 + K) return s;
  return -1;
}

void make(Pos& p, Rules r, const Move& m) {
  const int8_t pc = p.sq[m.from];
  p.sq[m.to] = pc;
  p.sq[m.from] = -1;
  if (r == RULES_FIDE) {
    const int color = color_of(pc);
    if (kind_of(pc) == P) {
      if (m.to == p.ep) p.sq[(m.from & ~7) | (m.to & 7)] = -1;
      if (m.promo) p.sq[m.to] = static_cast<int8_t>(color * 8 + m.promo);
    }
    if (kind_of(pc) == K && (m.to - m.from == 2 || m.from - m.to == 2)) {
      const int rank = m.from & ~7;
      if (m.to > m.from) {
        p.sq[rank + 5] = p.sq[rank + 7];
        p.sq[rank + 7] = -1;
      } else {
        p.sq[rank + 3] = p.sq[rank + 0];
        p.sq[rank + 0] = -1;
      }
    }
    for (int s : {static_cast<int>(m.from), static_cast<int>(m.to)}) {
      if (s == 4) p.castle &= ~(CW_K | CW_Q);
      if (s == 0) p.castle &= ~CW_Q;
      if (s == 7) p.castle &= ~CW_K;
      if (s == 60) p.castle &= ~(CB_K | CB_Q);
      if (s == 56) p.castle &= ~CB_Q;
      if (s == 63) p.castle &= ~CB_K;
    }
    const int delta = m.to - m.from;
    p.ep = (kind_of(pc) == P && (delta == 16 || delta == -16)) ? static_cast<int8_t>((m.from + m.to) / 2) : -1;
  }
  p.stm ^= 1;
}

static bool legal_after(const Pos& p, const Move& m) {
  Pos q = p;
  make(q, RULES_FIDE, m);
  const int ks = king_square(q, p.stm);
  return ks < 0 || !attacked(q, ks, p.stm ^ 1);
}

int gen_moves(const Pos& p, Rules r, Move* out) {
  int n = 0;
  const bool fide = r == RULES_FIDE;
  for (int f = 0; f < 64; ++f) {
    const int8_t pc = p.sq[f];
    if (pc < 0 || color_of(pc) != p.stm) continue;
    uint64_t t = piece_targets(p, f, fide);
    if (fide && kind_of(pc) == K) {
      // castling: king on its home square with the right still held
      const int home = p.stm ? 60 : 4;
      const int them = p.stm ^ 1;
      const uint8_t rk = p.stm ? CB_K : CW_K, rq = p.stm ? CB_Q : CW_Q;
      const int8_t rook = static_cast<int8_t>(p.stm * 8 + R);
      if (f == home && !attacked(p, home, them)) {
        if ((p.castle & rk) && p.sq[home + 3] == rook && p.sq[home + 1] < 0 && p.sq[home + 2] < 0 &&
            !attacked(p, home + 1, them) && !attacked(p, home + 2, them))
          t |= 1ull << (home + 2);
        if ((p.castle & rq) && p.sq[home - 4] == rook && p.sq[home - 1] < 0 && p.sq[home - 2] < 0 &&
            p.sq[home - 3] < 0 && !attacked(p, home - 1, them) && !attacked(p, home - 2, them))
          t |= 1ull << (home - 2);
      }
    }
    while (t) {
      const int to = __builtin_ctzll(t);
      t &= t - 1;
      const bool promo = fide && kind_of(pc) == P && (to >> 3) == (p.stm ? 0 : 7);
      for (int k = promo ? 1 : 0; k <= (promo ? 4 : 0); ++k) {
        const Move m{static_cast<uint8_t>(f), static_cast<uint8_t>(to), static_cast<uint8_t>(k)};
        if (fide && !legal_after(p, m)) continue;
        out[n++] = m;
      }
    }
  }
  return n;
}

uint8_t validate(const Pos& p, Rules r, uint16_t move) {
  if (move & kOorFlag) return V_OOR;
  const int f = move & 63, t = (move >> 6) & 63, promo = (move >> 12) & 7;
  if (p.sq[f] < 0) return V_NO_PIECE;
  if (color_of(p.sq[f]) != p.stm) return V_WRONG_TURN;
  if (r == RULES_REF) return ((piece_targets(p, f, false) >> t) & 1) ? V_OK : V_ILLEGAL;
  Move ms[256];
  const int n = gen_moves(p, r, ms);
  for (int i = 0; i < n; ++i)
    if (ms[i].from == f && ms[i].to == t && ms[i].promo == promo) return V_OK;
  return V_ILLEGAL;
}

uint8_t apply_info(const Pos& p, const Move& m) {
  return static_cast<uint8_t>(kind_of(p.sq[m.from]) | ((p.sq[m.to] >= 0) ? 8 : 0));
}

static uint64_t perft_rec(const Pos& p, Rules r, unsigned depth) {
  Move ms[256];
  const int n = gen_moves(p, r, ms);
  if (depth == 1) return static_cast<uint64_t>(n);
  uint64_t total = 0;
  for (int i = 0; i < n; ++i) {
    Pos q = p;
    make(q, r, ms[i]);
    total += perft_rec(q, r, depth - 1);
  }
  return total;
}

template <class F>
static void parallel_for(size_t n, unsigned threads, F&& fn) {
  if (threads <= 1 || n <= 1) {
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

uint64_t perft(const Pos& p, Rules r, unsigned depth, unsigned threads, std::vector<uint64_t>* divide) {
  if (depth == 0) return 1;
  Move roots[256];
  const int n = gen_moves(p, r, roots);
  std::vector<uint64_t> per(n, 0);
  if (depth == 1) {
    for (int i = 0; i < n; ++i) per[i] = 1;
  } else {
    // tasks: every grandchild (or child when depth == 2) of the root
    struct Task {
      int root;
      Pos pos;
    };
    std::vector<Task> tasks;
    for (int i = 0; i < n; ++i) {
      Pos c = p;
      make(c, r, roots[i]);
      if (depth == 2) {
        tasks.push_back({i, c});
        continue;
      }
      Move ms[256];
      const int m = gen_moves(c, r, ms);
      for (int j = 0; j < m; ++j) {
        Pos g = c;
        make(g, r, ms[j]);
        tasks.push_back({i, g});
      }
    }
    const unsigned sub = depth == 2 ? 1 : depth - 2;
    std::vector<uint64_t> res(tasks.size());
    parallel_for(tasks.size(), threads, [&](size_t k) { res[k] = perft_rec(tasks[k].pos, r, sub); });
    for (size_t k = 0; k < tasks.size(); ++k) per[tasks[k].root] += res[k];
  }
  uint64_t total = 0;
  for (auto v : per) total += v;
  if (divide) *divide = per;
  return total;
}

static inline uint64_t splitmix_next(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void gen_games(uint64_t seed, uint64_t first_game, uint32_t n_games, uint32_t n_plies,
               uint32_t noise_per_256, Rules r, uint16_t* out, unsigned threads) {
  parallel_for(n_games, threads, [&](size_t g) {
    uint64_t s = seed ^ (first_game + g);
    Pos p;
    startpos(p);
    Move ms[256];
    bool over = false;
    for (uint32_t ply = 0; ply < n_plies; ++ply) {
      uint16_t* slot = out + static_cast<size_t>(ply) * n_games + g;
      if (over) {
        *slot = kSentinel;
        continue;
      }
      const int n = gen_moves(p, r, ms);
      if (n == 0) {
        over = true;
        *slot = kSentinel;
        continue;
      }
      const uint64_t x = splitmix_next(s);
      uint16_t m;
      if ((x & 0xFF) < noise_per_256) {
        m = static_cast<uint16_t>((x >> 8) & 0xFFF);
      } else {
        const uint64_t k = ((x >> 32) * static_cast<uint64_t>(n)) >> 32;
        m = encode(ms[k]);
      }
      *slot = m;
      if (validate(p, r, m) == V_OK)
        make(p, r, Move{static_cast<uint8_t>(m & 63), static_cast<uint8_t>((m >> 6) & 63),
                        static_cast<uint8_t>((m >> 12) & 7)});
    }
  });
}

void replay(const Pos* start, const uint16_t* moves, uint32_t n_games, uint32_t n_plies, Rules r,
            uint64_t* bitmap, uint64_t* digests, ReplayStats* stats, unsigned threads) {
  const uint32_t words = (n_games + 63) / 64;
  if (bitmap) std::memset(bitmap, 0, sizeof(uint64_t) * words * n_plies);
  // one task per 64-game word so bitmap words are owned by a single thread
  std::vector<ReplayStats> part(words, ReplayStats{0, 0, 0, 0, 0});
  parallel_for(words, threads, [&](size_t w) {
    ReplayStats& st = part[w];
    for (uint32_t g = static_cast<uint32_t>(w * 64); g < n_games && g < (w + 1) * 64; ++g) {
      Pos p;
      if (start) p = *start; else startpos(p);
      for (uint32_t ply = 0; ply < n_plies; ++ply) {
        const uint16_t m = moves[static_cast<size_t>(ply) * n_games + g];
        if (m == kSentinel) continue;
        ++st.validated;
        const uint8_t v = validate(p, r, m);
        if (v == V_OK) {
          ++st.accepted;
          if (bitmap) bitmap[static_cast<size_t>(ply) * words + w] |= 1ull << (g & 63);
          make(p, r, Move{static_cast<uint8_t>(m & 63), static_cast<uint8_t>((m >> 6) & 63),
                          static_cast<uint8_t>((m >> 12) & 7)});
        } else {
          ++st.rejected;
        }
      }
      const uint64_t d = digest(p);
      if (digests) digests[g] = d;
      st.digest_sum += d;
      st.digest_xor ^= d;
    }
  });
  ReplayStats tot{0, 0, 0, 0, 0};
  for (auto& s : part) {
    tot.validated += s.validated;
    tot.accepted += s.accepted;
    tot.rejected += s.rejected;
    tot.digest_sum += s.digest_sum;
    tot.digest_xor ^= s.digest_xor;
  }
  if (stats) *stats = tot;
}

}  // namespace fastcpu
