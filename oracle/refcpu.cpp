// oracle/refcpu.cpp -- TEST INFRASTRUCTURE ONLY.  See refcpu.hpp.
//
// Every function cites the reference lines it restates.  The deliberate
// per-call board clones are kept: they are the reference's cost model, and this
// file doubles as the "reference-faithful" CPU baseline in bench.py.
#include "refcpu.hpp"

#include <cstdlib>
#include <sstream>

namespace refcpu {

const char* verdict_message(uint8_t v) {
  switch (v) {
    case V_OK: return "";
    case V_NO_PIECE: return "No piece at the source location";       // chess.rs:104-106
    case V_WRONG_TURN: return "It's not this piece's turn to move";  // chess.rs:113-115
    case V_ILLEGAL: return "Invalid move for the piece";             // chess.rs:119-121
    case V_OOR: return "index out of bounds";                         // Rust panic text
    case V_BAD_TURN: return "Correct color";                          // .expect() panic text
  }
  return "?";
}

// chess.rs:383-434 -- rows 1..6 empty, back ranks RNBQKBNR, pawns on rows 1 and 6.
Board Board::initial() {
  Board b;
  b.rows.assign(8, Row{});
  for (auto& r : b.rows) r.cells.assign(8, Cell{});
  static const char* back = "RNBQKBNR";
  for (int y = 0; y < 8; ++y) {
    b.rows[0].cells[y].piece = Piece{0, std::string(1, back[y])};
    b.rows[7].cells[y].piece = Piece{1, std::string(1, back[y])};
    b.rows[1].cells[y].piece = Piece{0, "P"};
    b.rows[6].cells[y].piece = Piece{1, "P"};
  }
  return b;
}

// chess.rs:436-440
const Piece* Board::get_piece_at(const std::vector<uint32_t>& c) const {
  const auto& cell = rows.at(c[0]).cells.at(c[1]);
  return cell.piece ? &*cell.piece : nullptr;
}
// chess.rs:442-447 -- "enemy" is any colour different from the mover's.
bool Board::has_enemy_piece(const std::vector<uint32_t>& c, int32_t color) const {
  const Piece* p = get_piece_at(c);
  return p != nullptr && p->color != color;
}
// chess.rs:449-451
bool Board::is_empty(const std::vector<uint32_t>& c) const { return get_piece_at(c) == nullptr; }
// chess.rs:453-455
bool Board::is_empty_or_enemy(const std::vector<uint32_t>& c, int32_t color) const {
  return is_empty(c) || has_enemy_piece(c, color);
}

// chess.rs:12-20
GameState GameState::create(const std::string& white, const std::string& black) {
  GameState g;
  g.white_player = white;
  g.black_player = black;
  g.turn = 0;
  g.history = std::string();
  g.board = Board::initial();
  return g;
}

static inline int32_t signum(int32_t v) { return (v > 0) - (v < 0); }

// chess.rs:214-254 (pawn).  dir +1 for colour 0 else -1; double push only from
// row 1/6 with the middle square empty; diagonal only onto an enemy piece.
static bool pawn_ok(const Piece& p, const Location& from, const Location& to, int32_t dx,
                    int32_t dy, const Board& b) {
  const int32_t dir = (p.color == 0) ? 1 : -1;
  const int32_t start_row = (p.color == 0) ? 1 : 6;
  if (dy == 0 && dx == dir) return b.is_empty(to.coords);
  if (dy == 0 && dx == 2 * dir && static_cast<int32_t>(from.coords[0]) == start_row) {
    // chess.rs:241-244 builds a Location (vector + Piece copy) for the middle square.
    Location mid{{static_cast<uint32_t>(static_cast<int32_t>(from.coords[0]) + dir), from.coords[1]},
                 Piece{p.color, "P"}};
    return b.is_empty(to.coords) && b.is_empty(mid.coords);
  }
  if (std::abs(dy) == 1 && dx == dir) return b.has_enemy_piece(to.coords, p.color);
  return false;
}

// Shared path walk of chess.rs:272-284 (rook) and :319-332 (bishop): every square
// strictly between from and to must be empty; each probe allocates a Location.
static bool path_clear(const Piece& p, const Location& from, const Location& to, int32_t sx,
                       int32_t sy, const Board& b) {
  int32_t x = static_cast<int32_t>(from.coords[0]) + sx;
  int32_t y = static_cast<int32_t>(from.coords[1]) + sy;
  const int32_t tx = static_cast<int32_t>(to.coords[0]);
  const int32_t ty = static_cast<int32_t>(to.coords[1]);
  while (x != tx || y != ty) {
    Location probe{{static_cast<uint32_t>(x), static_cast<uint32_t>(y)}, Piece{p.color, p.kind}};
    if (!b.is_empty(probe.coords)) return false;
    x += sx;
    y += sy;
  }
  return true;
}

// chess.rs:256-287
static bool rook_ok(const Piece& p, const Location& from, const Location& to, int32_t dx,
                    int32_t dy, const Board& b) {
  if (dx != 0 && dy != 0) return false;
  if (!path_clear(p, from, to, signum(dx), signum(dy), b)) return false;
  return b.is_empty_or_enemy(to.coords, p.color);
}

// chess.rs:289-300
static bool knight_ok(const Piece& p, const Location&, const Location& to, int32_t dx, int32_t dy,
                      const Board& b) {
  const int32_t ax = std::abs(dx), ay = std::abs(dy);
  return ((ax == 2 && ay == 1) || (ax == 1 && ay == 2)) && b.is_empty_or_enemy(to.coords, p.color);
}

// chess.rs:302-335
static bool bishop_ok(const Piece& p, const Location& from, const Location& to, int32_t dx,
                      int32_t dy, const Board& b) {
  if (std::abs(dx) != std::abs(dy)) return false;
  if (!path_clear(p, from, to, signum(dx), signum(dy), b)) return false;
  return b.is_empty_or_enemy(to.coords, p.color);
}

// chess.rs:337-348
static bool queen_ok(const Piece& p, const Location& from, const Location& to, int32_t dx,
                     int32_t dy, const Board& b) {
  return rook_ok(p, from, to, dx, dy, b) || bishop_ok(p, from, to, dx, dy, b);
}

// chess.rs:350-360 -- no castling, no check test.
static bool king_ok(const Piece& p, const Location&, const Location& to, int32_t dx, int32_t dy,
                    const Board& b) {
  return std::abs(dx) <= 1 && std::abs(dy) <= 1 && b.is_empty_or_enemy(to.coords, p.color);
}

// chess.rs:199-212 -- dispatch on the exact kind string; anything else cannot move.
bool can_move_to(const Piece& p, const Location& from, const Location& to, const Board& b) {
  const int32_t dx = static_cast<int32_t>(to.coords[0]) - static_cast<int32_t>(from.coords[0]);
  const int32_t dy = static_cast<int32_t>(to.coords[1]) - static_cast<int32_t>(from.coords[1]);
  if (p.kind == "P") return pawn_ok(p, from, to, dx, dy, b);
  if (p.kind == "R") return rook_ok(p, from, to, dx, dy, b);
  if (p.kind == "N") return knight_ok(p, from, to, dx, dy, b);
  if (p.kind == "B") return bishop_ok(p, from, to, dx, dy, b);
  if (p.kind == "Q") return queen_ok(p, from, to, dx, dy, b);
  if (p.kind == "K") return king_ok(p, from, to, dx, dy, b);
  return false;
}

static bool in_range(const Board& b, const Position& p) {
  return p.x < b.rows.size() && p.y < b.rows[p.x].cells.size();
}

// chess.rs:82-98 -- both squares are looked up (through a full board clone each)
// before any rule is checked; an out-of-range index panics in the reference.
uint8_t GameState::validate_move(const Position& from, const Position& to) const {
  if (!in_range(*board, from) || !in_range(*board, to)) return V_OOR;
  Board clone_a = *board;  // chess.rs:85
  Location lf{{from.x, from.y}, clone_a.rows[from.x].cells[from.y].piece};
  Board clone_b = *board;  // chess.rs:92
  Location lt{{to.x, to.y}, clone_b.rows[to.x].cells[to.y].piece};
  return validate_move_inner(lf, lt);
}

// chess.rs:100-125
uint8_t GameState::validate_move_inner(const Location& from, const Location& to) const {
  if (!from.piece) return V_NO_PIECE;
  if (turn != 0 && turn != 1) return V_BAD_TURN;  // Color::from_i32(..).expect panics
  if (from.piece->color != turn) return V_WRONG_TURN;
  if (!can_move_to(*from.piece, from, to, *board)) return V_ILLEGAL;
  return V_OK;
}

// chess.rs:127-131
static std::string square_name(const Position& p) {
  std::string s;
  s.push_back(static_cast<char>('a' + static_cast<uint8_t>(p.y)));
  s += std::to_string(p.x + 1);
  return s;
}

// chess.rs:133-154 -- kind letter unless pawn; pawn captures prefix the file.
static std::string notation(const Position& from, const Position& to, const Piece& p, bool capture) {
  std::string s;
  if (p.kind != "P") s += p.kind;
  if (capture) {
    if (p.kind == "P") s.push_back(static_cast<char>('a' + static_cast<uint8_t>(from.y)));
    s.push_back('x');
  }
  s += square_name(to);
  return s;
}

// chess.rs:156-184 -- n counts whitespace tokens already in the history, so the
// numbers run 1, 3, 5, ... (each entry "k. san" is two tokens).
void GameState::update_history(const Position& from, const Position& to) {
  const Piece& mover = *board->rows[from.x].cells[from.y].piece;
  const bool capture = board->rows[to.x].cells[to.y].piece.has_value();
  std::string san = notation(from, to, mover, capture);
  // chess.rs:169-175: history.split_whitespace().count() -- Rust's
  // char::is_whitespace, i.e. the Unicode White_Space set, over UTF-8 text
  // (an ASCII-only split would miss e.g. U+3000 or U+00A0 in a name-bearing
  // start history)
  auto white = [](uint32_t c) {
    return (c >= 0x09 && c <= 0x0D) || c == 0x20 || c == 0x85 || c == 0xA0 || c == 0x1680 ||
           (c >= 0x2000 && c <= 0x200A) || c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F || c == 0x3000;
  };
  size_t n = 0;
  bool in_word = false;
  const std::string& hs = *history;
  for (size_t i = 0; i < hs.size();) {
    const unsigned char c0 = (unsigned char)hs[i];
    const int len = c0 < 0x80 ? 1 : c0 < 0xE0 ? 2 : c0 < 0xF0 ? 3 : 4;
    uint32_t c = len == 1 ? c0 : len == 2 ? (c0 & 0x1F) : len == 3 ? (c0 & 0x0F) : (c0 & 0x07);
    for (int k = 1; k < len && i + k < hs.size(); ++k) c = (c << 6) | ((unsigned char)hs[i + k] & 0x3F);
    i += len;
    if (white(c)) in_word = false;
    else if (!in_word) { in_word = true; ++n; }
  }
  std::string& h = *history;
  if (n != 0) h.push_back(' ');
  h += std::to_string(n + 1);
  h += ". ";
  h += san;
}

// chess.rs:43-80
uint8_t GameState::apply_move(const Position& from, const Position& to, bool record_history) {
  const uint8_t v = validate_move(from, to);  // chess.rs:44-46
  if (v != V_OK) return v;
  if (record_history) update_history(from, to);  // chess.rs:48
  Board clone_a = *board;                        // chess.rs:52
  Location lf{{from.x, from.y}, clone_a.rows[from.x].cells[from.y].piece};
  Board clone_b = *board;                        // chess.rs:59
  Location lt{{to.x, to.y}, clone_b.rows[to.x].cells[to.y].piece};
  if (lt.piece && lt.piece->color == turn) return V_ILLEGAL;  // chess.rs:64-70 (unreachable)
  board->rows[lt.coords[0]].cells[lt.coords[1]].piece = lf.piece;  // chess.rs:72-73
  board->rows[lf.coords[0]].cells[lf.coords[1]].piece.reset();     // chess.rs:74-75
  turn = (turn + 1) % 2;                                           // chess.rs:77
  return V_OK;
}

// ---------------------------------------------------------------- adapters
static const char* kKindNames[7] = {"P", "N", "B", "R", "Q", "K", "X"};

void board_from_cells(const int8_t* cells, Board& out) {
  out.rows.assign(8, Row{});
  for (int x = 0; x < 8; ++x) {
    out.rows[x].cells.assign(8, Cell{});
    for (int y = 0; y < 8; ++y) {
      const int8_t c = cells[8 * x + y];
      if (c < 0) continue;
      out.rows[x].cells[y].piece = Piece{c >> 3, kKindNames[c & 7]};
    }
  }
}

static int kind_index(const std::string& k) {
  for (int i = 0; i < 6; ++i)
    if (k == kKindNames[i]) return i;
  return 6;
}

void board_to_cells(const Board& b, int8_t* cells) {
  for (int x = 0; x < 8; ++x)
    for (int y = 0; y < 8; ++y) {
      const auto& p = b.rows[x].cells[y].piece;
      cells[8 * x + y] = p ? static_cast<int8_t>(p->color * 8 + kind_index(p->kind)) : -1;
    }
}

// ABI nibble per square (include/dchess.h): bb[0] = black bit, bb[1..3] = bits of
// the kind code P=1 N=2 K=3 other=4 B=5 R=6 Q=7.  Restated independently here.
void board_to_quad(const Board& b, uint64_t bb[4]) {
  static const int code[7] = {1, 2, 5, 6, 7, 3, 4};
  bb[0] = bb[1] = bb[2] = bb[3] = 0;
  for (int x = 0; x < 8; ++x)
    for (int y = 0; y < 8; ++y) {
      const auto& p = b.rows[x].cells[y].piece;
      if (!p) continue;
      const uint64_t m = 1ull << (8 * x + y);
      const int k = code[kind_index(p->kind)];
      if (p->color == 1) bb[0] |= m;
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

// Final-state digest (DESIGN.md "digest"): folds bb[3], bb[2], bb[1], bb[0] into
// a seed carrying the side to move.
uint64_t state_digest(const GameState& g) {
  uint64_t bb[4];
  board_to_quad(*g.board, bb);
  uint64_t h = 0x6A09E667F3BCC909ull ^ static_cast<uint64_t>(g.turn & 1);
  h = fmix64(h ^ bb[3]);
  h = fmix64(h ^ bb[2]);
  h = fmix64(h ^ bb[1]);
  h = fmix64(h ^ bb[0]);
  return h;
}

// perft(pos, d) = sum over accepted (f,t) of perft(apply(pos,f,t), d-1).
// Brute force over all 4096 pairs, exactly as a caller of validate_move would.
uint64_t perft(const GameState& g, unsigned depth, uint64_t* divide) {
  if (depth == 0) return 1;
  uint64_t total = 0;
  for (uint32_t f = 0; f < 64; ++f)
    for (uint32_t t = 0; t < 64; ++t) {
      const Position pf{f >> 3, f & 7}, pt{t >> 3, t & 7};
      if (g.validate_move(pf, pt) != V_OK) continue;
      uint64_t n;
      if (depth == 1) {
        n = 1;
      } else {
        GameState child = g;
        child.apply_move(pf, pt, /*record_history=*/false);
        n = perft(child, depth - 1, nullptr);
      }
      if (divide) divide[f * 64 + t] = n;
      total += n;
    }
  return total;
}

}  // namespace refcpu
