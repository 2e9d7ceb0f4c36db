// chess_state.cpp -- see chess_state.hpp.
#include "chess_state.hpp"

namespace dchess {

namespace {
const char* kKinds[7] = {"P", "N", "B", "R", "Q", "K", "X"};

int kind_index(const std::string& k) {
  for (int i = 0; i < 6; ++i)
    if (k == kKinds[i]) return i;
  return 6;  // any other kind string: immovable (chess.rs:210)
}

void check(int status, const char* what) {
  if (status != DC_SUCCESS) throw std::runtime_error(std::string(what) + ": " + dc_strerror(status));
}

std::optional<AppError> verdict_to_result(uint8_t v) {
  if (v == DC_V_OK) return std::nullopt;
  if (v == DC_V_OOR) throw Panic("index out of bounds");  // chess.rs:85,92 panic
  return AppError{dc_verdict_message(v)};
}
}  // namespace

namespace {
// serde_json string literal (serde_json 1.0 ser.rs ESCAPE table).
void json_str(const std::string& v, std::string& out) {
  static const char hex[] = "0123456789abcdef";
  out += '"';
  for (unsigned char ch : v) {
    switch (ch) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\b': out += "\\b"; break;
      case '\t': out += "\\t"; break;
      case '\n': out += "\\n"; break;
      case '\f': out += "\\f"; break;
      case '\r': out += "\\r"; break;
      default:
        if (ch < 0x20) {
          out += "\\u00";
          out += hex[ch >> 4];
          out += hex[ch & 15];
        } else {
          out += (char)ch;
        }
    }
  }
  out += '"';
}
}  // namespace

std::string GameState::to_json() const {
  std::string j = "{\"turn\":" + std::to_string(turn) + ",\"white_player\":";
  json_str(white_player, j);
  j += ",\"black_player\":";
  json_str(black_player, j);
  j += ",\"history\":";
  if (history) json_str(*history, j);
  else j += "null";
  j += ",\"board\":{\"rows\":[";
  for (int x = 0; x < 8; ++x) {
    j += x ? ",{\"cells\":[" : "{\"cells\":[";
    for (int y = 0; y < 8; ++y) {
      if (y) j += ',';
      const auto& p = board[x][y];
      if (!p) {
        j += "{\"piece\":null}";
      } else {
        j += "{\"piece\":{\"color\":" + std::to_string(p->color) + ",\"kind\":";
        json_str(p->kind, j);
        j += "}}";
      }
    }
    j += "]}";
  }
  j += "]}}";
  return j;
}

std::string GameState::state_hash() const {
  const std::string j = to_json();
  uint8_t h[32];
  check(dc_keccak256(j.data(), j.size(), h), "dc_keccak256");
  static const char hex[] = "0123456789abcdef";
  std::string s = "0x";
  for (uint8_t b : h) {
    s += hex[b >> 4];
    s += hex[b & 15];
  }
  return s;
}

Engine::Engine(int device) { check(dc_ctx_create(device, &ctx_), "dc_ctx_create"); }
Engine::~Engine() {
  if (ctx_) dc_ctx_destroy(ctx_);
}

GameState GameState::create(const std::string& white, const std::string& black) {
  GameState g;
  g.white_player = white;
  g.black_player = black;
  g.turn = 0;
  g.history = std::string();
  dc_pos p;
  check(dc_startpos(&p), "dc_startpos");
  int8_t cells[64];
  uint8_t turn = 0;
  check(dc_pos_to_cells(&p, cells, &turn), "dc_pos_to_cells");
  for (int s = 0; s < 64; ++s)
    if (cells[s] >= 0) g.board[s / 8][s % 8] = Piece{cells[s] >> 3, kKinds[cells[s] & 7]};
  return g;
}

dc_pos GameState::to_pos() const {
  if (turn != 0 && turn != 1) throw Panic("Correct color");  // Color::from_i32(..).expect, chess.rs:110
  int8_t cells[64];
  for (int x = 0; x < 8; ++x)
    for (int y = 0; y < 8; ++y) {
      const auto& p = board[x][y];
      cells[8 * x + y] = p ? static_cast<int8_t>(p->color * 8 + kind_index(p->kind)) : int8_t(DC_CELL_EMPTY);
      if (p && p->color != 0 && p->color != 1) throw std::invalid_argument("piece colour outside {0,1}");
    }
  dc_pos out;
  check(dc_pos_from_cells(cells, static_cast<uint8_t>(turn), &out), "dc_pos_from_cells");
  return out;
}

std::optional<AppError> GameState::validate_move(Engine& e, const Position& from, const Position& to) const {
  const dc_pos p = to_pos();
  const uint16_t m = dc_move_pack(from.x, from.y, to.x, to.y);
  uint8_t v = 0;
  check(dc_validate_batch(e.ctx(), DC_RULES_REF, &p, &m, 1, &v), "dc_validate_batch");
  return verdict_to_result(v);
}

std::optional<AppError> GameState::apply_move(Engine& e, const Position& from, const Position& to) {
  dc_pos p = to_pos();
  const uint16_t m = dc_move_pack(from.x, from.y, to.x, to.y);
  uint8_t v = 0, info = 0;
  check(dc_apply_batch(e.ctx(), DC_RULES_REF, &p, &m, 1, &v, &info), "dc_apply_batch");
  if (auto err = verdict_to_result(v)) return err;  // rejected: state untouched (chess.rs:44-46)
  // update_history (chess.rs:156-184) from the kernel's mover kind / capture
  // flag, formatted by the ABI's dc_history_append (split_whitespace numbering)
  std::string& h = *history;
  size_t len = 0;
  check(dc_history_append(h.c_str(), &m, &info, 1, 1, nullptr, 0, &len), "dc_history_append");
  std::string out(len + 1, '\0');
  check(dc_history_append(h.c_str(), &m, &info, 1, 1, out.data(), out.size(), &len), "dc_history_append");
  out.resize(len);
  h = out;
  // the board after the move, from the kernel's position (unknown kinds never move)
  int8_t cells[64];
  uint8_t t = 0;
  check(dc_pos_to_cells(&p, cells, &t), "dc_pos_to_cells");
  Board nb;
  for (int s = 0; s < 64; ++s) {
    if (cells[s] < 0) continue;
    std::string kind = kKinds[cells[s] & 7];
    if (kind == "X") kind = board[s / 8][s % 8]->kind;
    nb[s / 8][s % 8] = Piece{cells[s] >> 3, kind};
  }
  board = nb;
  turn = t;
  return std::nullopt;
}

std::vector<std::optional<AppError>> GameState::validate_many(Engine& e, const std::vector<GameState>& states,
                                                              const std::vector<std::pair<Position, Position>>& moves) {
  if (states.size() != moves.size()) throw std::invalid_argument("states/moves size mismatch");
  std::vector<dc_pos> pos(states.size());
  std::vector<uint16_t> mv(states.size());
  for (size_t i = 0; i < states.size(); ++i) {
    pos[i] = states[i].to_pos();
    mv[i] = dc_move_pack(moves[i].first.x, moves[i].first.y, moves[i].second.x, moves[i].second.y);
  }
  std::vector<uint8_t> v(states.size());
  check(dc_validate_batch(e.ctx(), DC_RULES_REF, pos.data(), mv.data(), static_cast<uint32_t>(v.size()), v.data()),
        "dc_validate_batch");
  std::vector<std::optional<AppError>> out;
  out.reserve(v.size());
  for (uint8_t x : v) {
    if (x == DC_V_OOR) out.push_back(AppError{"index out of bounds"});
    else out.push_back(x == DC_V_OK ? std::nullopt : std::optional<AppError>(AppError{dc_verdict_message(x)}));
  }
  return out;
}

}  // namespace dchess
