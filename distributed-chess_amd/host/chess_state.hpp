// chess_state.hpp -- C++ host mirror of the reference's move-validation surface.
//
// The reference host code is Rust (core/src/chess.rs); no Rust toolchain exists
// in this image, so the host side above the C ABI (include/dchess.h) is this
// C++ restatement of the same API: GameState / Position / Piece with
// validate_move (chess.rs:82-98) and apply_move (chess.rs:43-80), errors as
// AppError::InternalGameError strings (core/src/errors.rs:9).  Every verdict
// and state update comes from the gfx950 kernels through dc_validate_batch /
// dc_apply_batch; only history formatting (chess.rs:127-184) happens here,
// from the mover kind and capture flag the kernel returns.
#pragma once
#include <array>
#include <cstdint>
#include <optional>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/dchess.h"

namespace dchess {

// AppError::InternalGameError(String), core/src/errors.rs:9.
struct AppError {
  std::string message;
};

// A Rust panic in the reference (index out of bounds, Color::from_i32(..).expect).
struct Panic : std::runtime_error {
  using std::runtime_error::runtime_error;
};

struct Position {  // proto query.Position
  uint32_t x = 0, y = 0;
};

struct Piece {  // proto game.Piece
  int32_t color = 0;
  std::string kind;
  bool operator==(const Piece& o) const { return color == o.color && kind == o.kind; }
};

// One dc_ctx (one device, one stream); not thread-safe, like the ABI.
class Engine {
 public:
  explicit Engine(int device = 0);
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;
  dc_ctx* ctx() const { return ctx_; }

 private:
  dc_ctx* ctx_ = nullptr;
};

using Board = std::array<std::array<std::optional<Piece>, 8>, 8>;

struct GameState {  // proto game.GameState, core/proto/game.proto:7-13
  int32_t turn = 0;
  std::string white_player, black_player;
  std::optional<std::string> history;
  Board board;

  static GameState create(const std::string& white, const std::string& black);  // chess.rs:12-20

  // Ok(()) -> std::nullopt; Err(AppError) -> the error.  Coordinates >= 8 or a
  // turn outside {0,1} throw Panic, as the reference panics.
  std::optional<AppError> validate_move(Engine& e, const Position& from, const Position& to) const;
  std::optional<AppError> apply_move(Engine& e, const Position& from, const Position& to);

  // Batched form for callers that validate many (state, move) pairs at once.
  static std::vector<std::optional<AppError>> validate_many(Engine& e, const std::vector<GameState>& states,
                                                            const std::vector<std::pair<Position, Position>>& moves);

  dc_pos to_pos() const;

  // serde_json::to_string(&GameState) (fields in proto order, None -> null,
  // prost i32 enums as numbers, serde_json string escapes) and
  // calculate_game_state_hash (core/src/consensus/hotstuff.rs:153-166):
  // "0x" + hex(keccak256(json)), keccak through dc_keccak256.
  std::string to_json() const;
  std::string state_hash() const;
};

}  // namespace dchess
