// tests/cpp/test_chess_rs.cpp -- the reference's unit tests
// (/root/reference/core/src/chess.rs:499-557) restated against the C++ host
// mirror (distributed-chess_amd/host/chess_state.hpp), i.e. through the C ABI
// to the gfx950 kernels.  Exit code 0 = all pass.  Run by tests/test_cpp_host.py.
#include <cstdio>
#include <cstring>

#include "../../distributed-chess_amd/host/chess_state.hpp"

using dchess::AppError;
using dchess::Engine;
using dchess::GameState;
using dchess::Position;

static int failures = 0;
#define CHECK(cond)                                                  \
  do {                                                               \
    if (!(cond)) {                                                   \
      std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);  \
      ++failures;                                                    \
    }                                                                \
  } while (0)

// chess.rs:504-514
static void test_initial_game_state() {
  GameState g = GameState::create("Alice", "Bob");
  CHECK(g.turn == 0);
  CHECK(g.white_player == "Alice");
  CHECK(g.black_player == "Bob");
}

// chess.rs:516-530
static void test_pawn_valid_move(Engine& e) {
  GameState g = GameState::create("Alice", "Bob");
  CHECK(!g.validate_move(e, Position{1, 0}, Position{3, 0}));
  g.turn = 1;
  CHECK(!g.validate_move(e, Position{6, 0}, Position{5, 0}));
}

// chess.rs:532-539
static void test_rook_invalid_move(Engine& e) {
  GameState g = GameState::create("Alice", "Bob");
  CHECK(g.validate_move(e, Position{0, 0}, Position{2, 2}).has_value());
}

// chess.rs:541-556
static void test_turn_logic(Engine& e) {
  GameState g = GameState::create("Alice", "Bob");
  g.turn = 0;
  CHECK(!g.validate_move(e, Position{1, 0}, Position{2, 0}));
  g.turn = 1;
  CHECK(!g.validate_move(e, Position{6, 0}, Position{5, 0}));
}

// Beyond the reference's tests: error strings, apply + history.
static void test_errors_and_history(Engine& e) {
  GameState g = GameState::create("Alice", "Bob");
  auto r = g.validate_move(e, Position{3, 3}, Position{4, 3});
  CHECK(r && r->message == "No piece at the source location");
  r = g.validate_move(e, Position{6, 0}, Position{5, 0});
  CHECK(r && r->message == "It's not this piece's turn to move");
  r = g.validate_move(e, Position{0, 2}, Position{2, 4});
  CHECK(r && r->message == "Invalid move for the piece");
  bool panicked = false;
  try {
    g.validate_move(e, Position{8, 0}, Position{0, 0});
  } catch (const dchess::Panic&) {
    panicked = true;
  }
  CHECK(panicked);
  CHECK(!g.apply_move(e, Position{1, 4}, Position{3, 4}));
  CHECK(!g.apply_move(e, Position{6, 4}, Position{4, 4}));
  CHECK(!g.apply_move(e, Position{0, 5}, Position{3, 2}));
  CHECK(*g.history == "1. e4 3. e5 5. Bc4");
  CHECK(g.turn == 1);
  CHECK(g.board[3][2] && g.board[3][2]->kind == "B" && !g.board[0][5]);
  auto rej = g.apply_move(e, Position{0, 0}, Position{2, 2});  // not black's piece
  CHECK(rej && rej->message == "It's not this piece's turn to move" && *g.history == "1. e4 3. e5 5. Bc4");
}

// --json: serde_json(GameState) + calculate_game_state_hash of a fixed state
// (host only, no device), checked by tests/test_cpp_host.py against the oracle.
static int print_json_case() {
  GameState g = GameState::create("Al\"ice\\", "B\tob\x01");
  g.history = std::string("1. e4 3. e5");
  g.board[3][4] = g.board[1][4];
  g.board[1][4].reset();
  g.board[4][4] = g.board[6][4];
  g.board[6][4].reset();
  g.board[5][5] = dchess::Piece{1, "Dragon"};
  std::printf("%s\n%s\n", g.to_json().c_str(), g.state_hash().c_str());
  g.history.reset();
  g.turn = 1;
  std::printf("%s\n%s\n", g.to_json().c_str(), g.state_hash().c_str());
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && std::strcmp(argv[1], "--json") == 0) return print_json_case();
  try {
    Engine e(0);
    test_initial_game_state();
    test_pawn_valid_move(e);
    test_rook_invalid_move(e);
    test_turn_logic(e);
    test_errors_and_history(e);
  } catch (const std::exception& ex) {
    std::printf("ERROR %s\n", ex.what());
    return 2;
  }
  std::printf("%s (%d failures)\n", failures ? "FAILED" : "OK", failures);
  return failures ? 1 : 0;
}
