/*
 * dchess.h -- C ABI of the MI355X chess state-transition engine.
 *
 * Drop-in boundary for the reference's move-validation call surface
 * (dorlneylon/distributed-chess @ 2024-10-22, core/src/chess.rs):
 *
 *   reference (Rust inherent methods)                      replaced by
 *   -----------------------------------------------------  ------------------------------
 *   GameState::validate_move(&self,&Position,&Position)    dc_validate_batch (n >= 1)
 *       core/src/chess.rs:82-98, called from
 *       core/src/consensus/hotstuff.rs:138 (is_valid_tx)
 *   GameState::apply_move(&mut self,Position,Position)     dc_apply_batch
 *       core/src/chess.rs:43-80, called from
 *       core/src/consensus/hotstuff.rs:52 (commit_block)
 *   GameState::new / Board::new                            dc_startpos
 *       core/src/chess.rs:12-20, :383-434
 *   proto GameState.board (core/proto/game.proto:7-40)     dc_pos_from_cells / dc_pos_to_cells
 *   Position{x,y} pairs (core/proto/query.proto:46-49)     dc_move_pack
 *   AppError::InternalGameError(String)                    dc_verdict_message
 *       core/src/errors.rs:9, strings chess.rs:104-121
 *   (absent in the reference)                  dc_replay, dc_gen_games, dc_perft
 *
 * Conventions
 *   - Every call returns int status: DC_SUCCESS (0) or a negative DC_E* code.
 *     Nothing panics or aborts across the ABI; a rejected move is a verdict
 *     (data), never an error.
 *   - Buffers are caller-owned HOST memory unless the name ends in _device,
 *     in which case they are device pointers on the context's device.
 *   - A dc_ctx is bound to one device and one HIP stream and is not thread-safe:
 *     use one context per thread.  Host-memory calls block until results are
 *     on the host (wrap them in tokio::task::spawn_blocking on the Rust side).
 *   - All arithmetic is integer; results are bit-exact with the reference.
 *
 * There is no CPU fallback behind this ABI: if no gfx950 device is present,
 * dc_ctx_create fails with DC_ENODEV.
 */
#ifndef DCHESS_H
#define DCHESS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ status */
#define DC_SUCCESS 0
#define DC_EINVAL (-1)       /* bad argument (null pointer, bad cell, bad turn, bad FEN) */
#define DC_EHIP (-2)         /* HIP runtime failure */
#define DC_ENOMEM (-3)       /* device or host allocation failed */
#define DC_ENODEV (-4)       /* no usable gfx950 device */
#define DC_ERCCL (-5)        /* RCCL failure (dc_multi_*) */
#define DC_EUNSUPPORTED (-6) /* request outside what this build supports */

/* ----------------------------------------------------------------- verdicts
 * In the reference's check order (chess.rs:82-125), with OOR first because the
 * reference indexes both squares before any rule check (chess.rs:85,92). */
#define DC_V_OK 0
#define DC_V_NO_PIECE 1   /* "No piece at the source location"     chess.rs:104-106 */
#define DC_V_WRONG_TURN 2 /* "It's not this piece's turn to move"  chess.rs:113-115 */
#define DC_V_ILLEGAL 3    /* "Invalid move for the piece"          chess.rs:119-121 */
#define DC_V_OOR 4        /* coordinate >= 8: the reference panics (chess.rs:85,92) */

/* ------------------------------------------------------------------- rules */
#define DC_RULES_REF 0  /* bit-exact with core/src/chess.rs (geometry only) */
#define DC_RULES_FIDE 1 /* standard chess: castling, en passant, promotion, no self-check */

/* ---------------------------------------------------------------- position
 * Quad-bitboard: square s = 8*x + y (x = row, 0 = White's back rank; y = column),
 * the 4-bit nibble of square s is (bb[0]>>s &1) | (bb[1]>>s &1)<<1 | ... :
 *   bb[0]            : 1 = black piece
 *   bb[1],bb[2],bb[3]: bits 0,1,2 of the kind code
 *                      P=1 N=2 K=3 OTHER=4 B=5 R=6 Q=7   (0 = empty square)
 * so  diagonal sliders = bb[3]&bb[1], orthogonal sliders = bb[3]&bb[2].
 * OTHER is a piece whose kind string is not one of "P","N","B","R","Q","K":
 * it never moves (chess.rs:210) but blocks and can be captured.
 * stm: side to move, 0 White / 1 Black (proto Color, game.proto:20-23).
 * castle (FIDE): bit0 White O-O, bit1 White O-O-O, bit2 Black O-O, bit3 Black O-O-O.
 * ep (FIDE): en-passant target square or -1.  Both are ignored under DC_RULES_REF. */
typedef struct dc_pos {
  uint64_t bb[4];
  uint8_t stm;
  uint8_t castle;
  int8_t ep;
  uint8_t reserved0;
  uint32_t reserved1;
} dc_pos; /* 40 bytes */

/* -------------------------------------------------------------------- moves
 * uint16: from | to<<6 | promo<<12, promo 0 none, 1 N, 2 B, 3 R, 4 Q (FIDE only;
 * ignored under REF, where a Position pair carries no promotion).
 * Bit 15 (DC_MOVE_OOR) marks a move with a coordinate >= 8: verdict DC_V_OOR.
 * 0xFFFF (DC_MOVE_NONE) pads replay games that ended: skipped, not counted. */
#define DC_MOVE_OOR 0x8000u
#define DC_MOVE_NONE 0xFFFFu

/* Cell encoding of dc_pos_from_cells / dc_pos_to_cells (the proto board flattened):
 * cells[8*x+y] = -1 for an empty cell, else color*8 + kind with
 * kind 0 P, 1 N, 2 B, 3 R, 4 Q, 5 K, 6 OTHER; color 0 White, 1 Black. */
#define DC_CELL_EMPTY (-1)

typedef struct dc_ctx dc_ctx;

typedef struct dc_replay_stats {
  uint64_t validated;  /* non-sentinel plies (accepted + rejected) */
  uint64_t accepted;
  uint64_t rejected;
  uint64_t digest_sum; /* sum of per-game final-state digests (mod 2^64) */
  uint64_t digest_xor; /* xor of per-game final-state digests */
} dc_replay_stats;

typedef struct dc_kernel_stats {
  uint64_t launches;  /* launches of the kernel since the last reset */
  double total_ms;    /* summed HIP-event duration of those launches */
  uint64_t units;     /* work units those launches processed (leaves, moves, ...) */
} dc_kernel_stats;

/* ------------------------------------------------------------------ context */
int dc_ctx_create(int device, dc_ctx** out);
int dc_ctx_destroy(dc_ctx* ctx);
int dc_ctx_device(const dc_ctx* ctx);
/* hipStream_t of the context, as void* (so callers can order their own work). */
void* dc_ctx_stream(dc_ctx* ctx);
const char* dc_strerror(int status);
/* Exact reference error text for verdicts 1..3 (chess.rs:104-121); "" for OK. */
const char* dc_verdict_message(uint8_t verdict);
int dc_version(void);

/* Per-kernel HIP-event timing (enable, read, reset).  Kernel names:
 * "validate", "replay", "gen_games", "expand_count", "expand_write", "count1", "count2". */
int dc_ctx_set_profiling(dc_ctx* ctx, int enable);
int dc_ctx_kernel_stats(dc_ctx* ctx, const char* kernel, dc_kernel_stats* out);
int dc_ctx_reset_stats(dc_ctx* ctx);

/* Device memory owned by the caller, on the context's device (for the *_device
 * entry points, so a host program needs no other GPU runtime). */
int dc_device_alloc(dc_ctx* ctx, size_t bytes, void** d_ptr);
int dc_device_free(dc_ctx* ctx, void* d_ptr);
int dc_memcpy_h2d(dc_ctx* ctx, void* d_dst, const void* src, size_t bytes);
int dc_memcpy_d2h(dc_ctx* ctx, void* dst, const void* d_src, size_t bytes);

/* ----------------------------------------------------------------- adapters
 * Pure data-layout conversions on the host (no rule evaluation). */
int dc_startpos(dc_pos* out); /* Board::new + turn White, chess.rs:12-20,383-434 */
int dc_pos_from_cells(const int8_t cells[64], uint8_t turn, dc_pos* out);
int dc_pos_to_cells(const dc_pos* pos, int8_t cells[64], uint8_t* turn);
int dc_pos_from_fen(const char* fen, dc_pos* out);
/* Position{x,y} pair -> move word; any coordinate >= 8 sets DC_MOVE_OOR. */
uint16_t dc_move_pack(uint32_t from_x, uint32_t from_y, uint32_t to_x, uint32_t to_y);
/* A block's Transaction.action lists (core/proto/query.proto:46-49, the u32
 * Position pairs of is_valid_tx's action[0..2], hotstuff.rs:138) -> move words:
 * actions[4i .. 4i+4) = from.x, from.y, to.x, to.y (the dc_verify_tx_batch
 * layout, so one packed block feeds both checks); moves[i] = dc_move_pack of
 * them, DC_MOVE_OOR for any coordinate >= 8 (where the reference panics). */
int dc_move_pack_batch(const uint32_t* actions, uint32_t n, uint16_t* moves);

/* ------------------------------------------------------------- validation
 * verdicts[i] = verdict of moves[i] in pos[i] (rules per call). */
int dc_validate_batch(dc_ctx* ctx, uint32_t rules, const dc_pos* pos, const uint16_t* moves, uint32_t n,
                      uint8_t* verdicts);
/* Validate and, where accepted, make the move in place (pos[i] updated, turn
 * flipped); rejected positions are left untouched (chess.rs:44-46).
 * info[i] (optional) = moved kind (cell kind 0..6) | 8 if the target held a piece,
 * which is what update_history needs (chess.rs:156-167). */
int dc_apply_batch(dc_ctx* ctx, uint32_t rules, dc_pos* pos, const uint16_t* moves, uint32_t n,
                   uint8_t* verdicts, uint8_t* info);

/* The live validator (opt-in, per context): with lease_us > 0, every
 * dc_validate_batch / dc_apply_batch call of at most 64 moves on this context
 * is served by one resident GPU wave that polls a pinned mailbox (no kernel
 * launch per call) -- the n = 1 call is_valid_tx makes before a replica signs
 * its vote (core/src/consensus/hotstuff.rs:138, :52).  Results are identical
 * to the launched path.  The wave leaves after lease_us microseconds without a
 * call (at most 60 s; the next call restarts it), on dc_live_validator(ctx, 0)
 * and in dc_ctx_destroy.  At most one wave is resident per process: a live
 * call that starts its context's wave stops the others' first.  Every other
 * call of this library that uses the device (perft, replay, hashing,
 * signatures, launched validate / apply, device memory, dc_ctx_destroy) stops
 * the resident wave first and keeps new ones from starting until it returns:
 * HIP maps a process's streams onto a few hardware queues, and work queued
 * behind a resident wave -- and hipFree, which waits for every stream -- would
 * otherwise wait for its lease.  GPU work the CALLER issues itself (its own
 * kernels, hipDeviceSynchronize, hipFree) while a wave is resident can wait
 * for the lease: switch the validator off (lease 0) before such work. */
int dc_live_validator(dc_ctx* ctx, uint32_t lease_us);

/* ------------------------------------------------------------------ replay
 * Replays n_games games of n_plies ply-major moves (moves[ply*n_games + g])
 * from *start (NULL = startpos).  Per ply: verdict; apply only if accepted
 * (core/src/consensus/hotstuff.rs:52-56).  bitmap (optional) is ply-major
 * [n_plies][ceil(n_games/64)] of accept bits; digests (optional) [n_games]. */
int dc_replay(dc_ctx* ctx, uint32_t rules, const dc_pos* start, const uint16_t* moves, uint32_t n_games,
              uint32_t n_plies, uint64_t* bitmap, uint64_t* digests, dc_replay_stats* stats);
int dc_replay_device(dc_ctx* ctx, uint32_t rules, const dc_pos* start, const uint16_t* d_moves,
                     uint32_t n_games, uint32_t n_plies, uint64_t* d_bitmap, uint64_t* d_digests,
                     dc_replay_stats* stats);

/* Replay for a resyncing replica (the history-rebuild path): dc_replay plus
 * info (ply-major [n_plies][n_games] bytes, like the moves): for an accepted
 * ply the moved piece's cell kind (0 P .. 5 K) | 8 if the target held a piece
 * -- dc_apply_batch's info, what update_history needs (chess.rs:156-167) --
 * and 0xFF for a rejected or DC_MOVE_NONE ply.  RULES_REF only (else
 * DC_EUNSUPPORTED), and n_games * n_plies * 2 < 4 GiB per call.
 * Replaces commit_block's per-move apply_move + update_history loop
 * (core/src/consensus/hotstuff.rs:41-56) for a whole move log at once. */
int dc_replay_info(dc_ctx* ctx, uint32_t rules, const dc_pos* start, const uint16_t* moves, uint32_t n_games,
                   uint32_t n_plies, uint64_t* bitmap, uint64_t* digests, uint8_t* info, dc_replay_stats* stats);
int dc_replay_info_device(dc_ctx* ctx, uint32_t rules, const dc_pos* start, const uint16_t* d_moves,
                          uint32_t n_games, uint32_t n_plies, uint64_t* d_bitmap, uint64_t* d_digests,
                          uint8_t* d_info, dc_replay_stats* stats);
/* GameState::update_history (chess.rs:127-184) over one game's plies, on the
 * host: history (NUL-terminated UTF-8, NULL = "") followed by one
 * "N. <notation>" token pair per accepted ply (info != 0xFF), numbered as the
 * reference numbers them (N = 1 + the whitespace-separated tokens already
 * present: 1, 3, 5, ...).  moves/info of ply p at [p * stride] (stride =
 * n_games for a column of dc_replay_info's ply-major arrays).  *out_len = the
 * result's length; out (capacity out_cap, incl. the NUL) receives it, or
 * DC_EINVAL if out_cap is too small (out_cap = 0 only sizes it). */
int dc_history_append(const char* history, const uint16_t* moves, const uint8_t* info, uint32_t n_plies,
                      size_t stride, char* out, size_t out_cap, size_t* out_len);

/* Seeded synthetic games: rng = splitmix64 from seed ^ game_id;
 * per ply one draw r: (r & 0xFF) < noise_per_256 -> move (r>>8)&0xFFF, else the
 * ((r>>32)*n>>32)-th legal move in (from, to, promo) order; no legal move ->
 * DC_MOVE_NONE for the rest of the game.  Output ply-major [n_plies][n_games]. */
int dc_gen_games(dc_ctx* ctx, uint32_t rules, uint64_t seed, uint64_t first_game, uint32_t n_games,
                 uint32_t n_plies, uint32_t noise_per_256, uint16_t* out);
int dc_gen_games_device(dc_ctx* ctx, uint32_t rules, uint64_t seed, uint64_t first_game, uint32_t n_games,
                        uint32_t n_plies, uint32_t noise_per_256, uint16_t* d_out);

/* ------------------------------------------------------------- state hash
 * The hash a replica compares before voting: keccak256(serde_json(GameState))
 * (core/src/consensus/hotstuff.rs:153-166 calculate_game_state_hash; the same
 * keccak-of-JSON as BlockBuilder::build, core/src/consensus/types.rs:45-55).
 *
 * dc_keccak256: alloy-primitives keccak256 (Keccak-256, padding 0x01..0x80)
 * of one byte string, on the host -- the single-state path of the host
 * mirrors.
 *
 * dc_state_hash: for every game of a replay batch, the hash of its FINAL
 * GameState, on the GPU: start (dc_pos; NULL = startpos; turn = start.stm)
 * plus the game's accepted moves (RULES_REF, chess.rs:43-80), each one's
 * notation appended to `history` (chess.rs:127-184; the start history is
 * shared by all games, NUL-terminated UTF-8, "" for GameState::new).  Player
 * names: UTF-8 bytes names[names_off[2g] .. names_off[2g+1]) (white) and
 * [names_off[2g+1] .. names_off[2g+2]) (black); names_off has 2*n_games+1
 * entries.  hashes[32 g .. 32 g + 32) = the 32 digest bytes (alloy B256;
 * "0x" + hex of them is calculate_game_state_hash's String).  A start board
 * holding pieces of unknown kind returns DC_EUNSUPPORTED (their proto kind
 * string is not representable in a dc_pos).
 *
 * dc_state_hash_device: the same with d_names, d_names_off, d_moves and
 * d_hashes in device memory (raw UTF-8, as for dc_state_hash; history stays a
 * host string).  serde_json's escaping of the names runs on the device; a
 * decreasing offset pair is taken as an empty name (dc_state_hash rejects it
 * with DC_EINVAL).  Escaped text past 4 GiB returns DC_EUNSUPPORTED. */
int dc_keccak256(const void* data, size_t len, uint8_t out[32]);
int dc_state_hash(dc_ctx* ctx, const dc_pos* start, const char* history, const char* names,
                  const uint32_t* names_off, const uint16_t* moves, uint32_t n_games, uint32_t n_plies,
                  uint8_t* hashes);
int dc_state_hash_device(dc_ctx* ctx, const dc_pos* start, const char* history, const char* d_names,
                         const uint32_t* d_names_off, const uint16_t* d_moves, uint32_t n_games, uint32_t n_plies,
                         uint8_t* d_hashes);

/* ---------------------------------------------------- transaction signatures
 * The other per-transaction check of is_valid_tx (core/src/consensus/hotstuff.rs:139):
 * App::validate_signature (hotstuff.rs:168-208), batched on the GPU.  Per
 * transaction i:
 *   strings[str_off[4i+0] .. str_off[4i+1])  white_player (UTF-8)
 *   strings[str_off[4i+1] .. str_off[4i+2])  black_player
 *   strings[str_off[4i+2] .. str_off[4i+3])  signature (hex text, 64 bytes r||s)
 *   strings[str_off[4i+3] .. str_off[4i+4])  pub_key (hex text: 33, 64 or 65 bytes)
 *   actions[4i .. 4i+4) = action[0].x, action[0].y, action[1].x, action[1].y
 *   turns[i] (optional; NULL or -1 = skip) = the game's turn: after a valid
 *   signature, pub_key must equal the string of the player to move
 *   (hotstuff.rs:141-148), else DC_SIG_WRONG_OWNER.
 * The signed message is serde_json {"whitePlayer","blackPlayer","action":[{x,y},{x,y}]}
 * (hotstuff.rs:169-179), hashed with SHA-256; verification follows
 * libsecp256k1 0.7.1 (Message mod n, parse_standard_slice, parse_slice,
 * verify without a low-s rule).  Verdicts in the reference's check order: */
#define DC_SIG_OK 0
#define DC_SIG_BAD_SIG_HEX 1  /* hex::decode(signature) failed            hotstuff.rs:183-184 */
#define DC_SIG_BAD_SIG 2      /* Signature::parse_standard_slice failed    hotstuff.rs:186-191 */
#define DC_SIG_BAD_PK_HEX 3   /* hex::decode(pub_key) failed               hotstuff.rs:193-194 */
#define DC_SIG_BAD_PK 4       /* PublicKey::parse_slice failed             hotstuff.rs:195-200 */
#define DC_SIG_INVALID 5      /* verify() false: "invalid signature"       hotstuff.rs:202-206 */
#define DC_SIG_WRONG_OWNER 6  /* pub_key is not the mover: "invalud turn"  hotstuff.rs:141-148 */
int dc_verify_tx_batch(dc_ctx* ctx, const char* strings, const uint32_t* str_off, const uint32_t* actions,
                       const int8_t* turns, uint32_t n, uint8_t* verdicts);
int dc_verify_tx_batch_device(dc_ctx* ctx, const char* d_strings, const uint32_t* d_str_off,
                              const uint32_t* d_actions, const int8_t* d_turns, uint32_t n, uint8_t* d_verdicts);
/* Text for a DC_SIG_* verdict ("" for OK; codes 5 and 6 are the reference's strings). */
const char* dc_sig_verdict_message(uint8_t verdict);

/* -------------------------------------------------------------------- perft
 * perft(pos, depth) = number of leaf nodes of the move tree (under
 * REF the tree is every (from,to) pair validate_move accepts).  divide[i] is the
 * count below root move root_moves[i]; both arrays need room for 256 entries
 * (pass NULL to skip).  Root moves are in (from, to, promo) order. */
int dc_perft(dc_ctx* ctx, uint32_t rules, const dc_pos* pos, uint32_t depth, uint64_t* divide,
             uint16_t* root_moves, uint32_t* n_root, uint64_t* total);
/* One shard of perft for data-parallel runs: the frontier at ply `split_depth`
 * (N nodes) is built deterministically, and this call counts only the subtrees
 * of the STRIDED shard of it -- frontier nodes shard, shard + n_shards,
 * shard + 2*n_shards, ... < N (the front end selects them by index: REF depth
 * 6/7 at split 3 in k_front, else k_make_count over the top kernel's move
 * words; strided shards hold equal leaf counts to about 1 %, contiguous ones
 * did not).  Summing divide[] over all shards (e.g. an RCCL all-reduce) gives
 * dc_perft's result exactly. */
int dc_perft_shard(dc_ctx* ctx, uint32_t rules, const dc_pos* pos, uint32_t depth, uint32_t split_depth,
                   uint32_t shard, uint32_t n_shards, uint64_t* divide, uint16_t* root_moves,
                   uint32_t* n_root, uint64_t* total);

/* n_runs perfts of *pos (depth >= 2; shard as dc_perft_shard) enqueued back to
 * back on the context stream with no host round trip between them.  Run i
 * leaves its result in DEVICE memory d_out[258 i .. 258 i + 258):
 *   [0, 256) divide per root move (0 past n_root; root-move order as dc_perft)
 *   [256]    n_root | overflow << 32  (overflow != 0: redo with dc_perft_shard)
 *   [257]    total leaves of this shard
 * Returns once the runs are enqueued; dc_ctx_synchronize (or an event on
 * dc_ctx_stream) orders the caller after them.  For throughput work (a suite
 * of repeated perfts, the bench's timed steps, a device-side all-reduce of
 * each run's divide vector). */
int dc_perft_repeat_device(dc_ctx* ctx, uint32_t rules, const dc_pos* pos, uint32_t depth, uint32_t split_depth,
                           uint32_t shard, uint32_t n_shards, uint32_t n_runs, uint64_t* d_out);

/* perft of a batch of n_pos (1..DC_PERFT_BATCH_MAX) positions with the same side
 * to move, counted as one tree: their root moves (at most 256 in all; more is
 * DC_EUNSUPPORTED) share the divide tags, so every level -- the final stage's
 * included -- holds all positions and runs one grid instead of one per position
 * (a perft suite: BASELINE configs[2], the six published positions at depth 5).
 * totals[i] = perft(pos[i], depth); divide / root_moves as dc_perft over the
 * concatenated root moves, root_pos[k] = the position root move k belongs to
 * (each may be NULL; room for 256 entries). */
#define DC_PERFT_BATCH_MAX 8
int dc_perft_batch(dc_ctx* ctx, uint32_t rules, const dc_pos* pos, uint32_t n_pos, uint32_t depth, uint64_t* totals,
                   uint64_t* divide, uint16_t* root_moves, uint8_t* root_pos, uint32_t* n_root);
/* n_runs batch perfts enqueued as dc_perft_repeat_device does (depth >= 2, one
 * shard): run i's 258-word record in DEVICE memory holds the concatenated
 * divide ([257] = the batch's total); per-position totals are the sums of the
 * divide entries over dc_perft_batch's root_pos. */
int dc_perft_batch_repeat_device(dc_ctx* ctx, uint32_t rules, const dc_pos* pos, uint32_t n_pos, uint32_t depth,
                                 uint32_t split_depth, uint32_t n_runs, uint64_t* d_out);
/* Blocks until all work queued on the context stream has finished. */
int dc_ctx_synchronize(dc_ctx* ctx);

/* ------------------------------------------------------------- multi-GPU
 * One process, n_devices GPUs, one RCCL communicator (ncclCommInitAll); device
 * i counts strided shard i of the frontier (dc_perft_shard) and divide[] is
 * combined with ncclAllReduce(ncclUint64, ncclSum) over xGMI. */
int dc_multi_perft(const int* devices, int n_devices, uint32_t rules, const dc_pos* pos, uint32_t depth,
                   uint64_t* divide, uint16_t* root_moves, uint32_t* n_root, uint64_t* total);

/* Replay shard contract: game ids [0, n_games) are split into
 * contiguous ranges of whole 64-game bitmap words -- with W = ceil(n_games/64)
 * words and P = ceil(W/n_shards), shard s holds games [min(n_games, min(W, sP)*64),
 * min(n_games, min(W, (s+1)P)*64)) -- so its ply-major accept bitmap is the
 * word-column block [first/64, first/64 + ceil(count/64)) of every ply row of
 * the whole batch's bitmap.  Data-parallel callers (one process per GPU)
 * replay their own range and combine: validated / accepted / rejected /
 * digest_sum add (mod 2^64), digest_xor xors, bitmaps are gathered. */
int dc_replay_shard_range(uint64_t n_games, uint32_t shard, uint32_t n_shards, uint64_t* first, uint64_t* count);
/* The combine of the shards' bitmaps (host memory): gathered = n_shards blocks
 * [n_plies][per] with per = ceil(ceil(n_games/64) / n_shards) (each shard's
 * ply-major bitmap padded to `per` words per row, as a gather collects them);
 * bitmap = the whole batch's [n_plies][ceil(n_games/64)].  dc_multi_replay's
 * last step, and the layout a torch.distributed caller's gather produces. */
int dc_replay_scatter_shards(uint64_t n_games, uint32_t n_shards, uint32_t n_plies, const uint64_t* gathered,
                             uint64_t* bitmap);
/* The seeded games [0, n_games) (dc_gen_games' generator: seed, n_plies,
 * noise_per_256) generated and replayed on n_devices GPUs of one process,
 * shard i on device i.  bitmap (optional, HOST) = the whole batch's ply-major
 * [n_plies][ceil(n_games/64)] accept bitmap: the shards' bitmaps are gathered
 * to devices[0] with ncclGather over xGMI, then copied out; stats = the
 * combined counters. */
int dc_multi_replay(const int* devices, int n_devices, uint32_t rules, uint64_t seed, uint64_t n_games,
                    uint32_t n_plies, uint32_t noise_per_256, uint64_t* bitmap, dc_replay_stats* stats);

#ifdef __cplusplus
}
#endif
#endif /* DCHESS_H */
