// dc_hash.hip -- the consensus state hash of replayed games on gfx950.
//
//   k_state_hash_ref   one lane per game: replay (RULES_REF), serialise the
//                      final GameState as serde_json, keccak256 it
//
// What a replica computes before voting is keccak256(serde_json(GameState))
// (core/src/consensus/hotstuff.rs:153-166; the same hash over a block at
// core/src/consensus/types.rs:45-55).  For a batch of games this kernel gives
// every game's final-state hash: a replay that ends in the value a replica
// compares, i.e. a resync engine.
//
// The final state of game g: the start (turn, board, history) with the game's
// accepted moves applied (chess.rs:43-80) and each one's notation appended to
// the history (chess.rs:127-184: "N. san", N = whitespace tokens so far + 1).
// JSON layout (serde_json, struct fields in prost's proto order, game.proto:7-40):
//   {"turn":T,"white_player":"W","black_player":"B","history":"H",
//    "board":{"rows":[{"cells":[{"piece":null},{"piece":{"color":0,"kind":"R"}},...]},...]}}
// The start history arrives JSON-escaped from the host (one short string per
// batch); the player names are escaped on the device (k_escape_len -> scan ->
// k_escape_write, below) from raw UTF-8 resident in HBM; the tokens the kernel
// appends are plain ASCII.
//
// Per lane: pass 1 learns the final turn (the first JSON field); pass 2
// streams the JSON bytes into the sponge, making only the accepted moves.
// Since round 5 the host runs the replay kernel's per-ply info pass first
// (info: verdict, mover kind, capture per ply), so pass 1 is the accepted
// plies' parity and pass 2 validates nothing.  Without info (a batch past
// the replay kernel's one buffer descriptor), pass 1 replays the game
// (ref_verdict + make per ply) and keeps each ply's verdict as one bit in LDS
// (the first kAccPlies plies; later plies are validated again in pass 2).
// Bytes are produced into the lane's 136-byte block in LDS by a small piece
// state machine (template strings, names, start history, per-move tokens,
// board cells); every lane emits exactly one block per step, so the
// permutations of a wave run together until its lanes' streams end.
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include "dc_common.h"
#include "dc_hash.h"
#include "dc_keccak.h"

DC_BBPROF_DEFINE(hash)  // measurement builds only (tools/bbprof.py)

namespace dc {

// ----------------------------------------------------------- JSON templates
// All fixed strings in one blob; a piece is (offset, length) in it.
struct JsonTpl {
  char s[768];
  uint16_t off[32], len[32];
};
enum : int {
  T_TURN = 0,   // {"turn":
  T_DIGITS,     // 01
  T_WP,         // ,"white_player":"
  T_BP,         // ","black_player":"
  T_HIST,       // ","history":"
  T_BOARD,      // ","board":{"rows":[
  T_ROW,        // {"cells":[
  T_ROW_END,    // ]},   (the last row drops the comma)
  T_END,        // ]}}
  T_NULL,       // {"piece":null},   (the last cell of a row drops the comma)
  T_CELL0,      // {"piece":{"color":0,"kind":"P"}},  ... 12 cells: colour-major P N B R Q K
  T_NULLRUN = T_CELL0 + 12,  // T_NULL eight times: a run of k empty cells is its first 15 k bytes
  T_BOARD_ROW,  // ","board":{"rows":[{"cells":[   (T_BOARD + T_ROW: DC_HASH_MERGE)
  T_ROW_SEP,    // ]},{"cells":[                  (T_ROW_END + T_ROW)
  T_LAST,       // ]}]}}                          (the last row's end + T_END)
  T_COUNT
};

constexpr JsonTpl make_json_tpl() {
  JsonTpl t{};
  const char* strs[T_COUNT] = {"{\"turn\":", "01", ",\"white_player\":\"", "\",\"black_player\":\"",
                               "\",\"history\":\"", "\",\"board\":{\"rows\":[", "{\"cells\":[", "]},", "]}}",
                               "{\"piece\":null},", nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                               nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                               "\",\"board\":{\"rows\":[{\"cells\":[", "]},{\"cells\":[", "]}]}}"};
  int p = 0;
  for (int i = 0; i < T_COUNT; ++i) {
    t.off[i] = (uint16_t)p;
    if (i == T_NULLRUN) {
      for (int r = 0; r < 8; ++r)
        for (const char* c = strs[T_NULL]; *c; ++c) t.s[p++] = *c;
    } else if (strs[i]) {
      for (const char* c = strs[i]; *c; ++c) t.s[p++] = *c;
    } else {  // {"piece":{"color":C,"kind":"K"}},
      const int k = i - T_CELL0;
      const char kinds[6] = {'P', 'N', 'B', 'R', 'Q', 'K'};
      const char* a = "{\"piece\":{\"color\":";
      for (const char* c = a; *c; ++c) t.s[p++] = *c;
      t.s[p++] = (char)('0' + k / 6);
      const char* b = ",\"kind\":\"";
      for (const char* c = b; *c; ++c) t.s[p++] = *c;
      t.s[p++] = kinds[k % 6];
      t.s[p++] = '"';
      t.s[p++] = '}';
      t.s[p++] = '}';
      t.s[p++] = ',';
    }
    t.len[i] = (uint16_t)(p - t.off[i]);
  }
  return t;
}
__constant__ JsonTpl g_json_tpl = make_json_tpl();
constexpr JsonTpl kJsonTpl = make_json_tpl();
constexpr u32 kCellNullOff = kJsonTpl.off[T_NULL], kCellNullLen = kJsonTpl.len[T_NULL];
constexpr u32 kCell0Off = kJsonTpl.off[T_CELL0], kCellLen = kJsonTpl.len[T_CELL0];
constexpr bool cells_even() {
  for (int k = 1; k < 12; ++k)
    if (kJsonTpl.len[T_CELL0 + k] != kCellLen || kJsonTpl.off[T_CELL0 + k] != kCell0Off + k * kCellLen) return false;
  return true;
}
static_assert(cells_even(), "the 12 piece-cell templates are consecutive and of one length");
constexpr u32 kNullRunOff = kJsonTpl.off[T_NULLRUN];
static_assert(kJsonTpl.len[T_NULLRUN] == 8 * kCellNullLen, "eight null cells");
static_assert(kNullRunOff + 8 * kCellNullLen + 8 <= sizeof(kJsonTpl.s), "copy8 may read 7 bytes past a piece");
// DC_HASH_NULLRUN (round 6): a run of empty cells in a row is one piece (the
// first 15 k bytes of T_NULLRUN), so the board's ~32 empty cells take ~10
// trips of the fill loop instead of 32.
#ifndef DC_HASH_NULLRUN
#define DC_HASH_NULLRUN 1
#endif
// DC_HASH_MERGE (round 6): fewer trips of the fill loop -- the row boundaries
// as one piece each (T_BOARD_ROW, T_ROW_SEP, T_LAST instead of two), and up to
// two accepted moves' tokens per token piece.
#ifndef DC_HASH_MERGE
#define DC_HASH_MERGE 1
#endif
// DC_HASH_TOK3 (round 6): three tokens per piece while the move numbers are
// BCD (a token then has at most 15 bytes), two otherwise; the token area grows
// to 46 B a lane and the block rows shrink to 144 B to keep three blocks' LDS
// under 160 KB.
#ifndef DC_HASH_TOK3
#define DC_HASH_TOK3 1
#endif
constexpr u32 kTokPerPiece = DC_HASH_MERGE ? 2 : 1;
// DC_HASH_PF (round 6): with the replay pre-pass (info), the token loop takes
// each ply's info byte and move word from a queue of DC_HASH_PF plies loaded
// ahead (0: loaded where used, the move's load waiting on the info byte's).
// Same box, alternating: 4 against 0, kernel 3.26-3.29 -> 3.15-3.20 ms
// (profiles/r06/ab_hash_pf.txt); 8 against 4 within 0.5 % (ab_hash_pf8.txt).
#ifndef DC_HASH_PF
#define DC_HASH_PF 4
#endif
// DC_HASH_P1 (round 6): pass 1's parity of the accepted plies reads this many
// info bytes per batch of loads (1: one load, one wait per ply).  16 against
// 1, same box, alternating: kernel 3.08-3.10 -> 2.92-2.95 ms
// (profiles/r06/ab_hash_p1.txt): every wave of a round starts with this loop
// at once, so its round trips had nothing to overlap.  40 measured slower
// than 16 (2.97-3.02 against 2.92-2.98 ms, ab_hash_p1_40.txt).
#ifndef DC_HASH_P1
#define DC_HASH_P1 16
#endif
// DC_HASH_GLB8 (round 6): pieces in global memory (the names, the start
// history) are copied 8 loads at a time instead of one load and wait a byte.
// Same box, alternating: kernel 2.92-2.94 ms either way (the names are ~24
// bytes a game; profiles/r06/ab_hash_glb8.txt), so off.
#ifndef DC_HASH_GLB8
#define DC_HASH_GLB8 0
#endif

// kind code (dc_ref.h: P=1 N=2 K=3 X=4 B=5 R=6 Q=7) -> index in P N B R Q K; 6 = unknown
__device__ __forceinline__ u32 kind_index(u32 code) {
  return code == KC_P ? 0 : code == KC_N ? 1 : code == KC_B ? 2 : code == KC_R ? 3 : code == KC_Q ? 4
       : code == KC_K ? 5 : 6;
}

// a + 2 on 32-bit packed BCD (7 digits: callers keep the numbers below 10^7)
__device__ __forceinline__ u32 bcd_add2(u32 a) {
  const u32 t1 = a + 0x06666666u, t2 = t1 + 2, t3 = t1 ^ 2;
  const u32 t5 = ~(t2 ^ t3) & 0x11111110u;  // the digits that carried
  return t2 - ((t5 >> 2) | (t5 >> 3));
}

constexpr u32 kHashThreads = 256;
// one token is at most 18 bytes (" " + 10 digits + ". " + kind + file + "x" +
// square); 36 B holds two and keeps three 256-thread blocks' LDS under 160 KB
constexpr u32 kTokBytes = DC_HASH_TOK3 ? 46 : 36;
constexpr u32 kAccPlies = 128;  // per-lane verdict bits kept from pass 1 (4 dwords of LDS)
// DC_HASH_COPY8 (round 5): pieces whose bytes sit in LDS (templates, move
// tokens) are copied 8 bytes a step -- eight ds_read_u8 then eight ds_write_b8
// at immediate offsets, one wait -- instead of a generic-pointer byte loop that
// waits on every byte.  A step may read up to 7 bytes past its piece (LDS: in
// the block's allocation, or 0 past it) and write up to 7 past the block's
// byte 135, so each lane's block row is kBlkRow (>= 143) bytes; the bytes
// written past a piece are overwritten by the next piece or by the padding.
#ifndef DC_HASH_COPY8
#define DC_HASH_COPY8 1
#endif
// DC_HASH_FUSE (round 5): a piece fetched in the fill loop is copied in the
// same trip (round 4 spent one trip on the fetch and the next on the copy).
#ifndef DC_HASH_FUSE
#define DC_HASH_FUSE 1
#endif
constexpr u32 kBlkRow = DC_HASH_COPY8 ? (DC_HASH_TOK3 ? 144 : 152) : kKeccakRate;  // 152 = 38 dwords: 2-way banks for the u64 absorb reads

// Stages of a lane's JSON stream (in order).
enum : u32 {
  S_TURN, S_DIGIT, S_WP, S_WNAME, S_BP, S_BNAME, S_HIST, S_HSTART, S_TOKENS, S_BOARD, S_ROW, S_CELL, S_ROW_END,
  S_END, S_DONE
};

__global__ __launch_bounds__(kHashThreads) void k_state_hash_ref(Board start, u32 stm0, const uint16_t* __restrict__ moves,
                                                                  u32 n_games, u32 n_plies,
                                                                  const char* __restrict__ hist, u32 hist_len,
                                                                  u32 hist_tokens, const char* __restrict__ names,
                                                                  const u32* __restrict__ names_off,
                                                                  const uint8_t* __restrict__ info,
                                                                  uint8_t* __restrict__ out,
                                                                  const Board* __restrict__ fboards, u32 bcd_max) {
  // templates and the lanes' move tokens in one LDS pool (a piece in LDS is an
  // offset into it; names and the start history are global pointers)
  constexpr u32 kTplBytes = sizeof(g_json_tpl.s);
  __shared__ char lpool[kTplBytes + kHashThreads * kTokBytes];
  __shared__ __attribute__((aligned(8))) uint8_t blk[kHashThreads][kBlkRow];
  char* const tpl = lpool;
  __shared__ u32 accb[kAccPlies / 32][kHashThreads];  // [word][lane]: bank per lane
  const u32 tid = threadIdx.x;
  for (u32 i = tid; i < sizeof(g_json_tpl.s); i += kHashThreads) tpl[i] = g_json_tpl.s[i];
  __syncthreads();
  const u32 g = blockIdx.x * kHashThreads + tid;
  const bool active = g < n_games;
  // ---- pass 1: the final turn
  // info != nullptr (round 5): the replay kernel ran first (k_replay_ref4's
  // INFO form, dc_replay_info's per-ply byte: the mover's kind | 8 on a
  // capture, 0xFF for a rejected move), so the turn is the accepted plies'
  // parity and pass 2 reads kind and capture from it; no ply is validated here
  u32 stm = stm0;
  if (active && info) {
    // DC_HASH_P1 bytes loaded before any is used (round 6: one at a time, the
    // loop waited a memory round trip per ply, every wave of a round at once)
    u32 p = 0;
#if DC_HASH_P1 > 1
    for (; p + DC_HASH_P1 <= n_plies; p += DC_HASH_P1) {
      u32 cb[DC_HASH_P1];
#pragma unroll
      for (int j = 0; j < DC_HASH_P1; ++j) cb[j] = info[(size_t)(p + j) * n_games + g];
#pragma unroll
      for (int j = 0; j < DC_HASH_P1; ++j) stm ^= (u32)(cb[j] != 0xFFu);
    }
#endif
    for (; p < n_plies; ++p) stm ^= (u32)(info[(size_t)p * n_games + g] != 0xFFu);
  } else if (active) {
    Board b = start;
    u32 bits = 0;
    for (u32 p = 0; p < n_plies; ++p) {
      const u32 m = moves[(size_t)p * n_games + g];
      const bool ok = m != 0xFFFFu && ref_verdict(b, stm, m) == V_OK;
      if (ok) {
        ref_make(b, (int)(m & 63), (int)((m >> 6) & 63));
        stm ^= 1;
      }
      bits |= (u32)ok << (p & 31);
      if ((p & 31) == 31 || p + 1 == n_plies) {
        if (p < kAccPlies) accb[p >> 5][tid] = bits;
        bits = 0;
      }
    }
  }
  // ---- pass 2: stream the JSON into the sponge
  // The stream is a sequence of pieces (src, rem): template strings and tokens
  // in LDS, names and the start history in global memory, all read through
  // generic (flat) pointers so the byte copy has one code path.  A piece is
  // chosen once (the divergent part) and then copied in runs.
  // fboards (round 6, with info): the final board comes from the replay
  // kernel's info pass, so no move is made here (the tokens need only the
  // info bytes; ref_make per accepted move was 5 % of the kernel's issue)
  Board b = (fboards && active) ? fboards[g] : start;
  u32 cur = stm0, ply = 0, ntok = hist_tokens;
  // the move number ntok + 1 as packed BCD, one decimal digit per nibble,
  // advanced by a BCD add per token (round 6: the divisions by 10 of the
  // digit loop were 5.8 % of the kernel's issue, tools/bbprof.py)
  // (32-bit: every number of the batch below bcd_max <= 10^7, else the divisions)
  const bool bcd_ok = (u64)hist_tokens + 2ull * n_plies + 1 < (u64)min(bcd_max, 10000000u);  // kernel-uniform
  u32 bcd = 0;
  if (bcd_ok)
    for (u32 v = hist_tokens + 1, sh = 0; v; v /= 10, sh += 4) bcd |= (v % 10) << sh;
  u32 stage = active ? S_TURN : S_DONE;
  // the current piece: lpool[loff...] (glb false) or src[...] (glb true)
  const char* src = nullptr;
  bool glb = false;
  u32 loff = g_json_tpl.off[T_TURN];
  u32 rem = active ? g_json_tpl.len[T_TURN] : 0u;
  u32 row = 0, col = 0;
  u32 wn0 = 0, wn1 = 0, bn1 = 0;
  if (active) {
    wn0 = names_off[2 * g];
    wn1 = names_off[2 * g + 1];
    bn1 = names_off[2 * g + 2];
  }
#if DC_HASH_PF
  u32 pq_c[DC_HASH_PF], pq_m[DC_HASH_PF];  // plies ply .. ply + DC_HASH_PF - 1 (clamped to the last)
#pragma unroll
  for (int j = 0; j < DC_HASH_PF; ++j) {
    pq_c[j] = pq_m[j] = 0;
    if (info && active && n_plies) {
      const u32 pn = min((u32)j, n_plies - 1);
      pq_c[j] = info[(size_t)pn * n_games + g];
      pq_m[j] = moves[(size_t)pn * n_games + g];
    }
  }
#endif
  const u32 tok_off = kTplBytes + tid * kTokBytes;
  char* mytok = lpool + tok_off;
  auto tpl_piece = [&](int i, u32 drop) {
    glb = false;
    loff = g_json_tpl.off[i];
    rem = g_json_tpl.len[i] - drop;
  };
  auto glb_piece = [&](const char* p, u32 n) {
    glb = true;
    src = p;
    rem = n;
  };
  // The piece after the current one (rem == 0: the stream has ended).
  auto next_piece = [&]() {
    for (;;) {
      switch (stage) {
        case S_TURN:
          stage = S_DIGIT;
          tpl_piece(T_DIGITS, 1);
          loff += stm;
          break;
        case S_DIGIT: stage = S_WP; tpl_piece(T_WP, 0); break;
        case S_WP: stage = S_WNAME; glb_piece(names + wn0, wn1 - wn0); break;
        case S_WNAME: stage = S_BP; tpl_piece(T_BP, 0); break;
        case S_BP: stage = S_BNAME; glb_piece(names + wn1, bn1 - wn1); break;
        case S_BNAME: stage = S_HIST; tpl_piece(T_HIST, 0); break;
        case S_HIST: stage = S_HSTART; glb_piece(hist, hist_len); break;
        case S_HSTART:
        case S_TOKENS: {
          stage = S_TOKENS;
          // the next accepted moves (up to kTokPerPiece): their tokens "[ ]N. san"
          rem = 0;
          u32 n = 0, got = 0;
          const u32 tok_max = (DC_HASH_TOK3 && bcd_ok) ? 3u : kTokPerPiece;  // kernel-uniform
          while (ply < n_plies && got < tok_max) {
            const u32 p = ply++;
            u32 code = 0, m = 0;
#if DC_HASH_PF
            if (info) {  // kernel-uniform
              code = pq_c[0];
              m = pq_m[0];
#pragma unroll
              for (int j = 0; j + 1 < DC_HASH_PF; ++j) {
                pq_c[j] = pq_c[j + 1];
                pq_m[j] = pq_m[j + 1];
              }
              const u32 pn = min(p + DC_HASH_PF, n_plies - 1);
              pq_c[DC_HASH_PF - 1] = info[(size_t)pn * n_games + g];
              pq_m[DC_HASH_PF - 1] = moves[(size_t)pn * n_games + g];
              if (code == 0xFFu) continue;  // rejected
            } else
#endif
            {
              if (info) {  // kernel-uniform
                code = info[(size_t)p * n_games + g];
                if (code == 0xFFu) continue;  // rejected
              } else if (p < kAccPlies && ((accb[p >> 5][tid] >> (p & 31)) & 1) == 0) {
                continue;  // rejected in pass 1
              }
              m = moves[(size_t)p * n_games + g];
              if (!info && p >= kAccPlies && (m == 0xFFFFu || ref_verdict(b, cur, m) != V_OK)) continue;
            }
            const int f = (int)(m & 63), t = (int)((m >> 6) & 63);
            // info's kinds are P0 N1 B2 R3 Q4 K5 (kind_index's order; an unknown kind never moves)
            const u32 ki = info ? (code & 7u) : kind_index(nibble(b, f) >> 1);
            const bool cap = info ? (code & 8u) != 0 : ((occupied(b) >> t) & 1) != 0;
            if (ntok) mytok[n++] = ' ';
            // N's decimal digits straight into the token from the BCD (round 4
            // built them in a dynamically indexed register array: 29 % of the
            // kernel's issue cycles in tools/bbprof.py's count)
            if (bcd_ok) {
              const u32 nd = max(1u, (35u - (u32)__clz((int)bcd)) >> 2);
              for (u32 i = 0; i < nd; ++i) mytok[n + i] = (char)('0' + __builtin_amdgcn_ubfe(bcd, 4 * (nd - 1 - i), 4));
              n += nd;
            } else {  // digits written last-first
              u32 v = ntok + 1, nd = 1;
              for (u32 q = v; q >= 10; q /= 10) ++nd;
              for (u32 i = nd; i-- > 0;) {
                mytok[n + i] = (char)('0' + v % 10);
                v /= 10;
              }
              n += nd;
            }
            mytok[n++] = '.';
            mytok[n++] = ' ';
            if (ki != 0) mytok[n++] = "PNBRQK"[ki];
            if (cap) {
              if (ki == 0) mytok[n++] = (char)('a' + (f & 7));
              mytok[n++] = 'x';
            }
            mytok[n++] = (char)('a' + (t & 7));
            mytok[n++] = (char)('1' + (t >> 3));
            if (!fboards) ref_make(b, f, t);  // (kernel-uniform)
            cur ^= 1;
            ntok += 2;
            if (bcd_ok) bcd = bcd_add2(bcd);
            ++got;
          }
          if (n) {
            glb = false;
            loff = tok_off;
            rem = n;
          } else {
#if DC_HASH_MERGE
            stage = S_ROW;  // the board's header and its first row's (row 0)
            row = 0;
            tpl_piece(T_BOARD_ROW, 0);
#else
            stage = S_BOARD;
            tpl_piece(T_BOARD, 0);
#endif
          }
          break;
        }
        case S_BOARD:
          stage = S_ROW;
          row = 0;
          tpl_piece(T_ROW, 0);
          break;
        case S_ROW_END:
          if (row == 7) {
            stage = S_END;
            tpl_piece(T_END, 0);
            break;
          }
          ++row;
          stage = S_ROW;
          tpl_piece(T_ROW, 0);
          break;
        case S_ROW:
        case S_CELL: {
          if (stage == S_CELL && col == 7) {
#if DC_HASH_MERGE
            if (row == 7) {  // the last row's end and the board's and object's
              stage = S_END;
              tpl_piece(T_LAST, 0);
            } else {  // this row's end and the next row's header
              ++row;
              stage = S_ROW;
              tpl_piece(T_ROW_SEP, 0);
            }
#else
            stage = S_ROW_END;
            tpl_piece(T_ROW_END, row == 7 ? 1u : 0u);
#endif
            break;
          }
          col = stage == S_ROW ? 0u : col + 1;
          stage = S_CELL;
#if DC_HASH_NULLRUN
          {
            // empty cells from col on in this row (bit 8 stops the run at the row's end)
            const u32 occ8 = (u32)(occupied(b) >> (8 * row)) & 0xFFu;
            const u32 run = (u32)__builtin_ctz((occ8 | 0x100u) >> col);
            if (run) {
              glb = false;
              loff = kNullRunOff;
              rem = kCellNullLen * run - (col + run == 8 ? 1u : 0u);
              col += run - 1;  // the run's last cell
              break;
            }
          }
#endif
          const u32 nib = nibble(b, (int)(8 * row + col));
          const u32 ki = kind_index(nib >> 1);
          // the cell templates' offsets and lengths as constants (round 6:
          // the per-lane index into g_json_tpl made two global loads a cell)
          const u32 k = 6 * (nib & 1) + (ki < 6 ? ki : 0);
          glb = false;
          loff = (nib >> 1) == 0 ? kCellNullOff : kCell0Off + kCellLen * k;
          rem = ((nib >> 1) == 0 ? kCellNullLen : kCellLen) - (col == 7 ? 1u : 0u);
          break;
        }
        default:  // S_END
          stage = S_DONE;
          rem = 0;
          return;
      }
      if (rem) return;  // names and the start history may be empty
    }
  };
  uint64_t a[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) a[i] = 0;
  bool finished = !active;
  uint8_t* my = blk[tid];
  for (;;) {
    if (__ballot(!finished) == 0) break;
    if (!finished) {
      // fill this step's 136-byte block
      u32 fill = 0;
      while (fill < (u32)kKeccakRate && stage != S_DONE) {
        if (rem == 0) {
          next_piece();  // the next non-empty piece, or the stream's end
#if DC_HASH_FUSE
          if (stage == S_DONE) break;  // (the fetch falls through to the copy: one loop trip per piece)
#else
          continue;
#endif
        }
        const u32 n = min(rem, (u32)kKeccakRate - fill);
        if (glb) {
#if DC_HASH_GLB8
          // 8 loads issued before any store (clamped to the piece's last byte;
          // the up to 7 bytes written past it are overwritten, as in COPY8)
          for (u32 k = 0; k < n; k += 8) {
            char v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = src[min(k + (u32)j, n - 1)];
#pragma unroll
            for (int j = 0; j < 8; ++j) my[fill + k + j] = (uint8_t)v[j];
          }
#else
          for (u32 k = 0; k < n; ++k) my[fill + k] = (uint8_t)src[k];
#endif
          src += n;
        } else {
#if DC_HASH_COPY8
          for (u32 k = 0; k < n; k += 8) {
            const char* a = lpool + loff + k;
            uint8_t* d = my + fill + k;
            char v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = a[j];
#pragma unroll
            for (int j = 0; j < 8; ++j) d[j] = (uint8_t)v[j];
          }
#else
          for (u32 k = 0; k < n; ++k) my[fill + k] = (uint8_t)lpool[loff + k];
#endif
          loff += n;
        }
        rem -= n;
        fill += n;
      }
      if (fill < (u32)kKeccakRate) {  // the stream ended in this block: Keccak padding
        my[fill] = 0x01;
        for (u32 k = fill + 1; k < (u32)kKeccakRate; ++k) my[k] = 0;
        my[kKeccakRate - 1] |= 0x80;
        finished = true;
      }
      const uint64_t* w = reinterpret_cast<const uint64_t*>(my);
#pragma unroll
      for (int i = 0; i < kKeccakRate / 8; ++i) a[i] ^= w[i];
      keccak_f1600(a);
    }
  }
  if (active) {
    uint64_t* o = reinterpret_cast<uint64_t*>(out + (size_t)32 * g);
    o[0] = a[0];
    o[1] = a[1];
    o[2] = a[2];
    o[3] = a[3];
  }
}

// ------------------------------------------------- serde_json name escaping
// serde_json 1.0's string escape (ser.rs ESCAPE table, the format_escaped_str
// that serialises GameState's white_player / black_player, game.proto:9-10):
// '"' and '\\' and \b \t \n \f \r take two bytes, every other byte < 0x20
// six (\u00xx, lowercase hex), every other byte -- UTF-8 included -- one.
// One lane per string; names are short, so a lane walks its bytes.
__device__ __forceinline__ u32 esc_len(u32 ch) {
  if (ch >= 0x20) return (ch == '"' || ch == '\\') ? 2u : 1u;
  return (ch == 8 || ch == 9 || ch == 10 || ch == 12 || ch == 13) ? 2u : 6u;
}

__global__ __launch_bounds__(256) void k_escape_len(const char* __restrict__ names, const u32* __restrict__ off,
                                                   u32 n_str, u32* __restrict__ lens) {
  const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n_str) return;
  u32 len = 0;
  if (i < n_str) {
    const u32 a = off[i], b = off[i + 1];
    for (u32 k = a; k < b; ++k) len += esc_len((unsigned char)names[k]);  // b < a (malformed): empty
  }
  lens[i] = len;  // lens[n_str] = 0: the scan's last entry is the total
}

// esc64: the exclusive scan of the lengths (u64, so a total past 4 GiB is seen
// on the host before anything is written); out_off: the same as u32, for the
// hash kernel.
__global__ __launch_bounds__(256) void k_escape_write(const char* __restrict__ names, const u32* __restrict__ off,
                                                     u32 n_str, const u64* __restrict__ esc64,
                                                     u32* __restrict__ out_off, char* __restrict__ out) {
  const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n_str) return;
  out_off[i] = (u32)esc64[i];
  if (i == n_str) return;
  const u32 a = off[i], b = off[i + 1];
  char* o = out + esc64[i];
  for (u32 k = a; k < b; ++k) {
    const u32 ch = (unsigned char)names[k];
    const u32 l = esc_len(ch);
    if (l == 1) {
      *o++ = (char)ch;
    } else if (l == 2) {
      o[0] = '\\';
      o[1] = ch == '"' ? '"' : ch == '\\' ? '\\' : ch == 8 ? 'b' : ch == 9 ? 't' : ch == 10 ? 'n' : ch == 12 ? 'f' : 'r';
      o += 2;
    } else {
      o[0] = '\\';
      o[1] = 'u';
      o[2] = '0';
      o[3] = '0';
      o[4] = (char)('0' + (ch >> 4));
      const u32 lo = ch & 15;
      o[5] = (char)(lo < 10 ? '0' + lo : 'a' + lo - 10);
      o += 6;
    }
  }
}

// The fast path's check (round 6): flag[0] = 1 if any byte of names[0 ..
// off[n_str]) needs a JSON escape or an offset decreases; else the names are
// their own serde_json escapes and the hash kernel reads them in place (no
// per-name scan and copy).  Byte-parallel and coalesced.
__global__ __launch_bounds__(256) void k_names_plain(const char* __restrict__ names, const u32* __restrict__ off,
                                                    u32 n_str, u32* __restrict__ flag) {
  const u64 total = off[n_str];
  const u64 stride = (u64)gridDim.x * blockDim.x;
  bool bad = false;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const u32 ch = (unsigned char)names[i];
    bad |= ch < 0x20 || ch == '"' || ch == '\\';
  }
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n_str; i += stride) bad |= off[i] > off[i + 1];
  if (__ballot(bad) != 0 && lane_id() == 0) atomicOr(flag, 1u);
}

hipError_t launch_names_plain(hipStream_t st, const char* names, const u32* off, u32 n_str, u32* flag) {
  hipError_t e = hipMemsetAsync(flag, 0, sizeof(u32), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_names_plain, dim3(2048), dim3(256), 0, st, names, off, n_str, flag);
  return hipGetLastError();
}

size_t escape_scan_tmp_bytes(u32 n_str) {
  size_t bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveScan(nullptr, bytes, (const u32*)nullptr, (u64*)nullptr, hipcub::Sum(), (u64)0,
                                          (int)(n_str + 1));
  return bytes;
}

hipError_t launch_escape_len_scan(hipStream_t st, const char* names, const u32* off, u32 n_str, u64 base, u32* lens,
                                  void* tmp, size_t tmp_bytes, u64* esc64) {
  hipLaunchKernelGGL(k_escape_len, dim3(blocks_for((u64)n_str + 1, 256)), dim3(256), 0, st, names, off, n_str, lens);
  return hipcub::DeviceScan::ExclusiveScan(tmp, tmp_bytes, lens, esc64, hipcub::Sum(), base, (int)(n_str + 1), st);
}

hipError_t launch_escape_write(hipStream_t st, const char* names, const u32* off, u32 n_str, const u64* esc64,
                               u32* out_off, char* out) {
  hipLaunchKernelGGL(k_escape_write, dim3(blocks_for((u64)n_str + 1, 256)), dim3(256), 0, st, names, off, n_str, esc64,
                     out_off, out);
  return hipGetLastError();
}

hipError_t launch_state_hash_ref(hipStream_t st, const Board& start, u32 stm0, const uint16_t* moves, u32 n_games,
                                 u32 n_plies, const char* hist, u32 hist_len, u32 hist_tokens, const char* names,
                                 const u32* names_off, const uint8_t* info, uint8_t* out, const Board* final_boards,
                                 u32 bcd_max) {
  if (n_games == 0) return hipSuccess;
  hipLaunchKernelGGL(k_state_hash_ref, dim3(blocks_for(n_games, kHashThreads)), dim3(kHashThreads), 0, st, start, stm0,
                     moves, n_games, n_plies, hist, hist_len, hist_tokens, names, names_off, info, out,
                     info ? final_boards : nullptr, bcd_max);
  return hipGetLastError();
}

}  // namespace dc
