// dc_ref.h -- the reference's move rules (RULES_REF) as set-wise bitboard code.
//
// Semantics restated from /root/reference/core/src/chess.rs:
//   validate_move  chess.rs:82-125   (OOR first, then NO_PIECE, WRONG_TURN, ILLEGAL)
//   can_move_to    chess.rs:199-212  (dispatch on kind; unknown kind never moves)
//   pawn           chess.rs:214-254  (push, double from row 1/6, diagonal onto enemy;
//                                     no en passant, no promotion)
//   rook/bishop    chess.rs:256-335  (aligned, path empty, target empty-or-enemy)
//   knight/king    chess.rs:289-300, :350-360 (no castling, no check test)
//   apply_move     chess.rs:43-80    (to <- from, from <- empty, turn flips)
// "Enemy" is any piece whose colour differs from the mover's (chess.rs:444).
//
// Board: quad-bitboard of include/dchess.h -- b0 = black, b1..b3 = kind bits,
// kind codes P=1 N=2 K=3 OTHER=4 B=5 R=6 Q=7.
#pragma once
#include <type_traits>

#include "dc_bits.h"
#include "dc_kernels.h"

namespace dc {

enum : u32 { V_OK = 0, V_NO_PIECE = 1, V_WRONG_TURN = 2, V_ILLEGAL = 3, V_OOR = 4 };
enum : u32 { KC_P = 1, KC_N = 2, KC_K = 3, KC_X = 4, KC_B = 5, KC_R = 6, KC_Q = 7 };

__device__ __forceinline__ u64 occupied(const Board& b) { return b.b1 | b.b2 | b.b3; }
__device__ __forceinline__ u32 nibble(const Board& b, int s) {
  return (u32)(((b.b0 >> s) & 1) | (((b.b1 >> s) & 1) << 1) | (((b.b2 >> s) & 1) << 2) |
               (((b.b3 >> s) & 1) << 3));
}

// Own pieces split into the move classes the generator iterates.
struct Sides {
  u64 occ, own, enemy, empty, notown;
  u64 P, N, K, D, O;  // pawns, knights, kings, diagonal sliders (B,Q), orthogonal (R,Q)
};

template <int STM>
__device__ __forceinline__ Sides sides(const Board& b) {
  Sides s;
  s.occ = occupied(b);
  s.own = STM ? b.b0 : (s.occ & ~b.b0);
  s.enemy = s.occ ^ s.own;
  s.empty = ~s.occ;
  s.notown = ~s.own;
  const u64 lo = b.b1, mid = b.b2, hi = b.b3;
  s.P = s.own & lo & ~(mid | hi);
  s.N = s.own & mid & ~(lo | hi);
  s.K = s.own & lo & mid & ~hi;
  s.D = s.own & hi & lo;
  s.O = s.own & hi & mid;
  return s;
}

// Pawn target sets (per direction class; sources = target - delta).
template <int STM>
struct PawnDir {
  static constexpr int F = STM ? -8 : 8;      // forward
  static constexpr int CW = STM ? -9 : 7;     // capture toward column y-1
  static constexpr int CE = STM ? -7 : 9;     // capture toward column y+1
  static constexpr u64 ROW_AFTER1 = STM ? kRow(5) : kRow(2);  // single pushes from the start row land here
  static constexpr u64 ROW_DBL = STM ? kRow(4) : kRow(3);     // ... and double pushes land here
};

// Moves of the king(s) onto `allowed`.  One king (the norm): the 3x3 pattern
// shifted to its square, with the wrap file masked -- one variable 64-bit
// shift instead of eight.  Several kings (possible through the cells adapter)
// fall back to per-direction popcounts.
__device__ __forceinline__ u32 king_moves(u64 k, u64 allowed) {
  if ((k & (k - 1)) == 0) {
    if (!k) return 0;
    const int s = lsb(k);
#if DC_ATT_TAB
    return pc(kAtt.king[s & 63] & allowed);  // (& 63: the load may be speculated above the k == 0 exit)
#endif
    constexpr u64 kAtB2 = 0x0000000000070507ull;  // a1 b1 c1 a2 c2 a3 b3 c3 around b2 (9)
    const u64 att = s >= 9 ? (kAtB2 << (s - 9)) : (kAtB2 >> (9 - s));
    const int f = s & 7;
    const u64 wrap = f == 0 ? kNotH : (f == 7 ? kNotA : kAll);
    return pc(and3(att, wrap, allowed));
  }
  return pc(sh<8>(k) & allowed) + pc(sh<-8>(k) & allowed) + pc(and3(sh<1>(k), kNotA, allowed)) +
         pc(and3(sh<-1>(k), kNotH, allowed)) + pc(and3(sh<9>(k), kNotA, allowed)) +
         pc(and3(sh<7>(k), kNotH, allowed)) + pc(and3(sh<-7>(k), kNotA, allowed)) +
         pc(and3(sh<-9>(k), kNotH, allowed));
}

// Knight moves onto `allowed`: per knight one kAtt row and one popcount (the
// norm is at most two knights: ~26 VALU against 40 for the eight direction
// terms).  DC_KNIGHT_TAB=0: the direction terms (A/B).
#ifndef DC_KNIGHT_TAB
#define DC_KNIGHT_TAB 1
#endif
__device__ __forceinline__ u32 knight_moves(u64 n, u64 allowed) {
#if DC_KNIGHT_TAB
  u32 c = 0;
  for (; n; n &= n - 1) c += pc(kAtt.knight[lsb(n) & 63] & allowed);
  return c;
#else
  return pc(and3(sh<17>(n), kNotA, allowed)) + pc(and3(sh<15>(n), kNotH, allowed)) +
         pc(and3(sh<10>(n), kNotAB, allowed)) + pc(and3(sh<6>(n), kNotGH, allowed)) +
         pc(and3(sh<-6>(n), kNotAB, allowed)) + pc(and3(sh<-10>(n), kNotGH, allowed)) +
         pc(and3(sh<-15>(n), kNotA, allowed)) + pc(and3(sh<-17>(n), kNotH, allowed));
#endif
}

// Bulk count of REF moves for the side to move: the number of (from,to) pairs
// validate_move accepts.  Every term is a popcount over one direction class, so
// multiplicity is exact (two knights reaching one square count twice).  Wrap
// guards are applied on the target side so each leaper term is one shift, one
// bitop3 (shifted & guard & ~own) and one popcount.
template <int STM>
__device__ __forceinline__ u32 ref_count_sides(const Sides& s) {
  typedef PawnDir<STM> PD;
  const u64 push1 = sh<PD::F>(s.P) & s.empty;
  const u64 push2 = and3(sh<PD::F>(push1), PD::ROW_DBL, s.empty);
  u32 c = pc(push1 | push2);  // (disjoint: a landing square's mid square is empty)
  c += pc(and3(sh<PD::CW>(s.P), kNotH, s.enemy));  // toward column y-1: wraps land on file h
  c += pc(and3(sh<PD::CE>(s.P), kNotA, s.enemy));  // toward column y+1: wraps land on file a
  const u64 no = s.notown;
  c += knight_moves(s.N, no);
  c += king_moves(s.K, no);
  const u64 e = s.empty;
  c += pc(ray_attacks<8, kAll>(s.O, e) & no) + pc(ray_attacks<-8, kAll>(s.O, e) & no);
  c += pc(ray_moves<1, kNotA>(s.O, e, no)) + pc(ray_moves<-1, kNotH>(s.O, e, no));
  c += pc(ray_moves<9, kNotA>(s.D, e, no)) + pc(ray_moves<-9, kNotH>(s.D, e, no));
  c += pc(ray_moves<7, kNotH>(s.D, e, no)) + pc(ray_moves<-7, kNotA>(s.D, e, no));
  return c;
}

template <int STM>
__device__ __forceinline__ u32 ref_count(const Board& b) {
  return ref_count_sides<STM>(sides<STM>(b));
}

// Moves of the side to move whose source lies in M (ref_count with every piece
// class restricted to M; targets unrestricted).
template <int STM>
__device__ __forceinline__ u32 ref_count_from(const Board& b, u64 M) {
  Sides s = sides<STM>(b);
  s.P &= M;
  s.N &= M;
  s.K &= M;
  s.D &= M;
  s.O &= M;
  return ref_count_sides<STM>(s);
}

// ------------------------------------------------ side-to-move view (k_gen_games_ref)
// The REF rules are symmetric under a vertical flip that swaps the colours, so
// any position can be evaluated as "White to move": rows reversed (byte swap,
// square s -> s ^ 56) and, when Black is to move, the colour plane replaced
// by the other side's pieces.  A wave whose lanes hold games with different
// sides to move then runs one code path (ref_count<0>), not both.
__device__ __forceinline__ u64 flip_rows(u64 x) { return __builtin_bswap64(x); }

__device__ __forceinline__ Board white_view(const Board& b, u32 stm) {
  if (!stm) return b;  // (callers keep this branch-free: see view_sel)
  const u64 occ = occupied(b);
  return Board{flip_rows(b.b0 ^ occ), flip_rows(b.b1), flip_rows(b.b2), flip_rows(b.b3)};
}

// Branch-free select of the two views (stm is per lane).
__device__ __forceinline__ Board view_sel(const Board& b, u32 stm) {
  const u64 occ = occupied(b);
  const u64 m = 0ull - (u64)(stm & 1);
  auto pick = [&](u64 a, u64 f) { return (a & ~m) | (f & m); };
  return Board{pick(b.b0, flip_rows(b.b0 ^ occ)), pick(b.b1, flip_rows(b.b1)), pick(b.b2, flip_rows(b.b2)),
               pick(b.b3, flip_rows(b.b3))};
}

// Slider propagators of one white-to-move board, per direction: the empty
// squares (wrap-masked) and their 2- and 4-step products.  A source-restricted
// count needs occluded fills from several generator subsets over ONE
// occupancy (k_gen_games_ref's binary search), so the propagators are built
// once per ply and each fill is then 3 shift/bitop3 steps.
struct Props {
  u64 p1[8], p2[8], p4[8];
};

template <int S, u64 M>
__device__ __forceinline__ void prop_dir(u64 empty, u64& p1, u64& p2, u64& p4) {
  p1 = empty & M;
  p2 = p1 & sh<S>(p1);
  p4 = p2 & sh<2 * S>(p2);
}

__device__ __forceinline__ Props make_props(u64 e) {
  Props p;
  prop_dir<8, kAll>(e, p.p1[0], p.p2[0], p.p4[0]);
  prop_dir<-8, kAll>(e, p.p1[1], p.p2[1], p.p4[1]);
  prop_dir<1, kNotA>(e, p.p1[2], p.p2[2], p.p4[2]);
  prop_dir<-1, kNotH>(e, p.p1[3], p.p2[3], p.p4[3]);
  prop_dir<9, kNotA>(e, p.p1[4], p.p2[4], p.p4[4]);
  prop_dir<-9, kNotH>(e, p.p1[5], p.p2[5], p.p4[5]);
  prop_dir<7, kNotH>(e, p.p1[6], p.p2[6], p.p4[6]);
  prop_dir<-7, kNotA>(e, p.p1[7], p.p2[7], p.p4[7]);
  return p;
}

template <int S, u64 M, int I>
__device__ __forceinline__ u64 fill_props(u64 g, const Props& p, u64 allowed) {
  g = or_and(g, p.p1[I], sh<S>(g));
  g = or_and(g, p.p2[I], sh<2 * S>(g));
  g = or_and(g, p.p4[I], sh<4 * S>(g));
  return and3(sh<S>(g), M, allowed);
}

// ref_count<0> restricted to sources in Msrc, with the slider fills over the
// precomputed propagators.
__device__ __forceinline__ u32 ref_count_from_w(const Sides& s, const Props& pr, u64 Msrc) {
  const u64 P = s.P & Msrc, N = s.N & Msrc, K = s.K & Msrc, D = s.D & Msrc, O = s.O & Msrc;
  const u64 e = s.empty, no = s.notown;
  const u64 push1 = sh<8>(P) & e;
  u32 c = pc(push1) + pc(and3(sh<8>(push1), kRow(3), e));
  c += pc(and3(sh<7>(P), kNotH, s.enemy)) + pc(and3(sh<9>(P), kNotA, s.enemy));
  c += pc(and3(sh<17>(N), kNotA, no)) + pc(and3(sh<15>(N), kNotH, no));
  c += pc(and3(sh<10>(N), kNotAB, no)) + pc(and3(sh<6>(N), kNotGH, no));
  c += pc(and3(sh<-6>(N), kNotAB, no)) + pc(and3(sh<-10>(N), kNotGH, no));
  c += pc(and3(sh<-15>(N), kNotA, no)) + pc(and3(sh<-17>(N), kNotH, no));
  c += king_moves(K, no);
  c += pc(fill_props<8, kAll, 0>(O, pr, no)) + pc(fill_props<-8, kAll, 1>(O, pr, no));
  c += pc(fill_props<1, kNotA, 2>(O, pr, no)) + pc(fill_props<-1, kNotH, 3>(O, pr, no));
  c += pc(fill_props<9, kNotA, 4>(D, pr, no)) + pc(fill_props<-9, kNotH, 5>(D, pr, no));
  c += pc(fill_props<7, kNotH, 6>(D, pr, no)) + pc(fill_props<-7, kNotA, 7>(D, pr, no));
  return c;
}

// Target set of the White piece on square f of a white-to-move board: every
// piece class evaluated set-wise from the one-bit source (no branch on the
// kind; the classes of other kinds come out empty).
__device__ __forceinline__ u64 ref_piece_targets_w(const Board& b, int f) {
  Sides s = sides<0>(b);
  const u64 bit = 1ull << f;
  const u64 P = s.P & bit, N = s.N & bit, K = s.K & bit, D = s.D & bit, O = s.O & bit;
  const u64 e = s.empty, no = s.notown;
  const u64 push1 = sh<8>(P) & e;
  u64 t = push1 | and3(sh<8>(push1), kRow(3), e);
  t |= ((sh<7>(P) & kNotH) | (sh<9>(P) & kNotA)) & s.enemy;
  u64 l = (sh<17>(N) & kNotA) | (sh<15>(N) & kNotH) | (sh<10>(N) & kNotAB) | (sh<6>(N) & kNotGH);
  l |= (sh<-6>(N) & kNotAB) | (sh<-10>(N) & kNotGH) | (sh<-15>(N) & kNotA) | (sh<-17>(N) & kNotH);
  l |= sh<8>(K) | sh<-8>(K) | (sh<1>(K) & kNotA) | (sh<-1>(K) & kNotH) | (sh<9>(K) & kNotA) | (sh<7>(K) & kNotH) |
       (sh<-7>(K) & kNotA) | (sh<-9>(K) & kNotH);
  l |= ray_attacks<8, kAll>(O, e) | ray_attacks<-8, kAll>(O, e) | ray_attacks<1, kNotA>(O, e) |
       ray_attacks<-1, kNotH>(O, e);
  l |= ray_attacks<9, kNotA>(D, e) | ray_attacks<-9, kNotH>(D, e) | ray_attacks<7, kNotH>(D, e) |
       ray_attacks<-7, kNotA>(D, e);
  return t | (l & no);
}

// ------------------------------------------------ split count (k_count2c)
// For the side SIDE in `b`: the moves of its knights, kings and sliders (the
// part of ref_count that a quiet move of the OTHER side leaves unchanged unless
// it touches a slider ray), and in `att` the union of its slider rays -- every
// square a ray reaches, up to and including the first occupied one.
//
// Why a quiet move m = (f -> t, t empty) by the other side keeps this part: the
// SIDE's own set is unchanged (nothing of SIDE is captured), so leaper targets
// (not-own squares) are unchanged; a slider ray changes only if it reached f
// (f empties, the ray now runs on) or t (t fills, the ray now stops there),
// i.e. only if f or t is in `att`.  Then only SIDE's pawn moves need
// recounting in the child (ref_pawn_count_child).  Checked on random positions
// (including unknown-kind pieces) against the oracle: DESIGN.md §3.
template <int SIDE>
__device__ __forceinline__ u32 ref_count_nonpawn(const Board& b, u64& att) {
  const Sides s = sides<SIDE>(b);
  const u64 no = s.notown, n = s.N, e = s.empty;
  u32 c = pc(and3(sh<17>(n), kNotA, no)) + pc(and3(sh<15>(n), kNotH, no));
  c += pc(and3(sh<10>(n), kNotAB, no)) + pc(and3(sh<6>(n), kNotGH, no));
  c += pc(and3(sh<-6>(n), kNotAB, no)) + pc(and3(sh<-10>(n), kNotGH, no));
  c += pc(and3(sh<-15>(n), kNotA, no)) + pc(and3(sh<-17>(n), kNotH, no));
  c += king_moves(s.K, no);
  const u64 a0 = ray_attacks<8, kAll>(s.O, e), a1 = ray_attacks<-8, kAll>(s.O, e);
  const u64 a2 = ray_attacks<1, kNotA>(s.O, e), a3 = ray_attacks<-1, kNotH>(s.O, e);
  const u64 a4 = ray_attacks<9, kNotA>(s.D, e), a5 = ray_attacks<-9, kNotH>(s.D, e);
  const u64 a6 = ray_attacks<7, kNotH>(s.D, e), a7 = ray_attacks<-7, kNotA>(s.D, e);
  c += pc(a0 & no) + pc(a1 & no) + pc(a2 & no) + pc(a3 & no);
  c += pc(a4 & no) + pc(a5 & no) + pc(a6 & no) + pc(a7 & no);
  att = bop3<0xFE>(bop3<0xFE>(a0, a1, a2), bop3<0xFE>(a3, a4, a5), a6 | a7);  // 0xFE = a | b | c
  return c;
}

// ref_count_nonpawn with the slider groups kept apart for the group-wise
// recount (c2c_diag): also `orth` = the orthogonal rays plus the orthogonal
// sliders themselves (a move touching it changes that group's count) and
// `diag` = the diagonal group's move count.
template <int SIDE>
__device__ __forceinline__ u32 ref_count_nonpawn_g(const Board& b, u64& att, u64& orth, u32& diag) {
  const Sides s = sides<SIDE>(b);
  const u64 no = s.notown, n = s.N, e = s.empty;
  // the king first: its several-kings branch would otherwise split a block
  // holding all eight knight shifts live (spills at the 128-VGPR budget)
  u32 c = king_moves(s.K, no);
  c += knight_moves(n, no);
  asm volatile("" : "+v"(c));  // the leaper terms reduced here, not sunk past the fills
  const u64 a0 = ray_attacks<8, kAll>(s.O, e), a1 = ray_attacks<-8, kAll>(s.O, e);
  const u64 a2 = ray_attacks<1, kNotA>(s.O, e), a3 = ray_attacks<-1, kNotH>(s.O, e);
  const u64 a4 = ray_attacks<9, kNotA>(s.D, e), a5 = ray_attacks<-9, kNotH>(s.D, e);
  const u64 a6 = ray_attacks<7, kNotH>(s.D, e), a7 = ray_attacks<-7, kNotA>(s.D, e);
  c += pc(a0 & no) + pc(a1 & no) + pc(a2 & no) + pc(a3 & no);
  diag = pc(a4 & no) + pc(a5 & no) + pc(a6 & no) + pc(a7 & no);
  const u64 ao = bop3<0xFE>(a0, a1, a2) | a3;
  orth = ao | s.O;
  att = bop3<0xFE>(ao, bop3<0xFE>(a4, a5, a6), a7);
  return c + diag;
}

// Knight and king attack sets of one square: the pattern around c3 / b2
// shifted to s, the files a shift wraps into masked (king_moves' trick).
__device__ __forceinline__ u64 knight_att_sq(int s) {
#if DC_ATT_TAB
  return kAtt.knight[s];
#endif
  constexpr u64 kAtC3 = 0x0000000A1100110Aull;  // b1 d1 a2 e2 a4 e4 b5 d5 around c3 (18)
  const u64 a = s >= 18 ? (kAtC3 << (s - 18)) : (kAtC3 >> (18 - s));
  const int f = s & 7;
  return a & (f <= 1 ? kNotGH : (f >= 6 ? kNotAB : kAll));
}
__device__ __forceinline__ u64 king_att_sq(int s) {
#if DC_ATT_TAB
  return kAtt.king[s];
#endif
  constexpr u64 kAtB2 = 0x0000000000070507ull;
  const u64 a = s >= 9 ? (kAtB2 << (s - 9)) : (kAtB2 >> (9 - s));
  const int f = s & 7;
  return a & (f == 0 ? kNotH : (f == 7 ? kNotA : kAll));
}

// count_O of the child P∘(f -> t) (the other side's move; O = SIDE to move in
// the child) when O's orthogonal group is unchanged (f, t off `orth` of
// ref_count_nonpawn_g): from the parent's base (O's knight/king/slider moves)
// and diag (its diagonal group's share),
//   count = base - diag + diag group in the child + O's pawns in the child
//           + [capture] (O's knights/kings attacking t, now an enemy square,
//              minus the captured knight's or king's own moves).
// Knights and kings see only the own/not-own status of their targets, which a
// move changes at t alone (and only by a capture); the pawn terms and the
// diagonal fills are recomputed on the child's occupancy.
template <int SIDE>
__device__ __forceinline__ u32 ref_count_child_diag(const Board& b, int f, int t, u32 base_minus_diag) {
  typedef PawnDir<SIDE> PD;
  const u64 occ = occupied(b);
  const u64 bf = 1ull << f, bt = 1ull << t;
  const u64 own0 = SIDE ? b.b0 : (occ & ~b.b0);
  const u64 own = own0 & ~bt;                 // O's pieces in the child
  const u64 occc = bop3<0xBA>(occ, bf, bt);   // (occ & ~f) | t
  const u64 e = ~occc, no = ~own, enemy = occc ^ own;
  const u64 D = and3(own, b.b3, b.b1);
  u32 c = base_minus_diag;
  c += pc(ray_moves<9, kNotA>(D, e, no)) + pc(ray_moves<-9, kNotH>(D, e, no));
  c += pc(ray_moves<7, kNotH>(D, e, no)) + pc(ray_moves<-7, kNotA>(D, e, no));
  const u64 P = and_andn(own, b.b1, b.b2 | b.b3);
  const u64 push1 = sh<PD::F>(P) & e;
  c += pc(or_and(push1, sh<PD::F>(push1) & PD::ROW_DBL, e));  // single | double pushes (disjoint)
  c += pc(and3(sh<PD::CW>(P), kNotH, enemy)) + pc(and3(sh<PD::CE>(P), kNotA, enemy));
  const u64 kn = knight_att_sq(t), kg = king_att_sq(t);
  const u64 N = and_andn(own, b.b2, b.b1 | b.b3), K = and_andn(own, b.b1 & b.b2, b.b3);
  const u32 xk = (u32)(((b.b1 >> t) & 1) | (((b.b2 >> t) & 1) << 1) | (((b.b3 >> t) & 1) << 2));
  const u32 gain = pc(kn & N) + pc(kg & K);
  const u32 lost = xk == KC_N ? pc(kn & ~own0) : (xk == KC_K ? pc(kg & ~own0) : 0u);
  return ((own0 >> t) & 1) ? c + gain - lost : c;
}

// Pawn moves of SIDE in the child reached from `b` by the other side's quiet
// move f -> t (f occupied by the mover, t empty): the pawn terms of ref_count
// on the child's occupancy, without making the child.
template <int SIDE>
__device__ __forceinline__ u32 ref_pawn_count_child(const Board& b, int f, int t) {
  typedef PawnDir<SIDE> PD;
  const u64 occ = occupied(b);
  const u64 own = SIDE ? b.b0 : (occ & ~b.b0);
  const u64 P = and_andn(own, b.b1, b.b2 | b.b3);
  const u64 ft = (1ull << f) | (1ull << t);
  const u64 empty_c = ~(occ ^ ft);
  const u64 enemy_c = (occ & ~own) ^ ft;  // the mover's pieces after the move
  const u64 push1 = sh<PD::F>(P) & empty_c;
  const u64 push2 = and3(sh<PD::F>(push1), PD::ROW_DBL, empty_c);
  return pc(push1 | push2) + pc(and3(sh<PD::CW>(P), kNotH, enemy_c)) + pc(and3(sh<PD::CE>(P), kNotA, enemy_c));
}

// ------------------------------------------------ bulk split (k_count2c)
// Pawn-sensitive squares of SIDE in `b` and SIDE's pawn-move count there.
// For a quiet move f -> t of the other side (t empty, nothing captured), the
// change in SIDE's pawn-move count is g(t) - g(f) (+1 correction when f, t are
// the mid and landing squares of one double push), where
//   g(x) = #SIDE pawns attacking x - [x is a push square of a SIDE pawn]
//          - [x is the mid square of a double push whose landing is empty]
//          - [x is the landing square of a double push whose mid is empty]
// (derivation: DESIGN.md §3).  g vanishes outside
//   G = pawn attacks | push squares | double-push landings with empty mid,
// (mid squares are push squares), so a quiet move with f, t outside G leaves
// SIDE's pawn count unchanged -- and the correction case has t or f on a mid
// square, inside G.
template <int SIDE>
__device__ __forceinline__ u64 ref_pawn_sensitive(const Board& b, u32& pawn_cnt) {
  typedef PawnDir<SIDE> PD;
  const Sides s = sides<SIDE>(b);
  const u64 q1 = sh<PD::F>(s.P);
  const u64 cw = sh<PD::CW>(s.P) & kNotH, ce = sh<PD::CE>(s.P) & kNotA;
  const u64 push1 = q1 & s.empty;
  const u64 land = sh<PD::F>(push1) & PD::ROW_DBL;  // landings whose mid is empty
  pawn_cnt = pc(or_and(push1, land, s.empty)) + pc(cw & s.enemy) + pc(ce & s.enemy);
  return bop3<0xFE>(q1, cw, ce) | land;
}

// ref_pawn_sensitive plus the weight planes of g on the parent (DC_C2C_GCORR):
//   g(x) = [x in cw] + [x in ce] - [x in q1] - [x in mid] - [x in land]
// (cw/ce: SIDE's pawn capture squares, q1: its push squares, mid: middle
// squares of a double push whose landing is empty, land: landings whose
// middle is empty).  For a quiet move f -> t of the other side with f off G
// and t empty, SIDE's pawn-move count in the child is pawn_cnt + g(t)
// (tools/ref_gsplit_proto.py: 0 mismatches against the oracle).  P1 / N1: the
// squares where g = +1 / -1; BIG: |g| = 2 (rare; such targets stay enumerated).
template <int SIDE>
__device__ __forceinline__ u64 ref_pawn_planes(const Board& b, u32& pawn_cnt, u64& P1, u64& N1, u64& BIG) {
  typedef PawnDir<SIDE> PD;
  const Sides s = sides<SIDE>(b);
  const u64 q1 = sh<PD::F>(s.P);
  const u64 cw = sh<PD::CW>(s.P) & kNotH, ce = sh<PD::CE>(s.P) & kNotA;
  const u64 push1 = q1 & s.empty;
  const u64 land = sh<PD::F>(push1) & PD::ROW_DBL;  // landings whose mid is empty
  pawn_cnt = pc(or_and(push1, land, s.empty)) + pc(cw & s.enemy) + pc(ce & s.enemy);
  const u64 mid = and3(q1, PD::ROW_AFTER1, sh<-PD::F>(s.empty & PD::ROW_DBL));  // mids whose landing is empty
  const u64 nd = mid | land;  // disjoint rows; mid is inside q1
  const u64 s1 = cw ^ ce, s2 = cw & ce, n1 = q1 ^ nd, n2 = q1 & nd;  // g = (s1 + 2 s2) - (n1 + 2 n2)
  const u64 sp = s1 | s2, sn = n1 | n2;
  P1 = (s2 & n1) | (s1 & ~sn);
  N1 = (n2 & s1) | (n1 & ~sp);
  BIG = (s2 & ~sn) | (n2 & ~sp);
  return bop3<0xFE>(q1, cw, ce) | land;
}

// Moves of STM in `b` with source in Fs and target in Ts ("simple" moves;
// Ts holds empty squares only, so pawn captures never count): ref_count<STM>
// with the sources and targets restricted.  Slider targets of sources in Fs
// are the fill from (sliders & Fs): a target whose nearest slider behind it is
// outside Fs is shadowed by that slider.
template <int STM>
__device__ __forceinline__ u32 ref_count_simple(const Board& b, u64 Fs, u64 Ts) {
  const Sides s = sides<STM>(b);
  typedef PawnDir<STM> PD;
  const u64 push1 = sh<PD::F>(s.P & Fs) & s.empty;
  u32 c = pc(push1 & Ts) + pc(and3(sh<PD::F>(push1), PD::ROW_DBL, Ts));
  const u64 n = s.N & Fs;
  c += pc(and3(sh<17>(n), kNotA, Ts)) + pc(and3(sh<15>(n), kNotH, Ts));
  c += pc(and3(sh<10>(n), kNotAB, Ts)) + pc(and3(sh<6>(n), kNotGH, Ts));
  c += pc(and3(sh<-6>(n), kNotAB, Ts)) + pc(and3(sh<-10>(n), kNotGH, Ts));
  c += pc(and3(sh<-15>(n), kNotA, Ts)) + pc(and3(sh<-17>(n), kNotH, Ts));
  c += king_moves(s.K & Fs, Ts);
  const u64 e = s.empty, o = s.O & Fs, d = s.D & Fs;
  c += pc(ray_attacks<8, kAll>(o, e) & Ts) + pc(ray_attacks<-8, kAll>(o, e) & Ts);
  c += pc(ray_moves<1, kNotA>(o, e, Ts)) + pc(ray_moves<-1, kNotH>(o, e, Ts));
  c += pc(ray_moves<9, kNotA>(d, e, Ts)) + pc(ray_moves<-9, kNotH>(d, e, Ts));
  c += pc(ray_moves<7, kNotH>(d, e, Ts)) + pc(ray_moves<-7, kNotA>(d, e, Ts));
  return c;
}

// Two occluded fills toward S sharing the propagator masks (one pass per
// direction keeps few masks live; see ref_parent_split).
template <int S, u64 M>
__device__ __forceinline__ void ray_attacks2(u64 g1, u64 g2, u64 empty, u64& r1, u64& r2) {
  u64 pro = empty & M;
  g1 = or_and(g1, pro, sh<S>(g1));
  g2 = or_and(g2, pro, sh<S>(g2));
  pro &= sh<S>(pro);
  g1 = or_and(g1, pro, sh<2 * S>(g1));
  g2 = or_and(g2, pro, sh<2 * S>(g2));
  pro &= sh<2 * S>(pro);
  g1 = or_and(g1, pro, sh<4 * S>(g1));
  g2 = or_and(g2, pro, sh<4 * S>(g2));
  r1 = sh<S>(g1) & M;
  r2 = sh<S>(g2) & M;
}

// Everything k_count2c needs per parent P (side STM to move, opponent O):
//   base, att = ref_count_nonpawn<O>;  pawn_o (and G) = ref_pawn_sensitive<O>;
//   Fs = own & ~(att | G), Ts = empty & ~(att | G);
//   n_total = ref_count<STM>, n_simple = ref_count_simple<STM>(Fs, Ts),
// with STM's all-source and Fs-source fills fused per direction.  Computed
// as four separate functions, the compiler kept every direction's fill masks
// live across them (CSE) and spilled 184 B per lane -- 0.9 GB of scratch
// traffic per perft(7) launch (rocprofv3 FETCH_SIZE).
struct ParentSplit {
  u64 att, Fs, Ts, orth;
  u32 base, pawn_o, n_total, n_simple, diag;
  u32 gcorr;  // (GCORR) sum of g(t) over the simple moves, mod 2^32 (may be negative)
};

// GCORR (round 5): a quiet move with f off att and G and t off att (and off
// BIG) is simple too, its child's count corrected by g(t) (ref_pawn_planes):
// Ts = empty & ~(att | BIG) instead of empty & ~(att | G), and each class's
// simple targets are also counted on the g = +1 and g = -1 planes.  80 % of
// the quiet children round 4 enumerated for a pawn recount become simple
// (tools/ref_gsplit_proto.py).
#ifndef DC_C2C_GCORR
#define DC_C2C_GCORR 1
#endif

// GROUPS: also orth/diag (ref_count_nonpawn_g) for the group-wise recount.
// TGT: also the side to move's slider target sets per direction (tgt[0..7]
// in ref_for_each_special's slide order), so the enumeration of the special
// moves reuses these fills instead of running them again (DC_C2C_REUSE).
template <int STM, bool GROUPS = false, bool TGT = false>
__device__ __forceinline__ void ref_parent_split(const Board& b, ParentSplit& r, u64* tgt = nullptr) {
  if constexpr (GROUPS) r.base = ref_count_nonpawn_g<1 - STM>(b, r.att, r.orth, r.diag);
  else r.base = ref_count_nonpawn<1 - STM>(b, r.att);
  const Sides s = sides<STM>(b);
#if DC_C2C_GCORR
  u64 P1, N1, BIG;
  const u64 Fs = s.own & ~(r.att | ref_pawn_planes<1 - STM>(b, r.pawn_o, P1, N1, BIG));
  const u64 Ts = s.empty & ~(r.att | BIG), no = s.notown;
  u32 gp = 0, gn = 0;
  // a class's simple targets X on the two weight planes
  auto wgt = [&](u64 x) {
    gp += pc(x & P1);
    gn += pc(x & N1);
  };
#else
  const u64 keep = ~(r.att | ref_pawn_sensitive<1 - STM>(b, r.pawn_o));
  const u64 Fs = s.own & keep, Ts = s.empty & keep, no = s.notown;
  auto wgt = [](u64) {};
#endif
  r.Fs = Fs;
  r.Ts = Ts;
  u64 e = s.empty;
  asm volatile("" : "+v"(e));  // opaque copy: no reuse of the opponent's fill masks
  typedef PawnDir<STM> PD;
  const u64 push1 = sh<PD::F>(s.P) & e, push1s = sh<PD::F>(s.P & Fs) & e;
  // single and double pushes land on disjoint squares: one popcount each
  u32 t = pc(or_and(push1, sh<PD::F>(push1) & PD::ROW_DBL, e));
  const u64 pm = bop3<0xA8>(push1s, sh<PD::F>(push1s) & PD::ROW_DBL, Ts);  // (a | b) & c
  u32 m = pc(pm);
  wgt(pm);
  t += pc(and3(sh<PD::CW>(s.P), kNotH, s.enemy)) + pc(and3(sh<PD::CE>(s.P), kNotA, s.enemy));
  using std::integral_constant;
#if DC_KNIGHT_TAB
  // per knight: its kAtt row counts toward t and, from a source in Fs, m
  for (u64 n = s.N; n; n &= n - 1) {
    const int f = lsb(n) & 63;
    const u64 a = kAtt.knight[f];
    t += pc(a & no);
    const u64 x = ((Fs >> f) & 1) ? a & Ts : 0ull;
    m += pc(x);
    wgt(x);
  }
#else
  const u64 n = s.N, ns = s.N & Fs;
  auto leap = [&](auto dtag, u64 guard) {
    constexpr int D = decltype(dtag)::value;
    t += pc(and3(sh<D>(n), guard, no));
    const u64 x = and3(sh<D>(ns), guard, Ts);
    m += pc(x);
    wgt(x);
  };
  leap(integral_constant<int, 17>{}, kNotA);
  leap(integral_constant<int, 15>{}, kNotH);
  leap(integral_constant<int, 10>{}, kNotAB);
  leap(integral_constant<int, 6>{}, kNotGH);
  leap(integral_constant<int, -6>{}, kNotAB);
  leap(integral_constant<int, -10>{}, kNotGH);
  leap(integral_constant<int, -15>{}, kNotA);
  leap(integral_constant<int, -17>{}, kNotH);
#endif
  if (DC_ATT_TAB && (s.K & (s.K - 1)) == 0) {  // one king (or none): one attack set for both counts
    const u64 ka = s.K ? kAtt.king[lsb(s.K) & 63] : 0ull;
    t += pc(ka & no);
    const u64 x = (s.K & Fs) ? ka & Ts : 0ull;
    m += pc(x);
    wgt(x);
  } else {
    t += king_moves(s.K, no);
    m += king_moves(s.K & Fs, Ts);
#if DC_C2C_GCORR
    for (u64 k = s.K & Fs; k; k &= k - 1) wgt(king_att_sq(lsb(k)) & Ts);  // several kings (cells adapter)
#endif
  }
#ifndef DC_C2C_KSKIP
#define DC_C2C_KSKIP 1
#endif
  // KSKIP: the simple moves' fill (from the sliders in Fs) differs from the
  // full one only where a slider stands on a K square (off Fs); a wave none of
  // whose lanes has such a slider in the class skips that second fill
  // (one wave-uniform branch per slider class, ballot)
  auto slide = [&](u64 sl, auto stag, auto mtag, auto itag, auto two) {
    constexpr int S = decltype(stag)::value;
    constexpr u64 M = decltype(mtag)::value;
    u64 ra, rs;
    if constexpr (decltype(two)::value) {
      ray_attacks2<S, M>(sl, sl & Fs, e, ra, rs);
    } else {
      ra = ray_attacks<S, M>(sl, e);
      rs = ra;
    }
    const u64 rt = ra & no, st = rs & Ts;
    t += pc(rt);
    m += pc(st);
    wgt(st);
    // (TGT) the special targets only: t in Ts is simple iff its source is
    // in Fs, i.e. iff t is in the fill from the sliders in Fs (rs)
    if constexpr (TGT) tgt[decltype(itag)::value] = and_andn(ra, no, st);
  };
  using K = std::integral_constant<u64, kAll>;
  using NA = std::integral_constant<u64, kNotA>;
  using NH = std::integral_constant<u64, kNotH>;
  auto orth = [&](auto two) {
    slide(s.O, integral_constant<int, 8>{}, K{}, integral_constant<int, 0>{}, two);
    slide(s.O, integral_constant<int, -8>{}, K{}, integral_constant<int, 1>{}, two);
    slide(s.O, integral_constant<int, 1>{}, NA{}, integral_constant<int, 2>{}, two);
    slide(s.O, integral_constant<int, -1>{}, NH{}, integral_constant<int, 3>{}, two);
  };
  auto diag = [&](auto two) {
    slide(s.D, integral_constant<int, 9>{}, NA{}, integral_constant<int, 4>{}, two);
    slide(s.D, integral_constant<int, -9>{}, NH{}, integral_constant<int, 5>{}, two);
    slide(s.D, integral_constant<int, 7>{}, NH{}, integral_constant<int, 6>{}, two);
    slide(s.D, integral_constant<int, -7>{}, NA{}, integral_constant<int, 7>{}, two);
  };
  using T2 = std::true_type;
  using T1 = std::false_type;
  if (!DC_C2C_KSKIP || __ballot((s.O & ~Fs) != 0) != 0) orth(T2{});
  else orth(T1{});
  if (!DC_C2C_KSKIP || __ballot((s.D & ~Fs) != 0) != 0) diag(T2{});
  else diag(T1{});
  r.n_total = t;
  r.n_simple = m;
#if DC_C2C_GCORR
  r.gcorr = gp - gn;
#else
  r.gcorr = 0;
#endif
}

// The knight and king moves of ref_for_each_special(_pre), in one order both
// share.  DC_ENUM_PIECE (round 4): per piece -- the source's attack set from
// kAtt, its special targets (not both f in Fs and t in Ts) walked in one loop --
// instead of one loop per direction: a wave pays the slowest lane of every
// loop it enters, and 16 direction loops (each with its own setup) cost more
// than 2-3 piece loops (tools/bbprof_inline.py: the enumeration was 25 % of
// k_count3c's VALU issue cycles).
#ifndef DC_ENUM_PIECE
#define DC_ENUM_PIECE 1
#endif
template <class Leap, class Visit>
__device__ __forceinline__ void special_leapers(u64 n, u64 k, u64 no, u64 Fs, u64 Ts, Leap&& leap, Visit&& visit) {
#if DC_ENUM_PIECE
  auto piece = [&](int f, u64 att) {
    const u64 simple = ((Fs >> f) & 1) ? Ts : 0ull;
    u64 targets = att & no & ~simple;
    while (targets) {
      const int t = lsb(targets);
      targets &= targets - 1;
      visit(f, t);
    }
  };
  for (; n; n &= n - 1) {
    const int f = lsb(n);
    piece(f, kAtt.knight[f]);
  }
  for (; k; k &= k - 1) {
    const int f = lsb(k);
    piece(f, kAtt.king[f]);
  }
#else
  (void)visit;
  leap(sh<17>(n & kNotH) & no, 17, sh<17>(Fs) & Ts);
  leap(sh<15>(n & kNotA) & no, 15, sh<15>(Fs) & Ts);
  leap(sh<10>(n & kNotGH) & no, 10, sh<10>(Fs) & Ts);
  leap(sh<6>(n & kNotAB) & no, 6, sh<6>(Fs) & Ts);
  leap(sh<-6>(n & kNotGH) & no, -6, sh<-6>(Fs) & Ts);
  leap(sh<-10>(n & kNotAB) & no, -10, sh<-10>(Fs) & Ts);
  leap(sh<-15>(n & kNotH) & no, -15, sh<-15>(Fs) & Ts);
  leap(sh<-17>(n & kNotA) & no, -17, sh<-17>(Fs) & Ts);
  leap(sh<8>(k) & no, 8, sh<8>(Fs) & Ts);
  leap(sh<-8>(k) & no, -8, sh<-8>(Fs) & Ts);
  leap(sh<1>(k & kNotH) & no, 1, sh<1>(Fs) & Ts);
  leap(sh<-1>(k & kNotA) & no, -1, sh<-1>(Fs) & Ts);
  leap(sh<9>(k & kNotH) & no, 9, sh<9>(Fs) & Ts);
  leap(sh<7>(k & kNotA) & no, 7, sh<7>(Fs) & Ts);
  leap(sh<-7>(k & kNotH) & no, -7, sh<-7>(Fs) & Ts);
  leap(sh<-9>(k & kNotA) & no, -9, sh<-9>(Fs) & Ts);
#endif
}

// ref_for_each_move<STM> without the simple moves (source in Fs, target in
// Ts): leaper and pawn classes drop them set-wise before the bit loop (the
// source of target t is t - delta), slider classes per move once the source
// is known.
template <int STM, class Visit>
__device__ __forceinline__ void ref_for_each_special(const Board& b, u64 Fs, u64 Ts, Visit&& visit) {
  const Sides s = sides<STM>(b);
  typedef PawnDir<STM> PD;
  const u64 no = s.notown, e = s.empty;
  auto leap = [&](u64 targets, int delta, u64 simple) {
    targets &= ~simple;
    while (targets) {
      const int t = lsb(targets);
      targets &= targets - 1;
      visit(t - delta, t);
    }
  };
  const u64 push1 = sh<PD::F>(s.P) & e;
  leap(push1, PD::F, sh<PD::F>(Fs) & Ts);
  leap(sh<PD::F>(push1 & PD::ROW_AFTER1) & e, 2 * PD::F, sh<2 * PD::F>(Fs) & Ts);
  leap(sh<PD::CW>(s.P & kNotA) & s.enemy, PD::CW, 0);
  leap(sh<PD::CE>(s.P & kNotH) & s.enemy, PD::CE, 0);
  special_leapers(s.N, s.K, no, Fs, Ts, leap, visit);
  auto slide = [&](u64 targets, auto dtag) {
    constexpr int D = decltype(dtag)::value;
    while (targets) {
      const int t = lsb(targets);
      targets &= targets - 1;
      const int f = slider_source<D>(s.occ, t);
      if (((Fs >> f) & (Ts >> t) & 1) == 0) visit(f, t);
    }
  };
  using std::integral_constant;
  slide(ray_attacks<8, kAll>(s.O, e) & no, integral_constant<int, 0>{});
  slide(ray_attacks<-8, kAll>(s.O, e) & no, integral_constant<int, 1>{});
  slide(ray_attacks<1, kNotA>(s.O, e) & no, integral_constant<int, 2>{});
  slide(ray_attacks<-1, kNotH>(s.O, e) & no, integral_constant<int, 3>{});
  slide(ray_attacks<9, kNotA>(s.D, e) & no, integral_constant<int, 4>{});
  slide(ray_attacks<-9, kNotH>(s.D, e) & no, integral_constant<int, 5>{});
  slide(ray_attacks<7, kNotH>(s.D, e) & no, integral_constant<int, 6>{});
  slide(ray_attacks<-7, kNotA>(s.D, e) & no, integral_constant<int, 7>{});
}

// ref_for_each_special with the slider target sets given (tgt[0..7]: the
// special targets of the fills ref_parent_split<STM, G, true> already made,
// simple ones removed); same visiting order.
template <int STM, class Visit>
__device__ __forceinline__ void ref_for_each_special_pre(const Board& b, u64 Fs, u64 Ts, const u64* tgt, Visit&& visit) {
  const Sides s = sides<STM>(b);
  typedef PawnDir<STM> PD;
  const u64 no = s.notown, e = s.empty;
  auto leap = [&](u64 targets, int delta, u64 simple) {
    targets &= ~simple;
    while (targets) {
      const int t = lsb(targets);
      targets &= targets - 1;
      visit(t - delta, t);
    }
  };
  const u64 push1 = sh<PD::F>(s.P) & e;
  leap(push1, PD::F, sh<PD::F>(Fs) & Ts);
  leap(sh<PD::F>(push1 & PD::ROW_AFTER1) & e, 2 * PD::F, sh<2 * PD::F>(Fs) & Ts);
  leap(sh<PD::CW>(s.P & kNotA) & s.enemy, PD::CW, 0);
  leap(sh<PD::CE>(s.P & kNotH) & s.enemy, PD::CE, 0);
  special_leapers(s.N, s.K, no, Fs, Ts, leap, visit);
  auto slide = [&](u64 targets, auto dtag) {
    constexpr int D = decltype(dtag)::value;
    while (targets) {
      const int t = lsb(targets);
      targets &= targets - 1;
      visit(slider_source<D>(s.occ, t), t);  // (tgt holds special targets only)
    }
  };
  using std::integral_constant;
  slide(tgt[0], integral_constant<int, 0>{});
  slide(tgt[1], integral_constant<int, 1>{});
  slide(tgt[2], integral_constant<int, 2>{});
  slide(tgt[3], integral_constant<int, 3>{});
  slide(tgt[4], integral_constant<int, 4>{});
  slide(tgt[5], integral_constant<int, 5>{});
  slide(tgt[6], integral_constant<int, 6>{});
  slide(tgt[7], integral_constant<int, 7>{});
}

// Runtime side-to-move version.
__device__ __forceinline__ u32 ref_count_rt(const Board& b, u32 stm) {
  return stm ? ref_count<1>(b) : ref_count<0>(b);
}

// apply_move's board effect (chess.rs:72-77): the mover's nibble goes to t
// (overwriting any captured piece, kings included), f becomes empty.
__device__ __forceinline__ void ref_make(Board& b, int f, int t) {
  const u64 keep = ~((1ull << f) | (1ull << t));
  b.b0 = (b.b0 & keep) | (((b.b0 >> f) & 1) << t);
  b.b1 = (b.b1 & keep) | (((b.b1 >> f) & 1) << t);
  b.b2 = (b.b2 & keep) | (((b.b2 >> f) & 1) << t);
  b.b3 = (b.b3 & keep) | (((b.b3 >> f) & 1) << t);
}

// validate_move on one (position, move word).  Verdict order chess.rs:82-125.
// Branch-free: every per-kind rule (chess.rs:214-360) is evaluated as a
// predicate and the mover's kind selects one, so lanes holding different
// pieces never serialise on a switch.  The core takes the board's facts the
// rules read -- the mover's nibble, t occupied / own, the double push's mid
// square occupied, the squares between f and t empty -- so the live validator
// can gather them across lanes instead of assembling the board.
__device__ __forceinline__ u32 ref_verdict_core(u32 stm, u32 m, u32 nib, u32 t_occ, u32 t_own, u32 mid_occ, u32 clear) {
  const int f = (int)(m & 63), t = (int)((m >> 6) & 63);
  const u32 kind = nib >> 1;
  const int dx = (t >> 3) - (f >> 3), dy = (t & 7) - (f & 7);
  const int ax = dx < 0 ? -dx : dx, ay = dy < 0 ? -dy : dy;
  const int dir = stm ? -1 : 1;
  const u32 on_start = (u32)((f >> 3) == (stm ? 6 : 1));
  const u32 push = (u32)(dy == 0) & (u32)(dx == dir) & (t_occ ^ 1);
  const u32 dbl = (u32)(dy == 0) & (u32)(dx == 2 * dir) & on_start & (t_occ ^ 1) & (mid_occ ^ 1);
  const u32 cap = (u32)(ay == 1) & (u32)(dx == dir) & t_occ & (t_own ^ 1);
  const u32 pawn_ok = push | dbl | cap;
  const u32 knight_ok = (u32)((ax == 1 && ay == 2) || (ax == 2 && ay == 1));
  const u32 king_ok = (u32)(ax <= 1) & (u32)(ay <= 1);
  const u32 orth = (u32)(dx == 0) | (u32)(dy == 0);
  const u32 diag = (u32)(ax == ay);
  // kind codes: P=1 N=2 K=3 X=4 B=5 R=6 Q=7
  const u32 line_ok = ((kind == KC_B) ? diag : (kind == KC_R) ? orth : (kind == KC_Q) ? (orth | diag) : 0u) & clear;
  const u32 step_ok = (kind == KC_P) ? pawn_ok : (kind == KC_N) ? knight_ok : (kind == KC_K) ? king_ok : 0u;
  const u32 ok = (line_ok | step_ok) & (t_own ^ 1);
  u32 v = ok ? V_OK : V_ILLEGAL;
  v = ((nib & 1) != stm) ? V_WRONG_TURN : v;
  v = (kind == 0) ? V_NO_PIECE : v;
  v = (m & 0x8000u) ? V_OOR : v;
  return v;
}

__device__ __forceinline__ u32 ref_verdict(const Board& b, u32 stm, u32 m) {
  const int f = (int)(m & 63), t = (int)((m >> 6) & 63);
  const u64 occ = occupied(b);
  const u64 own = stm ? b.b0 : (occ & ~b.b0);
  const u32 t_occ = (u32)(occ >> t) & 1, t_own = (u32)(own >> t) & 1;
  const u32 mid_occ = (u32)(occ >> ((f + t) >> 1)) & 1;  // only meaningful for a double push
  const u32 clear = (u32)((between(f, t) & occ) == 0);
  return ref_verdict_core(stm, m, nibble(b, f), t_occ, t_own, mid_occ, clear);
}

__device__ __forceinline__ u64 board_digest(const Board& b, u32 stm) {
  u64 h = 0x6A09E667F3BCC909ull ^ (u64)(stm & 1);
  h = fmix64(h ^ b.b3);
  h = fmix64(h ^ b.b2);
  h = fmix64(h ^ b.b1);
  h = fmix64(h ^ b.b0);
  return h;
}

// Target set of one REF piece (for the canonical-order generator).
__device__ __forceinline__ u64 ref_piece_targets(const Board& b, int f, u32 stm, u32 kind) {
  const u64 occ = occupied(b);
  const u64 own = stm ? b.b0 : (occ & ~b.b0);
  const u64 enemy = occ & ~own, empty = ~occ, no = ~own;
  const u64 bit = 1ull << f;
  switch (kind) {
    case KC_P: {
      u64 p1, p2, c;
      if (stm == 0) {
        p1 = (bit << 8) & empty;
        p2 = ((p1 & kRow(2)) << 8) & empty;
        c = (((bit & kNotA) << 7) | ((bit & kNotH) << 9)) & enemy;
      } else {
        p1 = (bit >> 8) & empty;
        p2 = ((p1 & kRow(5)) >> 8) & empty;
        c = (((bit & kNotA) >> 9) | ((bit & kNotH) >> 7)) & enemy;
      }
      return p1 | p2 | c;
    }
    case KC_N:
      return (sh<17>(bit & kNotH) | sh<15>(bit & kNotA) | sh<10>(bit & kNotGH) | sh<6>(bit & kNotAB) |
              sh<-6>(bit & kNotGH) | sh<-10>(bit & kNotAB) | sh<-15>(bit & kNotH) | sh<-17>(bit & kNotA)) &
             no;
    case KC_K:
      return (sh<8>(bit) | sh<-8>(bit) | sh<1>(bit & kNotH) | sh<-1>(bit & kNotA) | sh<9>(bit & kNotH) |
              sh<7>(bit & kNotA) | sh<-7>(bit & kNotH) | sh<-9>(bit & kNotA)) &
             no;
    case KC_B:
    case KC_R:
    case KC_Q: {
      u64 a = 0;
      if (kind != KC_B)
        a |= ray_attacks<8, kAll>(bit, empty) | ray_attacks<-8, kAll>(bit, empty) |
             ray_attacks<1, kNotA>(bit, empty) | ray_attacks<-1, kNotH>(bit, empty);
      if (kind != KC_R)
        a |= ray_attacks<9, kNotA>(bit, empty) | ray_attacks<-9, kNotH>(bit, empty) |
             ray_attacks<7, kNotH>(bit, empty) | ray_attacks<-7, kNotA>(bit, empty);
      return a & no;
    }
    default: return 0;
  }
}

// ------------------------------------------------------------------------
// Move classes for enumeration.  Class c's target set and source rule:
//   0 push1, 1 push2, 2 capture toward y-1, 3 capture toward y+1,
//   4..11 knight offsets, 12..19 king offsets, 20..23 orthogonal rays N,S,E,W,
//   24..27 diagonal rays NE,SW,NW,SE.
// The visitor gets (from, to) for every move; order is class-major, target
// ascending within a class (deterministic).
template <int STM, class Visit>
__device__ __forceinline__ void ref_for_each_move(const Board& b, Visit&& visit) {
  const Sides s = sides<STM>(b);
  typedef PawnDir<STM> PD;
  const u64 no = s.notown, e = s.empty;
  auto leap = [&](u64 targets, int delta) {
    while (targets) {
      const int t = lsb(targets);
      targets &= targets - 1;
      visit(t - delta, t);
    }
  };
  const u64 push1 = sh<PD::F>(s.P) & e;
  leap(push1, PD::F);
  leap(sh<PD::F>(push1 & PD::ROW_AFTER1) & e, 2 * PD::F);
  leap(sh<PD::CW>(s.P & kNotA) & s.enemy, PD::CW);
  leap(sh<PD::CE>(s.P & kNotH) & s.enemy, PD::CE);
  const u64 n = s.N;
  leap(sh<17>(n & kNotH) & no, 17);
  leap(sh<15>(n & kNotA) & no, 15);
  leap(sh<10>(n & kNotGH) & no, 10);
  leap(sh<6>(n & kNotAB) & no, 6);
  leap(sh<-6>(n & kNotGH) & no, -6);
  leap(sh<-10>(n & kNotAB) & no, -10);
  leap(sh<-15>(n & kNotH) & no, -15);
  leap(sh<-17>(n & kNotA) & no, -17);
  const u64 k = s.K;
  leap(sh<8>(k) & no, 8);
  leap(sh<-8>(k) & no, -8);
  leap(sh<1>(k & kNotH) & no, 1);
  leap(sh<-1>(k & kNotA) & no, -1);
  leap(sh<9>(k & kNotH) & no, 9);
  leap(sh<7>(k & kNotA) & no, 7);
  leap(sh<-7>(k & kNotH) & no, -7);
  leap(sh<-9>(k & kNotA) & no, -9);
  auto slide = [&](u64 targets, auto dtag) {
    constexpr int D = decltype(dtag)::value;
    while (targets) {
      const int t = lsb(targets);
      targets &= targets - 1;
      visit(slider_source<D>(s.occ, t), t);
    }
  };
  slide(ray_attacks<8, kAll>(s.O, e) & no, std::integral_constant<int, 0>{});
  slide(ray_attacks<-8, kAll>(s.O, e) & no, std::integral_constant<int, 1>{});
  slide(ray_attacks<1, kNotA>(s.O, e) & no, std::integral_constant<int, 2>{});
  slide(ray_attacks<-1, kNotH>(s.O, e) & no, std::integral_constant<int, 3>{});
  slide(ray_attacks<9, kNotA>(s.D, e) & no, std::integral_constant<int, 4>{});
  slide(ray_attacks<-9, kNotH>(s.D, e) & no, std::integral_constant<int, 5>{});
  slide(ray_attacks<7, kNotH>(s.D, e) & no, std::integral_constant<int, 6>{});
  slide(ray_attacks<-7, kNotA>(s.D, e) & no, std::integral_constant<int, 7>{});
}


// ref_for_each_move's classes in four contiguous groups (so the groups in
// order 0..3 give ref_for_each_move's order): 0 pawns (push1, push2, both
// captures), 1 knights, 2 king + orthogonal rays, 3 diagonal rays.
// ref_group_count<STM, G> = the number of moves ref_group_moves<STM, G> visits.
// k_level_moves enumerates one group per wave, so a lane walks a quarter of
// its position's moves.
template <int STM, int G, class Visit>
__device__ __forceinline__ void ref_group_moves(const Board& b, Visit&& visit) {
  const Sides s = sides<STM>(b);
  typedef PawnDir<STM> PD;
  const u64 no = s.notown, e = s.empty;
  auto leap = [&](u64 targets, int delta) {
    while (targets) {
      const int t = lsb(targets);
      targets &= targets - 1;
      visit(t - delta, t);
    }
  };
  auto slide = [&](u64 targets, auto dtag) {
    constexpr int D = decltype(dtag)::value;
    while (targets) {
      const int t = lsb(targets);
      targets &= targets - 1;
      visit(slider_source<D>(s.occ, t), t);
    }
  };
  if constexpr (G == 0) {
    const u64 push1 = sh<PD::F>(s.P) & e;
    leap(push1, PD::F);
    leap(sh<PD::F>(push1 & PD::ROW_AFTER1) & e, 2 * PD::F);
    leap(sh<PD::CW>(s.P & kNotA) & s.enemy, PD::CW);
    leap(sh<PD::CE>(s.P & kNotH) & s.enemy, PD::CE);
  } else if constexpr (G == 1) {
    const u64 n = s.N;
    leap(sh<17>(n & kNotH) & no, 17);
    leap(sh<15>(n & kNotA) & no, 15);
    leap(sh<10>(n & kNotGH) & no, 10);
    leap(sh<6>(n & kNotAB) & no, 6);
    leap(sh<-6>(n & kNotGH) & no, -6);
    leap(sh<-10>(n & kNotAB) & no, -10);
    leap(sh<-15>(n & kNotH) & no, -15);
    leap(sh<-17>(n & kNotA) & no, -17);
  } else if constexpr (G == 2) {
    const u64 k = s.K;
    leap(sh<8>(k) & no, 8);
    leap(sh<-8>(k) & no, -8);
    leap(sh<1>(k & kNotH) & no, 1);
    leap(sh<-1>(k & kNotA) & no, -1);
    leap(sh<9>(k & kNotH) & no, 9);
    leap(sh<7>(k & kNotA) & no, 7);
    leap(sh<-7>(k & kNotH) & no, -7);
    leap(sh<-9>(k & kNotA) & no, -9);
    slide(ray_attacks<8, kAll>(s.O, e) & no, std::integral_constant<int, 0>{});
    slide(ray_attacks<-8, kAll>(s.O, e) & no, std::integral_constant<int, 1>{});
    slide(ray_attacks<1, kNotA>(s.O, e) & no, std::integral_constant<int, 2>{});
    slide(ray_attacks<-1, kNotH>(s.O, e) & no, std::integral_constant<int, 3>{});
  } else {
    slide(ray_attacks<9, kNotA>(s.D, e) & no, std::integral_constant<int, 4>{});
    slide(ray_attacks<-9, kNotH>(s.D, e) & no, std::integral_constant<int, 5>{});
    slide(ray_attacks<7, kNotH>(s.D, e) & no, std::integral_constant<int, 6>{});
    slide(ray_attacks<-7, kNotA>(s.D, e) & no, std::integral_constant<int, 7>{});
  }
}

template <int STM, int G>
__device__ __forceinline__ u32 ref_group_count(const Board& b) {
  const Sides s = sides<STM>(b);
  typedef PawnDir<STM> PD;
  const u64 no = s.notown, e = s.empty;
  if constexpr (G == 0) {
    const u64 push1 = sh<PD::F>(s.P) & e;
    return pc(push1) + pc(and3(sh<PD::F>(push1), PD::ROW_DBL, e)) + pc(and3(sh<PD::CW>(s.P), kNotH, s.enemy)) +
           pc(and3(sh<PD::CE>(s.P), kNotA, s.enemy));
  } else if constexpr (G == 1) {
    const u64 n = s.N;
    return pc(and3(sh<17>(n), kNotA, no)) + pc(and3(sh<15>(n), kNotH, no)) + pc(and3(sh<10>(n), kNotAB, no)) +
           pc(and3(sh<6>(n), kNotGH, no)) + pc(and3(sh<-6>(n), kNotAB, no)) + pc(and3(sh<-10>(n), kNotGH, no)) +
           pc(and3(sh<-15>(n), kNotA, no)) + pc(and3(sh<-17>(n), kNotH, no));
  } else if constexpr (G == 2) {
    return king_moves(s.K, no) + pc(ray_attacks<8, kAll>(s.O, e) & no) + pc(ray_attacks<-8, kAll>(s.O, e) & no) +
           pc(ray_moves<1, kNotA>(s.O, e, no)) + pc(ray_moves<-1, kNotH>(s.O, e, no));
  } else {
    return pc(ray_moves<9, kNotA>(s.D, e, no)) + pc(ray_moves<-9, kNotH>(s.D, e, no)) +
           pc(ray_moves<7, kNotH>(s.D, e, no)) + pc(ray_moves<-7, kNotA>(s.D, e, no));
  }
}

}  // namespace dc
