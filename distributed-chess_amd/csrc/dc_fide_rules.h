// dc_fide_rules.h -- RULES_FIDE (standard chess) on the quad-bitboard.
//
// The reference validator has no check, pin, castling, en-passant or
// promotion logic; BASELINE configs[2]/[4] quote standard perft
// (Kiwipete & the standard suite), so this second rule set shares the board,
// the kernels and the ABI, and is pinned by the published perft tables
// (tests/golden/oracle_golden.json "perft_fide") and by fastcpu.
//
// Legal generation is set-wise: one analysis per position (enemy attack map
// with our king removed, checkers via a ray scan from the king, pinned pieces,
// check mask), then free pieces are handled by direction class exactly like
// RULES_REF and the few pinned pieces / en-passant / castling individually.
//
// Per-node state beside the board: meta = castle rights (bits 0-3: K Q k q)
// | en-passant target square << 4 | 0x400 when valid (dc_fide.h pack_meta).
#pragma once
#include "dc_ref.h"

namespace dc {

enum : u32 { CR_WK = 1, CR_WQ = 2, CR_BK = 4, CR_BQ = 8, META_EP_VALID = 0x400 };

__device__ __forceinline__ int meta_ep(u32 meta) { return (meta & META_EP_VALID) ? (int)((meta >> 4) & 63) : -1; }

template <int SIDE>
__device__ __forceinline__ u64 pawn_attacks(u64 p) {
  if constexpr (SIDE == 0) return sh<7>(p & kNotA) | sh<9>(p & kNotH);
  else return sh<-9>(p & kNotA) | sh<-7>(p & kNotH);
}
__device__ __forceinline__ u64 knight_attacks(u64 n) {
  return sh<17>(n & kNotH) | sh<15>(n & kNotA) | sh<10>(n & kNotGH) | sh<6>(n & kNotAB) | sh<-6>(n & kNotGH) |
         sh<-10>(n & kNotAB) | sh<-15>(n & kNotH) | sh<-17>(n & kNotA);
}
__device__ __forceinline__ u64 king_attacks(u64 k) {
  return sh<8>(k) | sh<-8>(k) | sh<1>(k & kNotH) | sh<-1>(k & kNotA) | sh<9>(k & kNotH) | sh<7>(k & kNotA) |
         sh<-7>(k & kNotH) | sh<-9>(k & kNotA);
}
// TAB: king and knight attack sets from kAtt (one L1 load per piece instead
// of eight shifts) -- the final stage's leaf counts only (k_count2b); the
// single-workgroup top plies are latency-bound and keep the shifts
#ifndef DC_FIDE_TAB_UNCOND
#define DC_FIDE_TAB_UNCOND 0
#endif
#ifndef DC_FIDE_TAB_PARTS
#define DC_FIDE_TAB_PARTS 7  // (diagnostics) 1 king sets, 2 enemy knight sets, 4 own knight counts
#endif
template <bool TAB>
__device__ __forceinline__ u64 king_attacks_t(u64 k) {
  if constexpr (TAB && (DC_FIDE_TAB_PARTS & 1)) {
#if DC_FIDE_TAB_UNCOND == 1
    // (diagnostics) the load issued by every lane, outside the branch
    u64 t = kAtt.king[lsb(k | (1ull << 63)) & 63];
    asm volatile("" : "+v"(t));
    if ((k & (k - 1)) == 0) return k ? t : 0ull;
#elif DC_FIDE_TAB_UNCOND == 2
    // (diagnostics) the load waited for at once
    if ((k & (k - 1)) == 0) {
      u64 t = k ? kAtt.king[lsb(k) & 63] : 0ull;
      asm volatile("s_waitcnt vmcnt(0)" : "+v"(t)::"memory");
      return t;
    }
#elif DC_FIDE_TAB_UNCOND == 3
    // (diagnostics) the table address in VGPRs (no SGPR base operand)
    if ((k & (k - 1)) == 0) {
      const u64* base = &kAtt.king[0];
      asm volatile("" : "+v"(base));
      return k ? base[lsb(k) & 63] : 0ull;
    }
#else
    if ((k & (k - 1)) == 0) return k ? kAtt.king[lsb(k) & 63] : 0ull;
#endif
  }
  return king_attacks(k);
}
template <bool TAB>
__device__ __forceinline__ u64 knight_attacks_t(u64 n) {
  if constexpr (TAB && (DC_FIDE_TAB_PARTS & 2)) {
    u64 a = 0;
    for (; n; n &= n - 1) a |= kAtt.knight[lsb(n) & 63];
    return a;
  }
  return knight_attacks(n);
}
__device__ __forceinline__ u64 orth_attacks(u64 s, u64 empty) {
  return ray_attacks<8, kAll>(s, empty) | ray_attacks<-8, kAll>(s, empty) | ray_attacks<1, kNotA>(s, empty) |
         ray_attacks<-1, kNotH>(s, empty);
}
__device__ __forceinline__ u64 diag_attacks(u64 s, u64 empty) {
  return ray_attacks<9, kNotA>(s, empty) | ray_attacks<-9, kNotH>(s, empty) | ray_attacks<7, kNotH>(s, empty) |
         ray_attacks<-7, kNotA>(s, empty);
}

// Lines through a square (full file, rank, diagonal, anti-diagonal).
struct Lines {
  u64 file, rank, diag, anti;
};
__device__ __forceinline__ Lines lines_of(int s) {
  const int x = s >> 3, y = s & 7;
  const int d = x - y, a = x + y - 7;
  Lines l;
  l.file = kFileA << y;
  l.rank = 0xFFull << (8 * x);
  l.diag = d >= 0 ? (kDiagMain << (8 * d)) : (kDiagMain >> (-8 * d));
  l.anti = a >= 0 ? (kDiagAnti << (8 * a)) : (kDiagAnti >> (-8 * a));
  return l;
}
__device__ __forceinline__ u64 above_mask(int s) { return ~((2ull << s) - 1); }  // squares > s (s=63: 0)
__device__ __forceinline__ u64 below_mask(int s) { return (1ull << s) - 1; }     // squares < s

// The full line through a and b (0 if they are not aligned).
__device__ __forceinline__ u64 line_through(int a, int b) {
  const Lines l = lines_of(a);
  const u64 bb = 1ull << b;
  return (l.file & bb) ? l.file : (l.rank & bb) ? l.rank : (l.diag & bb) ? l.diag : (l.anti & bb) ? l.anti : 0;
}

// Attacks of a single slider along one line (both directions), classical
// nearest-blocker method.
__device__ __forceinline__ u64 line_attacks(int s, u64 line, u64 occ) {
  const u64 up = line & above_mask(s), dn = line & below_mask(s);
  const u64 bu = occ & up, bd = occ & dn;
  const u64 segu = bu ? (up & ((2ull << lsb(bu)) - 1)) : up;            // up to and including first blocker
  const u64 segd = bd ? (dn & ~((1ull << msb(bd)) - 1)) : dn;            // down to and including first blocker
  return segu | segd;
}

// Side-relative view of a position.
template <int STM>
struct FPos {
  u64 occ, us, them, empty;
  u64 P, N, D, O, K;       // ours (D: bishops+queens, O: rooks+queens)
  u64 tP, tN, tD, tO, tK;  // theirs
};

template <int STM>
__device__ __forceinline__ FPos<STM> fpos(const Board& b) {
  FPos<STM> f;
  f.occ = occupied(b);
  f.us = STM ? b.b0 : (f.occ & ~b.b0);
  f.them = f.occ ^ f.us;
  f.empty = ~f.occ;
  const u64 lo = b.b1, mid = b.b2, hi = b.b3;
  const u64 p = lo & ~(mid | hi), n = mid & ~(lo | hi), k = lo & mid & ~hi, dg = hi & lo, og = hi & mid;
  f.P = p & f.us;
  f.N = n & f.us;
  f.K = k & f.us;
  f.D = dg & f.us;
  f.O = og & f.us;
  f.tP = p & f.them;
  f.tN = n & f.them;
  f.tK = k & f.them;
  f.tD = dg & f.them;
  f.tO = og & f.them;
  return f;
}

// Per-position legality analysis.
struct Analysis {
  u64 danger;    // squares attacked by the opponent (our king removed from occupancy)
  u64 checkers;  // opponent pieces giving check
  u64 cmask;     // targets that resolve a single check (all ones when not in check)
  u64 pinned;    // our pieces pinned to our king
  int ksq;       // our king square, -1 if none
};

// Branch-free on purpose: with `checkers |= m1; return;` on one path and
// `pinned |= m1` on another, the compiler merged the two stores into one
// store through a selected address (&a.checkers or &a.pinned), which kept the
// whole Analysis in scratch memory (round 3: 536 B/lane in k_count2b<Fide>).
// Two unconditional value updates keep both in registers.
// kup / kdn: the squares above / below the king (above_mask / below_mask),
// made once by analyse before its gates.
template <int STM, int D>
__device__ __forceinline__ void scan_dir(const FPos<STM>& f, u64 kup, u64 kdn, const Lines& l, u64& checkers,
                                         u64& pinned) {
  constexpr bool UP = (D & 1) == 0;  // 0 N, 2 E, 4 NE, 6 NW go to higher squares
  const u64 line = (D < 2) ? l.file : (D < 4) ? l.rank : (D < 6) ? l.diag : l.anti;
  const u64 ray = line & (UP ? kup : kdn);
  const u64 sl = (D < 4) ? f.tO : f.tD;
  const u64 blk = f.occ & ray;
  // first and second occupied squares on the ray (bits; 0 when absent)
  const u64 m1 = UP ? (blk & (0ull - blk)) : (blk ? (1ull << msb(blk)) : 0ull);
  const u64 rest = blk & ~m1;
  const u64 m2 = UP ? (rest & (0ull - rest)) : (rest ? (1ull << msb(rest)) : 0ull);
  checkers |= m1 & sl;
  pinned |= ((m2 & sl) ? (m1 & f.us) : 0ull);
}

#ifndef DC_FIDE_SNIPER
#define DC_FIDE_SNIPER 1
#endif
#ifndef DC_FIDE_LAZY_DANGER
#define DC_FIDE_LAZY_DANGER 0  // 1: fide_count computes the attack map only in waves that need it (2: also
                               // the split's passes) -- measured slower, off
#endif
// with_danger = false (wave-uniform): no attack map; danger reads "every
// square attacked", i.e. no king move and no castling -- for callers whose
// lanes have neither a free square next to the king nor an open castling path
template <int STM, bool TAB = false>
__device__ __forceinline__ Analysis analyse(const FPos<STM>& f, bool with_danger = true) {
  constexpr int THEM = 1 - STM;
  Analysis a;
  const u64 empty_nk = f.empty | f.K;
  a.danger = ~0ull;
  if (with_danger)
    a.danger = pawn_attacks<THEM>(f.tP) | knight_attacks_t<TAB>(f.tN) | king_attacks_t<TAB>(f.tK) |
               orth_attacks(f.tO, empty_nk) | diag_attacks(f.tD, empty_nk);
  a.checkers = 0;
  a.pinned = 0;
  a.ksq = f.K ? lsb(f.K) : -1;
  a.cmask = ~0ull;
  if (a.ksq < 0) return a;
  a.checkers = (pawn_attacks<STM>(f.K) & f.tP) | (knight_attacks(f.K) & f.tN);
  const Lines l = lines_of(a.ksq);
  // The king's half-line masks are made here, before the line gates, and kept
  // opaque.  Left to the compiler they were made between a gate's 64-bit
  // compare and its branch, the second shift overwriting the compare's
  // operands: the three-instruction window in which a co-resident wave's
  // single-issue VALU instruction made the round-4 table variant miscount
  // (tools/vccz_check.py --shape).
  u64 kup = above_mask(a.ksq), kdn = below_mask(a.ksq);
  asm volatile("" : "+v"(kup), "+v"(kdn));
  u64 chk = a.checkers, pin = 0;
#if DC_FIDE_SNIPER == 2
  // (diagnostics) the same gate as a per-lane branch (no __ballot)
  if ((l.file & f.tO) != 0) {
    scan_dir<STM, 0>(f, kup, kdn, l, chk, pin);
    scan_dir<STM, 1>(f, kup, kdn, l, chk, pin);
  }
  if ((l.rank & f.tO) != 0) {
    scan_dir<STM, 2>(f, kup, kdn, l, chk, pin);
    scan_dir<STM, 3>(f, kup, kdn, l, chk, pin);
  }
  if ((l.diag & f.tD) != 0) {
    scan_dir<STM, 4>(f, kup, kdn, l, chk, pin);
    scan_dir<STM, 5>(f, kup, kdn, l, chk, pin);
  }
  if ((l.anti & f.tD) != 0) {
    scan_dir<STM, 6>(f, kup, kdn, l, chk, pin);
    scan_dir<STM, 7>(f, kup, kdn, l, chk, pin);
  }
#elif DC_FIDE_SNIPER
  // a line through the king with no enemy slider of its kind on it can hold
  // neither a slider check nor a pin: a wave none of whose lanes has one
  // skips that line's two scans (round 4: the eight scans were ~19 % of the
  // FIDE final stage, tools/bbprof_inline.py)
  // Round 6: the four gates' operands are made together before the first gate
  // (opaque), and each stays live past its own branch (an empty asm reading
  // it after the if), so no VALU write can land on a gate compare's source
  // registers between the compare and its VCCZ branch -- the shape
  // tools/vccz_check.py --any flagged in 16 FIDE kernels after round 5 (there
  // the next gate's v_and_b32 overwrote them).
  u64 g_file = l.file & f.tO, g_rank = l.rank & f.tO, g_diag = l.diag & f.tD, g_anti = l.anti & f.tD;
  asm volatile("" : "+v"(g_file), "+v"(g_rank), "+v"(g_diag), "+v"(g_anti));
  if (__ballot(g_file != 0)) {
    scan_dir<STM, 0>(f, kup, kdn, l, chk, pin);
    scan_dir<STM, 1>(f, kup, kdn, l, chk, pin);
  }
  asm volatile("" ::"v"(g_file));
  if (__ballot(g_rank != 0)) {
    scan_dir<STM, 2>(f, kup, kdn, l, chk, pin);
    scan_dir<STM, 3>(f, kup, kdn, l, chk, pin);
  }
  asm volatile("" ::"v"(g_rank));
  if (__ballot(g_diag != 0)) {
    scan_dir<STM, 4>(f, kup, kdn, l, chk, pin);
    scan_dir<STM, 5>(f, kup, kdn, l, chk, pin);
  }
  asm volatile("" ::"v"(g_diag));
  if (__ballot(g_anti != 0)) {
    scan_dir<STM, 6>(f, kup, kdn, l, chk, pin);
    scan_dir<STM, 7>(f, kup, kdn, l, chk, pin);
  }
  asm volatile("" ::"v"(g_anti));
#else
  scan_dir<STM, 0>(f, kup, kdn, l, chk, pin);
  scan_dir<STM, 1>(f, kup, kdn, l, chk, pin);
  scan_dir<STM, 2>(f, kup, kdn, l, chk, pin);
  scan_dir<STM, 3>(f, kup, kdn, l, chk, pin);
  scan_dir<STM, 4>(f, kup, kdn, l, chk, pin);
  scan_dir<STM, 5>(f, kup, kdn, l, chk, pin);
  scan_dir<STM, 6>(f, kup, kdn, l, chk, pin);
  scan_dir<STM, 7>(f, kup, kdn, l, chk, pin);
#endif
  a.checkers = chk;
  a.pinned = pin;
  if (chk) a.cmask = chk | between(a.ksq, lsb(chk));
  return a;
}

// Is our king attacked after the en-passant capture from->to (captured pawn on cap)?
template <int STM>
__device__ __forceinline__ bool ep_legal(const FPos<STM>& f, int ksq, int from, int to, int cap) {
  if (ksq < 0) return true;
  constexpr int THEM = 1 - STM;
  const u64 occ = (f.occ ^ (1ull << from) ^ (1ull << cap)) | (1ull << to);
  const u64 tP = f.tP & ~(1ull << cap);
  const u64 k = 1ull << ksq;
  if (pawn_attacks<STM>(k) & tP) return false;
  if (knight_attacks(k) & f.tN) return false;
  if (king_attacks(k) & f.tK) return false;
  const Lines l = lines_of(ksq);
  if ((line_attacks(ksq, l.file, occ) | line_attacks(ksq, l.rank, occ)) & f.tO) return false;
  if ((line_attacks(ksq, l.diag, occ) | line_attacks(ksq, l.anti, occ)) & f.tD) return false;
  (void)THEM;
  return true;
}

template <int STM>
struct FDir {
  static constexpr int F = STM ? -8 : 8;
  static constexpr int CW = STM ? -9 : 7;
  static constexpr int CE = STM ? -7 : 9;
  static constexpr u64 ROW_AFTER1 = STM ? kRow(5) : kRow(2);
  static constexpr u64 LAST = STM ? kRow(0) : kRow(7);
  static constexpr int HOME = STM ? 60 : 4;
  static constexpr u32 RK = STM ? CR_BK : CR_WK;
  static constexpr u32 RQ = STM ? CR_BQ : CR_WQ;
};

// Does any lane of the wave need the attack map: a free square next to the
// king or an open castling path (`meta`'s rights, the squares between king
// and rook empty)?
template <int STM>
__device__ __forceinline__ bool wave_needs_danger(const FPos<STM>& f, u32 meta) {
  typedef FDir<STM> FD;
  const int h = FD::HOME;
  const bool castle_open = ((f.K >> h) & 1) && (((meta & FD::RK) && !((f.occ >> (h + 1)) & 3)) ||
                                                 ((meta & FD::RQ) && !((f.occ >> (h - 3)) & 7)));
  return __ballot((king_attacks(f.K) & ~f.us) != 0 || castle_open) != 0;
}

// Castling targets (king destination squares) -- only when not in check.
template <int STM>
__device__ __forceinline__ u64 castle_targets(const FPos<STM>& f, const Analysis& a, u32 meta, const Board& b) {
  typedef FDir<STM> FD;
  if (a.checkers || a.ksq != FD::HOME) return 0;
  u64 t = 0;
  const int h = FD::HOME;
  const u64 rooks = f.O & ~f.D;  // rooks proper (not queens)
  if ((meta & FD::RK) && (rooks >> (h + 3) & 1) && !((f.occ >> (h + 1)) & 3) && !((a.danger >> (h + 1)) & 3))
    t |= 1ull << (h + 2);
  if ((meta & FD::RQ) && (rooks >> (h - 4) & 1) && !((f.occ >> (h - 3)) & 7) && !((a.danger >> (h - 2)) & 3))
    t |= 1ull << (h - 2);
  (void)b;
  return t;
}

// Number of legal moves (promotions count 4).  TAB: see king_attacks_t.
template <int STM, bool TAB = false>
__device__ __forceinline__ u32 fide_count(const Board& b, u32 meta) {
  typedef FDir<STM> FD;
  const FPos<STM> f = fpos<STM>(b);
  // the attack map is needed only for king moves and castling: a wave none of
  // whose lanes has a free square next to its king or an open castling path
  // skips it (a third of perft(7)'s leaf parents; siblings share their king's
  // surroundings)
#if DC_FIDE_LAZY_DANGER
  const Analysis a = analyse<STM, TAB>(f, wave_needs_danger<STM>(f, meta));
#else
  const Analysis a = analyse<STM, TAB>(f);
#endif
  const u64 notus = ~f.us;
  u32 c = pc(king_attacks_t<TAB>(f.K) & notus & ~a.danger);
  if (a.checkers & (a.checkers - 1)) return c;  // double check: king moves only
  const u64 tm = notus & a.cmask;
  // free (unpinned) pieces, one popcount per direction class
  const u64 Pf = f.P & ~a.pinned;
  const u64 push1 = sh<FD::F>(Pf) & f.empty;
  const u64 push2 = sh<FD::F>(push1 & FD::ROW_AFTER1) & f.empty & a.cmask;
  const u64 p1 = push1 & a.cmask;
  const u64 cw = sh<FD::CW>(Pf & kNotA) & f.them & a.cmask;
  const u64 ce = sh<FD::CE>(Pf & kNotH) & f.them & a.cmask;
  c += pc(p1) + pc(push2) + pc(cw) + pc(ce) + 3 * (pc(p1 & FD::LAST) + pc(cw & FD::LAST) + pc(ce & FD::LAST));
  const u64 n = f.N & ~a.pinned;
  if constexpr (TAB && (DC_FIDE_TAB_PARTS & 4)) {
    for (u64 k = n; k; k &= k - 1) c += pc(kAtt.knight[lsb(k) & 63] & tm);
  } else {
    c += pc(sh<17>(n & kNotH) & tm) + pc(sh<15>(n & kNotA) & tm) + pc(sh<10>(n & kNotGH) & tm) +
         pc(sh<6>(n & kNotAB) & tm) + pc(sh<-6>(n & kNotGH) & tm) + pc(sh<-10>(n & kNotAB) & tm) +
         pc(sh<-15>(n & kNotH) & tm) + pc(sh<-17>(n & kNotA) & tm);
  }
  const u64 e = f.empty, O = f.O & ~a.pinned, D = f.D & ~a.pinned;
  c += pc(ray_attacks<8, kAll>(O, e) & tm) + pc(ray_attacks<-8, kAll>(O, e) & tm) +
       pc(ray_attacks<1, kNotA>(O, e) & tm) + pc(ray_attacks<-1, kNotH>(O, e) & tm);
  c += pc(ray_attacks<9, kNotA>(D, e) & tm) + pc(ray_attacks<-9, kNotH>(D, e) & tm) +
       pc(ray_attacks<7, kNotH>(D, e) & tm) + pc(ray_attacks<-7, kNotA>(D, e) & tm);
  // pinned pieces move only along their pin line (never when in check)
  if (!a.checkers) {
    u64 pins = a.pinned;
    while (pins) {
      const int s = lsb(pins);
      pins &= pins - 1;
      const u64 line = line_through(a.ksq, s);
      const u64 bit = 1ull << s;
      u64 t;
      if (bit & f.P) {
        const u64 q1 = sh<FD::F>(bit) & f.empty;
        t = (q1 | (sh<FD::F>(q1 & FD::ROW_AFTER1) & f.empty) | (pawn_attacks<STM>(bit) & f.them)) & line;
        c += pc(t) + 3 * pc(t & FD::LAST);
      } else if (bit & (f.O | f.D)) {
        const bool orth_line = (line == lines_of(s).file) || (line == lines_of(s).rank);
        if ((orth_line && (bit & f.O)) || (!orth_line && (bit & f.D)))
          c += pc(line_attacks(s, line, f.occ) & notus);
      }
    }
  }
  // en passant (full legality test; also covers pinned capturers)
  const int ep = meta_ep(meta);
  if (ep >= 0) {
    u64 cand = pawn_attacks<1 - STM>(1ull << ep) & f.P;
    while (cand) {
      const int s = lsb(cand);
      cand &= cand - 1;
      c += ep_legal<STM>(f, a.ksq, s, ep, ep - FD::F) ? 1u : 0u;
    }
  }
  c += pc(castle_targets<STM>(f, a, meta, b));
  return c;
}

// Enumerates legal moves: visit(from, to, promo).  Deterministic order.
template <int STM, class Visit>
__device__ __forceinline__ void fide_for_each_move(const Board& b, u32 meta, Visit&& visit) {
  typedef FDir<STM> FD;
  const FPos<STM> f = fpos<STM>(b);
  const Analysis a = analyse<STM>(f);
  const u64 notus = ~f.us;
  auto emit = [&](int from, u64 targets) {
    while (targets) {
      const int t = lsb(targets);
      targets &= targets - 1;
      visit(from, t, 0);
    }
  };
  auto emit_pawn = [&](u64 targets, int delta) {
    while (targets) {
      const int t = lsb(targets);
      targets &= targets - 1;
      if ((1ull << t) & FD::LAST) {
        for (int pr = 1; pr <= 4; ++pr) visit(t - delta, t, pr);
      } else {
        visit(t - delta, t, 0);
      }
    }
  };
  if (a.ksq >= 0) emit(a.ksq, (king_attacks(f.K) & notus & ~a.danger) | castle_targets<STM>(f, a, meta, b));
  if (a.checkers & (a.checkers - 1)) return;
  const u64 tm = notus & a.cmask;
  const u64 Pf = f.P & ~a.pinned;
  const u64 push1 = sh<FD::F>(Pf) & f.empty;
  emit_pawn(push1 & a.cmask, FD::F);
  emit_pawn(sh<FD::F>(push1 & FD::ROW_AFTER1) & f.empty & a.cmask, 2 * FD::F);
  emit_pawn(sh<FD::CW>(Pf & kNotA) & f.them & a.cmask, FD::CW);
  emit_pawn(sh<FD::CE>(Pf & kNotH) & f.them & a.cmask, FD::CE);
  const u64 n = f.N & ~a.pinned;
  auto leap = [&](u64 targets, int delta) {
    while (targets) {
      const int t = lsb(targets);
      targets &= targets - 1;
      visit(t - delta, t, 0);
    }
  };
  leap(sh<17>(n & kNotH) & tm, 17);
  leap(sh<15>(n & kNotA) & tm, 15);
  leap(sh<10>(n & kNotGH) & tm, 10);
  leap(sh<6>(n & kNotAB) & tm, 6);
  leap(sh<-6>(n & kNotGH) & tm, -6);
  leap(sh<-10>(n & kNotAB) & tm, -10);
  leap(sh<-15>(n & kNotH) & tm, -15);
  leap(sh<-17>(n & kNotA) & tm, -17);
  const u64 e = f.empty, O = f.O & ~a.pinned, D = f.D & ~a.pinned;
  auto slide = [&](u64 targets, auto dtag) {
    constexpr int DD = decltype(dtag)::value;
    while (targets) {
      const int t = lsb(targets);
      targets &= targets - 1;
      visit(slider_source<DD, false>(f.occ, t), t, 0);
    }
  };
  slide(ray_attacks<8, kAll>(O, e) & tm, std::integral_constant<int, 0>{});
  slide(ray_attacks<-8, kAll>(O, e) & tm, std::integral_constant<int, 1>{});
  slide(ray_attacks<1, kNotA>(O, e) & tm, std::integral_constant<int, 2>{});
  slide(ray_attacks<-1, kNotH>(O, e) & tm, std::integral_constant<int, 3>{});
  slide(ray_attacks<9, kNotA>(D, e) & tm, std::integral_constant<int, 4>{});
  slide(ray_attacks<-9, kNotH>(D, e) & tm, std::integral_constant<int, 5>{});
  slide(ray_attacks<7, kNotH>(D, e) & tm, std::integral_constant<int, 6>{});
  slide(ray_attacks<-7, kNotA>(D, e) & tm, std::integral_constant<int, 7>{});
  if (!a.checkers) {
    u64 pins = a.pinned;
    while (pins) {
      const int s = lsb(pins);
      pins &= pins - 1;
      const u64 line = line_through(a.ksq, s);
      const u64 bit = 1ull << s;
      if (bit & f.P) {
        const u64 q1 = sh<FD::F>(bit) & f.empty;
        u64 t = (q1 | (sh<FD::F>(q1 & FD::ROW_AFTER1) & f.empty) | (pawn_attacks<STM>(bit) & f.them)) & line;
        while (t) {
          const int to = lsb(t);
          t &= t - 1;
          if ((1ull << to) & FD::LAST) {
            for (int pr = 1; pr <= 4; ++pr) visit(s, to, pr);
          } else {
            visit(s, to, 0);
          }
        }
      } else if (bit & (f.O | f.D)) {
        const Lines ls = lines_of(s);
        const bool orth_line = (line == ls.file) || (line == ls.rank);
        if ((orth_line && (bit & f.O)) || (!orth_line && (bit & f.D))) emit(s, line_attacks(s, line, f.occ) & notus);
      }
    }
  }
  const int ep = meta_ep(meta);
  if (ep >= 0) {
    u64 cand = pawn_attacks<1 - STM>(1ull << ep) & f.P;
    while (cand) {
      const int s = lsb(cand);
      cand &= cand - 1;
      if (ep_legal<STM>(f, a.ksq, s, ep, ep - FD::F)) visit(s, ep, 0);
    }
  }
}

// ------------------------------------------- simple children (final stage)
// For a parent P (side STM to move, opponent THEM), a legal STM move f -> t is
// *simple* when it is quiet (t empty; no promotion, castling, en passant or
// double push), STM is not in check, and neither square is in a set where a
// change of occupancy or of STM's attacks could change THEM's legal moves:
//   all      THEM's king zone Z' (king, neighbours, back-rank castling squares
//            while THEM has a right), THEM's slider rays and pawn push /
//            double-push / capture squares, the squares between Z' and an STM
//            slider attacking it, and the pin segments from THEM's king (king
//            -> THEM piece -> up to the next piece)
//   fsrc     (f only) a first piece seen from Z' with an STM slider of the
//            line's kind behind it (moving it uncovers an attack), and an STM
//            piece first on a line from THEM's king with a THEM piece second
//            (moving it can pin that piece)
//   t_orth / t_diag  (t only, rook/queen and bishop/queen movers) the open
//            lines of sight from Z'
//   lk/ln/lp (king/knight/pawn movers) squares from which such a piece hits Z'
// The child's THEM count then equals c0 = THEM's legal moves in P with THEM
// to move and no en-passant square.  Pinned with the oracle on random
// descendants of the published suite positions (tools/fide_simple_proto.py:
// 0 mismatches, 47 % of the children of startpos ply-5 parents simple);
// the GPU tests pin the kernel through the published perft tables.
struct Sens {
  u64 all, fsrc, t_orth, t_diag, lk, ln, lp;
};

template <int S, u64 M, int SO, u64 MO>
__device__ __forceinline__ void sens_dir(u64 zp, u64 e_nk, u64 occ_nk, u64 st, u64& all, u64& fsrc, u64& tt) {
  const u64 fd = ray_attacks<S, M>(zp, e_nk);   // seen from Z' toward S (first piece included)
  const u64 rd = ray_attacks<SO, MO>(st, e_nk);  // STM sliders of the kind, looking back
  const u64 b1 = fd & occ_nk;
  tt |= fd & e_nk;
  all |= (fd & rd & e_nk) | (b1 & st);
  fsrc |= b1 & rd;
}

// From THEM's king along direction D (scan_dir's numbering): when the first
// piece is THEM's, the squares up to and including the second piece (the
// first excluded): a change there can make or break a pin.  When the first
// piece is STM's and the second THEM's, moving the first can pin the second
// (a slider behind it): the first goes into fsrc.
template <int D>
__device__ __forceinline__ u64 pin_seg(const Lines& l, int ksq, u64 occ, u64 them, u64& fsrc) {
  constexpr bool UP = (D & 1) == 0;
  const u64 line = (D < 2) ? l.file : (D < 4) ? l.rank : (D < 6) ? l.diag : l.anti;
  const u64 ray = line & (UP ? above_mask(ksq) : below_mask(ksq));
  const u64 blk = occ & ray;
  const u64 m1 = UP ? (blk & (0ull - blk)) : (blk ? (1ull << msb(blk)) : 0ull);
  const u64 rest = blk & ~m1;
  const u64 m2 = UP ? (rest & (0ull - rest)) : (rest ? (1ull << msb(rest)) : 0ull);
  const u64 upto = UP ? (m2 ? ((m2 << 1) - 1) : ~0ull) : (m2 ? ~(m2 - 1) : ~0ull);  // m2 = bit 63: (0 - 1) = all
  fsrc |= (m2 & them) ? (m1 & ~them) : 0ull;
  return (m1 & them) ? (ray & upto & ~m1) : 0ull;
}

template <int STM>
__device__ __forceinline__ Sens fide_sens(const Board& b, u32 meta) {
  constexpr int THEM = 1 - STM;
  typedef FDir<THEM> TD;
  const FPos<STM> f = fpos<STM>(b);
  Sens s{~0ull, 0, 0, 0, 0, 0, 0};  // all = every square: no child simple
  if (!f.tK || (f.tK & (f.tK - 1)) || !f.K || (f.K & (f.K - 1))) return s;
  const u64 ro = orth_attacks(f.tO, f.empty) | diag_attacks(f.tD, f.empty);
  if ((ro & f.K) || (pawn_attacks<STM>(f.K) & f.tP) || (knight_attacks(f.K) & f.tN)) return s;  // STM in check
  const u64 push = sh<TD::F>(f.tP);
  const u32 rights = meta & (THEM ? (CR_BK | CR_BQ) : (CR_WK | CR_WQ));
  const u64 zp = f.tK | king_attacks(f.tK) | (rights ? (THEM ? (0x7Eull << 56) : 0x7Eull) : 0ull);
  u64 all = ro | push | sh<TD::F>(push & TD::ROW_AFTER1) | pawn_attacks<THEM>(f.tP) | zp;
  const u64 occ_nk = f.occ & ~f.tK, e_nk = ~occ_nk;
  u64 fsrc = 0, to = 0, td = 0;
  sens_dir<8, kAll, -8, kAll>(zp, e_nk, occ_nk, f.O, all, fsrc, to);
  sens_dir<-8, kAll, 8, kAll>(zp, e_nk, occ_nk, f.O, all, fsrc, to);
  sens_dir<1, kNotA, -1, kNotH>(zp, e_nk, occ_nk, f.O, all, fsrc, to);
  sens_dir<-1, kNotH, 1, kNotA>(zp, e_nk, occ_nk, f.O, all, fsrc, to);
  sens_dir<9, kNotA, -9, kNotH>(zp, e_nk, occ_nk, f.D, all, fsrc, td);
  sens_dir<-9, kNotH, 9, kNotA>(zp, e_nk, occ_nk, f.D, all, fsrc, td);
  sens_dir<7, kNotH, -7, kNotA>(zp, e_nk, occ_nk, f.D, all, fsrc, td);
  sens_dir<-7, kNotA, 7, kNotH>(zp, e_nk, occ_nk, f.D, all, fsrc, td);
  const int ksq = lsb(f.tK);
  const Lines l = lines_of(ksq);
  all |= pin_seg<0>(l, ksq, f.occ, f.them, fsrc) | pin_seg<1>(l, ksq, f.occ, f.them, fsrc) |
         pin_seg<2>(l, ksq, f.occ, f.them, fsrc) | pin_seg<3>(l, ksq, f.occ, f.them, fsrc) |
         pin_seg<4>(l, ksq, f.occ, f.them, fsrc) | pin_seg<5>(l, ksq, f.occ, f.them, fsrc) |
         pin_seg<6>(l, ksq, f.occ, f.them, fsrc) | pin_seg<7>(l, ksq, f.occ, f.them, fsrc);
  s.all = all;
  s.fsrc = fsrc;
  s.t_orth = to;
  s.t_diag = td;
  s.lk = king_attacks(zp);
  s.ln = knight_attacks(zp);
  s.lp = pawn_attacks<THEM>(zp);  // an STM pawn there attacks Z'
  return s;
}

// fide_for_each_move restricted to the children that are not simple (same
// order as fide_for_each_move with the simple ones left out); returns the
// number of simple children.  `sn(k)` reads one of the sets below, made by
// sens_masks from a Sens: the final stage keeps them in LDS and reads them
// where they are used, so they hold no registers across the enumeration loops.
enum : int {
  SN_ALL = 0,  // all
  SN_SRC,      // all | fsrc (f of any mover)
  SN_TORTH,    // all | t_orth (t of a rook/queen mover)
  SN_TDIAG,    // all | t_diag (t of a bishop/queen mover)
  SN_LK, SN_LN, SN_LP,
  SN_COUNT
};
__device__ __forceinline__ void sens_masks(const Sens& s, u64 (&m)[SN_COUNT]) {
  m[SN_ALL] = s.all;
  m[SN_SRC] = s.all | s.fsrc;
  m[SN_TORTH] = s.all | s.t_orth;
  m[SN_TDIAG] = s.all | s.t_diag;
  m[SN_LK] = s.lk;
  m[SN_LN] = s.ln;
  m[SN_LP] = s.lp;
}
template <int STM, class SensAt, class Visit>
__device__ __forceinline__ u32 fide_for_each_split(const Board& b, u32 meta, SensAt&& sn, Visit&& visit) {
  typedef FDir<STM> FD;
  const FPos<STM> f = fpos<STM>(b);
  const Analysis a = analyse<STM>(f, DC_FIDE_LAZY_DANGER < 2 || wave_needs_danger<STM>(f, meta));
  const u64 notus = ~f.us;
  u32 ns = 0;
  auto emit = [&](int from, u64 targets) {
    while (targets) {
      const int t = lsb(targets);
      targets &= targets - 1;
      visit(from, t, 0);
    }
  };
  auto emit_pawn = [&](u64 targets, int delta) {
    while (targets) {
      const int t = lsb(targets);
      targets &= targets - 1;
      if ((1ull << t) & FD::LAST) {
        for (int pr = 1; pr <= 4; ++pr) visit(t - delta, t, pr);
      } else {
        visit(t - delta, t, 0);
      }
    }
  };
  if (a.ksq >= 0) {
    const u64 kt = king_attacks(f.K) & notus & ~a.danger;
    const u64 ks = (f.K & (sn(SN_SRC) | sn(SN_LK))) ? 0ull : and_andn(kt, f.empty, sn(SN_ALL) | sn(SN_LK));
    ns += pc(ks);
    emit(a.ksq, (kt & ~ks) | castle_targets<STM>(f, a, meta, b));
  }
  if (a.checkers & (a.checkers - 1)) return ns;
  const u64 tm = notus & a.cmask;
  const u64 Pf = f.P & ~a.pinned;
  const u64 push1 = sh<FD::F>(Pf) & f.empty;
  // (in check, the `all` set is every square: nothing below is simple)
  const u64 ps = sh<FD::F>(Pf & ~(sn(SN_SRC) | sn(SN_LP))) & f.empty & ~(sn(SN_ALL) | sn(SN_LP) | FD::LAST);
  ns += pc(ps);
  emit_pawn((push1 & a.cmask) & ~ps, FD::F);
  emit_pawn(sh<FD::F>(push1 & FD::ROW_AFTER1) & f.empty & a.cmask, 2 * FD::F);
  emit_pawn(sh<FD::CW>(Pf & kNotA) & f.them & a.cmask, FD::CW);
  emit_pawn(sh<FD::CE>(Pf & kNotH) & f.them & a.cmask, FD::CE);
  const u64 n = f.N & ~a.pinned;
  const u64 nsrc = n & ~(sn(SN_SRC) | sn(SN_LN)), nt = f.empty & ~(sn(SN_ALL) | sn(SN_LN));
  auto leap = [&](u64 targets, u64 simple, int delta) {
    ns += pc(simple);
    targets &= ~simple;
    while (targets) {
      const int t = lsb(targets);
      targets &= targets - 1;
      visit(t - delta, t, 0);
    }
  };
  leap(sh<17>(n & kNotH) & tm, sh<17>(nsrc & kNotH) & nt, 17);
  leap(sh<15>(n & kNotA) & tm, sh<15>(nsrc & kNotA) & nt, 15);
  leap(sh<10>(n & kNotGH) & tm, sh<10>(nsrc & kNotGH) & nt, 10);
  leap(sh<6>(n & kNotAB) & tm, sh<6>(nsrc & kNotAB) & nt, 6);
  leap(sh<-6>(n & kNotGH) & tm, sh<-6>(nsrc & kNotGH) & nt, -6);
  leap(sh<-10>(n & kNotAB) & tm, sh<-10>(nsrc & kNotAB) & nt, -10);
  leap(sh<-15>(n & kNotH) & tm, sh<-15>(nsrc & kNotH) & nt, -15);
  leap(sh<-17>(n & kNotA) & tm, sh<-17>(nsrc & kNotA) & nt, -17);
  const u64 e = f.empty, O = f.O & ~a.pinned, D = f.D & ~a.pinned;
  auto slide = [&](u64 targets, auto dtag) {
    constexpr int DD = decltype(dtag)::value;
    while (targets) {
      const int t = lsb(targets);
      targets &= targets - 1;
      const int src = slider_source<DD, false>(f.occ, t);
      // a rook/bishop mover is tested against its own line kind, a queen
      // against both; captures are never simple
      const bool q = ((f.O & f.D) >> src) & 1;
      u32 bad = (u32)(f.occ >> t) | (u32)(sn(SN_SRC) >> src) | (u32)(sn(DD < 4 ? SN_TORTH : SN_TDIAG) >> t);
      if (q) bad |= (u32)(sn(DD < 4 ? SN_TDIAG : SN_TORTH) >> t);
      // ns updated unconditionally: `else ++ns` let the compiler merge the two
      // counter updates of the counting pass (the visitor's and ns) into one
      // through a selected address, which kept both in scratch memory
      ns += (bad & 1) ^ 1u;
      if (bad & 1) visit(src, t, 0);
    }
  };
  slide(ray_attacks<8, kAll>(O, e) & tm, std::integral_constant<int, 0>{});
  slide(ray_attacks<-8, kAll>(O, e) & tm, std::integral_constant<int, 1>{});
  slide(ray_attacks<1, kNotA>(O, e) & tm, std::integral_constant<int, 2>{});
  slide(ray_attacks<-1, kNotH>(O, e) & tm, std::integral_constant<int, 3>{});
  slide(ray_attacks<9, kNotA>(D, e) & tm, std::integral_constant<int, 4>{});
  slide(ray_attacks<-9, kNotH>(D, e) & tm, std::integral_constant<int, 5>{});
  slide(ray_attacks<7, kNotH>(D, e) & tm, std::integral_constant<int, 6>{});
  slide(ray_attacks<-7, kNotA>(D, e) & tm, std::integral_constant<int, 7>{});
  if (!a.checkers) {
    u64 pins = a.pinned;
    while (pins) {
      const int s = lsb(pins);
      pins &= pins - 1;
      const u64 line = line_through(a.ksq, s);
      const u64 bit = 1ull << s;
      if (bit & f.P) {
        const u64 q1 = sh<FD::F>(bit) & f.empty;
        u64 t = (q1 | (sh<FD::F>(q1 & FD::ROW_AFTER1) & f.empty) | (pawn_attacks<STM>(bit) & f.them)) & line;
        while (t) {
          const int to = lsb(t);
          t &= t - 1;
          if ((1ull << to) & FD::LAST) {
            for (int pr = 1; pr <= 4; ++pr) visit(s, to, pr);
          } else {
            visit(s, to, 0);
          }
        }
      } else if (bit & (f.O | f.D)) {
        const Lines ls = lines_of(s);
        const bool orth_line = (line == ls.file) || (line == ls.rank);
        if ((orth_line && (bit & f.O)) || (!orth_line && (bit & f.D))) emit(s, line_attacks(s, line, f.occ) & notus);
      }
    }
  }
  const int ep = meta_ep(meta);
  if (ep >= 0) {
    u64 cand = pawn_attacks<1 - STM>(1ull << ep) & f.P;
    while (cand) {
      const int s = lsb(cand);
      cand &= cand - 1;
      if (ep_legal<STM>(f, a.ksq, s, ep, ep - FD::F)) visit(s, ep, 0);
    }
  }
  return ns;
}

// The counting pass of the split without enumerating: fide_for_each_split's
// visits (returned) and its simple children (ns), set-wise -- the same
// classification, so the slot offsets it yields match the enumeration that
// fills them.  Sliders: the targets of sources off SN_SRC come from fills of
// those sources alone (the others still block: they stay occupied), rooks and
// bishops tested against their line kind's target set, queens against both.
template <int STM, class SensAt>
__device__ __forceinline__ u32 fide_count_split(const Board& b, u32 meta, SensAt&& sn, u32& ns_out) {
  typedef FDir<STM> FD;
  const FPos<STM> f = fpos<STM>(b);
  const Analysis a = analyse<STM>(f, DC_FIDE_LAZY_DANGER < 2 || wave_needs_danger<STM>(f, meta));
  const u64 notus = ~f.us;
  u32 c = 0, ns = 0;
  if (a.ksq >= 0) {
    const u64 kt = king_attacks(f.K) & notus & ~a.danger;
    const u64 ks = (f.K & (sn(SN_SRC) | sn(SN_LK))) ? 0ull : and_andn(kt, f.empty, sn(SN_ALL) | sn(SN_LK));
    ns += pc(ks);
    c += pc(kt & ~ks) + pc(castle_targets<STM>(f, a, meta, b));
  }
  if (a.checkers & (a.checkers - 1)) {
    ns_out = ns;
    return c;
  }
  const u64 tm = notus & a.cmask;
  const u64 Pf = f.P & ~a.pinned;
  const u64 push1 = sh<FD::F>(Pf) & f.empty;
  const u64 ps = sh<FD::F>(Pf & ~(sn(SN_SRC) | sn(SN_LP))) & f.empty & ~(sn(SN_ALL) | sn(SN_LP) | FD::LAST);
  const u64 p1 = push1 & a.cmask & ~ps;
  const u64 push2 = sh<FD::F>(push1 & FD::ROW_AFTER1) & f.empty & a.cmask;
  const u64 cw = sh<FD::CW>(Pf & kNotA) & f.them & a.cmask;
  const u64 ce = sh<FD::CE>(Pf & kNotH) & f.them & a.cmask;
  ns += pc(ps);
  c += pc(p1) + pc(push2) + pc(cw) + pc(ce) + 3 * (pc(p1 & FD::LAST) + pc(cw & FD::LAST) + pc(ce & FD::LAST));
  const u64 n = f.N & ~a.pinned;
  const u64 nsrc = n & ~(sn(SN_SRC) | sn(SN_LN)), nt = f.empty & ~(sn(SN_ALL) | sn(SN_LN));
  auto leap = [&](u64 targets, u64 simple) {
    ns += pc(simple);
    c += pc(targets & ~simple);
  };
  leap(sh<17>(n & kNotH) & tm, sh<17>(nsrc & kNotH) & nt);
  leap(sh<15>(n & kNotA) & tm, sh<15>(nsrc & kNotA) & nt);
  leap(sh<10>(n & kNotGH) & tm, sh<10>(nsrc & kNotGH) & nt);
  leap(sh<6>(n & kNotAB) & tm, sh<6>(nsrc & kNotAB) & nt);
  leap(sh<-6>(n & kNotGH) & tm, sh<-6>(nsrc & kNotGH) & nt);
  leap(sh<-10>(n & kNotAB) & tm, sh<-10>(nsrc & kNotAB) & nt);
  leap(sh<-15>(n & kNotH) & tm, sh<-15>(nsrc & kNotH) & nt);
  leap(sh<-17>(n & kNotA) & tm, sh<-17>(nsrc & kNotA) & nt);
  const u64 e = f.empty, O = f.O & ~a.pinned, D = f.D & ~a.pinned;
  const u64 q = O & D, qs = q & ~sn(SN_SRC);
  const u64 rs = O & ~q & ~sn(SN_SRC), bs = D & ~q & ~sn(SN_SRC);
  const u64 qt = ~(sn(SN_TORTH) | sn(SN_TDIAG)) & e;
  const u64 ot = ~sn(SN_TORTH) & e, dt = ~sn(SN_TDIAG) & e;
  auto slide = [&](u64 all_t, u64 simple) {
    ns += pc(simple);
    c += pc(all_t & ~simple);
  };
  slide(ray_attacks<8, kAll>(O, e) & tm, (ray_attacks<8, kAll>(rs, e) & ot) | (ray_attacks<8, kAll>(qs, e) & qt));
  slide(ray_attacks<-8, kAll>(O, e) & tm, (ray_attacks<-8, kAll>(rs, e) & ot) | (ray_attacks<-8, kAll>(qs, e) & qt));
  slide(ray_attacks<1, kNotA>(O, e) & tm, (ray_attacks<1, kNotA>(rs, e) & ot) | (ray_attacks<1, kNotA>(qs, e) & qt));
  slide(ray_attacks<-1, kNotH>(O, e) & tm, (ray_attacks<-1, kNotH>(rs, e) & ot) | (ray_attacks<-1, kNotH>(qs, e) & qt));
  slide(ray_attacks<9, kNotA>(D, e) & tm, (ray_attacks<9, kNotA>(bs, e) & dt) | (ray_attacks<9, kNotA>(qs, e) & qt));
  slide(ray_attacks<-9, kNotH>(D, e) & tm, (ray_attacks<-9, kNotH>(bs, e) & dt) | (ray_attacks<-9, kNotH>(qs, e) & qt));
  slide(ray_attacks<7, kNotH>(D, e) & tm, (ray_attacks<7, kNotH>(bs, e) & dt) | (ray_attacks<7, kNotH>(qs, e) & qt));
  slide(ray_attacks<-7, kNotA>(D, e) & tm, (ray_attacks<-7, kNotA>(bs, e) & dt) | (ray_attacks<-7, kNotA>(qs, e) & qt));
  if (!a.checkers) {
    u64 pins = a.pinned;
    while (pins) {
      const int s = lsb(pins);
      pins &= pins - 1;
      const u64 line = line_through(a.ksq, s);
      const u64 bit = 1ull << s;
      if (bit & f.P) {
        const u64 q1 = sh<FD::F>(bit) & f.empty;
        const u64 t = (q1 | (sh<FD::F>(q1 & FD::ROW_AFTER1) & f.empty) | (pawn_attacks<STM>(bit) & f.them)) & line;
        c += pc(t) + 3 * pc(t & FD::LAST);
      } else if (bit & (f.O | f.D)) {
        const Lines ls = lines_of(s);
        const bool orth_line = (line == ls.file) || (line == ls.rank);
        if ((orth_line && (bit & f.O)) || (!orth_line && (bit & f.D))) c += pc(line_attacks(s, line, f.occ) & notus);
      }
    }
  }
  const int ep = meta_ep(meta);
  if (ep >= 0) {
    u64 cand = pawn_attacks<1 - STM>(1ull << ep) & f.P;
    while (cand) {
      const int s = lsb(cand);
      cand &= cand - 1;
      c += ep_legal<STM>(f, a.ksq, s, ep, ep - FD::F) ? 1u : 0u;
    }
  }
  ns_out = ns;
  return c;
}

// Promotion piece -> kind code (1 N, 2 B, 3 R, 4 Q).
__device__ __forceinline__ u32 promo_code(int promo) {
  return promo == 1 ? KC_N : promo == 2 ? KC_B : promo == 3 ? KC_R : KC_Q;
}

__device__ __forceinline__ u32 castle_clear(int s) {
  return s == 0 ? CR_WQ : s == 4 ? (CR_WK | CR_WQ) : s == 7 ? CR_WK : s == 56 ? CR_BQ : s == 60 ? (CR_BK | CR_BQ)
       : s == 63 ? CR_BK : 0u;
}

__device__ __forceinline__ void clear_sq(Board& b, int s) {
  const u64 k = ~(1ull << s);
  b.b0 &= k;
  b.b1 &= k;
  b.b2 &= k;
  b.b3 &= k;
}

// Makes a legal move; returns the new meta.
template <int STM>
__device__ __forceinline__ u32 fide_make(Board& b, u32 meta, int f, int t, int promo) {
  typedef FDir<STM> FD;
  const u32 kind = nibble(b, f) >> 1;
  const int ep = meta_ep(meta);
  ref_make(b, f, t);
  if (kind == KC_P) {
    if (t == ep) clear_sq(b, t - FD::F);
    if (promo) {
      const u32 code = promo_code(promo);
      const u64 m = 1ull << t;
      b.b1 = (b.b1 & ~m) | ((code & 1) ? m : 0);
      b.b2 = (b.b2 & ~m) | ((code & 2) ? m : 0);
      b.b3 = (b.b3 & ~m) | ((code & 4) ? m : 0);
    }
  } else if (kind == KC_K && (t - f == 2 || f - t == 2)) {
    if (t > f) ref_make(b, f + 3, f + 1);
    else ref_make(b, f - 4, f - 1);
  }
  u32 rights = (meta & 15) & ~(castle_clear(f) | castle_clear(t));
  u32 nep = 0;
  if (kind == KC_P && (t - f == 16 || f - t == 16)) nep = META_EP_VALID | ((u32)((f + t) >> 1) << 4);
  return rights | nep;
}

// Legal target set of the piece on s (for validation and the canonical-order
// generator).  Promotion multiplicity is applied by the caller.
template <int STM>
__device__ __forceinline__ u64 fide_piece_targets(const Board& b, u32 meta, const FPos<STM>& f, const Analysis& a, int s) {
  typedef FDir<STM> FD;
  const u64 bit = 1ull << s;
  const u64 notus = ~f.us;
  if (bit & f.K) {
    if (s != a.ksq) return 0;  // extra kings (not reachable under FIDE) never move
    return (king_attacks(bit) & notus & ~a.danger) | castle_targets<STM>(f, a, meta, b);
  }
  if (a.checkers & (a.checkers - 1)) return 0;
  if (a.pinned & bit && a.checkers) return 0;
  u64 t;
  if (bit & f.P) {
    const u64 q1 = sh<FD::F>(bit) & f.empty;
    t = (q1 | (sh<FD::F>(q1 & FD::ROW_AFTER1) & f.empty) | (pawn_attacks<STM>(bit) & f.them)) & a.cmask;
  } else if (bit & f.N) {
    t = knight_attacks(bit) & notus & a.cmask;
  } else if (bit & (f.O | f.D)) {
    const Lines l = lines_of(s);
    t = 0;
    if (bit & f.O) t |= line_attacks(s, l.file, f.occ) | line_attacks(s, l.rank, f.occ);
    if (bit & f.D) t |= line_attacks(s, l.diag, f.occ) | line_attacks(s, l.anti, f.occ);
    t &= notus & a.cmask;
  } else {
    return 0;  // unknown kind: never moves
  }
  if (a.pinned & bit) t &= line_through(a.ksq, s);
  if (bit & f.P) {
    const int ep = meta_ep(meta);
    if (ep >= 0 && (pawn_attacks<STM>(bit) & (1ull << ep)) && ep_legal<STM>(f, a.ksq, s, ep, ep - FD::F))
      t |= 1ull << ep;
  }
  return t;
}

// validate_move under FIDE rules.  Same verdict order as REF; a promotion move
// must name its piece (promo 1..4) and any other move must have promo 0.
template <int STM>
__device__ __forceinline__ u32 fide_verdict_stm(const Board& b, u32 meta, u32 m) {
  typedef FDir<STM> FD;
  const int s = (int)(m & 63), t = (int)((m >> 6) & 63);
  const u32 promo = (m >> 12) & 7;
  const FPos<STM> f = fpos<STM>(b);
  const Analysis a = analyse<STM>(f);
  const u64 targets = fide_piece_targets<STM>(b, meta, f, a, s);
  if (!((targets >> t) & 1)) return V_ILLEGAL;
  const bool is_promo = ((1ull << s) & f.P) && ((1ull << t) & FD::LAST);
  if (is_promo ? (promo < 1 || promo > 4) : (promo != 0)) return V_ILLEGAL;
  return V_OK;
}

__device__ __forceinline__ u32 fide_verdict(const Board& b, u32 stm, u32 meta, u32 m) {
  if (m & 0x8000u) return V_OOR;
  const u32 nib = nibble(b, (int)(m & 63));
  if ((nib >> 1) == 0) return V_NO_PIECE;
  if ((nib & 1) != stm) return V_WRONG_TURN;
  return stm ? fide_verdict_stm<1>(b, meta, m) : fide_verdict_stm<0>(b, meta, m);
}

__device__ __forceinline__ u32 fide_count_rt(const Board& b, u32 stm, u32 meta) {
  return stm ? fide_count<1>(b, meta) : fide_count<0>(b, meta);
}

__device__ __forceinline__ u32 fide_make_rt(Board& b, u32 stm, u32 meta, int f, int t, int promo) {
  return stm ? fide_make<1>(b, meta, f, t, promo) : fide_make<0>(b, meta, f, t, promo);
}

// k-th legal move in (from, to, promo) order.
template <int STM>
__device__ __forceinline__ u32 fide_kth_move_stm(const Board& b, u32 meta, u32 k) {
  typedef FDir<STM> FD;
  const FPos<STM> f = fpos<STM>(b);
  const Analysis a = analyse<STM>(f);
  u64 own = f.us;
  while (own) {
    const int s = lsb(own);
    own &= own - 1;
    u64 t = fide_piece_targets<STM>(b, meta, f, a, s);
    const bool pawn = ((1ull << s) & f.P) != 0;
    while (t) {
      const int to = lsb(t);
      t &= t - 1;
      const u32 mult = (pawn && ((1ull << to) & FD::LAST)) ? 4u : 1u;
      if (k < mult) return (u32)s | ((u32)to << 6) | ((mult == 4 ? k + 1 : 0u) << 12);
      k -= mult;
    }
  }
  return 0xFFFFu;
}

__device__ __forceinline__ u32 fide_kth_move(const Board& b, u32 stm, u32 meta, u32 k) {
  return stm ? fide_kth_move_stm<1>(b, meta, k) : fide_kth_move_stm<0>(b, meta, k);
}

}  // namespace dc
