// test_secp.cpp -- host build of dc_secp.h / dc_txsig.h (the exact code the
// gfx950 kernel k_verify_tx runs) driven line by line from stdin, so
// tests/test_txsig.py can check field, scalar, point and whole-transaction
// results against oracle/txsig.py without a GPU.  Test infrastructure only.
//
// Commands (numbers: 64 hex digits, big-endian; strings: hex of their bytes,
// "-" for the empty string):
//   fe_mul A B | fe_sqr A | fe_add A B | fe_sub A B | fe_inv A | fe_sqrt A
//   sc_mul A B | sc_inv A | mulg K | mulq K QX QY | hash W B FX FY TX TY
//   tx W B FX FY TX TY SIG PK TURN
//   timed R   then tx lines, then "end": the G table is built first, then the
//             parsed transactions are checked R times under a steady_clock;
//             prints the verdicts of one pass and "ns <elapsed of all passes>"
//             (bench.py's cpu_baseline of the signature leg)
#include <chrono>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "../../distributed-chess_amd/csrc/dc_txsig.h"

using namespace dc::secp;

static void rd(u32 (&r)[8], const std::string& h) {
  std::string s = std::string(64 - h.size(), '0') + h;
  hex_limbs(r, s.c_str());
}
static std::string wr(const u32 (&a)[8]) {
  char b[65];
  for (int i = 0; i < 8; ++i) snprintf(b + 8 * i, 9, "%08x", a[7 - i]);
  return std::string(b, 64);
}
static std::string unhex(const std::string& h) {
  if (h == "-") return "";
  std::string o;
  for (size_t i = 0; i + 1 < h.size(); i += 2) o.push_back((char)std::stoi(h.substr(i, 2), nullptr, 16));
  return o;
}

static std::vector<Ge>& gtab() {
  static std::vector<Ge> t;
  if (t.empty()) {
    t.resize(kGTabEntries);
    for (int i = 0; i < kGTabRows; ++i)
      for (int j = 0; j < 256; ++j) gtab_entry(t[256 * i + j], i, j);
  }
  return t;
}

struct TxIn {
  std::string w, b, sig, pk;
  u32 act[4];
  int turn;
};

static TxIn parse_tx(std::istringstream& in) {
  TxIn t;
  t.turn = -1;
  in >> t.w >> t.b >> t.act[0] >> t.act[1] >> t.act[2] >> t.act[3] >> t.sig >> t.pk >> t.turn;
  t.w = unhex(t.w);
  t.b = unhex(t.b);
  t.sig = unhex(t.sig);
  t.pk = unhex(t.pk);
  return t;
}

static u32 run_tx(const TxIn& t) {
  uint8_t blk[64];
  return check_tx(t.w.data(), (u32)t.w.size(), t.b.data(), (u32)t.b.size(), t.act, t.sig.data(), (u32)t.sig.size(),
                  t.pk.data(), (u32)t.pk.size(), t.turn, gtab().data(), BlkRef{blk, 4});
}

// "timed R": only the verify loop is inside the clock (no process start-up,
// no G-table build, no parsing)
static void timed(int reps) {
  std::vector<TxIn> txs;
  std::string line;
  while (std::getline(std::cin, line)) {
    std::istringstream in(line);
    std::string op;
    in >> op;
    if (op == "end") break;
    if (op == "tx") txs.push_back(parse_tx(in));
  }
  gtab();
  std::vector<u32> v(txs.size());
  u32 sink = 0;
  const auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < reps; ++r)
    for (size_t i = 0; i < txs.size(); ++i) {
      v[i] = run_tx(txs[i]);
      sink += v[i];
    }
  const auto t1 = std::chrono::steady_clock::now();
  for (u32 x : v) std::cout << x << "\n";
  std::cout << "ns " << std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count() << " " << (sink & 0)
            << "\n";
  std::cout.flush();
}

int main() {
  std::string line;
  while (std::getline(std::cin, line)) {
    std::istringstream in(line);
    std::string op;
    in >> op;
    if (op.empty()) continue;
    if (op == "timed") {
      int reps = 1;
      in >> reps;
      timed(reps);
      continue;
    }
    if (op.rfind("fe_", 0) == 0) {
      std::string a, b;
      in >> a >> b;
      Fe x, y, r;
      u32 t[8];
      rd(t, a);
      fe_canon(x, t);
      if (!b.empty()) {
        rd(t, b);
        fe_canon(y, t);
      }
      if (op == "fe_mul") fe_mul(r, x, y);
      else if (op == "fe_sqr") fe_sqr(r, x);
      else if (op == "fe_add") fe_add(r, x, y);
      else if (op == "fe_sub") fe_sub(r, x, y);
      else if (op == "fe_inv") fe_inv(r, x);
      else fe_pow_sqrt(r, x);
      std::cout << wr(r.v) << "\n";
    } else if (op.rfind("sc_", 0) == 0) {
      std::string a, b;
      in >> a >> b;
      Sc x, y, r;
      u32 t[8];
      rd(t, a);
      sc_canon(x, t);
      if (op == "sc_mul") {
        rd(t, b);
        sc_canon(y, t);
        sc_mul(r, x, y);
      } else {
        sc_inv(r, x);
      }
      std::cout << wr(r.v) << "\n";
    } else if (op == "mulg" || op == "mulq") {
      std::string k, qx, qy;
      in >> k >> qx >> qy;
      Sc s, zero;
      u32 t[8];
      rd(t, k);
      sc_canon(s, t);
      set_zero(zero.v);
      Ge q;
      Gej r;
      if (op == "mulg") {
        ge_generator(q);
        ecmult(r, q, zero, s, gtab().data());  // through the G table
      } else {
        rd(q.x.v, qx);
        rd(q.y.v, qy);
        ecmult(r, q, s, zero, gtab().data());  // through the windowed Q part
      }
      if (r.inf) {
        std::cout << "inf\n";
      } else {
        Ge a;
        gej_to_ge(a, r);
        std::cout << wr(a.x.v) << " " << wr(a.y.v) << "\n";
      }
    } else if (op == "hash" || op == "tx") {
      std::string w, b, sig, pk;
      u32 act[4];
      int turn = -1;
      in >> w >> b >> act[0] >> act[1] >> act[2] >> act[3];
      w = unhex(w);
      b = unhex(b);
      uint8_t blk[64];
      if (op == "hash") {
        u32 h[8];
        message_hash(h, w.data(), (u32)w.size(), b.data(), (u32)b.size(), act, BlkRef{blk, 4});
        for (int i = 0; i < 8; ++i) printf("%08x", h[i]);
        printf("\n");
        fflush(stdout);
        continue;
      }
      in >> sig >> pk >> turn;
      sig = unhex(sig);
      pk = unhex(pk);
      const u32 v = check_tx(w.data(), (u32)w.size(), b.data(), (u32)b.size(), act, sig.data(), (u32)sig.size(),
                             pk.data(), (u32)pk.size(), turn, gtab().data(), BlkRef{blk, 4});
      std::cout << v << "\n";
    } else {
      std::cout << "?\n";
    }
    std::cout.flush();
  }
  return 0;
}
