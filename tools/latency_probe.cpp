// latency_probe.cpp -- the live consensus call timed at the C ABI, the way the
// Rust host would make it: dc_validate_batch with n = 1 on a
// host dc_pos and move, timed with steady_clock per call, on the launched
// path and with dc_live_validator.  No Python between the clock and the ABI.
//   build: g++ -O2 -std=c++17 tools/latency_probe.cpp -Iinclude -Ldistributed-chess_amd -ldchess
//          -Wl,-rpath,$ORIGIN/../distributed-chess_amd -o tools/latency_probe
//   run:   tools/latency_probe [calls]   -> one JSON line
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../include/dchess.h"

struct Stats {
  double median, p99, min;
};

static Stats run(dc_ctx* c, int calls, const dc_pos& p, uint16_t mv, bool* ok) {
  std::vector<double> t(calls);
  uint8_t v = 0xFF;
  for (int i = 0; i < 200; ++i) dc_validate_batch(c, DC_RULES_REF, &p, &mv, 1, &v);
  for (int i = 0; i < calls; ++i) {
    const auto t0 = std::chrono::steady_clock::now();
    const int r = dc_validate_batch(c, DC_RULES_REF, &p, &mv, 1, &v);
    const auto t1 = std::chrono::steady_clock::now();
    if (r != DC_SUCCESS || v != DC_V_OK) *ok = false;
    t[i] = std::chrono::duration<double, std::micro>(t1 - t0).count();
  }
  std::sort(t.begin(), t.end());
  return Stats{t[calls / 2], t[(size_t)(calls * 0.99)], t[0]};
}

int main(int argc, char** argv) {
  const int calls = argc > 1 ? std::atoi(argv[1]) : 5000;
  dc_ctx* c = nullptr;
  if (dc_ctx_create(0, &c) != DC_SUCCESS) {
    std::printf("{\"error\": \"dc_ctx_create\"}\n");
    return 1;
  }
  dc_pos p;
  dc_startpos(&p);
  const uint16_t mv = dc_move_pack(1, 4, 3, 4);  // e2e4
  bool ok = true;
  const Stats a = run(c, calls, p, mv, &ok);
  dc_live_validator(c, 1000000);
  const Stats b = run(c, calls, p, mv, &ok);
  dc_live_validator(c, 0);
  dc_ctx_destroy(c);
  std::printf(
      "{\"calls\": %d, \"parity\": %s, \"launched\": {\"median_us\": %.3f, \"p99_us\": %.3f, \"min_us\": %.3f}, "
      "\"live\": {\"median_us\": %.3f, \"p99_us\": %.3f, \"min_us\": %.3f}}\n",
      calls, ok ? "true" : "false", a.median, a.p99, a.min, b.median, b.p99, b.min);
  return ok ? 0 : 2;
}
