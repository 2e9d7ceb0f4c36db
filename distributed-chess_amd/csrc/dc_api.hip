// dc_api.hip -- implementation of include/dchess.h (host side of the engine).
//
// Owns the per-device context (stream, grow-only device buffers, HIP-event
// kernel timing) and drives the kernels of dc_kernels.hip.  No rule is ever
// evaluated on the host: every verdict, count and state update comes from a
// gfx950 kernel, and every entry point fails with DC_ENODEV when no device
// is usable -- there is no CPU fallback.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "../../include/dchess.h"
#include "dc_fide.h"
#include "dc_hash.h"
#include "dc_keccak.h"
#include "dc_kernels.h"
#include "dc_perft.h"
#include "dc_txsig_k.h"

using dc::Board;
using dc::DevPos;
using dc::u32;
using dc::u64;

static_assert(sizeof(dc_pos) == sizeof(DevPos), "dc_pos / DevPos layout");

// ------------------------------------------------------------------ buffers
// Bumped whenever any device buffer moves: captured perft graphs hold raw
// pointers and are re-captured after a bump.
static std::atomic<uint64_t> g_alloc_epoch{0};

// hipFree (and hipHostFree) wait for every stream of the device, a resident
// live-validator wave's included (dc_live_validator): a buffer grown or freed
// while any context's wave runs would block for that wave's lease (up to 60 s).
// LiveHold stops every resident wave of the process first and keeps new ones
// from starting while it is held (those calls take the launched path).
struct LiveHold {
  LiveHold();
  ~LiveHold();
};

template <class T>
struct DBuf {
  T* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t n) {
    if (n <= cap) return hipSuccess;
    LiveHold hold;
    g_alloc_epoch.fetch_add(1);
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(n, 64);
    want = want + want / 4;  // grow with headroom
    hipError_t e = hipMalloc(&p, want * sizeof(T));
    if (e != hipSuccess) {
      p = nullptr;
      return e;
    }
    cap = want;
    return hipSuccess;
  }
  void release() {
    if (p) {
      LiveHold hold;
      (void)hipFree(p);
    }
    p = nullptr;
    cap = 0;
  }
};

struct PendingEvent {
  std::string name;
  hipEvent_t a, b;
  u64 units;
};

struct KStat {
  u64 launches = 0;
  double ms = 0;
  u64 units = 0;
};

// Small validate / apply batches (the live consensus call is n = 1: one move
// per block, core/src/consensus/types.rs:10) are staged in one pinned host
// block that the kernel reads and writes in place: no DMA copies, one launch
// and one stream sync per call.  (Three pageable hipMemcpyAsync per call cost
// about 20 of its ~33 us, round 2.)
constexpr uint32_t kHostIoBatch = 4096;
struct HostIo {
  dc_pos pos[kHostIoBatch];
  uint16_t moves[kHostIoBatch];
  uint8_t verdicts[kHostIoBatch];
  uint8_t info[kHostIoBatch];
  uint32_t done;  // one-block launches (n <= 256): the kernel's completion flag (publish_done)
};
constexpr uint32_t kHostFlagBatch = 256;

struct dc_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool profiling = false;
  std::vector<hipEvent_t> event_pool;
  std::vector<PendingEvent> pending;
  std::map<std::string, KStat> stats;

  // perft frontier (ping-pong), top-level scratch and per-run control block
  DBuf<Board> nodes[2];
  DBuf<uint16_t> tags[2];
  DBuf<uint16_t> meta[2];  // FIDE castle/ep per node
  DBuf<Board> top_nodes;
  DBuf<uint16_t> top_tags, top_meta;
  DBuf<u32> counts, counts2;        // a level's move counts; counts2: the next level's,
  DBuf<u64> chunk_sum, chunk_sum2;  // made by the k_level_write that writes it
  DBuf<u64> chunk_base;
  DBuf<dc::PerftResult> res;
  DBuf<dc::Range> rng;
  DBuf<u64> desc;
  DBuf<u64> dfs_stack;  // K4 frames (dc_perft.hip k_perft_dfs)
  DBuf<Board> root;
  DBuf<uint16_t> root_meta;
  DBuf<dc::ResultCursor> rcur;  // dc_perft_repeat_device: where the next run's result goes
  dc::PerftResult* res_host = nullptr;  // pinned
  u64* replay_host = nullptr;            // pinned: the replay kernel's five counters
  u32* plain_host = nullptr;             // pinned: the state hash's names check (k_names_plain's flag)
  hipEvent_t plain_ev = nullptr;         // ... recorded after its readback
  struct HostIo* host_io = nullptr;      // pinned: small validate / apply batches, read and written in place
  uint32_t io_seq = 0;                   // last completion flag value published into host_io->done
  // dc_live_validator: the resident wave's mailbox (pinned, coherent), its
  // stream, the requests it has served and its lease (0: off)
  dc::LiveBox* live = nullptr;
  hipStream_t live_stream = nullptr;
  uint32_t live_seq = 0;
  uint32_t live_lease_us = 0;
  bool live_running = false;
  uint32_t live_timeout_us = 5000000;  // a call the wave neither answers nor leaves in this long is DC_EHIP
  std::mutex live_mu;  // the wave's state: held by live calls and by LiveHold's stop from another thread
  // The last perft launch sequence, captured as a hipGraph (see perft_run).
  struct PerftKey {
    u32 rules, depth, split, shard, n_shards, stm, k4;
    u32 n_root;  // root positions expanded together (dc_perft_batch; 1 otherwise)
    uint64_t epoch;
    // the capacities a captured graph was sized with (test knobs
    // DCHESS_PERFT_WIDE_MAX / _WIDE_LEVEL_MAX): a changed knob re-captures
    uint64_t wide_words, wide_level;
    bool front;  // the sequence is k_front + k_count3c
    bool operator==(const PerftKey& o) const {
      return rules == o.rules && depth == o.depth && split == o.split && shard == o.shard &&
             n_shards == o.n_shards && stm == o.stm && k4 == o.k4 && n_root == o.n_root && epoch == o.epoch &&
             wide_words == o.wide_words && wide_level == o.wide_level && front == o.front;
    }
  } pkey{};
  hipGraphExec_t pgraph = nullptr;
  // dc_perft_repeat_device's graph: the same sequence without the root upload
  // and the result readback (the root stays on the device between runs)
  hipGraphExec_t rgraph = nullptr;
  // ... and kRepeatBatch runs in one graph: consecutive graph launches leave
  // ~8.6 us between one graph's last kernel and the next graph's first
  // (rocprofv3 kernel trace, round 4), kernels within a graph none
  hipGraphExec_t rgraph_batch = nullptr;
  PerftKey rkey{};
  // the last perft_impl needed the exact (host-sized) rerun: its speculative
  // level capacities overflow, so dc_perft_repeat_device must not replay them
  bool last_exact = false;
  // the last perft_impl ran the one-launch front end (k_front); false when it
  // declined the position (the legacy chain ran) or was not eligible
  bool last_front = false;
  const char* last_final = "count2";  // timing name of the last perft's final stage
  struct RootStage {
    Board b[dc::kMaxPerftRoots];
    uint16_t meta[dc::kMaxPerftRoots];
    u32 n;
  }* root_host = nullptr;  // pinned
  // batch / replay scratch
  DBuf<DevPos> pos;
  DBuf<uint16_t> moves;
  DBuf<uint8_t> verdicts, info;
  DBuf<uint8_t> replay_info;  // dc_replay_info / the state hash's first pass: ply-major [n_plies][n_games] move info
  DBuf<Board> hash_boards;    // the state hash's first pass: every game's final board (round 6)
  DBuf<char> hash_text;    // escaped start history | escaped names of dc_state_hash*
  DBuf<u32> hash_off;      // the names' escaped offsets into hash_text
  DBuf<u32> esc_lens;      // device escaping scratch: per-name escaped lengths,
  DBuf<u64> esc64;         // their scan,
  DBuf<uint8_t> scan_tmp;  // the scan's temporary storage
  DBuf<char> names_raw;    // dc_state_hash (host buffers): the raw names staged
  DBuf<u32> names_raw_off;
  std::string hist_text;   // the escaped start history (host side of the H2D copy)
  DBuf<uint8_t> hashes;
  DBuf<u64> bitmap, digests, stats5;
  // the state hash's replay pre-pass is skipped past this many bytes of its
  // buffers (unlimited; dc_test_hash_prepass_max lowers it to test the fallback)
  u64 hash_prepass_max = ~0ull;
  // the hash kernel keeps move numbers as 32-bit BCD below this bound (at most
  // 10^7; dc_test_hash_bcd_max lowers it to test the division fallback)
  u32 hash_bcd_max = 10000000u;
  DBuf<u32> move_words;  // k_count3c: the final stage's parents as move words below their grandparents
  DBuf<u64> move_words64;  // ... as 64-bit words (REF perft(8): more than 2^20 grandparents)
  DBuf<dc::Range> slice_rng;  // the sliced final stage (REF perft(9)): one slice's node and word Ranges
  DBuf<u32> slice_ctr;        // ... and its group counter
  DBuf<u32> top_words;   // k_expand_top's last ply as move words (k_make_count makes it)
  DBuf<uint8_t> front_st;  // k_front's look-back slots, a dc::FrontState (zeroed once; k_count3c re-zeroes them)
  DBuf<u32> front_spill;   // k_front's spill rows (items past one LDS window)
  uint8_t* front_st_zeroed = nullptr;
  // transaction-signature check: staged strings / offsets / actions / turns,
  // and the G table (built on first use)
  DBuf<char> tx_text;
  DBuf<u32> tx_off, tx_act;
  DBuf<int8_t> tx_turn;
  DBuf<uint8_t> tx_verdicts;
  DBuf<dc::secp::Ge> gtab;
  bool gtab_ready = false;

  ~dc_ctx() {
    LiveHold hold;  // pinned host frees below wait for every stream too
    tx_text.release();
    tx_off.release();
    tx_act.release();
    tx_turn.release();
    tx_verdicts.release();
    gtab.release();
    for (auto* b : {&nodes[0], &nodes[1], &top_nodes, &root}) b->release();
    for (auto* b : {&tags[0], &tags[1], &meta[0], &meta[1], &top_tags, &top_meta, &root_meta, &moves}) b->release();
    counts.release();
    counts2.release();
    chunk_sum.release();
    chunk_sum2.release();
    chunk_base.release();
    res.release();
    rng.release();
    desc.release();
    top_words.release();
    front_st.release();
    front_spill.release();
    move_words.release();
    dfs_stack.release();
    move_words64.release();
    slice_rng.release();
    slice_ctr.release();
    if (pgraph) (void)hipGraphExecDestroy(pgraph);
    if (rgraph) (void)hipGraphExecDestroy(rgraph);
    if (rgraph_batch) (void)hipGraphExecDestroy(rgraph_batch);
    if (res_host) (void)hipHostFree(res_host);
    if (replay_host) (void)hipHostFree(replay_host);
    if (plain_host) (void)hipHostFree(plain_host);
    if (plain_ev) (void)hipEventDestroy(plain_ev);
    if (host_io) (void)hipHostFree(host_io);
    if (live) (void)hipHostFree(live);
    if (live_stream) (void)hipStreamDestroy(live_stream);
    if (root_host) (void)hipHostFree(root_host);
    pos.release();
    verdicts.release();
    info.release();
    replay_info.release();
    hash_boards.release();
    hash_text.release();
    hash_off.release();
    esc_lens.release();
    esc64.release();
    scan_tmp.release();
    names_raw.release();
    names_raw_off.release();
    hashes.release();
    bitmap.release();
    digests.release();
    stats5.release();
    move_words.release();
    for (auto& p : pending) {
      (void)hipEventDestroy(p.a);
      (void)hipEventDestroy(p.b);
    }
    for (auto e : event_pool) (void)hipEventDestroy(e);
    if (stream) (void)hipStreamDestroy(stream);
  }

  hipEvent_t take_event() {
    if (!event_pool.empty()) {
      hipEvent_t e = event_pool.back();
      event_pool.pop_back();
      return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
  }
  // Brackets one launch with events on the context stream when profiling.
  template <class F>
  hipError_t timed(const char* name, u64 units, F&& launch) {
    if (!profiling) return launch();
    PendingEvent pe{name, take_event(), take_event(), units};
    (void)hipEventRecord(pe.a, stream);
    hipError_t e = launch();
    (void)hipEventRecord(pe.b, stream);
    pending.push_back(pe);
    return e;
  }
  // After a stream sync: fold pending events into stats.
  void harvest() {
    for (auto& p : pending) {
      float ms = 0;
      (void)hipEventElapsedTime(&ms, p.a, p.b);
      KStat& s = stats[p.name];
      s.launches++;
      s.ms += ms;
      s.units += p.units;
      event_pool.push_back(p.a);
      event_pool.push_back(p.b);
    }
    pending.clear();
  }
};

#define HIP_TRY(x)                                   \
  do {                                               \
    hipError_t _e = (x);                             \
    if (_e != hipSuccess) return map_hip_error(_e);  \
  } while (0)

static int map_hip_error(hipError_t e) {
  static const bool debug = std::getenv("DC_DEBUG") != nullptr;
  if (debug) std::fprintf(stderr, "dchess: HIP error %d (%s)\n", (int)e, hipGetErrorString(e));
  if (e == hipErrorOutOfMemory) return DC_ENOMEM;
  if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return DC_ENODEV;
  if (e == hipErrorNotSupported) return DC_EUNSUPPORTED;
  return DC_EHIP;
}

static int sync_ctx(dc_ctx* c) {
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->harvest();
  return DC_SUCCESS;
}

// Waits for a one-block validate/apply kernel through its host flag
// (publish_done) instead of a stream synchronisation: ~15 us less per n = 1
// call.  A stream that completes or fails without the flag is reported.
static uint32_t next_seq(dc_ctx* c) {
  if (++c->io_seq == 0) c->io_seq = 1;  // 0 is the flag's initial value
  return c->io_seq;
}
static int wait_host_flag(dc_ctx* c, const uint32_t* flag, uint32_t seq) {
  for (uint32_t k = 1;; ++k) {
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) return DC_SUCCESS;
    if ((k & 1023) == 0) {
      const hipError_t q = hipStreamQuery(c->stream);
      if (q == hipSuccess) return __atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq ? DC_SUCCESS : DC_EHIP;
      if (q != hipErrorNotReady) {
        const int e = sync_ctx(c);  // the stream's error
        return e != DC_SUCCESS ? e : DC_EHIP;
      }
    }
  }
}

static int enter(dc_ctx* c) {
  if (!c) return DC_EINVAL;
  HIP_TRY(hipSetDevice(c->device));
  return DC_SUCCESS;
}

#define ENTER(c)                      \
  do {                                \
    int _r = enter(c);                \
    if (_r != DC_SUCCESS) return _r;  \
  } while (0)

// Device work other than a live call: every resident live-validator wave of
// the process is stopped first and stays stopped for the call (LiveHold).
// HIP maps a process's streams onto at most GPU_MAX_HW_QUEUES (4) hardware
// queues, so a kernel launched on a stream that shares its queue with a
// resident wave would wait behind that wave for its whole lease (round 5:
// a perft blocked 20 s behind two 20 s leases in the live test module).
#define ENTER_WORK(c) \
  ENTER(c);           \
  LiveHold live_hold_

// ================================================================ context
extern "C" {

int dc_version(void) { return 100; }

const char* dc_strerror(int s) {
  switch (s) {
    case DC_SUCCESS: return "success";
    case DC_EINVAL: return "invalid argument";
    case DC_EHIP: return "HIP runtime error";
    case DC_ENOMEM: return "out of memory";
    case DC_ENODEV: return "no usable gfx950 device";
    case DC_ERCCL: return "RCCL error";
    case DC_EUNSUPPORTED: return "unsupported request";
  }
  return "unknown status";
}

const char* dc_verdict_message(uint8_t v) {
  switch (v) {
    case DC_V_OK: return "";
    case DC_V_NO_PIECE: return "No piece at the source location";       // chess.rs:104-106
    case DC_V_WRONG_TURN: return "It's not this piece's turn to move";  // chess.rs:113-115
    case DC_V_ILLEGAL: return "Invalid move for the piece";             // chess.rs:119-121
    case DC_V_OOR: return "Position out of range";
  }
  return "Unknown verdict";
}

int dc_ctx_create(int device, dc_ctx** out) {
  if (!out) return DC_EINVAL;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return DC_ENODEV;
  if (device < 0 || device >= n) return DC_ENODEV;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return DC_ENODEV;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return DC_ENODEV;  // code objects are gfx950-only
  HIP_TRY(hipSetDevice(device));
  dc_ctx* c = new dc_ctx();
  c->device = device;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return DC_EHIP;
  }
  *out = c;
  return DC_SUCCESS;
}

static int live_stop(dc_ctx* c);
// Contexts with the live validator on (registered by dc_live_validator,
// removed by dc_ctx_destroy) and the number of LiveHolds alive.  Lock order:
// g_live_mu, then a context's live_mu.
static std::mutex g_live_mu;
static std::set<dc_ctx*> g_live_ctxs;
static std::atomic<int> g_live_hold{0};

int dc_ctx_destroy(dc_ctx* c) {
  if (!c) return DC_EINVAL;
  (void)hipSetDevice(c->device);
  {
    std::lock_guard<std::mutex> g(g_live_mu);
    std::lock_guard<std::mutex> l(c->live_mu);
    (void)live_stop(c);
    g_live_ctxs.erase(c);
  }
  (void)hipStreamSynchronize(c->stream);
  delete c;
  return DC_SUCCESS;
}

int dc_ctx_device(const dc_ctx* c) { return c ? c->device : -1; }
void* dc_ctx_stream(dc_ctx* c) { return c ? (void*)c->stream : nullptr; }

int dc_ctx_set_profiling(dc_ctx* c, int enable) {
  if (!c) return DC_EINVAL;
  c->profiling = enable != 0;
  return DC_SUCCESS;
}

int dc_ctx_kernel_stats(dc_ctx* c, const char* kernel, dc_kernel_stats* out) {
  if (!c || !kernel || !out) return DC_EINVAL;
  auto it = c->stats.find(kernel);
  if (it == c->stats.end()) {
    *out = dc_kernel_stats{0, 0.0, 0};
  } else {
    out->launches = it->second.launches;
    out->total_ms = it->second.ms;
    out->units = it->second.units;
  }
  return DC_SUCCESS;
}

int dc_ctx_reset_stats(dc_ctx* c) {
  if (!c) return DC_EINVAL;
  c->stats.clear();
  return DC_SUCCESS;
}

int dc_device_alloc(dc_ctx* c, size_t bytes, void** d_ptr) {
  ENTER_WORK(c);
  if (!d_ptr) return DC_EINVAL;
  *d_ptr = nullptr;
  HIP_TRY(hipMalloc(d_ptr, std::max<size_t>(bytes, 1)));
  return DC_SUCCESS;
}

int dc_device_free(dc_ctx* c, void* d_ptr) {
  ENTER_WORK(c);
  if (d_ptr) HIP_TRY(hipFree(d_ptr));
  return DC_SUCCESS;
}

int dc_memcpy_h2d(dc_ctx* c, void* d_dst, const void* src, size_t bytes) {
  ENTER_WORK(c);
  if (bytes && (!d_dst || !src)) return DC_EINVAL;
  if (bytes) HIP_TRY(hipMemcpyAsync(d_dst, src, bytes, hipMemcpyHostToDevice, c->stream));
  return sync_ctx(c);
}

int dc_memcpy_d2h(dc_ctx* c, void* dst, const void* d_src, size_t bytes) {
  ENTER_WORK(c);
  if (bytes && (!dst || !d_src)) return DC_EINVAL;
  if (bytes) HIP_TRY(hipMemcpyAsync(dst, d_src, bytes, hipMemcpyDeviceToHost, c->stream));
  return sync_ctx(c);
}

// ================================================================ adapters
// Cell kind (P N B R Q K X) -> ABI kind code (P=1 N=2 B=5 R=6 Q=7 K=3 X=4).
static const int kCellToCode[7] = {1, 2, 5, 6, 7, 3, 4};
static const int kCodeToCell[8] = {-1, 0, 1, 5, 6, 2, 3, 4};

int dc_startpos(dc_pos* out) {
  if (!out) return DC_EINVAL;
  std::memset(out, 0, sizeof *out);
  out->bb[0] = dc::kStartB0;
  out->bb[1] = dc::kStartB1;
  out->bb[2] = dc::kStartB2;
  out->bb[3] = dc::kStartB3;
  out->stm = 0;
  out->castle = 15;
  out->ep = -1;
  return DC_SUCCESS;
}

int dc_pos_from_cells(const int8_t cells[64], uint8_t turn, dc_pos* out) {
  if (!cells || !out || turn > 1) return DC_EINVAL;  // Color::from_i32 panics otherwise (chess.rs:110)
  dc_pos p;
  std::memset(&p, 0, sizeof p);
  for (int s = 0; s < 64; ++s) {
    const int8_t c = cells[s];
    if (c == DC_CELL_EMPTY) continue;
    if (c < 0 || (c >> 3) > 1 || (c & 7) > 6) return DC_EINVAL;  // colour outside {0,1} is not representable
    const uint64_t m = 1ull << s;
    const int code = kCellToCode[c & 7];
    if (c >> 3) p.bb[0] |= m;
    if (code & 1) p.bb[1] |= m;
    if (code & 2) p.bb[2] |= m;
    if (code & 4) p.bb[3] |= m;
  }
  p.stm = turn;
  p.castle = 0;
  p.ep = -1;
  *out = p;
  return DC_SUCCESS;
}

int dc_pos_to_cells(const dc_pos* pos, int8_t cells[64], uint8_t* turn) {
  if (!pos || !cells) return DC_EINVAL;
  for (int s = 0; s < 64; ++s) {
    const int code = (int)(((pos->bb[1] >> s) & 1) | (((pos->bb[2] >> s) & 1) << 1) | (((pos->bb[3] >> s) & 1) << 2));
    if (code == 0) {
      cells[s] = DC_CELL_EMPTY;
      continue;
    }
    cells[s] = (int8_t)(((pos->bb[0] >> s) & 1) * 8 + kCodeToCell[code]);
  }
  if (turn) *turn = pos->stm;
  return DC_SUCCESS;
}

int dc_pos_from_fen(const char* fen, dc_pos* out) {
  if (!fen || !out) return DC_EINVAL;
  int8_t cells[64];
  std::memset(cells, DC_CELL_EMPTY, sizeof cells);
  int x = 7, y = 0;
  const char* s = fen;
  for (; *s && *s != ' '; ++s) {
    if (*s == '/') {
      if (y != 8 || x == 0) return DC_EINVAL;
      --x;
      y = 0;
      continue;
    }
    if (*s >= '1' && *s <= '8') {
      y += *s - '0';
      if (y > 8) return DC_EINVAL;
      continue;
    }
    static const char* kinds = "pnbrqk";
    const char* k = std::strchr(kinds, *s | 0x20);
    if (!k || y > 7) return DC_EINVAL;
    cells[8 * x + y] = (int8_t)(((*s >= 'a') ? 8 : 0) + (k - kinds));
    ++y;
  }
  if (x != 0 || y != 8) return DC_EINVAL;
  while (*s == ' ') ++s;
  uint8_t stm = 0;
  if (*s == 'b') stm = 1;
  else if (*s != 'w') return DC_EINVAL;
  ++s;
  while (*s == ' ') ++s;
  uint8_t castle = 0;
  for (; *s && *s != ' '; ++s) {
    switch (*s) {
      case 'K': castle |= 1; break;
      case 'Q': castle |= 2; break;
      case 'k': castle |= 4; break;
      case 'q': castle |= 8; break;
      case '-': break;
      default: return DC_EINVAL;
    }
  }
  while (*s == ' ') ++s;
  int8_t ep = -1;
  if (*s >= 'a' && *s <= 'h' && s[1] >= '1' && s[1] <= '8') ep = (int8_t)((s[1] - '1') * 8 + (s[0] - 'a'));
  int r = dc_pos_from_cells(cells, stm, out);
  if (r != DC_SUCCESS) return r;
  out->castle = castle;
  out->ep = ep;
  return DC_SUCCESS;
}

uint16_t dc_move_pack(uint32_t fx, uint32_t fy, uint32_t tx, uint32_t ty) {
  if (fx >= 8 || fy >= 8 || tx >= 8 || ty >= 8) return (uint16_t)DC_MOVE_OOR;
  return (uint16_t)((8 * fx + fy) | ((8 * tx + ty) << 6));
}

int dc_move_pack_batch(const uint32_t* actions, uint32_t n, uint16_t* moves) {
  if (n && (!actions || !moves)) return DC_EINVAL;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t* a = actions + (size_t)4 * i;
    moves[i] = dc_move_pack(a[0], a[1], a[2], a[3]);
  }
  return DC_SUCCESS;
}

// ========================================================= live validator
// dc_live_validator(ctx, lease_us): small validate / apply calls (n <= 64,
// not profiling) go to one resident wave (k_live, dc_moves.hip) through the
// stamped mailbox of dc_kernels.h instead of a kernel launch each.  The wave
// leaves after lease_us without a request (and on dc_live_validator(ctx, 0) or
// dc_ctx_destroy); the next call starts it again.  While it runs, a
// device-wide synchronisation (hipDeviceSynchronize) waits for its lease.
static int live_stop(dc_ctx* c) {
  if (!c->live_running) return DC_SUCCESS;
  __atomic_store_n(&c->live->ctl, 1u, __ATOMIC_RELEASE);
  const hipError_t e = hipStreamSynchronize(c->live_stream);
  __atomic_store_n(&c->live->ctl, 0u, __ATOMIC_RELEASE);
  c->live_running = false;
  return e == hipSuccess ? DC_SUCCESS : DC_EHIP;
}

LiveHold::LiveHold() {
  g_live_hold.fetch_add(1);
  std::lock_guard<std::mutex> g(g_live_mu);
  for (dc_ctx* c : g_live_ctxs) {
    std::lock_guard<std::mutex> l(c->live_mu);
    (void)live_stop(c);
  }
}
LiveHold::~LiveHold() { g_live_hold.fetch_sub(1); }

static int live_start(dc_ctx* c) {
  __atomic_store_n(&c->live->state, 0u, __ATOMIC_RELEASE);
  __atomic_store_n(&c->live->ctl, 0u, __ATOMIC_RELEASE);
  HIP_TRY(dc::launch_live(c->live_stream, c->live, c->live_seq, (u64)c->live_lease_us * 100));  // 100 MHz clock
  c->live_running = true;
  return DC_SUCCESS;
}

int dc_live_validator(dc_ctx* c, uint32_t lease_us) {
  ENTER(c);
  if (lease_us > 60u * 1000 * 1000) return DC_EINVAL;  // at most a minute
  if (lease_us && !c->live) {
    HIP_TRY(hipHostMalloc((void**)&c->live, sizeof(dc::LiveBox), hipHostMallocCoherent));
    std::memset((void*)c->live, 0, sizeof(dc::LiveBox));
  }
  if (lease_us && !c->live_stream) HIP_TRY(hipStreamCreateWithFlags(&c->live_stream, hipStreamNonBlocking));
  std::lock_guard<std::mutex> g(g_live_mu);
  std::lock_guard<std::mutex> l(c->live_mu);
  if (lease_us == 0) {
    const int e = live_stop(c);
    c->live_lease_us = 0;
    g_live_ctxs.erase(c);
    return e;
  }
  if (c->live_running && lease_us != c->live_lease_us) {
    const int e = live_stop(c);  // the running wave holds the old lease
    if (e != DC_SUCCESS) return e;
  }
  c->live_lease_us = lease_us;
  g_live_ctxs.insert(c);
  return DC_SUCCESS;
}

// Test hook (not in the header): the live call's no-answer timeout, so a test
// can force the timeout path and check the next call's verdicts.
extern "C" __attribute__((visibility("default"))) int dc_test_live_timeout(dc_ctx* c, uint32_t us) {
  if (!c) return DC_EINVAL;
  std::lock_guard<std::mutex> l(c->live_mu);
  c->live_timeout_us = us;
  return DC_SUCCESS;
}

// live_call's answer when a LiveHold is active: the caller takes the launched path.
constexpr int kLiveDeclined = -1000;

// Test hook (not in the header): 1 when the context's last perft ran the
// one-launch front end (k_front), 0 when it took the legacy chain.
extern "C" __attribute__((visibility("default"))) int dc_test_perft_last_front(const dc_ctx* c) {
  return c ? (int)c->last_front : -1;
}

// Test hook (not in the header): the state hash's pre-pass budget in bytes, so
// a test can force the hash kernel's own validation path and compare hashes.
extern "C" __attribute__((visibility("default"))) int dc_test_hash_prepass_max(dc_ctx* c, uint64_t bytes) {
  if (!c) return DC_EINVAL;
  c->hash_prepass_max = bytes;
  return DC_SUCCESS;
}

// Test hook (not in the header): the state hash's BCD move-number bound
// (clamped to 10^7), so a test can force the kernel's division path.
extern "C" __attribute__((visibility("default"))) int dc_test_hash_bcd_max(dc_ctx* c, uint32_t bound) {
  if (!c) return DC_EINVAL;
  c->hash_bcd_max = bound < 10000000u ? bound : 10000000u;
  return DC_SUCCESS;
}

// One request through the mailbox.  pos_out (apply) may alias pos.
// The whole call runs under g_live_mu (then c->live_mu), and whether a hold is
// active is decided under that lock: a LiveHold counts itself before it takes
// g_live_mu, so either this call sees it and declines, or the hold's
// constructor runs after this call and stops the wave it may have started.
// (Round 5 read the hold count and live_running before any lock: a hold that
// stopped the waves in between could be followed by a fresh wave, and the
// hold's hipFree then waited for that wave's lease.)
static int live_call(dc_ctx* c, bool apply, bool fide, const dc_pos* pos, const uint16_t* moves, uint32_t n,
                     uint8_t* verdicts, uint8_t* info, dc_pos* pos_out) {
  std::lock_guard<std::mutex> g(g_live_mu);
  if (g_live_hold.load() != 0) return kLiveDeclined;
  // About to start a wave: the process keeps one resident at a time, since
  // two contexts' live streams may share a hardware queue, where the second
  // wave would wait behind the first for its whole lease.
  if (!c->live_running) {
    for (dc_ctx* o : g_live_ctxs)
      if (o != c) {
        std::lock_guard<std::mutex> l(o->live_mu);
        (void)live_stop(o);
      }
  }
  std::lock_guard<std::mutex> lock(c->live_mu);
  dc::LiveBox* b = c->live;
  if (!c->live_running) {
    const int e = live_start(c);
    if (e != DC_SUCCESS) return e;
  }
  const uint32_t seq = c->live_seq + 1;
  const uint32_t st = dc::live_stamp(seq) << 16;
  if (seq % dc::kLiveClearEvery == 0) std::memset((void*)b->req, 0, sizeof(b->req));
  const uint32_t nw = apply ? dc::kLiveFields * n : n;  // response words read back
  for (uint32_t i = 0; i < nw; ++i) __atomic_store_n(&b->resp[i], 0u, __ATOMIC_RELAXED);
  for (uint32_t e = 0; e < n; ++e) {
    uint16_t h[dc::kLiveFields];
    std::memcpy(h, pos[e].bb, 32);
    h[16] = (uint16_t)(pos[e].stm | (pos[e].castle << 8));
    h[17] = (uint8_t)pos[e].ep;
    h[18] = moves[e];
    for (uint32_t k = 0; k < dc::kLiveFields; ++k) b->req[1 + k * n + e] = st | h[k];
  }
  __atomic_store_n(&b->req[0], st | n | ((uint32_t)apply << 7) | ((uint32_t)fide << 8), __ATOMIC_RELEASE);
  // spin on the response words; a wave that stopped (lease) before taking the
  // request is restarted -- it takes requests only before it publishes state 2
  auto complete = [&]() {
    for (uint32_t i = 0; i < nw; ++i)
      if ((__atomic_load_n(&b->resp[i], __ATOMIC_ACQUIRE) & 0xFFFF0000u) != st) return false;
    return true;
  };
  u64 spins = 0;
  const auto t0 = std::chrono::steady_clock::now();
  while (!complete()) {
    if ((++spins & 255) == 0) {
      if (__atomic_load_n(&b->state, __ATOMIC_ACQUIRE) == 2u) {
        HIP_TRY(hipStreamSynchronize(c->live_stream));
        c->live_running = false;
        if (complete()) break;
        const int e = live_start(c);
        if (e != DC_SUCCESS) return e;
      } else if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(c->live_timeout_us)) {
        (void)live_stop(c);
        // the request may still be in the mailbox, and a wave on its way out
        // may have answered it: clear it and burn its stamp, so the next
        // call's wave looks for seq + 1 and never takes this one for its own
        __atomic_store_n(&b->req[0], 0u, __ATOMIC_RELEASE);
        c->live_seq = seq;
        return DC_EHIP;  // the wave neither answered nor stopped
      }
    }
  }
  c->live_seq = seq;
  for (uint32_t e = 0; e < n; ++e) {
    const uint32_t w = b->resp[e];
    verdicts[e] = (uint8_t)(w & 0xFF);
    if (info) info[e] = (uint8_t)((w >> 8) & 0xFF);
    if (apply) {
      uint16_t h[dc::kLiveFields];
      for (uint32_t k = 1; k < dc::kLiveFields; ++k) h[k] = (uint16_t)b->resp[k * n + e];
      dc_pos q = pos[e];
      std::memcpy(q.bb, h + 1, 32);
      q.stm = (uint8_t)(h[17] & 0xFF);
      q.castle = (uint8_t)(h[17] >> 8);
      q.ep = (int8_t)(uint8_t)h[18];
      pos_out[e] = q;
    }
  }
  return DC_SUCCESS;
}

// (the hold count read here is only a hint; live_call decides under g_live_mu)
static bool live_eligible(const dc_ctx* c, uint32_t n) {
  return c->live_lease_us && n <= dc::kLiveMax && !c->profiling && g_live_hold.load() == 0;
}

// ============================================================== validation
int dc_validate_batch(dc_ctx* c, uint32_t rules, const dc_pos* pos, const uint16_t* moves, uint32_t n,
                      uint8_t* verdicts) {
  ENTER(c);
  if (rules > DC_RULES_FIDE || (n && (!pos || !moves || !verdicts))) return DC_EINVAL;
  if (n == 0) return DC_SUCCESS;
  if (live_eligible(c, n)) {
    const int e = live_call(c, false, rules == DC_RULES_FIDE, pos, moves, n, verdicts, nullptr, nullptr);
    if (e != kLiveDeclined) return e;
  }
  LiveHold live_hold_;  // the launched path (ENTER_WORK)
  if (n <= kHostIoBatch) {  // pinned, read in place by the kernel
    if (!c->host_io) {
      HIP_TRY(hipHostMalloc((void**)&c->host_io, sizeof(HostIo), hipHostMallocCoherent));
      c->host_io->done = 0;  // io_seq's values start at 1
    }
    HostIo* h = c->host_io;
    std::memcpy(h->pos, pos, sizeof(dc_pos) * n);
    std::memcpy(h->moves, moves, sizeof(uint16_t) * n);
    const DevPos* dp = reinterpret_cast<const DevPos*>(h->pos);
    const bool flag = n <= kHostFlagBatch && !c->profiling;
    const uint32_t seq = flag ? next_seq(c) : 0u;
    uint32_t* done = flag ? &h->done : nullptr;
    HIP_TRY(c->timed("validate", n, [&] {
      return rules == DC_RULES_REF ? dc::launch_validate_ref(c->stream, dp, h->moves, n, h->verdicts, done, seq)
                                   : dc::launch_validate_fide(c->stream, dp, h->moves, n, h->verdicts, done, seq);
    }));
    const int e = flag ? wait_host_flag(c, done, seq) : sync_ctx(c);
    if (e != DC_SUCCESS) return e;
    std::memcpy(verdicts, h->verdicts, n);
    return DC_SUCCESS;
  }
  HIP_TRY(c->pos.ensure(n));
  HIP_TRY(c->moves.ensure(n));
  HIP_TRY(c->verdicts.ensure(n));
  HIP_TRY(hipMemcpyAsync(c->pos.p, pos, sizeof(dc_pos) * n, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->moves.p, moves, sizeof(uint16_t) * n, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c->timed("validate", n, [&] {
    return rules == DC_RULES_REF ? dc::launch_validate_ref(c->stream, c->pos.p, c->moves.p, n, c->verdicts.p)
                                 : dc::launch_validate_fide(c->stream, c->pos.p, c->moves.p, n, c->verdicts.p);
  }));
  HIP_TRY(hipMemcpyAsync(verdicts, c->verdicts.p, n, hipMemcpyDeviceToHost, c->stream));
  return sync_ctx(c);
}

int dc_apply_batch(dc_ctx* c, uint32_t rules, dc_pos* pos, const uint16_t* moves, uint32_t n, uint8_t* verdicts,
                   uint8_t* info) {
  ENTER(c);
  if (rules > DC_RULES_FIDE || (n && (!pos || !moves || !verdicts))) return DC_EINVAL;
  if (n == 0) return DC_SUCCESS;
  if (live_eligible(c, n)) {
    const int e = live_call(c, true, rules == DC_RULES_FIDE, pos, moves, n, verdicts, info, pos);
    if (e != kLiveDeclined) return e;
  }
  LiveHold live_hold_;  // the launched path (ENTER_WORK)
  if (n <= kHostIoBatch) {  // pinned, read and written in place by the kernel
    if (!c->host_io) {
      HIP_TRY(hipHostMalloc((void**)&c->host_io, sizeof(HostIo), hipHostMallocCoherent));
      c->host_io->done = 0;  // io_seq's values start at 1
    }
    HostIo* h = c->host_io;
    std::memcpy(h->pos, pos, sizeof(dc_pos) * n);
    std::memcpy(h->moves, moves, sizeof(uint16_t) * n);
    DevPos* dp = reinterpret_cast<DevPos*>(h->pos);
    const bool flag = n <= kHostFlagBatch && !c->profiling;
    const uint32_t seq = flag ? next_seq(c) : 0u;
    uint32_t* done = flag ? &h->done : nullptr;
    HIP_TRY(c->timed("apply", n, [&] {
      return rules == DC_RULES_REF
                 ? dc::launch_apply_ref(c->stream, dp, h->moves, n, h->verdicts, h->info, done, seq)
                 : dc::launch_apply_fide(c->stream, dp, h->moves, n, h->verdicts, h->info, done, seq);
    }));
    const int e = flag ? wait_host_flag(c, done, seq) : sync_ctx(c);
    if (e != DC_SUCCESS) return e;
    std::memcpy(pos, h->pos, sizeof(dc_pos) * n);
    std::memcpy(verdicts, h->verdicts, n);
    if (info) std::memcpy(info, h->info, n);
    return DC_SUCCESS;
  }
  HIP_TRY(c->pos.ensure(n));
  HIP_TRY(c->moves.ensure(n));
  HIP_TRY(c->verdicts.ensure(n));
  HIP_TRY(c->info.ensure(n));
  HIP_TRY(hipMemcpyAsync(c->pos.p, pos, sizeof(dc_pos) * n, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->moves.p, moves, sizeof(uint16_t) * n, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c->timed("apply", n, [&] {
    return rules == DC_RULES_REF
               ? dc::launch_apply_ref(c->stream, c->pos.p, c->moves.p, n, c->verdicts.p, c->info.p)
               : dc::launch_apply_fide(c->stream, c->pos.p, c->moves.p, n, c->verdicts.p, c->info.p);
  }));
  HIP_TRY(hipMemcpyAsync(pos, c->pos.p, sizeof(dc_pos) * n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(verdicts, c->verdicts.p, n, hipMemcpyDeviceToHost, c->stream));
  if (info) HIP_TRY(hipMemcpyAsync(info, c->info.p, n, hipMemcpyDeviceToHost, c->stream));
  return sync_ctx(c);
}

// ================================================================== replay
static int replay_impl(dc_ctx* c, uint32_t rules, const dc_pos* start, const uint16_t* d_moves, uint32_t n_games,
                       uint32_t n_plies, u64* d_bitmap, u64* d_digests, dc_replay_stats* stats,
                       uint8_t* d_info = nullptr) {
  dc_pos s;
  if (start) s = *start;
  else dc_startpos(&s);
  if (s.stm > 1) return DC_EINVAL;
  // per-ply info: REF only (FIDE notation would need promotion/castling,
  // which the reference's update_history never sees); one buffer descriptor
  if (d_info && (rules != DC_RULES_REF || (u64)n_games * n_plies * 2 > 0xFFFFFFFFull)) return DC_EUNSUPPORTED;
  // stats5 = [5 totals | partials]; the reduction kernel writes all five totals
  HIP_TRY(c->stats5.ensure(5 + 5 * (size_t)dc::replay_partials(std::max<u32>(n_games, 1))));
  if (!c->replay_host) HIP_TRY(hipHostMalloc((void**)&c->replay_host, 5 * sizeof(u64)));
  u64* partial = c->stats5.p + 5;
  const Board b{s.bb[0], s.bb[1], s.bb[2], s.bb[3]};
  bool host_written = false;
  HIP_TRY(c->timed("replay", (u64)n_games * n_plies, [&] {
    return rules == DC_RULES_REF
               ? dc::launch_replay_ref(c->stream, b, s.stm, d_moves, n_games, n_plies, d_bitmap, d_digests, c->stats5.p,
                                       partial, c->replay_host, &host_written, d_info)
               : dc::launch_replay_fide(c->stream, reinterpret_cast<const DevPos&>(s), d_moves, n_games, n_plies,
                                        d_bitmap, d_digests, c->stats5.p, partial);
  }));
  u64 h[5] = {0, 0, 0, 0, 0};
  if (!host_written && n_games)
    HIP_TRY(hipMemcpyAsync(h, c->stats5.p, sizeof h, hipMemcpyDeviceToHost, c->stream));
  int r = sync_ctx(c);
  if (r != DC_SUCCESS) return r;
  if (host_written) std::memcpy(h, c->replay_host, sizeof h);
  if (stats) {
    stats->validated = h[0];
    stats->accepted = h[1];
    stats->rejected = h[2];
    stats->digest_sum = h[3];
    stats->digest_xor = h[4];
  }
  // patch the unit count to validated moves (non-sentinel plies)
  if (c->profiling) {
    auto& ks = c->stats["replay"];
    ks.units = ks.units - (u64)n_games * n_plies + h[0];
  }
  return DC_SUCCESS;
}

int dc_replay_device(dc_ctx* c, uint32_t rules, const dc_pos* start, const uint16_t* d_moves, uint32_t n_games,
                     uint32_t n_plies, uint64_t* d_bitmap, uint64_t* d_digests, dc_replay_stats* stats) {
  ENTER_WORK(c);
  if (rules > DC_RULES_FIDE || (n_games && n_plies && !d_moves)) return DC_EINVAL;
  return replay_impl(c, rules, start, d_moves, n_games, n_plies, reinterpret_cast<u64*>(d_bitmap),
                     reinterpret_cast<u64*>(d_digests), stats);
}

int dc_replay(dc_ctx* c, uint32_t rules, const dc_pos* start, const uint16_t* moves, uint32_t n_games,
              uint32_t n_plies, uint64_t* bitmap, uint64_t* digests, dc_replay_stats* stats) {
  ENTER_WORK(c);
  if (rules > DC_RULES_FIDE || (n_games && n_plies && !moves)) return DC_EINVAL;
  const size_t nm = (size_t)n_games * n_plies;
  const size_t words = (size_t)((n_games + 63) / 64) * n_plies;
  HIP_TRY(c->moves.ensure(std::max<size_t>(nm, 1)));
  if (bitmap) HIP_TRY(c->bitmap.ensure(std::max<size_t>(words, 1)));
  if (digests) HIP_TRY(c->digests.ensure(std::max<size_t>(n_games, 1)));
  if (nm) HIP_TRY(hipMemcpyAsync(c->moves.p, moves, nm * sizeof(uint16_t), hipMemcpyHostToDevice, c->stream));
  int r = replay_impl(c, rules, start, c->moves.p, n_games, n_plies, bitmap ? c->bitmap.p : nullptr,
                      digests ? c->digests.p : nullptr, stats);
  if (r != DC_SUCCESS) return r;
  if (bitmap && words)
    HIP_TRY(hipMemcpyAsync(bitmap, c->bitmap.p, words * sizeof(u64), hipMemcpyDeviceToHost, c->stream));
  if (digests && n_games)
    HIP_TRY(hipMemcpyAsync(digests, c->digests.p, (size_t)n_games * sizeof(u64), hipMemcpyDeviceToHost, c->stream));
  return sync_ctx(c);
}

int dc_replay_info_device(dc_ctx* c, uint32_t rules, const dc_pos* start, const uint16_t* d_moves, uint32_t n_games,
                          uint32_t n_plies, uint64_t* d_bitmap, uint64_t* d_digests, uint8_t* d_info,
                          dc_replay_stats* stats) {
  ENTER_WORK(c);
  if (rules > DC_RULES_FIDE || (n_games && n_plies && (!d_moves || !d_info))) return DC_EINVAL;
  return replay_impl(c, rules, start, d_moves, n_games, n_plies, reinterpret_cast<u64*>(d_bitmap),
                     reinterpret_cast<u64*>(d_digests), stats, d_info);
}

int dc_replay_info(dc_ctx* c, uint32_t rules, const dc_pos* start, const uint16_t* moves, uint32_t n_games,
                   uint32_t n_plies, uint64_t* bitmap, uint64_t* digests, uint8_t* info, dc_replay_stats* stats) {
  ENTER_WORK(c);
  if (rules > DC_RULES_FIDE || (n_games && n_plies && (!moves || !info))) return DC_EINVAL;
  if (rules != DC_RULES_REF) return DC_EUNSUPPORTED;
  const size_t nm = (size_t)n_games * n_plies;
  // replay_impl's limit (n_games * n_plies * 2 < 4 GiB), checked before any
  // buffer is sized or any byte is copied
  if (nm * 2 >= (1ull << 32)) return DC_EUNSUPPORTED;
  const size_t words = (size_t)((n_games + 63) / 64) * n_plies;
  HIP_TRY(c->moves.ensure(std::max<size_t>(nm, 1)));
  HIP_TRY(c->replay_info.ensure(std::max<size_t>(nm, 1)));
  if (bitmap) HIP_TRY(c->bitmap.ensure(std::max<size_t>(words, 1)));
  if (digests) HIP_TRY(c->digests.ensure(std::max<size_t>(n_games, 1)));
  if (nm) HIP_TRY(hipMemcpyAsync(c->moves.p, moves, nm * sizeof(uint16_t), hipMemcpyHostToDevice, c->stream));
  int r = replay_impl(c, rules, start, c->moves.p, n_games, n_plies, bitmap ? c->bitmap.p : nullptr,
                      digests ? c->digests.p : nullptr, stats, c->replay_info.p);
  if (r != DC_SUCCESS) return r;
  if (nm) HIP_TRY(hipMemcpyAsync(info, c->replay_info.p, nm, hipMemcpyDeviceToHost, c->stream));
  if (bitmap && words)
    HIP_TRY(hipMemcpyAsync(bitmap, c->bitmap.p, words * sizeof(u64), hipMemcpyDeviceToHost, c->stream));
  if (digests && n_games)
    HIP_TRY(hipMemcpyAsync(digests, c->digests.p, (size_t)n_games * sizeof(u64), hipMemcpyDeviceToHost, c->stream));
  return sync_ctx(c);
}

// ------------------------------------------------------------ state hashes
}  // extern "C"

namespace {

// serde_json's string escaping (serde_json 1.0 ser.rs ESCAPE table): '"' and
// '\\', \b \t \n \f \r, other bytes < 0x20 as \u00xx (lowercase hex); every
// other byte, UTF-8 included, verbatim.
void json_escape(const char* s, size_t n, std::string& out) {
  static const char hex[] = "0123456789abcdef";
  size_t clean = 0;  // fast path: a run of bytes that need no escape is appended whole
  while (clean < n) {
    const unsigned char ch = (unsigned char)s[clean];
    if (ch < 0x20 || ch == '"' || ch == '\\') break;
    ++clean;
  }
  out.append(s, clean);
  for (size_t i = clean; i < n; ++i) {
    const unsigned char ch = (unsigned char)s[i];
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
}

// Rust's str::split_whitespace().count() (char::is_whitespace = Unicode White_Space).
u32 count_ws_tokens(const char* s, size_t n) {
  auto is_ws = [](u32 c) {
    return (c >= 9 && c <= 13) || c == 32 || c == 0x85 || c == 0xA0 || c == 0x1680 || (c >= 0x2000 && c <= 0x200A) ||
           c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F || c == 0x3000;
  };
  u32 count = 0;
  bool in_tok = false;
  for (size_t i = 0; i < n;) {
    const unsigned char b0 = (unsigned char)s[i];
    u32 c = b0, len = 1;
    if (b0 >= 0xF0) { c = b0 & 7; len = 4; }
    else if (b0 >= 0xE0) { c = b0 & 15; len = 3; }
    else if (b0 >= 0xC0) { c = b0 & 31; len = 2; }
    for (u32 k = 1; k < len && i + k < n; ++k) c = (c << 6) | ((unsigned char)s[i + k] & 63);
    i += len;
    const bool ws = is_ws(c);
    if (!ws && !in_tok) ++count;
    in_tok = !ws;
  }
  return count;
}

// Enqueues the names check of stage_hash_text: k_names_plain's flag (0: no
// byte of any name needs escaping and the offsets are ordered) is read back
// into pinned memory, then plain_ev is recorded.  state_hash_impl enqueues it
// ahead of the replay pre-pass, so the host's wait for the flag ends while the
// GPU still runs the pass and the hash kernel is enqueued behind the pass
// (round 6: a stream-wide wait after the pass left the GPU idle between the
// two kernels).
int begin_names_check(dc_ctx* c, const char* d_names, const uint32_t* d_names_off, uint32_t n_games) {
  const u64 n_str = 2ull * n_games;
  if (n_str + 1 > 0x7FFFFFFFull) return DC_EUNSUPPORTED;  // hipcub's item count is an int
  if (!c->plain_host) HIP_TRY(hipHostMalloc((void**)&c->plain_host, sizeof(u32)));
  if (!c->plain_ev) HIP_TRY(hipEventCreateWithFlags(&c->plain_ev, hipEventDisableTiming));
  HIP_TRY(c->esc_lens.ensure(n_str + 1));
  HIP_TRY(dc::launch_names_plain(c->stream, d_names, d_names_off, (u32)n_str, c->esc_lens.p));
  HIP_TRY(hipMemcpyAsync(c->plain_host, c->esc_lens.p, sizeof(u32), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipEventRecord(c->plain_ev, c->stream));
  return DC_SUCCESS;
}

// Stages the hash kernel's text on the device: hash_text = the start history
// escaped on the host (one string per batch) followed by the player names
// escaped on the device from the raw UTF-8 in d_names (serde_json's table,
// k_escape_len / k_escape_write); hash_off = the names' escaped offsets.  One
// small readback sizes hash_text from the exact escaped total.  Runs after
// begin_names_check.
int stage_hash_text(dc_ctx* c, const char* history, const char* d_names, const uint32_t* d_names_off, uint32_t n_games,
                    u32* hist_len, u32* hist_tokens, const char** names_out, const u32** off_out) {
  const size_t hn = history ? std::strlen(history) : 0;
  c->hist_text.clear();
  json_escape(history ? history : "", hn, c->hist_text);
  if (c->hist_text.size() > 0xFFFFFFFFull) return DC_EUNSUPPORTED;
  *hist_len = (u32)c->hist_text.size();
  *hist_tokens = count_ws_tokens(history ? history : "", hn);
  const u64 n_str = 2ull * n_games;
  // Fast path (round 6): names with no byte to escape and ordered offsets are
  // their own serde_json escapes; the hash kernel then reads them in place and
  // the escaping kernels, scan and copy (~80 us per 1M games) are skipped.
  HIP_TRY(hipEventSynchronize(c->plain_ev));
  const u32 escapes = *c->plain_host;
  if (!escapes) {
    HIP_TRY(c->hash_text.ensure(std::max<size_t>(*hist_len, 1)));
    if (*hist_len)
      HIP_TRY(hipMemcpyAsync(c->hash_text.p, c->hist_text.data(), *hist_len, hipMemcpyHostToDevice, c->stream));
    *names_out = d_names;
    *off_out = d_names_off;
    return DC_SUCCESS;
  }
  const size_t tb = dc::escape_scan_tmp_bytes((u32)n_str);
  HIP_TRY(c->esc64.ensure(n_str + 1));
  HIP_TRY(c->scan_tmp.ensure(std::max<size_t>(tb, 1)));
  HIP_TRY(c->hash_off.ensure(n_str + 1));
  HIP_TRY(dc::launch_escape_len_scan(c->stream, d_names, d_names_off, (u32)n_str, *hist_len, c->esc_lens.p,
                                     c->scan_tmp.p, tb, c->esc64.p));
  u64 total = 0;
  HIP_TRY(hipMemcpyAsync(&total, c->esc64.p + n_str, sizeof(u64), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (total > 0xFFFFFFFFull) return DC_EUNSUPPORTED;  // the hash kernel's offsets are u32
  HIP_TRY(c->hash_text.ensure(std::max<size_t>(total, 1)));
  if (*hist_len)
    HIP_TRY(hipMemcpyAsync(c->hash_text.p, c->hist_text.data(), *hist_len, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(dc::launch_escape_write(c->stream, d_names, d_names_off, (u32)n_str, c->esc64.p, c->hash_off.p,
                                  c->hash_text.p));
  *names_out = c->hash_text.p;
  *off_out = c->hash_off.p;
  return DC_SUCCESS;
}

int state_hash_impl(dc_ctx* c, const dc_pos* start, const char* history, const char* d_names,
                    const uint32_t* d_names_off, const uint16_t* d_moves, uint32_t n_games, uint32_t n_plies,
                    uint8_t* d_hashes) {
  if (!d_names_off || (n_games && n_plies && !d_moves) || (n_games && !d_hashes)) return DC_EINVAL;
  dc_pos s0;
  if (start) s0 = *start;
  else dc_startpos(&s0);
  if (s0.stm > 1) return DC_EINVAL;
  // pieces of unknown kind keep a proto kind string this engine does not know
  if (s0.bb[3] & ~(s0.bb[1] | s0.bb[2])) return DC_EUNSUPPORTED;
  if (n_games == 0) return DC_SUCCESS;
  const Board b{s0.bb[0], s0.bb[1], s0.bb[2], s0.bb[3]};
  // The replay kernel first (round 5): its per-ply info byte (dc_replay_info's
  // form) gives the hash kernel each ply's verdict, mover kind and capture, so
  // the hash kernel validates nothing.  Batches past the replay kernel's one
  // buffer descriptor keep the hash kernel's own validation pass.
  const uint8_t* d_info = nullptr;
  {
    const int e = begin_names_check(c, d_names, d_names_off, n_games);
    if (e != DC_SUCCESS) return e;
  }
#ifndef DC_HASH_PRE
#define DC_HASH_PRE 1  // (0: the round-4 single kernel, for A/B only)
#endif
  // The pre-pass is an optimisation: when its buffers (up to ~2 GiB near the
  // move bound) cannot be had, or exceed the context's pre-pass budget (a test
  // hook), the hash kernel validates on its own instead of the call failing.
  // (round 6: the pass also leaves every game's final board, 32 B a game,
  // so the hash kernel makes no move)
  const u64 pre_bytes = (u64)n_games * n_plies + 8 * (5 + 5 * (u64)dc::replay_partials(n_games)) +
                        sizeof(Board) * (u64)n_games;
  bool pre = DC_HASH_PRE && n_plies > 0 && (u64)n_games * n_plies * 2 <= 0xFFFFFFFFull &&
             pre_bytes <= c->hash_prepass_max;
  if (pre && (c->replay_info.ensure((size_t)n_games * n_plies) != hipSuccess ||
              c->hash_boards.ensure(n_games) != hipSuccess ||
              c->stats5.ensure(5 + 5 * (size_t)dc::replay_partials(n_games)) != hipSuccess)) {
    (void)hipGetLastError();
    pre = false;
  }
  const Board* d_boards = nullptr;
  if (pre) {
    bool host_written = false;
    HIP_TRY(c->timed("state_hash_replay", (u64)n_games * n_plies, [&] {
      return dc::launch_replay_ref(c->stream, b, s0.stm, d_moves, n_games, n_plies, nullptr, nullptr, c->stats5.p,
                                   c->stats5.p + 5, nullptr, &host_written, c->replay_info.p, c->hash_boards.p);
    }));
    d_info = c->replay_info.p;
    d_boards = c->hash_boards.p;
  }
  // the names staged after the pass is enqueued: the staging waits only for the
  // names check enqueued ahead of the pass (begin_names_check), so the hash
  // kernel is enqueued while the GPU runs the pass (round 6)
  u32 hist_len = 0, hist_tokens = 0;
  const char* names = nullptr;
  const u32* names_off = nullptr;
  int e = stage_hash_text(c, history, d_names, d_names_off, n_games, &hist_len, &hist_tokens, &names, &names_off);
  if (e != DC_SUCCESS) return e;
  const char* text = c->hash_text.p;
  HIP_TRY(c->timed("state_hash", n_games, [&] {
    return dc::launch_state_hash_ref(c->stream, b, s0.stm, d_moves, n_games, n_plies, text, hist_len, hist_tokens,
                                     names, names_off, d_info, d_hashes, d_boards, c->hash_bcd_max);
  }));
  return sync_ctx(c);
}

}  // namespace

extern "C" {

// update_history (chess.rs:127-184) for one game's accepted plies, on the
// host: the reference's notation (convert_move_to_notation, :134-154) with its
// numbering quirk -- the move number is 1 + the number of whitespace-separated
// tokens already in the history (:169-183), so it runs 1, 3, 5, ... from "".
int dc_history_append(const char* history, const uint16_t* moves, const uint8_t* info, uint32_t n_plies,
                      size_t stride, char* out, size_t out_cap, size_t* out_len) {
  if ((n_plies && (!moves || !info)) || !out_len || (out_cap && !out)) return DC_EINVAL;
  if (stride == 0) stride = 1;
  std::string h = history ? history : "";
  size_t tokens = count_ws_tokens(h.c_str(), h.size());  // split_whitespace().count()
  static const char* kKind[7] = {"", "N", "B", "R", "Q", "K", ""};
  for (uint32_t p = 0; p < n_plies; ++p) {
    const uint8_t code = info[(size_t)p * stride];
    const uint16_t m = moves[(size_t)p * stride];
    if (code == 0xFF) continue;  // rejected or padded: not applied, no history entry
    if ((code & 7) > 5) return DC_EUNSUPPORTED;  // an OTHER piece never moves (chess.rs:210)
    const int f = m & 63, t = (m >> 6) & 63;
    std::string san = kKind[code & 7];
    if (code & 8) {
      if ((code & 7) == 0) san += (char)('a' + (f & 7));
      san += 'x';
    }
    san += (char)('a' + (t & 7));
    san += std::to_string((t >> 3) + 1);
    h += (tokens == 0 ? "" : " ") + std::to_string(tokens + 1) + ". " + san;
    tokens += 2;
  }
  *out_len = h.size();
  if (out_cap < h.size() + 1) return out_cap ? DC_EINVAL : DC_SUCCESS;
  std::memcpy(out, h.c_str(), h.size() + 1);
  return DC_SUCCESS;
}


int dc_keccak256(const void* data, size_t len, uint8_t out[32]) {
  if ((!data && len) || !out) return DC_EINVAL;
  dc::Keccak256 k;
  k.update(data, len);
  k.final(out);
  return DC_SUCCESS;
}

int dc_state_hash_device(dc_ctx* c, const dc_pos* start, const char* history, const char* d_names,
                         const uint32_t* d_names_off, const uint16_t* d_moves, uint32_t n_games, uint32_t n_plies,
                         uint8_t* d_hashes) {
  ENTER_WORK(c);
  return state_hash_impl(c, start, history, d_names, d_names_off, d_moves, n_games, n_plies, d_hashes);
}

int dc_state_hash(dc_ctx* c, const dc_pos* start, const char* history, const char* names, const uint32_t* names_off,
                  const uint16_t* moves, uint32_t n_games, uint32_t n_plies, uint8_t* hashes) {
  ENTER_WORK(c);
  if ((n_games && n_plies && !moves) || (n_games && !hashes)) return DC_EINVAL;
  const size_t nm = (size_t)n_games * n_plies;
  HIP_TRY(c->moves.ensure(std::max<size_t>(nm, 1)));
  HIP_TRY(c->hashes.ensure(std::max<size_t>((size_t)32 * n_games, 1)));
  if (nm) HIP_TRY(hipMemcpyAsync(c->moves.p, moves, nm * sizeof(uint16_t), hipMemcpyHostToDevice, c->stream));
  if (n_games) {
    if (!names || !names_off) return DC_EINVAL;
    const size_t n_off = (size_t)2 * n_games + 1;
    for (size_t i = 0; i + 1 < n_off; ++i)
      if (names_off[i + 1] < names_off[i]) return DC_EINVAL;
    const size_t raw = names_off[n_off - 1];
    HIP_TRY(c->names_raw.ensure(std::max<size_t>(raw, 1)));
    HIP_TRY(c->names_raw_off.ensure(n_off));
    if (raw) HIP_TRY(hipMemcpyAsync(c->names_raw.p, names, raw, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->names_raw_off.p, names_off, n_off * sizeof(u32), hipMemcpyHostToDevice, c->stream));
  }
  int r = state_hash_impl(c, start, history, c->names_raw.p, c->names_raw_off.p, c->moves.p, n_games, n_plies,
                          c->hashes.p);
  if (r != DC_SUCCESS) return r;
  if (n_games) HIP_TRY(hipMemcpyAsync(hashes, c->hashes.p, (size_t)32 * n_games, hipMemcpyDeviceToHost, c->stream));
  return sync_ctx(c);
}

// ------------------------------------------------ transaction signatures
const char* dc_sig_verdict_message(uint8_t v) {
  switch (v) {
    case DC_SIG_OK: return "";
    case DC_SIG_BAD_SIG_HEX: return "invalid signature hex";
    case DC_SIG_BAD_SIG: return "invalid signature encoding";
    case DC_SIG_BAD_PK_HEX: return "invalid public key hex";
    case DC_SIG_BAD_PK: return "invalid public key";
    case DC_SIG_INVALID: return "invalid signature";  // hotstuff.rs:204-206
    case DC_SIG_WRONG_OWNER: return "invalud turn";    // hotstuff.rs:147 (sic)
  }
  return "unknown verdict";
}

static int ensure_gtab(dc_ctx* c) {
  if (c->gtab_ready) return DC_SUCCESS;
  HIP_TRY(c->gtab.ensure(dc::secp::kGTabEntries));
  HIP_TRY(dc::launch_secp_gtab(c->stream, c->gtab.p));
  c->gtab_ready = true;
  return DC_SUCCESS;
}

int dc_verify_tx_batch_device(dc_ctx* c, const char* d_strings, const uint32_t* d_str_off, const uint32_t* d_actions,
                              const int8_t* d_turns, uint32_t n, uint8_t* d_verdicts) {
  ENTER_WORK(c);
  if (n == 0) return DC_SUCCESS;
  if (!d_strings || !d_str_off || !d_actions || !d_verdicts) return DC_EINVAL;
  int e = ensure_gtab(c);
  if (e != DC_SUCCESS) return e;
  HIP_TRY(c->timed("verify_tx", n, [&] {
    return dc::launch_verify_tx(c->stream, d_strings, d_str_off, d_actions, d_turns, n, c->gtab.p, d_verdicts);
  }));
  return sync_ctx(c);
}

int dc_verify_tx_batch(dc_ctx* c, const char* strings, const uint32_t* str_off, const uint32_t* actions,
                       const int8_t* turns, uint32_t n, uint8_t* verdicts) {
  ENTER_WORK(c);
  if (n == 0) return DC_SUCCESS;
  if (!strings || !str_off || !actions || !verdicts) return DC_EINVAL;
  const size_t no = (size_t)4 * n + 1;
  for (size_t i = 0; i + 1 < no; ++i)
    if (str_off[i + 1] < str_off[i]) return DC_EINVAL;
  const size_t nt = str_off[no - 1];
  HIP_TRY(c->tx_text.ensure(std::max<size_t>(nt, 1)));
  HIP_TRY(c->tx_off.ensure(no));
  HIP_TRY(c->tx_act.ensure((size_t)4 * n));
  HIP_TRY(c->tx_verdicts.ensure(n));
  if (turns) HIP_TRY(c->tx_turn.ensure(n));
  if (nt) HIP_TRY(hipMemcpyAsync(c->tx_text.p, strings, nt, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->tx_off.p, str_off, no * sizeof(u32), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->tx_act.p, actions, (size_t)4 * n * sizeof(u32), hipMemcpyHostToDevice, c->stream));
  if (turns) HIP_TRY(hipMemcpyAsync(c->tx_turn.p, turns, n, hipMemcpyHostToDevice, c->stream));
  const int r = dc_verify_tx_batch_device(c, c->tx_text.p, c->tx_off.p, c->tx_act.p, turns ? c->tx_turn.p : nullptr,
                                          n, c->tx_verdicts.p);
  if (r != DC_SUCCESS) return r;
  HIP_TRY(hipMemcpyAsync(verdicts, c->tx_verdicts.p, n, hipMemcpyDeviceToHost, c->stream));
  return sync_ctx(c);
}

int dc_gen_games_device(dc_ctx* c, uint32_t rules, uint64_t seed, uint64_t first_game, uint32_t n_games,
                        uint32_t n_plies, uint32_t noise_per_256, uint16_t* d_out) {
  ENTER_WORK(c);
  if (rules > DC_RULES_FIDE || (n_games && n_plies && !d_out) || noise_per_256 > 256) return DC_EINVAL;
  if (!n_games || !n_plies) return DC_SUCCESS;
  HIP_TRY(c->timed("gen_games", (u64)n_games * n_plies, [&] {
    return rules == DC_RULES_REF
               ? dc::launch_gen_games_ref(c->stream, seed, first_game, n_games, n_plies, noise_per_256, d_out)
               : dc::launch_gen_games_fide(c->stream, seed, first_game, n_games, n_plies, noise_per_256, d_out);
  }));
  return sync_ctx(c);
}

int dc_gen_games(dc_ctx* c, uint32_t rules, uint64_t seed, uint64_t first_game, uint32_t n_games, uint32_t n_plies,
                 uint32_t noise_per_256, uint16_t* out) {
  ENTER_WORK(c);
  if (rules > DC_RULES_FIDE || (n_games && n_plies && !out) || noise_per_256 > 256) return DC_EINVAL;
  const size_t nm = (size_t)n_games * n_plies;
  if (!nm) return DC_SUCCESS;
  HIP_TRY(c->moves.ensure(nm));
  int r = dc_gen_games_device(c, rules, seed, first_game, n_games, n_plies, noise_per_256, c->moves.p);
  if (r != DC_SUCCESS) return r;
  HIP_TRY(hipMemcpyAsync(out, c->moves.p, nm * sizeof(uint16_t), hipMemcpyDeviceToHost, c->stream));
  return sync_ctx(c);
}

}  // extern "C"

// =================================================================== perft
// Device-driven level pipeline (dc_perft.hip): the level sizes live in device
// Range descriptors, capacities are bounded on the host (n_bound x 64 children,
// within kSpecBudget bytes per level), and the host synchronises once at the
// end.  Writes past a capacity are dropped and flagged; the run is then
// repeated in exact mode, which reads every level size back before sizing the
// next (one sync per level).  Level order is deterministic, so ranks that
// rebuild the top levels agree on the frontier and take contiguous shards.
namespace {

constexpr u64 kBranchBound = 64;                    // speculative children per node
constexpr u64 kSpecBudget = 16ull << 30;            // bytes per speculative level (of 288 GB HBM)
constexpr u64 kNodeBytes = sizeof(Board) + 2 * sizeof(uint16_t);
// Deepest BFS level under REF: below it, K4 (k_perft_dfs) walks per lane.
// Ply 5 of startpos is 4.9M nodes (196 MB); a typical middlegame ply 5 stays
// within the speculative budget (Kiwipete's is 193M nodes, 6.6 GB).
constexpr u32 kDfsFrontier = 5;
// REF perft(8) takes the fused final stage from ply 5 instead (k_level_moves
// + k_count3c with 64-bit move words: startpos ply 6 is 120M words, 0.96 GB)
// while the words fit this capacity; a larger ply 6 (or DCHESS_PERFT_K4=1 in
// the environment, for tests) goes through K4 from ply 5.  REF perft(9) builds
// ply 6 as boards (startpos: 120M, 4.3 GB) and runs the fused stage over
// slices of kSliceNodes grandparents (each slice's words fit the capacity:
// 2^21 nodes x 256 moves); a ply 6 past kWideLevelBytes goes through K4.
constexpr u64 kWideWordsMax = 1ull << 29;  // 4.3 GB of words
constexpr u64 kSliceNodes = 1ull << 21;
constexpr u64 kWideLevelBytes = 48ull << 30;
// (DCHESS_PERFT_WIDE_MAX lowers it, so a test can take the fallback on a small tree)
u64 wide_words_max() {
  const char* e = std::getenv("DCHESS_PERFT_WIDE_MAX");
  const u64 v = e ? std::strtoull(e, nullptr, 10) : 0;
  return v ? std::min<u64>(v, kWideWordsMax) : kWideWordsMax;
}
// (DCHESS_PERFT_WIDE_LEVEL_MAX lowers kWideLevelBytes the same way)
u64 wide_level_bytes() {
  const char* e = std::getenv("DCHESS_PERFT_WIDE_LEVEL_MAX");
  const u64 v = e ? std::strtoull(e, nullptr, 10) : 0;
  return v ? std::min<u64>(v, kWideLevelBytes) : kWideLevelBytes;
}
bool perft_k4_forced() {
  const char* e = std::getenv("DCHESS_PERFT_K4");
  return e && e[0] == '1';
}

int ensure_level(dc_ctx* c, int b, u64 n, bool fide) {
  const size_t want = std::max<u64>(n, 1);
  HIP_TRY(c->nodes[b].ensure(want));
  HIP_TRY(c->tags[b].ensure(want));
  if (fide) HIP_TRY(c->meta[b].ensure(want));
  return DC_SUCCESS;
}

int read_range(dc_ctx* c, int level, u64* n) {
  dc::Range r;
  HIP_TRY(hipMemcpyAsync(&r, c->rng.p + level, sizeof r, hipMemcpyDeviceToHost, c->stream));
  int e = sync_ctx(c);
  if (e != DC_SUCCESS) return e;
  *n = r.hi - r.lo;
  return DC_SUCCESS;
}

static bool shard_contiguous() {
  static const bool v = [] {
    const char* e = dc::ab_env("DC_SHARD");
    return e && std::strcmp(e, "contig") == 0;
  }();
  return v;
}

// Writes *pos into the pinned root staging block.  Copies already queued on
// the stream (dc_perft_repeat_device returns with runs in flight, each reading
// the block when it executes) must see the value they were queued with, so a
// changed root first waits for the stream.  A capture only ever re-stages the
// root of the run that was just synchronised (the value is unchanged).
bool root_staged(const dc_ctx* c, const dc_pos* pos, u32 n) {
  if (c->root_host->n != n) return false;
  for (u32 i = 0; i < n; ++i) {
    const Board rb{pos[i].bb[0], pos[i].bb[1], pos[i].bb[2], pos[i].bb[3]};
    if (std::memcmp(&c->root_host->b[i], &rb, sizeof(Board)) != 0 ||
        c->root_host->meta[i] != dc::pack_meta(pos[i].castle, pos[i].ep))
      return false;
  }
  return true;
}

int write_root_host(dc_ctx* c, const dc_pos* pos, u32 n = 1) {
  if (root_staged(c, pos, n)) return DC_SUCCESS;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  HIP_TRY(hipStreamIsCapturing(c->stream, &cs));
  if (cs != hipStreamCaptureStatusNone) return DC_EHIP;  // unreachable: captures follow a synchronised run
  HIP_TRY(hipStreamSynchronize(c->stream));
  for (u32 i = 0; i < n; ++i) {
    c->root_host->b[i] = Board{pos[i].bb[0], pos[i].bb[1], pos[i].bb[2], pos[i].bb[3]};
    c->root_host->meta[i] = dc::pack_meta(pos[i].castle, pos[i].ep);
  }
  c->root_host->n = n;
  return DC_SUCCESS;
}

// the staged roots to the device root arrays (stream-ordered)
int upload_roots(dc_ctx* c, u32 n, bool meta = true) {
  HIP_TRY(hipMemcpyAsync(c->root.p, c->root_host->b, n * sizeof(Board), hipMemcpyHostToDevice, c->stream));
  if (meta)  // (REF reads no castle / ep: one graph node less per run)
    HIP_TRY(hipMemcpyAsync(c->root_meta.p, c->root_host->meta, n * sizeof(uint16_t), hipMemcpyHostToDevice,
                           c->stream));
  return DC_SUCCESS;
}

// DC_FUSED3=0 (A/B build): the last level is written and counted by k_count2c.
static bool fused3_enabled() {
  static const bool on = [] {
    const char* e = dc::ab_env("DC_FUSED3");
    return !(e && e[0] == '0');
  }();
  return on;
}

// FIDE depth 5: the top kernel stops one ply short (DC_FIDE_TOP3=1, A/B only:
// the round-4 plan, three plies in the one workgroup)
static bool fide_top_short() {
  static const bool on = [] {
    const char* e = dc::ab_env("DC_FIDE_TOP3");
    return !(e && e[0] == '1');
  }();
  return on;
}

// Enqueues one perft on the context stream up to (not including) the result
// copy.  *host_sync is set when a level size had to be read back on the host
// (exact mode or a level beyond the speculative budget): such a sequence
// depends on data and is never captured as a graph.
// DC_FRONT=0 (A/B build): REF perft(6) / perft(7) take the round-5 chain.
static bool front_enabled() {
  static const bool on = [] {
    const char* e = dc::ab_env("DC_FRONT");
    return !(e && e[0] == '0');
  }();
  return on;
}

// REF perft(6) / perft(7) of one root, unsharded or a strided shard of ply 3:
// the one-launch front end (k_front) + k_count3c.
static bool front_eligible(uint32_t rules, uint32_t depth, uint32_t split_depth, uint32_t n_shards, u32 n_pos) {
  if (rules != DC_RULES_REF || n_pos != 1 || (depth != 6 && depth != 7) || !front_enabled() || !fused3_enabled())
    return false;
  const u32 S = std::max<u32>(1, std::min(split_depth, depth - 2));
  return n_shards == 1 || (S == 3 && !shard_contiguous());
}

// k_front's sequence: the root upload (stage_root), k_front, k_count3c.
static int front_enqueue(dc_ctx* c, const dc_pos* pos, uint32_t depth, uint32_t shard, uint32_t n_shards,
                         bool stage_root) {
  if (!c->res_host) HIP_TRY(hipHostMalloc((void**)&c->res_host, sizeof(dc::PerftResult)));
  if (!c->root_host) {
    HIP_TRY(hipHostMalloc((void**)&c->root_host, sizeof(*c->root_host)));
    c->root_host->n = 0;
  }
  HIP_TRY(c->res.ensure(1));
  HIP_TRY(c->rng.ensure(16));
  HIP_TRY(c->root.ensure(dc::kMaxPerftRoots));
  HIP_TRY(c->root_meta.ensure(dc::kMaxPerftRoots));
  HIP_TRY(c->front_st.ensure(sizeof(dc::FrontState)));
  dc::FrontState* fst = reinterpret_cast<dc::FrontState*>(c->front_st.p);
  if (c->front_st_zeroed != c->front_st.p) {  // a new state block (stream-ordered before its first use)
    HIP_TRY(hipMemsetAsync(c->front_st.p, 0, sizeof(dc::FrontState), c->stream));
    c->front_st_zeroed = c->front_st.p;
  }
  // the grandparents' index is a move word's upper 20 bits
  const u32 cap_b = (u32)dc::kMoveWordNodesMax;
  const u64 cap_w = std::min<u64>((u64)cap_b * kBranchBound, 0xFFFFFFFFull);
  int e = ensure_level(c, 0, cap_b, false);
  if (e != DC_SUCCESS) return e;
  HIP_TRY(c->move_words.ensure(cap_w));
  HIP_TRY(c->front_spill.ensure(dc::front_spill_words()));
  if (stage_root) {
    e = write_root_host(c, pos, 1);
    if (e == DC_SUCCESS) e = upload_roots(c, 1, false);
    if (e != DC_SUCCESS) return e;
  }
  dc::Range* rng = c->rng.p + 8;  // [8] the grandparents, [9] the move words
  HIP_TRY(c->timed("front", 0, [&] {
    return dc::launch_front(c->stream, pos->stm, depth, c->root.p, shard, n_shards, c->nodes[0].p, c->tags[0].p,
                            cap_b, c->move_words.p, cap_w, c->res.p, rng, fst, c->front_spill.p);
  }));
  c->last_final = "count2";
  const int stm_g = pos->stm ^ (int)((depth - 3) & 1);  // the grandparents are ply depth - 3
  HIP_TRY(c->timed("count2", 0, [&] {
    return dc::launch_count3c(c->stream, stm_g, c->nodes[0].p, c->tags[0].p, rng, rng + 1, c->move_words.p,
                              c->res.p, nullptr, fst);
  }));
  return DC_SUCCESS;
}

int perft_enqueue(dc_ctx* c, uint32_t rules, const dc_pos* pos, uint32_t depth, uint32_t split_depth,
                  uint32_t shard, uint32_t n_shards, bool exact, bool* host_sync, bool stage_root = true,
                  u32 n_pos = 1, bool front = false) {
  if (front && !exact) return front_enqueue(c, pos, depth, shard, n_shards, stage_root);
  const bool fide = rules == DC_RULES_FIDE;
  const bool sharded = n_shards > 1;
  u32 F = depth >= 3 ? depth - 2 : 1;             // level handed to the final stage
  // REF perft(8) and (9): 64-bit move words below ply 5 or slices of ply 6 (see kWideWordsMax)
  // (the sliced stage indexes its grandparent level from 0: a contiguous shard
  // cut at that very level (DC_SHARD=contig, A/B build) starts elsewhere, so
  // that combination takes K4 instead)
  const bool contig_at_sliced = shard_contiguous() && sharded && depth == kDfsFrontier + 4 &&
                                std::max<u32>(1, std::min(split_depth, depth - 2)) == depth - 3;
  const bool wide = !fide && (depth == kDfsFrontier + 3 || depth == kDfsFrontier + 4) && !perft_k4_forced() &&
                    !contig_at_sliced;
  const bool sliced = wide && depth == kDfsFrontier + 4;
  // REF beyond ply kDfsFrontier: K4 walks the last Ldfs plies above the final
  // stage per lane (k_perft_dfs) instead of materialising those levels
  u32 Ldfs = 0;
  if (!fide && depth >= 3 && F > kDfsFrontier && !wide) {
    Ldfs = F - kDfsFrontier;
    F = kDfsFrontier;
    if (Ldfs > 3) return DC_EUNSUPPORTED;
  }
  const int final_plies = depth >= 3 ? 2 : 1;     // depth 1: no final stage
  const u32 S = std::max<u32>(1, std::min(split_depth, F));
  u32 T = exact ? 1 : std::min<u32>(F, 3);        // plies built by the single-workgroup top kernel
  // FIDE depth 5 (F = 3): the final stage's parents (Kiwipete: 97,862) made
  // inside the one workgroup were ~0.3 ms per position (rocprofv3, round 4);
  // stopping the top kernel one ply short leaves them to k_make_count and
  // k_level_write on every CU
  if (fide && !exact && T == F && F == 3 && fide_top_short()) T = F - 1;
  if (sharded) T = std::min(T, S);
  static const u64 kTopCap[4] = {1, 256, 256 * 256, 1ull << 20};
  // buffers (allocated before anything is enqueued)
  if (!c->res_host) HIP_TRY(hipHostMalloc((void**)&c->res_host, sizeof(dc::PerftResult)));
  if (!c->root_host) {
    HIP_TRY(hipHostMalloc((void**)&c->root_host, sizeof(*c->root_host)));
    c->root_host->n = 0;
  }
  HIP_TRY(c->res.ensure(1));
  HIP_TRY(c->rng.ensure(16));
  HIP_TRY(c->root.ensure(dc::kMaxPerftRoots));
  HIP_TRY(c->root_meta.ensure(dc::kMaxPerftRoots));
  HIP_TRY(c->top_nodes.ensure(kTopCap[1] + kTopCap[2]));
  HIP_TRY(c->top_tags.ensure(kTopCap[1] + kTopCap[2]));
  if (fide) HIP_TRY(c->top_meta.ensure(kTopCap[1] + kTopCap[2]));
  const u64 cap_T = kTopCap[T];
  int e = ensure_level(c, 0, cap_T, fide);
  if (e != DC_SUCCESS) return e;
  dc::TopScratch ts;
  for (int k = 0; k < 2; ++k) {
    const u64 off = k ? kTopCap[1] : 0;
    ts.nodes[k] = c->top_nodes.p + off;
    ts.tags[k] = c->top_tags.p + off;
    ts.meta[k] = fide ? c->top_meta.p + off : nullptr;
    ts.cap[k] = kTopCap[k + 1];
  }
  // root upload from pinned memory (stage_root = false: the caller staged it)
  if (stage_root) {
    e = write_root_host(c, pos, n_pos);
    if (e == DC_SUCCESS) e = upload_roots(c, n_pos, fide);
    if (e != DC_SUCCESS) return e;
  }
  // REF final stage over the last three plies (k_count3c): the level F is
  // never written; its parents' level is counted and scanned, then expanded
  // group by group inside the final stage.  Needs a level to expand (L < F)
  // that is not the shard level.
  const bool fused3 = !fide && Ldfs == 0 && final_plies == 2 && T < F && !(sharded && S == F) && fused3_enabled();
  // Capacity of level L + 1 (and the node guard of level L) in speculative
  // mode: the move-word level of the fused final stage, else a board level.
  auto spec_cap = [&](u32 lvl, u64 n_lvl, u64* guard) -> u64 {
    if (fused3 && wide && lvl + 1 == F) {  // 64-bit words: no grandparent limit
      *guard = 0;
      return std::min<u64>(n_lvl * kBranchBound, wide_words_max());
    }
    if (fused3 && lvl + 1 == F) {
      *guard = dc::kMoveWordNodesMax;
      return std::min<u64>(std::min<u64>(n_lvl, dc::kMoveWordNodesMax) * kBranchBound, 0xFFFFFFFFull);
    }
    *guard = 0;
    if (sliced && lvl + 2 == F)  // the sliced stage's grandparents (a lowered budget: tests)
      return std::min(n_lvl * kBranchBound, std::min(kSpecBudget, wide_level_bytes()) / kNodeBytes);
    return std::min(n_lvl * kBranchBound, kSpecBudget / kNodeBytes);
  };
  // The target ply of k_expand_top is made on many CUs by k_make_count (it
  // replaces that level's k_level_count) when that level is counted next.
  // A rank's strided shard of that ply (round 5): the words stay whole and
  // k_make_count makes only this rank's (word shard + i x n_shards), instead
  // of the one workgroup making the whole ply as boards and k_gather_shard
  // copying the shard out of it.
  const bool shard_words = !exact && sharded && S == T && T >= 2 && T < F && !shard_contiguous();
  bool top_words = !exact && T >= 2 && T < F && (!(sharded && S == T) || shard_words);
  if (top_words) HIP_TRY(c->top_words.ensure(cap_T));
  // the result block is cleared by k_expand_top itself (its first stores)
  HIP_TRY(c->timed("expand_top", 0, [&] {
    return dc::launch_expand_top(c->stream, rules, c->root.p, c->root_meta.p, pos->stm, T, ts, c->nodes[0].p,
                                 fide ? c->meta[0].p : nullptr, c->tags[0].p, cap_T, c->res.p, c->rng.p + T,
                                 top_words ? c->top_words.p : nullptr, n_pos);
  }));
  u32 L = T;
  u64 nb = cap_T;
  int buf = 0;
  // This rank's shard of level S: strided (default) or contiguous (DC_SHARD=contig).
  auto take_shard = [&]() -> int {
    if (shard_contiguous()) {
      HIP_TRY(dc::launch_slice(c->stream, c->rng.p + L, shard, n_shards));
      return DC_SUCCESS;
    }
    int e2 = ensure_level(c, buf ^ 1, nb, fide);
    if (e2 != DC_SUCCESS) return e2;
    HIP_TRY(dc::launch_gather_shard(c->stream, c->nodes[buf].p, fide ? c->meta[buf].p : nullptr, c->tags[buf].p,
                                    c->rng.p + L, shard, n_shards, c->nodes[buf ^ 1].p,
                                    fide ? c->meta[buf ^ 1].p : nullptr, c->tags[buf ^ 1].p));
    buf ^= 1;
    return DC_SUCCESS;
  };
  if (sharded && L == S) {
    if (shard_words) HIP_TRY(dc::launch_shard_range(c->stream, c->rng.p + L, shard, n_shards));
    else e = take_shard();
    if (e != DC_SUCCESS) return e;
  }
  // Level L's counts and chunk sums live in buffer pair cb; the k_level_write
  // that makes level L + 1 can count it into the other pair (counted: no
  // k_level_count launch for it).
  int cb = 0;
  bool counted = false;
  DBuf<u32>* cnt_buf[2] = {&c->counts, &c->counts2};
  DBuf<u64>* sum_buf[2] = {&c->chunk_sum, &c->chunk_sum2};
  // One level: counts + chunk sums, chunk scan into Range L+1 (capacity cap), then `write`.
  // count_next: level L + 1 will be counted by the write (its chunk sums are cleared here).
  auto count_and_scan = [&](int stm, u64 cap, int select_path, u64 guard, bool count_next) -> int {
    const u64 nch = std::max<u64>(dc::chunks_for(nb), 1);
    HIP_TRY(cnt_buf[cb]->ensure(std::max<u64>(nb, 1)));
    HIP_TRY(sum_buf[cb]->ensure(nch));
    HIP_TRY(c->chunk_base.ensure(nch));
    const u64 nch_next = std::max<u64>(dc::chunks_for(std::min<u64>(cap, 0xFFFFFFFFull)), 1);
    if (count_next) {
      HIP_TRY(cnt_buf[cb ^ 1]->ensure(std::max<u64>(std::min<u64>(cap, 0xFFFFFFFFull), 1)));
      HIP_TRY(sum_buf[cb ^ 1]->ensure(nch_next));
    }
    if (top_words) {  // level T, left as move words by k_expand_top
      top_words = false;
      HIP_TRY(c->timed("expand_count", 0, [&] {
        return dc::launch_make_count(c->stream, rules, stm ^ 1, ts.nodes[T - 2], ts.meta[T - 2], ts.tags[T - 2],
                                     c->top_words.p, c->rng.p + L, nb, c->nodes[buf].p,
                                     fide ? c->meta[buf].p : nullptr, c->tags[buf].p, cnt_buf[cb]->p, sum_buf[cb]->p,
                                     shard_words ? shard : 0u, shard_words ? n_shards : 1u);
      }));
    } else if (!counted) {
      HIP_TRY(c->timed("expand_count", 0, [&] {
        return dc::launch_level_count(c->stream, rules, stm, c->nodes[buf].p, fide ? c->meta[buf].p : nullptr,
                                      c->rng.p + L, nb, cnt_buf[cb]->p, sum_buf[cb]->p);
      }));
    }
    HIP_TRY(c->timed("scan", 0, [&] {
      return dc::launch_chunk_scan(c->stream, sum_buf[cb]->p, c->rng.p + L, c->chunk_base.p, c->rng.p + L + 1, cap,
                                   c->res.p, select_path, guard, count_next ? sum_buf[cb ^ 1]->p : nullptr, nch_next);
    }));
    return DC_SUCCESS;
  };
  while (L < F) {
    const int stm = pos->stm ^ (L & 1);
    if (exact) {
      *host_sync = true;
      e = read_range(c, L, &nb);
      if (e != DC_SUCCESS) return e;
    }
    if (fused3 && sliced && L + 1 == F) {
      // words of the whole level are never stored: per slice of grandparents,
      // k_level_moves writes that slice's words and k_count3c counts them
      e = count_and_scan(stm, ~0ull, 0, 0, false);
      if (e != DC_SUCCESS) return e;
      const u64 cap_w = std::min<u64>(kSliceNodes * 256, kWideWordsMax);
      HIP_TRY(c->move_words64.ensure(cap_w));
      HIP_TRY(c->slice_rng.ensure(2));
      HIP_TRY(c->slice_ctr.ensure(1));
      const u64 n_slices = std::max<u64>((nb + kSliceNodes - 1) / kSliceNodes, 1);
      c->last_final = "count2";
      for (u64 k = 0; k < n_slices; ++k) {
        const u64 s0 = k * kSliceNodes;
        HIP_TRY(dc::launch_wide_slice(c->stream, c->rng.p + L, c->chunk_base.p, c->rng.p + L + 1, s0, kSliceNodes,
                                      c->slice_rng.p, c->slice_ctr.p, c->res.p, cap_w));
        HIP_TRY(c->timed("level_moves", 0, [&] {
          return dc::launch_level_moves(c->stream, stm, c->nodes[buf].p + s0, c->slice_rng.p, kSliceNodes,
                                        cnt_buf[cb]->p + s0, c->chunk_base.p + dc::chunks_for(s0), c->move_words64.p,
                                        cap_w);
        }));
        HIP_TRY(c->timed("count2", 0, [&] {
          return dc::launch_count3c(c->stream, stm, c->nodes[buf].p + s0, c->tags[buf].p + s0, c->slice_rng.p,
                                    c->slice_rng.p + 1, c->move_words64.p, c->res.p, c->slice_ctr.p);
        }));
      }
      return DC_SUCCESS;
    }
    if (fused3 && L + 1 == F && (!exact || wide || nb <= dc::kMoveWordNodesMax)) {
      // one u32 move word per child (u64 when wide); in speculative mode a
      // grandparent level past kMoveWordNodesMax (a word level past
      // kWideWordsMax) is flagged on the device (exact rerun)
      u64 guard = 0;
      u64 cap_f = spec_cap(L, nb, &guard);
      e = count_and_scan(stm, exact ? ~0ull : cap_f, 0, exact ? 0 : guard, false);
      if (e != DC_SUCCESS) return e;
      if (exact) {
        *host_sync = true;
        e = read_range(c, L + 1, &cap_f);
        if (e != DC_SUCCESS) return e;
        if (wide && cap_f > wide_words_max()) {
          // too many words for the fused stage: K4 from this level (ply 5)
          Ldfs = F - L;
          F = L;
          break;
        }
        if (cap_f > 0xFFFFFFFFull) return DC_EUNSUPPORTED;
      }
      if (wide) HIP_TRY(c->move_words64.ensure(std::max<u64>(cap_f, 1)));
      else HIP_TRY(c->move_words.ensure(std::max<u64>(cap_f, 1)));
      HIP_TRY(c->timed("level_moves", 0, [&] {
        return wide ? dc::launch_level_moves(c->stream, stm, c->nodes[buf].p, c->rng.p + L, nb, cnt_buf[cb]->p,
                                             c->chunk_base.p, c->move_words64.p, cap_f)
                    : dc::launch_level_moves(c->stream, stm, c->nodes[buf].p, c->rng.p + L, nb, cnt_buf[cb]->p,
                                             c->chunk_base.p, c->move_words.p, cap_f);
      }));
      c->last_final = "count2";
      HIP_TRY(c->timed("count2", 0, [&] {
        return wide ? dc::launch_count3c(c->stream, stm, c->nodes[buf].p, c->tags[buf].p, c->rng.p + L,
                                         c->rng.p + L + 1, c->move_words64.p, c->res.p)
                    : dc::launch_count3c(c->stream, stm, c->nodes[buf].p, c->tags[buf].p, c->rng.p + L,
                                         c->rng.p + L + 1, c->move_words.p, c->res.p);
      }));
      return DC_SUCCESS;
    }
    // Speculative mode never reads a level size back: the next level gets
    // min(64 x bound, kSpecBudget) of capacity, a level past it is dropped and
    // flagged (k_chunk_scan) and the run redone in exact mode.  The level
    // kernels use resident grids over device Ranges, so a loose bound costs
    // memory, not launches.  (Reading the ply-4 size back cost perft(7) one
    // host sync mid-run and kept it out of the graph.)
    u64 guard_unused = 0;
    u64 cap_next = exact ? nb * kBranchBound : spec_cap(L, nb, &guard_unused);
    const bool exact_next = exact;
    // the write counts level L + 1 when that level is counted next (not the
    // final stage's level, not a level first cut to this rank's shard)
    // (speculative mode only: exact mode sizes the next level after the scan)
    const bool count_next = !exact && L + 1 < F && !(sharded && L + 1 == S);
    e = count_and_scan(stm, exact_next ? ~0ull : cap_next, 0, 0, count_next);
    if (e != DC_SUCCESS) return e;
    if (exact_next) {
      *host_sync = true;
      e = read_range(c, L + 1, &cap_next);
      if (e != DC_SUCCESS) return e;
      if (sliced && L + 2 == F && cap_next * kNodeBytes > wide_level_bytes()) {
        // the sliced stage's grandparent level would not fit: K4 from this level
        Ldfs = F - L;
        F = L;
        break;
      }
      if (cap_next > 0xFFFFFFFFull) return DC_EUNSUPPORTED;
    }
    e = ensure_level(c, buf ^ 1, cap_next, fide);
    if (e != DC_SUCCESS) return e;
    HIP_TRY(c->timed("expand_write", 0, [&] {
      return dc::launch_level_write(c->stream, rules, stm, c->nodes[buf].p, fide ? c->meta[buf].p : nullptr,
                                    c->tags[buf].p, c->rng.p + L, nb, cnt_buf[cb]->p, c->chunk_base.p,
                                    c->nodes[buf ^ 1].p, fide ? c->meta[buf ^ 1].p : nullptr, c->tags[buf ^ 1].p,
                                    cap_next, count_next ? cnt_buf[cb ^ 1]->p : nullptr,
                                    count_next ? sum_buf[cb ^ 1]->p : nullptr);
    }));
    buf ^= 1;
    counted = count_next;
    if (count_next) cb ^= 1;
    ++L;
    nb = cap_next;
    if (sharded && L == S) {
      e = take_shard();
      if (e != DC_SUCCESS) return e;
    }
  }
  const int stm = pos->stm ^ (L & 1);
  c->last_final = Ldfs > 0 ? "dfs" : final_plies == 2 ? "count2" : "count1";
  if (Ldfs > 0) {
    const u64 lanes = dc::dfs_lanes();
    if (Ldfs > 1) HIP_TRY(c->dfs_stack.ensure((size_t)(Ldfs - 1) * 7 * lanes));
    HIP_TRY(c->timed("dfs", 0, [&] {
      return dc::launch_perft_dfs(c->stream, stm ^ (int)(Ldfs & 1), Ldfs, c->nodes[buf].p, c->tags[buf].p,
                                  c->rng.p + L, c->res.p, Ldfs > 1 ? c->dfs_stack.p : nullptr, lanes);
    }));
  } else if (depth >= 2) {
    HIP_TRY(c->timed(final_plies == 2 ? "count2" : "count1", 0, [&] {
      return dc::launch_final(c->stream, rules, stm, final_plies, c->nodes[buf].p, fide ? c->meta[buf].p : nullptr,
                              c->tags[buf].p, c->rng.p + L, nb, c->res.p->divide, nullptr);
    }));
  }
  return DC_SUCCESS;
}

// DC_GRAPH=0 disables the perft graph (A/B).
static bool perft_graphs_enabled() {
  static const bool on = [] {
    const char* e = dc::ab_env("DC_GRAPH");
    return !(e && e[0] == '0');
  }();
  return on;
}

// One perft.  A repeated configuration (same rules, depth, shard, side to move
// and buffers) replays the launch sequence captured from its previous run as a
// hipGraph: the 12 stream operations of a perft(7) go to the GPU as one launch,
// which removes the per-kernel launch gaps.  The root position
// is read from the pinned staging block when the graph runs.
int perft_run(dc_ctx* c, uint32_t rules, const dc_pos* pos, uint32_t depth, uint32_t split_depth, uint32_t shard,
              uint32_t n_shards, bool exact, dc::PerftResult* out, u32 n_pos = 1, bool front = false) {
  const bool graphable = !exact && !c->profiling && perft_graphs_enabled();
  front = front && !exact;
  dc_ctx::PerftKey key{rules,  depth, split_depth, shard, n_shards, (u32)pos->stm, (u32)perft_k4_forced(), n_pos,
                       g_alloc_epoch.load(), wide_words_max(), wide_level_bytes(), front};
  if (graphable && c->pgraph && c->pkey == key) {
    int e = write_root_host(c, pos, n_pos);
    if (e != DC_SUCCESS) return e;
    HIP_TRY(hipGraphLaunch(c->pgraph, c->stream));
    e = sync_ctx(c);
    if (e != DC_SUCCESS) return e;
    *out = *c->res_host;
    return DC_SUCCESS;
  }
  bool host_sync = false;
  int e = perft_enqueue(c, rules, pos, depth, split_depth, shard, n_shards, exact, &host_sync, true, n_pos, front);
  if (e != DC_SUCCESS) return e;
  HIP_TRY(hipMemcpyAsync(c->res_host, c->res.p, sizeof(dc::PerftResult), hipMemcpyDeviceToHost, c->stream));
  e = sync_ctx(c);
  if (e != DC_SUCCESS) return e;
  *out = *c->res_host;
  if (!graphable || host_sync || out->overflow) return DC_SUCCESS;
  // capture the same sequence for the next call (best effort: any failure
  // leaves the plain path in place)
  if (c->pgraph) {
    (void)hipGraphExecDestroy(c->pgraph);
    c->pgraph = nullptr;
  }
  if (hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal) != hipSuccess) {
    (void)hipGetLastError();
    return DC_SUCCESS;
  }
  bool hs = false;
  int ce = perft_enqueue(c, rules, pos, depth, split_depth, shard, n_shards, false, &hs, true, n_pos, front);
  if (ce == DC_SUCCESS &&
      hipMemcpyAsync(c->res_host, c->res.p, sizeof(dc::PerftResult), hipMemcpyDeviceToHost, c->stream) != hipSuccess)
    ce = DC_EHIP;
  hipGraph_t g = nullptr;
  const hipError_t ee = hipStreamEndCapture(c->stream, &g);
  if (ce == DC_SUCCESS && ee == hipSuccess && !hs && g && key.epoch == g_alloc_epoch.load() &&
      hipGraphInstantiate(&c->pgraph, g, nullptr, nullptr, 0) == hipSuccess) {
    c->pkey = key;
  } else {
    c->pgraph = nullptr;
  }
  if (g) (void)hipGraphDestroy(g);
  (void)hipGetLastError();
  return DC_SUCCESS;
}

int perft_impl(dc_ctx* c, uint32_t rules, const dc_pos* pos, uint32_t depth, uint32_t split_depth, uint32_t shard,
               uint32_t n_shards, uint64_t* divide, uint16_t* root_moves, uint32_t* n_root, uint64_t* total,
               u32 n_pos = 1, uint8_t* root_parent = nullptr) {
  if (!pos || !total || rules > DC_RULES_FIDE || n_shards == 0 || shard >= n_shards || pos->stm > 1) return DC_EINVAL;
  if (depth > 12) return DC_EUNSUPPORTED;
  *total = 0;
  if (n_root) *n_root = 0;
  if (depth == 0) {
    *total = (shard == 0) ? 1 : 0;
    return DC_SUCCESS;
  }
  dc::PerftResult r;
  // the one-launch front end where eligible; a position it declines (a top
  // past its LDS bounds, a level past its capacity) takes the legacy chain,
  // and speculative capacities that overflow there the exact rerun
  bool front = front_eligible(rules, depth, split_depth, n_shards, n_pos);
  int e = perft_run(c, rules, pos, depth, split_depth, shard, n_shards, false, &r, n_pos, front);
  if (e == DC_SUCCESS && front && r.overflow && r.front_declined) {
    front = false;
    e = perft_run(c, rules, pos, depth, split_depth, shard, n_shards, false, &r, n_pos, false);
  }
  c->last_front = front;
  c->last_exact = e == DC_SUCCESS && r.overflow;
  if (c->last_exact) e = perft_run(c, rules, pos, depth, split_depth, shard, n_shards, true, &r, n_pos);
  if (e != DC_SUCCESS) return e;
  if (r.overflow) return DC_EUNSUPPORTED;  // more than 256 root moves, or a level beyond 2^32 nodes
  const u32 nr = r.n_root;
  if (n_root) *n_root = nr;
  if (root_moves) std::copy(r.root_moves, r.root_moves + nr, root_moves);
  if (root_parent) std::copy(r.root_parent, r.root_parent + nr, root_parent);
  u64 t = 0;
  for (u32 i = 0; i < nr; ++i) {
    const u64 v = depth == 1 ? (shard == 0 ? 1 : 0) : r.divide[i];
    t += v;
    if (divide) divide[i] = v;
  }
  *total = t;
  if (c->profiling && depth >= 2) {
    auto it = c->stats.find(c->last_final);  // the final stage that ran
    if (it != c->stats.end()) it->second.units += t;
  }
  return DC_SUCCESS;
}

}  // namespace

extern "C" {

int dc_perft(dc_ctx* c, uint32_t rules, const dc_pos* pos, uint32_t depth, uint64_t* divide, uint16_t* root_moves,
             uint32_t* n_root, uint64_t* total) {
  ENTER_WORK(c);
  return perft_impl(c, rules, pos, depth, 1, 0, 1, divide, root_moves, n_root, total);
}

int dc_perft_shard(dc_ctx* c, uint32_t rules, const dc_pos* pos, uint32_t depth, uint32_t split_depth, uint32_t shard,
                   uint32_t n_shards, uint64_t* divide, uint16_t* root_moves, uint32_t* n_root, uint64_t* total) {
  ENTER_WORK(c);
  return perft_impl(c, rules, pos, depth, split_depth, shard, n_shards, divide, root_moves, n_root, total);
}

// n_runs perfts of one position enqueued back to back on the context stream,
// each run's result left on the device (k_copy_result into d_out + 258 i): no
// host round trip between runs.  The first call of a configuration runs it once
// through perft_impl (host sync), which captures the launch sequence; later
// runs replay that hipGraph.  Returns once the runs are enqueued.
// n_runs runs on context c, the results at d_out + 258 (idx0 + stride i).
// Runs per batch graph of dc_perft_repeat_device (see dc_ctx::rgraph_batch).
constexpr u32 kRepeatBatch = 8;

static int repeat_runs(dc_ctx* c, uint32_t rules, const dc_pos* pos, uint32_t depth, uint32_t split_depth,
                       uint32_t shard, uint32_t n_shards, uint32_t n_runs, uint64_t* d_out, u32 idx0, u32 stride,
                       u32 n_pos = 1) {
  if (n_runs == 0) return DC_SUCCESS;
  HIP_TRY(c->rcur.ensure(1));  // before the key: an allocation moves the epoch
  // (a graph captured after a declined front holds the legacy chain: front false)
  dc_ctx::PerftKey key{rules,  depth, split_depth, shard, n_shards, (u32)pos->stm, (u32)perft_k4_forced(), n_pos,
                       g_alloc_epoch.load(), wide_words_max(), wide_level_bytes(),
                       front_eligible(rules, depth, split_depth, n_shards, n_pos)};
  const bool graphable = !c->profiling && perft_graphs_enabled();
  // capture `runs` runs of the sequence back to back (the result copy is part
  // of the graph: its destination is the cursor)
  auto capture = [&](u32 runs, hipGraphExec_t* out) {
    if (hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal) != hipSuccess) return false;
    bool hs = false;
    int ce = DC_SUCCESS;
    for (u32 r = 0; r < runs && ce == DC_SUCCESS && !hs; ++r) {
      ce = perft_enqueue(c, rules, pos, depth, split_depth, shard, n_shards, false, &hs, false, n_pos, key.front);
      if (ce == DC_SUCCESS && dc::launch_copy_result(c->stream, c->res.p, c->rcur.p) != hipSuccess) ce = DC_EHIP;
    }
    hipGraph_t g = nullptr;
    const hipError_t ee = hipStreamEndCapture(c->stream, &g);
    const bool ok = ce == DC_SUCCESS && ee == hipSuccess && !hs && g && key.epoch == g_alloc_epoch.load() &&
                    hipGraphInstantiate(out, g, nullptr, nullptr, 0) == hipSuccess;
    if (!ok) *out = nullptr;
    if (g) (void)hipGraphDestroy(g);
    (void)hipGetLastError();
    return ok;
  };
  if (!c->root_host || !(graphable && c->rgraph && c->rkey == key)) {
    // a plain run (host sync) sizes the buffers and stages the root; then the
    // sequence is captured without the root upload and the readback
    uint64_t total = 0;
    int e = perft_impl(c, rules, pos, depth, split_depth, shard, n_shards, nullptr, nullptr, nullptr, &total, n_pos);
    if (e != DC_SUCCESS) return e;
    if (c->last_exact) {
      // speculative capacities overflow for this configuration: exact runs
      // (one host sync per level), each result still left on the device
      HIP_TRY(dc::launch_set_result_cursor(c->stream, c->rcur.p, reinterpret_cast<u64*>(d_out), idx0, stride));
      for (u32 i = 0; i < n_runs; ++i) {
        bool hs = false;
        e = perft_enqueue(c, rules, pos, depth, split_depth, shard, n_shards, true, &hs, true, n_pos);
        if (e != DC_SUCCESS) return e;
        HIP_TRY(dc::launch_copy_result(c->stream, c->res.p, c->rcur.p));
      }
      return DC_SUCCESS;
    }
    key.epoch = g_alloc_epoch.load();
    key.front = c->last_front;
    if (graphable) {
      for (hipGraphExec_t* ge : {&c->rgraph, &c->rgraph_batch}) {
        if (*ge) (void)hipGraphExecDestroy(*ge);
        *ge = nullptr;
      }
      if (capture(1, &c->rgraph)) {
        c->rkey = key;
        if (n_runs >= kRepeatBatch) (void)capture(kRepeatBatch, &c->rgraph_batch);
      }
      (void)hipGetLastError();
    } else if (c->rgraph_batch) {
      (void)hipGraphExecDestroy(c->rgraph_batch);
      c->rgraph_batch = nullptr;
    }
  }
  const bool use_graph = graphable && c->rgraph && c->rkey == key;
  if (use_graph && !root_staged(c, pos, n_pos)) {
    // every staging copies root_host to the device root, so the device root
    // holds *pos once queued work is done if root_host does; else restage
    // (write_root_host waits for the runs still queued to read the pinned block)
    int e = write_root_host(c, pos, n_pos);
    if (e == DC_SUCCESS) e = upload_roots(c, n_pos);
    if (e != DC_SUCCESS) return e;
  }
  HIP_TRY(dc::launch_set_result_cursor(c->stream, c->rcur.p, reinterpret_cast<u64*>(d_out), idx0, stride));
  u32 i = 0;
  if (use_graph && n_runs >= kRepeatBatch && !c->rgraph_batch && c->rgraph) {
    // the key's one-run graph exists but no batch graph yet (an earlier call
    // had fewer runs): capture it now
    (void)capture(kRepeatBatch, &c->rgraph_batch);
  }
  if (use_graph && c->rgraph_batch)
    for (; i + kRepeatBatch <= n_runs; i += kRepeatBatch) HIP_TRY(hipGraphLaunch(c->rgraph_batch, c->stream));
  for (; i < n_runs; ++i) {
    if (use_graph) {
      HIP_TRY(hipGraphLaunch(c->rgraph, c->stream));  // perft + result copy
    } else {
      bool host_sync = false;
      int e = perft_enqueue(c, rules, pos, depth, split_depth, shard, n_shards, false, &host_sync, true, n_pos,
                            key.front);
      if (e != DC_SUCCESS) return e;
      HIP_TRY(dc::launch_copy_result(c->stream, c->res.p, c->rcur.p));
    }
  }
  return DC_SUCCESS;
}

int dc_perft_repeat_device(dc_ctx* c, uint32_t rules, const dc_pos* pos, uint32_t depth, uint32_t split_depth,
                           uint32_t shard, uint32_t n_shards, uint32_t n_runs, uint64_t* d_out) {
  ENTER_WORK(c);
  if (!pos || (n_runs && !d_out) || rules > DC_RULES_FIDE || n_shards == 0 || shard >= n_shards || pos->stm > 1)
    return DC_EINVAL;
  if (depth < 2 || depth > 12) return DC_EUNSUPPORTED;
  if (n_runs == 0) return DC_SUCCESS;
  // (round 4 measured alternating the runs over a second context, so one
  // run's front end would overlap the other's final stage: 1.03 against
  // 0.53 ms per perft(7) step; not kept)
  return repeat_runs(c, rules, pos, depth, split_depth, shard, n_shards, n_runs, d_out, 0, 1);
}

// A batch of root positions with the same side to move as one tree: the top
// kernel expands them together, their root moves (at most 256 in all) share
// the divide tags, and every level after it -- the final stage included --
// holds all of them, so the GPU runs one full grid per level instead of one
// small one per position (BASELINE configs[2]: six suite positions at depth 5).
static_assert(DC_PERFT_BATCH_MAX == dc::kMaxPerftRoots, "dchess.h batch bound");
static int batch_args(uint32_t rules, const dc_pos* pos, uint32_t n_pos, uint32_t depth) {
  if (!pos || n_pos == 0 || rules > DC_RULES_FIDE) return DC_EINVAL;
  if (n_pos > dc::kMaxPerftRoots || depth == 0 || depth > 12) return DC_EUNSUPPORTED;
  for (u32 i = 0; i < n_pos; ++i)
    if (pos[i].stm > 1 || pos[i].stm != pos[0].stm) return DC_EINVAL;
  return DC_SUCCESS;
}

int dc_perft_batch(dc_ctx* c, uint32_t rules, const dc_pos* pos, uint32_t n_pos, uint32_t depth, uint64_t* totals,
                   uint64_t* divide, uint16_t* root_moves, uint8_t* root_pos, uint32_t* n_root) {
  ENTER_WORK(c);
  int e = batch_args(rules, pos, n_pos, depth);
  if (e != DC_SUCCESS) return e;
  if (!totals) return DC_EINVAL;
  uint64_t div[256], total = 0;
  uint8_t parent[256];
  uint32_t nr = 0;
  e = perft_impl(c, rules, pos, depth, 1, 0, 1, div, root_moves, &nr, &total, n_pos, parent);
  if (e != DC_SUCCESS) return e;
  for (u32 i = 0; i < n_pos; ++i) totals[i] = 0;
  // a root move tagged with a position outside the batch can only come from a
  // device fault: an error, never a count folded into some position's total
  for (u32 k = 0; k < nr; ++k)
    if (parent[k] >= n_pos) return DC_EHIP;
  for (u32 k = 0; k < nr; ++k) totals[parent[k]] += div[k];
  if (divide) std::copy(div, div + nr, divide);
  if (root_pos) std::copy(parent, parent + nr, root_pos);
  if (n_root) *n_root = nr;
  return DC_SUCCESS;
}

int dc_perft_batch_repeat_device(dc_ctx* c, uint32_t rules, const dc_pos* pos, uint32_t n_pos, uint32_t depth,
                                 uint32_t split_depth, uint32_t n_runs, uint64_t* d_out) {
  ENTER_WORK(c);
  int e = batch_args(rules, pos, n_pos, depth);
  if (e != DC_SUCCESS) return e;
  if (n_runs && !d_out) return DC_EINVAL;
  if (depth < 2) return DC_EUNSUPPORTED;
  return repeat_runs(c, rules, pos, depth, split_depth, 0, 1, n_runs, d_out, 0, 1, n_pos);
}

int dc_ctx_synchronize(dc_ctx* c) {
  ENTER_WORK(c);
  return sync_ctx(c);
}

// One process, several GPUs: a host thread per device computes its shard of
// the frontier, then one grouped ncclAllReduce(ncclUint64, ncclSum) over the
// per-device divide[] vectors combines them over xGMI.
int dc_multi_perft(const int* devices, int n_devices, uint32_t rules, const dc_pos* pos, uint32_t depth,
                   uint64_t* divide, uint16_t* root_moves, uint32_t* n_root, uint64_t* total) {
  if (!devices || n_devices <= 0 || !pos || !total) return DC_EINVAL;
  std::vector<dc_ctx*> ctx(n_devices, nullptr);
  for (int i = 0; i < n_devices; ++i) {
    int r = dc_ctx_create(devices[i], &ctx[i]);
    if (r != DC_SUCCESS) {
      for (auto* x : ctx)
        if (x) dc_ctx_destroy(x);
      return r;
    }
  }
  const u32 split = depth >= 5 ? 3 : (depth >= 3 ? depth - 2 : 1);
  std::vector<int> rc(n_devices, DC_SUCCESS);
  std::vector<uint32_t> nroot(n_devices, 0);
  std::vector<uint16_t> rm(256);
  std::vector<std::thread> th;
  for (int i = 0; i < n_devices; ++i)
    th.emplace_back([&, i] {
      uint64_t tot = 0;
      rc[i] = dc_perft_shard(ctx[i], rules, pos, depth, split, (u32)i, (u32)n_devices, nullptr,
                             i == 0 ? rm.data() : nullptr, &nroot[i], &tot);
    });
  for (auto& t : th) t.join();
  int result = DC_SUCCESS;
  for (int r : rc)
    if (r != DC_SUCCESS) result = r;
  std::vector<u64> div(256, 0);
  // every shard rebuilds the same root moves: a disagreement is a bug, never summed over
  for (int i = 1; i < n_devices && result == DC_SUCCESS; ++i)
    if (nroot[i] != nroot[0]) result = DC_EHIP;
  if (result == DC_SUCCESS && depth > 0) {
    std::vector<ncclComm_t> comms(n_devices);
    if (ncclCommInitAll(comms.data(), n_devices, devices) != ncclSuccess) {
      result = DC_ERCCL;
    } else {
      if (ncclGroupStart() != ncclSuccess) result = DC_ERCCL;
      for (int i = 0; i < n_devices && result == DC_SUCCESS; ++i) {
        if (hipSetDevice(devices[i]) != hipSuccess) result = DC_EHIP;
        else if (ncclAllReduce(ctx[i]->res.p->divide, ctx[i]->res.p->divide, nroot[0], ncclUint64, ncclSum, comms[i],
                               ctx[i]->stream) != ncclSuccess)
          result = DC_ERCCL;
      }
      if (ncclGroupEnd() != ncclSuccess) result = DC_ERCCL;
      for (int i = 0; i < n_devices; ++i) {
        (void)hipSetDevice(devices[i]);
        if (hipStreamSynchronize(ctx[i]->stream) != hipSuccess) result = DC_EHIP;
      }
      if (result == DC_SUCCESS) {
        (void)hipSetDevice(devices[0]);
        if (hipMemcpy(div.data(), ctx[0]->res.p->divide, nroot[0] * sizeof(u64), hipMemcpyDeviceToHost) != hipSuccess)
          result = DC_EHIP;
      }
      for (auto& cm : comms) ncclCommDestroy(cm);
    }
  }
  if (result == DC_SUCCESS) {
    u64 t = 0;
    if (depth == 0) t = 1;
    for (u32 i = 0; i < nroot[0]; ++i) {
      t += div[i];
      if (divide) divide[i] = div[i];
    }
    if (depth == 1) {
      t = nroot[0];
      if (divide)
        for (u32 i = 0; i < nroot[0]; ++i) divide[i] = 1;
    }
    if (root_moves) std::copy(rm.begin(), rm.begin() + nroot[0], root_moves);
    if (n_root) *n_root = nroot[0];
    *total = t;
  }
  for (auto* x : ctx) dc_ctx_destroy(x);
  return result;
}


// ---------------------------------------------------------- multi-GPU replay
// Contiguous game-id ranges of whole 64-game bitmap words, so shard s's accept
// bitmap [n_plies][count/64] is a word-column block of the global ply-major
// bitmap [n_plies][ceil(n_games/64)], at word offset first/64.
int dc_replay_shard_range(uint64_t n_games, uint32_t shard, uint32_t n_shards, uint64_t* first, uint64_t* count) {
  if (!first || !count || n_shards == 0 || shard >= n_shards) return DC_EINVAL;
  const u64 words = (n_games + 63) / 64, per = (words + n_shards - 1) / n_shards;
  const u64 lo = std::min<u64>(n_games, std::min<u64>(words, (u64)shard * per) * 64);
  const u64 hi = std::min<u64>(n_games, std::min<u64>(words, (u64)(shard + 1) * per) * 64);
  *first = lo;
  *count = hi > lo ? hi - lo : 0;
  return DC_SUCCESS;
}

// One process, n_devices GPUs: device i generates (dc_gen_games_device) and
// replays (dc_replay_device) shard i of the game ids; the per-shard bitmaps
// go to device 0 with one ncclGather over xGMI (rccl.h:745) and from there to
// the host; the five counters are folded on the host (sums mod 2^64, xor).
// The gather layout of the replay shards (dc_replay_shard_range's contract):
// shard i's bitmap, padded to `per` words per ply row, is block i of
// `gathered` ([n_shards][n_plies][per]); its first ceil(count_i / 64) words of
// each row go to word first_i / 64 of the whole batch's row.
int dc_replay_scatter_shards(uint64_t n_games, uint32_t n_shards, uint32_t n_plies, const uint64_t* gathered,
                             uint64_t* bitmap) {
  if (n_shards == 0 || (n_games && n_plies && (!gathered || !bitmap))) return DC_EINVAL;
  const u64 words = (n_games + 63) / 64, per = (words + n_shards - 1) / n_shards;
  for (u32 i = 0; i < n_shards; ++i) {
    uint64_t first = 0, cnt = 0;
    const int r = dc_replay_shard_range(n_games, i, n_shards, &first, &cnt);
    if (r != DC_SUCCESS) return r;
    const u64 w_r = (cnt + 63) / 64;
    for (u32 p = 0; p < n_plies && w_r; ++p)
      std::memcpy(bitmap + (size_t)p * words + first / 64, gathered + ((size_t)i * n_plies + p) * per, w_r * 8);
  }
  return DC_SUCCESS;
}

int dc_multi_replay(const int* devices, int n_devices, uint32_t rules, uint64_t seed, uint64_t n_games,
                    uint32_t n_plies, uint32_t noise_per_256, uint64_t* bitmap, dc_replay_stats* stats) {
  if (!devices || n_devices <= 0 || rules > DC_RULES_FIDE || noise_per_256 > 256) return DC_EINVAL;
  const u64 words = (n_games + 63) / 64, per = (words + n_devices - 1) / n_devices;
  if (per * 64 > 0xFFFFFFFFull) return DC_EUNSUPPORTED;  // a shard's game count is a u32
  std::vector<dc_ctx*> ctx(n_devices, nullptr);
  for (int i = 0; i < n_devices; ++i) {
    int r = dc_ctx_create(devices[i], &ctx[i]);
    if (r != DC_SUCCESS) {
      for (auto* x : ctx)
        if (x) dc_ctx_destroy(x);
      return r;
    }
  }
  const size_t shard_words = (size_t)per * n_plies;  // every shard's bitmap padded to `per` words per ply
  std::vector<int> rc(n_devices, DC_SUCCESS);
  std::vector<dc_replay_stats> st(n_devices);
  std::vector<void*> d_moves(n_devices, nullptr), d_bm(n_devices, nullptr);
  void* d_all = nullptr;  // device 0: the gathered [n_devices][n_plies][per]
  std::vector<std::thread> th;
  for (int i = 0; i < n_devices; ++i)
    th.emplace_back([&, i] {
      uint64_t first = 0, cnt = 0;
      int r = dc_replay_shard_range(n_games, (u32)i, (u32)n_devices, &first, &cnt);
      if (r == DC_SUCCESS) r = dc_device_alloc(ctx[i], std::max<size_t>((size_t)cnt * n_plies * 2, 2), &d_moves[i]);
      if (r == DC_SUCCESS) r = dc_device_alloc(ctx[i], std::max<size_t>(shard_words * 8, 8), &d_bm[i]);
      if (r == DC_SUCCESS && i == 0 && bitmap)
        r = dc_device_alloc(ctx[i], std::max<size_t>(shard_words * 8 * n_devices, 8), &d_all);
      if (r == DC_SUCCESS && hipMemsetAsync(d_bm[i], 0, shard_words * 8, ctx[i]->stream) != hipSuccess) r = DC_EHIP;
      if (r == DC_SUCCESS)
        r = dc_gen_games_device(ctx[i], rules, seed, first, (u32)cnt, n_plies, noise_per_256,
                                static_cast<uint16_t*>(d_moves[i]));
      // the shard's bitmap rows are `per` words apart: replay into a dense
      // [n_plies][cnt/64] block, then spread the rows (dense = padded when full)
      if (r == DC_SUCCESS) {
        const u64 w_r = (cnt + 63) / 64;
        void* dense = d_bm[i];
        if (w_r != per && cnt) r = dc_device_alloc(ctx[i], (size_t)w_r * n_plies * 8, &dense);
        if (r == DC_SUCCESS)
          r = dc_replay_device(ctx[i], rules, nullptr, static_cast<uint16_t*>(d_moves[i]), (u32)cnt, n_plies,
                               static_cast<uint64_t*>(dense), nullptr, &st[i]);
        if (r == DC_SUCCESS && dense != d_bm[i]) {
          if (hipMemcpy2DAsync(d_bm[i], per * 8, dense, w_r * 8, w_r * 8, n_plies, hipMemcpyDeviceToDevice,
                               ctx[i]->stream) != hipSuccess)
            r = DC_EHIP;
          else
            r = sync_ctx(ctx[i]);
          dc_device_free(ctx[i], dense);
        }
      }
      rc[i] = r;
    });
  for (auto& t : th) t.join();
  int result = DC_SUCCESS;
  for (int r : rc)
    if (r != DC_SUCCESS) result = r;
  if (result == DC_SUCCESS && bitmap && n_plies && words) {
    std::vector<ncclComm_t> comms(n_devices);
    if (ncclCommInitAll(comms.data(), n_devices, devices) != ncclSuccess) {
      result = DC_ERCCL;
    } else {
      if (ncclGroupStart() != ncclSuccess) result = DC_ERCCL;
      for (int i = 0; i < n_devices && result == DC_SUCCESS; ++i) {
        if (hipSetDevice(devices[i]) != hipSuccess) result = DC_EHIP;
        else if (ncclGather(d_bm[i], i == 0 ? d_all : nullptr, shard_words, ncclUint64, 0, comms[i], ctx[i]->stream) !=
                 ncclSuccess)
          result = DC_ERCCL;
      }
      if (ncclGroupEnd() != ncclSuccess) result = DC_ERCCL;
      for (int i = 0; i < n_devices; ++i) {
        (void)hipSetDevice(devices[i]);
        if (hipStreamSynchronize(ctx[i]->stream) != hipSuccess) result = DC_EHIP;
      }
      for (auto& cm : comms) ncclCommDestroy(cm);
    }
    // device 0 -> host, then each shard's rows to word offset first_i / 64 of
    // every ply row (dc_replay_scatter_shards: the layout is host-tested)
    if (result == DC_SUCCESS) {
      std::vector<u64> all((size_t)n_devices * shard_words);
      (void)hipSetDevice(devices[0]);
      if (hipMemcpy(all.data(), d_all, all.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) result = DC_EHIP;
      else result = dc_replay_scatter_shards(n_games, (u32)n_devices, n_plies, reinterpret_cast<const uint64_t*>(all.data()), bitmap);
    }
  }
  if (result == DC_SUCCESS && stats) {
    dc_replay_stats t{0, 0, 0, 0, 0};
    for (auto& x : st) {
      t.validated += x.validated;
      t.accepted += x.accepted;
      t.rejected += x.rejected;
      t.digest_sum += x.digest_sum;
      t.digest_xor ^= x.digest_xor;
    }
    *stats = t;
  }
  for (int i = 0; i < n_devices; ++i) {
    if (d_moves[i]) dc_device_free(ctx[i], d_moves[i]);
    if (d_bm[i]) dc_device_free(ctx[i], d_bm[i]);
  }
  if (d_all) dc_device_free(ctx[0], d_all);
  for (auto* x : ctx) dc_ctx_destroy(x);
  return result;
}
}  // extern "C"
