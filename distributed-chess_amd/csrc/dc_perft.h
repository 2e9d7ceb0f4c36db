// dc_perft.h -- launch wrappers of the device-driven perft pipeline (dc_perft.hip).
#pragma once
#include "dc_kernels.h"

namespace dc {

// Index range of one frontier level, kept in device memory.
struct Range {
  u64 lo, hi;
};

// Device-resident result block of one perft run (read back with one copy).
struct PerftResult {
  u64 divide[256];
  uint16_t root_moves[256];
  u32 n_root;
  u32 overflow;
  u32 path;        // final stage: 0 descriptor list, 1 LDS count2
  u32 next_chunk;  // k_count2c's dynamic chunk counter (zeroed with the block)
  u64 level_n[16];
  u32 dfs_next;    // k_perft_dfs's frontier cursor (zeroed with the block)
  u32 front_declined;  // k_front: the top or a level did not fit it (overflow is set too): rerun without it
  uint8_t root_parent[256];  // which root position each root move belongs to (a batch: dc_perft_batch)
};

// Root positions one launch sequence can expand together (dc_perft_batch): the
// top kernel stages them in LDS; their root moves share the 256 divide tags.
constexpr u32 kMaxPerftRoots = 8;

// Scratch of the single-workgroup top expansion (plies 1 and 2).
struct TopScratch {
  Board* nodes[2];
  uint16_t* meta[2];
  uint16_t* tags[2];
  u64 cap[2];
};

hipError_t launch_expand_top(hipStream_t st, u32 rules, const Board* root, const uint16_t* root_meta, u32 stm0,
                             u32 target, const TopScratch& s, Board* out, uint16_t* out_meta, uint16_t* out_tags,
                             u64 cap_out, PerftResult* res, Range* out_rng, u32* words = nullptr, u32 n_root = 1);
// words != nullptr (target ply >= 2): k_expand_top leaves the target ply as
// move words {parent << 15 | f | t << 6 | promo << 12} over the previous top
// ply (s.nodes[target - 2]); launch_make_count then makes, stores and counts
// it (in place of launch_level_count).  stm_par = side to move at the parents.
// wsh / wstride (a rank's strided shard of the word level, round 5): child i of
// the made level is word wsh + i * wstride; the level's Range is the shard's
// (launch_shard_range).
hipError_t launch_make_count(hipStream_t st, u32 rules, int stm_par, const Board* par, const uint16_t* par_meta,
                             const uint16_t* par_tags, const u32* words, const Range* rng, u64 n_bound, Board* out,
                             uint16_t* out_meta, uint16_t* out_tags, u32* counts, u64* chunk_sum, u32 wsh = 0,
                             u32 wstride = 1);
// rng := the size of the strided shard `shard` of n_shards of the level rng
// (nodes shard, shard + n_shards, ...), as k_gather_shard's, without copying.
hipError_t launch_shard_range(hipStream_t st, Range* rng, u32 shard, u32 n_shards);
// Per level: count (+ chunk sums), one-workgroup chunk scan (-> next Range), write.
u64 chunks_for(u64 n);
hipError_t launch_level_count(hipStream_t st, u32 rules, int stm, const Board* nodes, const uint16_t* meta,
                              const Range* rng, u64 n_bound, u32* counts, u64* chunk_sum);
// guard != 0: a level `rng` of more than guard nodes is flagged as overflow
// (next = empty), as a total beyond cap is (the move-word path's node limit).
// zero_next != nullptr: also clears the next level's first chunk sums (at most
// zero_max), which launch_level_write(next_sum) then accumulates.
hipError_t launch_chunk_scan(hipStream_t st, const u64* chunk_sum, const Range* rng, u64* chunk_base, Range* next,
                             u64 cap, PerftResult* res, int select_path, u64 guard = 0, u64* zero_next = nullptr,
                             u64 zero_max = 0);
// next_counts != nullptr: the children's own move counts (next_counts[i]) and
// per-chunk sums (added into next_sum, cleared by the chunk scan) are made
// here, so the next level needs no launch_level_count.
hipError_t launch_level_write(hipStream_t st, u32 rules, int stm, const Board* nodes, const uint16_t* meta,
                              const uint16_t* tags, const Range* rng, u64 n_bound, const u32* counts,
                              const u64* chunk_base, Board* out, uint16_t* out_meta, uint16_t* out_tags, u64 cap,
                              u32* next_counts = nullptr, u64* next_sum = nullptr);
hipError_t launch_slice(hipStream_t st, Range* rng, u32 shard, u32 n_shards);
// out[0..256) = the run's divide (0 past n_root), out[256] = n_root | overflow << 32,
// out[257] = the total: one run's result kept on the device (dc_perft_repeat_device).
// The destination is read from a device-side cursor {base, run index} that the
// copy advances, so one captured graph (perft + copy) serves every run:
// launch_set_result_cursor points it at base, run 0.
// (stride: dc_perft_repeat_device's two pipelined contexts take every other run)
struct ResultCursor {
  u64* base;
  u32 idx, stride;
};
hipError_t launch_set_result_cursor(hipStream_t st, ResultCursor* cur, u64* base, u32 idx0 = 0, u32 stride = 1);
hipError_t launch_copy_result(hipStream_t st, const PerftResult* res, ResultCursor* cur);
// Strided shard: every n_shards-th node of the level, gathered to out[0..).
hipError_t launch_gather_shard(hipStream_t st, const Board* in, const uint16_t* in_meta, const uint16_t* in_tags,
                               Range* rng, u32 shard, u32 n_shards, Board* out, uint16_t* out_meta,
                               uint16_t* out_tags);
// plies = 1 (k_count1) or 2: the fused last two plies through LDS, k_count2b
// (256-parent blocks; res == nullptr) or the wave-level k_count2 (runs only
// when res->path == 1).
hipError_t launch_final(hipStream_t st, u32 rules, int stm, int plies, const Board* nodes, const uint16_t* meta,
                        const uint16_t* tags, const Range* rng, u64 n_bound, u64* divide, const PerftResult* res);

// REF, the last three plies without materialising the final stage's parents:
// after launch_level_count + launch_chunk_scan on the grandparent level `rng`
// (next Range = rng_ch = [0, children)), k_level_moves writes every child as a
// u32 move word {grandparent index << 12 | f | t << 6} (mw: children u32),
// then k_count3c counts plies +2 and +3 below every child.  A grandparent
// level of more than kMoveWordNodesMax nodes is flagged as overflow (exact
// rerun).  stm = side to move at the grandparents; res->next_chunk is the
// group counter.
// The node limit is checked by the scan that sizes the children (guard =
// kMoveWordNodesMax in launch_chunk_scan).
constexpr u64 kMoveWordNodesMax = 1ull << 20;
hipError_t launch_level_moves(hipStream_t st, int stm, const Board* nodes, const Range* rng, u64 n_bound,
                              const u32* counts, const u64* chunk_base, u32* mw, u64 mw_cap);
struct FrontState;
// fst != nullptr (after launch_front): the front end's look-back slots are
// cleared for the next run.  (Round 6 also tried the run's result record
// written by the last block to finish instead of k_copy_result: a done
// counter and a device fence per block cost more than the launch.)
hipError_t launch_count3c(hipStream_t st, int stm_g, const Board* nodes, const uint16_t* tags, const Range* rng,
                          const Range* rng_ch, const u32* mw, PerftResult* res, u32* counter = nullptr,
                          FrontState* fst = nullptr);
// The same with u64 words {grandparent index << 12 | f | t << 6} (no 2^20
// grandparent limit): REF perft(8)'s final stage below ply 5.
hipError_t launch_level_moves(hipStream_t st, int stm, const Board* nodes, const Range* rng, u64 n_bound,
                              const u32* counts, const u64* chunk_base, u64* mw, u64 mw_cap);
hipError_t launch_count3c(hipStream_t st, int stm_g, const Board* nodes, const uint16_t* tags, const Range* rng,
                          const Range* rng_ch, const u64* mw, PerftResult* res, u32* counter = nullptr);
// The sliced fused final stage (REF perft(9)): slice [s0, s0 + len) of the
// grandparent level `lvl` -> out[0] its node Range, out[1] its word Range,
// *counter = 0 (k_count3c's group counter for the slice); a slice of more
// than cap words sets res->overflow.
hipError_t launch_wide_slice(hipStream_t st, const Range* lvl, const u64* chunk_base, const Range* words_total,
                             u64 s0, u64 len, Range* out, u32* counter, PerftResult* res, u64 cap);

// REF perft(6) / perft(7) front end in one launch (k_front, round 6): the root
// (device) -> the final stage's grandparents (ply 3 at depth 6, ply 4 at depth 7)
// as boards + tags in out (capacity cap_b <= 2^20) and their children as u32
// move words in mw (capacity cap_w), rng_out[0] / rng_out[1] their Ranges;
// then launch_count3c(stm_g = side to move at the grandparents, rng_out,
// rng_out + 1, fst).  Unsharded, or this rank's strided shard of ply 3.  The
// state block (the items' look-back slots) must be zero before the first
// launch; the launch_count3c given it clears them again.  A top past the
// kernel's LDS bounds (more than 128 root moves or 2,048 ply-2 nodes), an item
// of more than 1,024 boards or a level past its capacity sets overflow and
// front_declined.
constexpr u32 kFrontItemsMax = 1u << 16;
struct FrontState {
  u32 n_items, pad;
  u64 agg[kFrontItemsMax];
  u64 incl[kFrontItemsMax];
};
// spill (front_spill_words() u32, or null): per-item rows for the words of
// items past one LDS window (no second walk).
u64 front_spill_words();
hipError_t launch_front(hipStream_t st, int stm0, u32 depth, const Board* root, u32 shard, u32 n_shards, Board* out,
                        uint16_t* out_tags, u32 cap_b, u32* mw, u64 cap_w, PerftResult* res, Range* rng_out,
                        FrontState* fst, u32* spill);

// K4 (REF): per-lane DFS over L plies below the frontier level `rng` (1 <= L <= 3),
// each level-L node bulk-counted over the last two plies (perft depth = frontier
// ply + L + 2).  stm_parent = side to move at the level-L nodes.  stack_frames
// holds (L - 1) x 7 x lanes u64 (null for L == 1); lanes = dfs_lanes().
u64 dfs_lanes();
hipError_t launch_perft_dfs(hipStream_t st, int stm_parent, u32 L, const Board* nodes, const uint16_t* tags,
                            const Range* rng, PerftResult* res, u64* stack_frames, u64 lanes);

}  // namespace dc
