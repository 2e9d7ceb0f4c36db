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
  u64 level_n[16];
};

hipError_t launch_expand_top(hipStream_t st, u32 rules, const Board* root, const uint16_t* root_meta, u32 stm0,
                             u32 target, Board* s_nodes, uint16_t* s_meta, uint16_t* s_tags, u64 cap_s, Board* out,
                             uint16_t* out_meta, uint16_t* out_tags, u64 cap_out, PerftResult* res, Range* out_rng);
hipError_t launch_count_children(hipStream_t st, u32 rules, int stm, const Board* nodes, const uint16_t* meta,
                                 const Range* rng, u64 n_bound, u32* counts);
hipError_t launch_scan_level(hipStream_t st, const u32* counts, const Range* rng, u64 n_bound, u64* offsets, u64* temp,
                             Range* next, u64 cap_next, PerftResult* res);
hipError_t launch_expand_write(hipStream_t st, u32 rules, int stm, const Board* nodes, const uint16_t* meta,
                               const uint16_t* tags, const Range* rng, u64 n_bound, const u64* offsets, Board* out,
                               uint16_t* out_meta, uint16_t* out_tags, u64 cap);
hipError_t launch_slice(hipStream_t st, Range* rng, u32 shard, u32 n_shards);
// plies = 1 (k_count1) or 2 (k_count2, the fused last two plies).
hipError_t launch_final(hipStream_t st, u32 rules, int stm, int plies, const Board* nodes, const uint16_t* meta,
                        const uint16_t* tags, const Range* rng, u64 n_bound, u64* divide);
// The last two plies through an 8-byte child-descriptor list: emit at scanned
// offsets (count with launch_count_children + launch_scan_level first), then
// one lane per child; drng = the descriptor list's Range from the scan.
hipError_t launch_emit_desc(hipStream_t st, u32 rules, int stm, const Board* nodes, const uint16_t* meta,
                            const Range* rng, u64 n_bound, const u64* offsets, u64* desc, u64 cap);
hipError_t launch_count_desc(hipStream_t st, u32 rules, int stm, const Board* nodes, const uint16_t* meta,
                             const uint16_t* tags, const u64* desc, const Range* drng, u64 n_bound, u64* divide);
size_t scan_temp_elems(u64 n);

}  // namespace dc
