// dc_fide.hip -- RULES_FIDE kernels (placeholder until the legal-move engine lands).
#include "dc_fide.h"

namespace dc {
hipError_t launch_validate_fide(hipStream_t, const DevPos*, const uint16_t*, u32, uint8_t*) { return hipErrorNotSupported; }
hipError_t launch_apply_fide(hipStream_t, DevPos*, const uint16_t*, u32, uint8_t*, uint8_t*) { return hipErrorNotSupported; }
hipError_t launch_replay_fide(hipStream_t, const DevPos&, const uint16_t*, u32, u32, u64*, u64*, u64*) { return hipErrorNotSupported; }
hipError_t launch_gen_games_fide(hipStream_t, u64, u64, u32, u32, u32, uint16_t*) { return hipErrorNotSupported; }
hipError_t launch_count_children_fide(hipStream_t, int, const Board*, const uint16_t*, u32, u32*) { return hipErrorNotSupported; }
hipError_t launch_expand_write_fide(hipStream_t, int, const Board*, const uint16_t*, const uint16_t*, u32, const u64*, Board*,
                                    uint16_t*, uint16_t*, uint16_t*, int) { return hipErrorNotSupported; }
hipError_t launch_count1_fide(hipStream_t, int, const Board*, const uint16_t*, const uint16_t*, u32, u64*) { return hipErrorNotSupported; }
hipError_t launch_count2_fide(hipStream_t, int, const Board*, const uint16_t*, const uint16_t*, u32, u64*, u32) { return hipErrorNotSupported; }
}  // namespace dc
