// Batched streaming history shift (misc.hip), used by the plan executor
// (capi.cpp) to issue a run of consecutive rave_shift_history ops as one launch.
#pragma once
#include "common.h"

namespace rave {
// kernel arguments by value (no device descriptor table): 24 x 40 bytes
constexpr int kShiftBatch = 24;
struct ShiftBatch {
    rave_shift_args a[kShiftBatch];
};
int shift_history_batch(const rave_shift_args* const* ops, int n, hipStream_t stream);
}  // namespace rave
