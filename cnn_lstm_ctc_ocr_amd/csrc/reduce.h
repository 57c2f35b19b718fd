// Deterministic column sums of f32 slab matrices (per-workgroup partial rows)
// shared by the BN backward, the conv bias gradients and ocrk_colsum.
#pragma once
#include "common.h"

namespace ocrk {

// Column sums of a [nslab][ld] f32 slab matrix over its first NC columns, in
// a fixed order with double accumulation, in two stages (stage 1 -> part
// [SLAB_P][NC] doubles, stage 2 -> the result). res[c] = sum (if res), and
// (accumulate ? += : =) into dst_lo[c] for c < split, dst_hi[c - split] above
// (either may be NULL).
constexpr int SLAB_P = 64;
int slab_sum(const float* slab, int nslab, int NC, double* part, float* res, float* dst_lo, float* dst_hi,
             int split, int accumulate, hipStream_t s, int ld = 0);

}  // namespace ocrk
