// Deterministic block-partial reductions shared by the small VALU kernels (gfx950).
//
// Float atomics make a sum's rounding depend on arrival order, so two runs of the same step
// differ in the last bits and a 20-step training curve drifts apart chaotically (SPPF's max-pool
// routing amplifies it).  These kernels instead combine their waves in a fixed order in LDS, write
// one partial row per workgroup and reduce the rows in a fixed order.
#pragma once
#include "common.h"

namespace ym {

// Workgroups of the small VALU kernels that emit [PARTIAL_BLOCKS][n] partial rows.
constexpr int PARTIAL_BLOCKS = 512;

// out[j] (+)= sum over r of part[r * ld + j], r in order; one launch, one thread per column
int colsum_launch(const float* part, int rows, int n, int64_t ld, float* out, int accumulate, hipStream_t st);

}  // namespace ym
