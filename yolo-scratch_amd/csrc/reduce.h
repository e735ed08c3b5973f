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

// ------------------------------------------------------------------ fixed-order wave combines (no float atomics)
// After the xor reductions, lane l < G of every wave holds the sums of channel group l (channels
// 8l..8l+7); the 4 waves are combined in wave order so every run rounds identically.
__device__ __forceinline__ void ordered_wave_add8(float* rs, float* rq, const float* ls, const float* lq, int g, int G) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    for (int w = 0; w < 4; ++w) {
        if (wave == w && lane < G)
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                rs[g * 8 + r] = (w ? rs[g * 8 + r] : 0.f) + ls[r];
                rq[g * 8 + r] = (w ? rq[g * 8 + r] : 0.f) + lq[r];
            }
        __syncthreads();
    }
}
// 8 channels x T taps per lane group (the stem's weight-gradient rows: T = 9 x input channels)
template <int T>
__device__ __forceinline__ void ordered_wave_add_taps(float* red, const float (*acc)[T], int g, int G) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    for (int w = 0; w < 4; ++w) {
        if (wave == w && lane < G)
#pragma unroll
            for (int r = 0; r < 8; ++r)
#pragma unroll
                for (int t = 0; t < T; ++t) red[(g * 8 + r) * T + t] = (w ? red[(g * 8 + r) * T + t] : 0.f) + acc[r][t];
        __syncthreads();
    }
}

// out[j] (+)= sum over r of part[r * ld + j], r in order; one launch, one thread per column
int colsum_launch(const float* part, int rows, int n, int64_t ld, float* out, int accumulate, hipStream_t st);

}  // namespace ym
