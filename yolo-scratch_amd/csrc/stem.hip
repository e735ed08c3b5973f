// The stem Conv block's backward (model.0: 1 -> c channels, 3x3 stride 2 on the fp32 image, BatchNorm2d,
// SiLU — /root/reference/yolo_scratch_cuda/models/yolo11_modules.py:21-33, yaml backbone row 0): the
// BatchNorm-backward apply fused into the weight gradient over the stored z.
//
// z of the stem is the largest tensor of the step (64 x 320 x 320 x 32 fp16 = 420 MB at s@640 bs64).
// The backward reads dy and the stored z once, forms dz = k1 (g - k2 - xhat k3) in registers (rounded
// to bf16 where the generic path stores it) and turns it straight into the weight-gradient partials
// against the image patches staged in LDS: dz never touches memory (0.45 -> 0.22 ms at s@640 bs64).
// (Round 2 also recomputed z from the image in the forward instead of storing it: 2.5 GB/step less
// traffic but VALU-bound passes, equal step time — removed)
#include <algorithm>

#include "common.h"
#include "reduce.h"

namespace ym {
namespace {

struct StemGeo {
    int N, H, W, OH, OW, C, stride, pad;
};

__device__ __forceinline__ float stem_dsilu(float u) {
    const float sg = __builtin_amdgcn_rcpf(1.0f + __expf(-u));
    return sg * (1.0f + u * (1.0f - sg));
}

__device__ __forceinline__ void load_w8(const float* __restrict__ w, int g, float (*wr)[9]) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int t = 0; t < 9; ++t) wr[r][t] = w[(g * 8 + r) * 9 + t];
}

__device__ __forceinline__ void load8f(const float* p, float* v) {
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = p[r];
}

// Output tiles of STH x STW pixels; a workgroup stages the tile's image window (stride <= 2) in LDS
// once, coalesced, then its threads — (pixel, 8-channel group) pairs — read their 3x3 patches from
// LDS.  (One thread per pixel reading its patch straight from the image made these kernels
// latency-bound: 9 dependent-address 4-byte loads per pixel, repeated by every channel group.)
constexpr int STH = 8, STW = 32;
constexpr int SIH = (STH - 1) * 2 + 3, SIW = (STW - 1) * 2 + 3;

struct StemTile {
    int n, oh0, ow0;
};

__device__ __forceinline__ StemTile stem_tile(const StemGeo& s, int t) {
    const int tw = (s.OW + STW - 1) / STW, th = (s.OH + STH - 1) / STH;
    StemTile T;
    const int c = t % tw, r = (t / tw) % th;
    T.n = t / (tw * th);
    T.oh0 = r * STH;
    T.ow0 = c * STW;
    return T;
}

__device__ __forceinline__ int stem_tiles(const StemGeo& s) {
    return s.N * ((s.OH + STH - 1) / STH) * ((s.OW + STW - 1) / STW);
}

// stage the image window of tile T (zero outside the image)
__device__ __forceinline__ void stem_stage(const float* __restrict__ img, const StemGeo& s, const StemTile& T,
                                           float* win) {
    const int ih0 = T.oh0 * s.stride - s.pad, iw0 = T.ow0 * s.stride - s.pad;
    const float* src = img + int64_t(T.n) * s.H * s.W;
    __syncthreads();
    for (int i = threadIdx.x; i < SIH * SIW; i += 256) {
        const int r = i / SIW, c = i - r * SIW;
        const int ih = ih0 + r, iw = iw0 + c;
        win[i] = (unsigned(ih) < unsigned(s.H) && unsigned(iw) < unsigned(s.W)) ? src[ih * s.W + iw] : 0.f;
    }
    __syncthreads();
}

// z of 8 channels of tile pixel (r, c): fp32 sums (zf) and the fp16-rounded values the stored path
// keeps (z); the 3x3 patch is returned for the weight gradient
__device__ __forceinline__ void stem_pix(const float (*wr)[9], const float* win, int stride, int r, int c, float* patch,
                                         float* zf, float* z) {
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) patch[kh * 3 + kw] = win[(r * stride + kh) * SIW + c * stride + kw];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        float acc = 0.f;
#pragma unroll
        for (int t = 0; t < 9; ++t) acc += wr[q][t] * patch[t];
        zf[q] = acc;
        z[q] = h2f(f2h(acc));
    }
}

// Visit every output pixel: fn(n, oh, ow, patch, zf, z, dy8) for the calling thread's 8 channels
// (G = C / 8 channel groups per pixel).  Software-pipelined over the block's tiles: while tile t is
// computed from LDS, the image window of tile t+1 and (DY) its dy values are already in flight in
// registers — one memory latency per tile would otherwise dominate (measured 9 us per 256-pixel tile).
template <int G, bool DY, class Fn, bool ZS = false>
__device__ __forceinline__ void stem_visit(const float* __restrict__ img, const StemGeo& s, const float (*wr)[9],
                                           float* win, const bf16_t* __restrict__ dy, int64_t d_bs, int64_t d_ld,
                                           Fn fn, const uint16_t* __restrict__ zst = nullptr) {
    // ZS: z is read from the stored dense fp16 [M][C] tensor (prefetched like dy) instead of recomputed
    constexpr int PPP = 256 / G, NP = STH * STW / PPP;          // pixels per pass, passes per tile
    constexpr int WI = (SIH * SIW + 255) / 256;                // window elements per thread
    const int pl = threadIdx.x / G, g = threadIdx.x % G;
    const int ntile = stem_tiles(s);
    float wv[WI];
    uint4 dv[DY ? NP : 1];
    uint4 zv[ZS ? NP : 1];
    auto fetch = [&](int t) {
        const StemTile T = stem_tile(s, t);
        const int ih0 = T.oh0 * s.stride - s.pad, iw0 = T.ow0 * s.stride - s.pad;
        const float* src = img + int64_t(T.n) * s.H * s.W;
#pragma unroll
        for (int k = 0; k < WI; ++k) {
            const int i = threadIdx.x + k * 256;
            const int r = i / SIW, c = i - r * SIW;
            const int ih = ih0 + r, iw = iw0 + c;
            wv[k] = (i < SIH * SIW && unsigned(ih) < unsigned(s.H) && unsigned(iw) < unsigned(s.W)) ? src[ih * s.W + iw]
                                                                                                 : 0.f;
        }
        if constexpr (DY) {
#pragma unroll
            for (int q = 0; q < NP; ++q) {
                const int p = q * PPP + pl, r = p / STW, c = p - r * STW;
                const int oh = min(T.oh0 + r, s.OH - 1), ow = min(T.ow0 + c, s.OW - 1);   // clamped: always in bounds
                dv[q] = *reinterpret_cast<const uint4*>(dy + int64_t(T.n) * d_bs + int64_t(oh * s.OW + ow) * d_ld + g * 8);
                if constexpr (ZS)
                    zv[q] = *reinterpret_cast<const uint4*>(zst + (int64_t(T.n) * s.OH * s.OW + int64_t(oh * s.OW + ow)) * s.C +
                                                            g * 8);
            }
        }
    };
    int t = blockIdx.x;
    if (t < ntile) fetch(t);
    for (; t < ntile; t += gridDim.x) {
        const StemTile T = stem_tile(s, t);
        __syncthreads();                       // the previous tile's patch reads are done
#pragma unroll
        for (int k = 0; k < WI; ++k) {
            const int i = threadIdx.x + k * 256;
            if (i < SIH * SIW) win[i] = wv[k];
        }
        uint4 cur[DY ? NP : 1], zcur[ZS ? NP : 1];
        if constexpr (DY) {
#pragma unroll
            for (int q = 0; q < NP; ++q) cur[q] = dv[q];
        }
        if constexpr (ZS) {
#pragma unroll
            for (int q = 0; q < NP; ++q) zcur[q] = zv[q];
        }
        __syncthreads();
        if (t + int(gridDim.x) < ntile) fetch(t + gridDim.x);
#pragma unroll
        for (int q = 0; q < NP; ++q) {
            const int p = q * PPP + pl, r = p / STW, c = p - r * STW;
            const int oh = T.oh0 + r, ow = T.ow0 + c;
            if (oh >= s.OH || ow >= s.OW) continue;
            float patch[9], zf[8], z[8];
            if constexpr (ZS) {
#pragma unroll
                for (int kh = 0; kh < 3; ++kh)
#pragma unroll
                    for (int kw = 0; kw < 3; ++kw)
                        patch[kh * 3 + kw] = win[(r * s.stride + kh) * SIW + c * s.stride + kw];
                const uint32_t u[4] = {zcur[q].x, zcur[q].y, zcur[q].z, zcur[q].w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    z[2 * e] = zf[2 * e] = h2f(uint16_t(u[e] & 0xffff));
                    z[2 * e + 1] = zf[2 * e + 1] = h2f(uint16_t(u[e] >> 16));
                }
            } else {
                stem_pix(wr, win, s.stride, r, c, patch, zf, z);
            }
            fn(T.n, oh, ow, patch, zf, z, cur[DY ? q : 0]);
        }
    }
}

__device__ __forceinline__ void unpack_bf8(uint4 v, float* d) {
    const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        d[2 * e] = bf2f(bf16_t(u[e] & 0xffff));
        d[2 * e + 1] = bf2f(bf16_t(u[e] >> 16));
    }
}

// dz = k1 (g - k2 - xhat k3), rounded to bf16 as the stored path stores it, straight into the
// weight-gradient partials part[block][co * 9 + t] = sum over the block's pixels of dz[co] * patch[t]
template <int G, bool ZS = false>
__global__ void __launch_bounds__(256) stem_bwd_wgrad_kernel(const bf16_t* __restrict__ dy, int64_t d_bs, int64_t d_ld,
                                                             const float* __restrict__ img, const float* __restrict__ w,
                                                             const float* __restrict__ bnv, const float* __restrict__ coef,
                                                             float* __restrict__ part, StemGeo s,
                                                             const uint16_t* __restrict__ zst = nullptr) {
    __shared__ float win[SIH * SIW];
    __shared__ float red[128 * 9];
    const int g = threadIdx.x % G, C = s.C;
    float wr[8][9], sc[8], sf[8], mu[8], rs[8], k1[8], k2[8], k3[8];
    if constexpr (!ZS) load_w8(w, g, wr);            // (the stored-z form never recomputes z)
    else
#pragma unroll
        for (int r = 0; r < 8; ++r)
#pragma unroll
            for (int t = 0; t < 9; ++t) wr[r][t] = 0.f;
    load8f(bnv + g * 8, sc);
    load8f(bnv + C + g * 8, sf);
    load8f(bnv + 2 * C + g * 8, mu);
    load8f(bnv + 3 * C + g * 8, rs);
    load8f(coef + g * 8, k1);
    load8f(coef + C + g * 8, k2);
    load8f(coef + 2 * C + g * 8, k3);
    float acc[8][9];
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[r][t] = 0.f;
    auto body = [&](int, int, int, const float* patch, const float*, const float* z, uint4 dv) {
        float d[8];
        unpack_bf8(dv, d);
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const float gg = d[r] * stem_dsilu(z[r] * sc[r] + sf[r]);
            const float xh = (z[r] - mu[r]) * rs[r];
            const float dz = bf2f(f2bf(k1[r] * (gg - k2[r] - xh * k3[r])));
#pragma unroll
            for (int t = 0; t < 9; ++t) acc[r][t] += dz * patch[t];
        }
    };
    stem_visit<G, true, decltype(body), ZS>(img, s, wr, win, dy, d_bs, d_ld, body, zst);
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int t = 0; t < 9; ++t)
            for (int o = G; o < 64; o <<= 1) acc[r][t] += __shfl_xor(acc[r][t], o, 64);
    ordered_wave_add_taps<9>(red, acc, g, G);
    for (int i = threadIdx.x; i < C * 9; i += 256) part[int64_t(blockIdx.x) * C * 9 + i] = red[i];
}

constexpr int STEM_WG_BLOCKS = 1024;   // weight-gradient partial rows

bool stem_shape_ok(int n, int h, int w, int oh, int ow, int c, int stride) {
    return (c == 16 || c == 32 || c == 64) && (stride == 1 || stride == 2) &&
           int64_t(n) * oh * ow < (int64_t(1) << 31) && int64_t(n) * h * w < (int64_t(1) << 31);
}

}  // namespace
}  // namespace ym

using namespace ym;

// the stored-z form: BatchNorm-backward apply + weight gradient of the stem in one pass over dy and
// the stored z (dz never written; replaces ym_bn_bwd_apply + ym_conv_first_wgrad)
extern "C" int ym_stem_bwd_wgrad_stored(const uint16_t* dy, int64_t d_bs, int64_t d_ld, const uint16_t* z,
                                        const float* img, const float* bnv, const float* coef, float* dw_oihw,
                                        float* workspace, size_t workspace_bytes, int n, int h, int w, int oh, int ow,
                                        int cout, int stride, int pad, void* stream) {
    YM_CHECK_ARG(dy && z && img && bnv && coef && dw_oihw, "ym_stem_bwd_wgrad_stored: null argument");
    YM_CHECK_ARG(stem_shape_ok(n, h, w, oh, ow, cout, stride) && d_ld % 8 == 0 && d_bs % 8 == 0,
                 "ym_stem_bwd_wgrad_stored: unsupported shape / unaligned view");
    YM_CHECK_ARG(workspace && workspace_bytes >= size_t(STEM_WG_BLOCKS) * size_t(cout) * 9 * sizeof(float),
                 "ym_stem_bwd_wgrad_stored: workspace too small");
    const StemGeo g{n, h, w, oh, ow, cout, stride, pad};
    hipStream_t st = as_stream(stream);
    const bf16_t* d = reinterpret_cast<const bf16_t*>(dy);
    if (cout == 16)
        hipLaunchKernelGGL((stem_bwd_wgrad_kernel<2, true>), dim3(STEM_WG_BLOCKS), dim3(256), 0, st, d, d_bs, d_ld, img,
                           nullptr, bnv, coef, workspace, g, z);
    else if (cout == 32)
        hipLaunchKernelGGL((stem_bwd_wgrad_kernel<4, true>), dim3(STEM_WG_BLOCKS), dim3(256), 0, st, d, d_bs, d_ld, img,
                           nullptr, bnv, coef, workspace, g, z);
    else
        hipLaunchKernelGGL((stem_bwd_wgrad_kernel<8, true>), dim3(STEM_WG_BLOCKS), dim3(256), 0, st, d, d_bs, d_ld, img,
                           nullptr, bnv, coef, workspace, g, z);
    colsum_launch(workspace, STEM_WG_BLOCKS, cout * 9, int64_t(cout) * 9, dw_oihw, 1, st);
    YM_LAUNCH_CHECK("ym_stem_bwd_wgrad_stored");
    return YM_OK;
}

extern "C" size_t ym_stem_bwd_wgrad_workspace_size(int cout) {
    return size_t(STEM_WG_BLOCKS) * size_t(cout > 0 ? cout : 0) * 9 * sizeof(float);
}
