// Non-GEMM graph ops of the YOLOv11 neck/backbone, NHWC bf16 (gfx950):
//   SPPF max-pool 5x5 s1 p2 fwd/bwd     (yolo11_modules.py:92-105)
//   nearest 2x upsample fwd/bwd         (configs/yolo11n_crater.yaml head rows 0, 3; nn.Upsample)
//   dtype/view conversions and the Detect-head gradient split (+ bias grads)
// Activation buffers are fp16, gradient buffers bf16 (see yolomi/graph.py).
#include <algorithm>

#include <cstdlib>

#include "common.h"
#include "reduce.h"

namespace ym {
namespace {

__device__ __forceinline__ void unpack8(uint4 v, float* f) {
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        f[2 * i] = bf2f(bf16_t(w[i] & 0xffff));
        f[2 * i + 1] = bf2f(bf16_t(w[i] >> 16));
    }
}
__device__ __forceinline__ uint4 pack8(const float* f) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = uint32_t(f2bf(f[2 * i])) | (uint32_t(f2bf(f[2 * i + 1])) << 16);
    return make_uint4(w[0], w[1], w[2], w[3]);
}
// activations are fp16, gradients bf16
__device__ __forceinline__ void unpack8h(uint4 v, float* f) {
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        f[2 * i] = h2f(uint16_t(w[i] & 0xffff));
        f[2 * i + 1] = h2f(uint16_t(w[i] >> 16));
    }
}
__device__ __forceinline__ uint4 pack8h(const float* f) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = pk2h(f[2 * i], f[2 * i + 1]);
    return make_uint4(w[0], w[1], w[2], w[3]);
}

int grid_for(int64_t work, int threads = 256, int cap = 8192) {
    int64_t g = (work + threads - 1) / threads;
    return int(std::max<int64_t>(1, std::min<int64_t>(g, cap)));
}

// ------------------------------------------------------------------ max pool 5x5, stride 1, pad 2 (SPPF)
// SPPF's chained pools run on fp32 values (the first-max routing of the backward must see the
// fp32 reference's ties).  Forward: one thread per (pixel, 4 channels), 32-bit index math; the
// window argmax (kh*5 + kw, first maximum in kh-major scan order, NaN wins as in ATen's CPU
// kernel) is kept as one byte per element so the backward is a gather instead of atomics.
__global__ void __launch_bounds__(256) maxpool5_f32_fwd_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                               uint8_t* __restrict__ code, uint16_t* __restrict__ yv,
                                                               int64_t y_bs, int64_t y_ld, int N, int H, int W, int C) {
    const int C4 = C >> 2;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= N * H * W * C4) return;
    const int c4 = i % C4, m = i / C4;
    const int HW = H * W, n = m / HW, pix = m - n * HW, h = pix / W, w = pix - h * W;
    float mx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    uint32_t cd[4] = {0, 0, 0, 0};
    bool first = true;
    for (int dh = -2; dh <= 2; ++dh) {
        const int ih = h + dh;
        if (ih < 0 || ih >= H) continue;
        for (int dw = -2; dw <= 2; ++dw) {
            const int iw = w + dw;
            if (iw < 0 || iw >= W) continue;
            const float4 v = *reinterpret_cast<const float4*>(x + (size_t(n * HW + ih * W + iw) * C + c4 * 4));
            const float vv[4] = {v.x, v.y, v.z, v.w};
            const uint32_t k = uint32_t((dh + 2) * 5 + dw + 2);
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (first || vv[r] > mx[r] || vv[r] != vv[r]) { mx[r] = vv[r]; cd[r] = k; }
            first = false;
        }
    }
    const size_t o = size_t(m) * C + c4 * 4;
    *reinterpret_cast<float4*>(y + o) = make_float4(mx[0], mx[1], mx[2], mx[3]);
    *reinterpret_cast<uint32_t*>(code + o) = cd[0] | (cd[1] << 8) | (cd[2] << 16) | (cd[3] << 24);
    uint2 hv;
    hv.x = pk2h(mx[0], mx[1]);
    hv.y = pk2h(mx[2], mx[3]);
    *reinterpret_cast<uint2*>(yv + n * y_bs + int64_t(pix) * y_ld + c4 * 4) = hv;
}

// dx[p] = init[p] + sum of dy[q] over the windows q whose argmax is p (gather, no atomics);
// out to a dense fp32 buffer and/or a bf16 gradient view (overwrite or accumulate)
__global__ void __launch_bounds__(256) maxpool5_f32_bwd_kernel(const uint8_t* __restrict__ code,
                                                               const float* __restrict__ dy,
                                                               const uint16_t* __restrict__ init, int64_t i_bs,
                                                               int64_t i_ld, float* __restrict__ dx,
                                                               uint16_t* __restrict__ dxv, int64_t v_bs, int64_t v_ld,
                                                               int accumulate, int N, int H, int W, int C) {
    const int C4 = C >> 2;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= N * H * W * C4) return;
    const int c4 = i % C4, m = i / C4;
    const int HW = H * W, n = m / HW, pix = m - n * HW, h = pix / W, w = pix - h * W;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int qh = h - 2; qh <= h + 2; ++qh) {
        if (qh < 0 || qh >= H) continue;
        for (int qw = w - 2; qw <= w + 2; ++qw) {
            if (qw < 0 || qw >= W) continue;
            const uint32_t want = uint32_t((h - qh + 2) * 5 + (w - qw + 2));
            const size_t o = size_t(n * HW + qh * W + qw) * C + c4 * 4;
            const uint32_t cq = *reinterpret_cast<const uint32_t*>(code + o);
            const bool hit[4] = {(cq & 0xff) == want, ((cq >> 8) & 0xff) == want, ((cq >> 16) & 0xff) == want,
                                 (cq >> 24) == want};
            if (hit[0] | hit[1] | hit[2] | hit[3]) {
                const float4 g = *reinterpret_cast<const float4*>(dy + o);
                acc[0] += hit[0] ? g.x : 0.f;
                acc[1] += hit[1] ? g.y : 0.f;
                acc[2] += hit[2] ? g.z : 0.f;
                acc[3] += hit[3] ? g.w : 0.f;
            }
        }
    }
    if (init) {
        const uint2 b = *reinterpret_cast<const uint2*>(init + n * i_bs + int64_t(pix) * i_ld + c4 * 4);
        acc[0] += bf2f(bf16_t(b.x & 0xffff)); acc[1] += bf2f(bf16_t(b.x >> 16));
        acc[2] += bf2f(bf16_t(b.y & 0xffff)); acc[3] += bf2f(bf16_t(b.y >> 16));
    }
    if (dx) *reinterpret_cast<float4*>(dx + size_t(m) * C + c4 * 4) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    if (dxv) {
        uint16_t* p = dxv + n * v_bs + int64_t(pix) * v_ld + c4 * 4;
        if (accumulate) {
            const uint2 b = *reinterpret_cast<const uint2*>(p);
            acc[0] += bf2f(bf16_t(b.x & 0xffff)); acc[1] += bf2f(bf16_t(b.x >> 16));
            acc[2] += bf2f(bf16_t(b.y & 0xffff)); acc[3] += bf2f(bf16_t(b.y >> 16));
        }
        *reinterpret_cast<uint2*>(p) = make_uint2(pk2bf(acc[0], acc[1]), pk2bf(acc[2], acc[3]));
    }
}

// LDS forms for maps that fit (SPPF runs on 1/32-scale maps: 10x10 .. 40x40): a block owns one
// image x CG channels of the whole map.  The forward is separable — row maxima first (first max in
// kw order, NaN wins), then the maximum of the five row results (first in kh order): the winner is
// the first maximum in kh-major scan order, the same element the direct 25-tap scan picks — so
// each input is read from HBM once and the window costs 10 LDS reads instead of 25 global ones.
// The backward stages the codes and dy of the map once and gathers in the same (qh, qw) order.
template <int CG>
__global__ void __launch_bounds__(256) maxpool5_lds_fwd_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                               uint8_t* __restrict__ code, uint16_t* __restrict__ yv,
                                                               int64_t y_bs, int64_t y_ld, int H, int W, int C) {
    extern __shared__ float sm[];
    const int HW = H * W, E = HW * CG;
    float* xs = sm;                                   // [HW][CG]
    float* rm = sm + E;                               // row maxima
    uint8_t* rk = reinterpret_cast<uint8_t*>(sm + 2 * E);   // their kw
    const int n = blockIdx.y, c0 = blockIdx.x * CG;
    const float* xb = x + (size_t(n) * HW) * C + c0;
    for (int e = threadIdx.x; e < E; e += 256) xs[e] = xb[size_t(e / CG) * C + (e % CG)];
    __syncthreads();
    for (int e = threadIdx.x; e < E; e += 256) {
        const int pix = e / CG, c = e % CG, h = pix / W, w = pix - h * W;
        float mx = 0.f;
        int k = 0;
        bool first = true;
#pragma unroll
        for (int dw = -2; dw <= 2; ++dw) {
            const int iw = w + dw;
            if (iw < 0 || iw >= W) continue;
            const float v = xs[(h * W + iw) * CG + c];
            if (first || v > mx || v != v) { mx = v; k = dw + 2; }
            first = false;
        }
        rm[e] = mx;
        rk[e] = uint8_t(k);
    }
    __syncthreads();
    for (int e = threadIdx.x; e < E; e += 256) {
        const int pix = e / CG, c = e % CG, h = pix / W, w = pix - h * W;
        float mx = 0.f;
        uint32_t cd = 0;
        bool first = true;
#pragma unroll
        for (int dh = -2; dh <= 2; ++dh) {
            const int ih = h + dh;
            if (ih < 0 || ih >= H) continue;
            const int q = (ih * W + w) * CG + c;
            const float v = rm[q];
            if (first || v > mx || v != v) { mx = v; cd = uint32_t((dh + 2) * 5) + rk[q]; }
            first = false;
        }
        const size_t o = (size_t(n) * HW + pix) * C + c0 + c;
        y[o] = mx;
        code[o] = uint8_t(cd);
        yv[n * y_bs + int64_t(pix) * y_ld + c0 + c] = f2h(mx);
    }
}

template <int CG>
__global__ void __launch_bounds__(256) maxpool5_lds_bwd_kernel(const uint8_t* __restrict__ code,
                                                               const float* __restrict__ dy,
                                                               const uint16_t* __restrict__ init, int64_t i_bs,
                                                               int64_t i_ld, float* __restrict__ dx,
                                                               uint16_t* __restrict__ dxv, int64_t v_bs, int64_t v_ld,
                                                               int accumulate, int H, int W, int C) {
    extern __shared__ float sm[];
    const int HW = H * W, E = HW * CG;
    float* gs = sm;                                   // [HW][CG] dy
    uint8_t* ks = reinterpret_cast<uint8_t*>(sm + E); // [HW][CG] codes
    const int n = blockIdx.y, c0 = blockIdx.x * CG;
    const size_t base = (size_t(n) * HW) * C + c0;
    for (int e = threadIdx.x; e < E; e += 256) {
        const size_t o = base + size_t(e / CG) * C + (e % CG);
        gs[e] = dy[o];
        ks[e] = code[o];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < E; e += 256) {
        const int pix = e / CG, c = e % CG, h = pix / W, w = pix - h * W;
        float acc = 0.f;
        for (int qh = h - 2; qh <= h + 2; ++qh) {
            if (qh < 0 || qh >= H) continue;
#pragma unroll
            for (int dq = -2; dq <= 2; ++dq) {
                const int qw = w + dq;
                if (qw < 0 || qw >= W) continue;
                const int q = (qh * W + qw) * CG + c;
                if (ks[q] == uint8_t((h - qh + 2) * 5 + (w - qw + 2))) acc += gs[q];
            }
        }
        if (init) acc += bf2f(bf16_t(init[n * i_bs + int64_t(pix) * i_ld + c0 + c]));
        if (dx) dx[base + size_t(pix) * C + c] = acc;
        if (dxv) {
            uint16_t* p = dxv + n * v_bs + int64_t(pix) * v_ld + c0 + c;
            if (accumulate) acc += bf2f(bf16_t(*p));
            *p = f2bf(acc);
        }
    }
}

// SPPF's three chained pools in ONE launch per direction (yolo11_modules.py:100-104): a block owns
// one image x CG channels of the map and keeps the chain in LDS — pool j+1 reads pool j's result
// where it was computed, so the fp32 intermediates never go to memory (the forward writes only the
// three argmax planes and the fp16 concat slices; the backward reads the three bf16 slice gradients
// and the codes and writes slice 0's).  Same window scans, tie rules and summation order as
// maxpool5_lds_fwd/bwd_kernel chained three times: bit-identical results.
template <int CG>
__global__ void __launch_bounds__(256) sppf_fwd_kernel(const float* __restrict__ x, uint8_t* __restrict__ code,
                                                       int64_t plane, uint16_t* __restrict__ y1,
                                                       uint16_t* __restrict__ y2, uint16_t* __restrict__ y3,
                                                       int64_t y_bs, int64_t y_ld, float* __restrict__ p_out, int H,
                                                       int W, int C) {
    extern __shared__ float sm[];
    const int HW = H * W, E = HW * CG;
    float* xs = sm;                                            // pool input   [HW][CG]
    float* ys = sm + E;                                        // pool output
    float* rm = sm + 2 * E;                                    // row maxima
    uint8_t* rk = reinterpret_cast<uint8_t*>(sm + 3 * E);      // their kw
    const int n = blockIdx.y, c0 = blockIdx.x * CG;
    const float* xb = x + (size_t(n) * HW) * C + c0;
    for (int e = threadIdx.x; e < E; e += 256) xs[e] = xb[size_t(e / CG) * C + (e % CG)];
    __syncthreads();
#pragma unroll 1
    for (int j = 0; j < 3; ++j) {
        uint16_t* yv = j == 0 ? y1 : j == 1 ? y2 : y3;
        for (int e = threadIdx.x; e < E; e += 256) {
            const int pix = e / CG, c = e % CG, h = pix / W, w = pix - h * W;
            float mx = 0.f;
            int k = 0;
            bool first = true;
#pragma unroll
            for (int dw = -2; dw <= 2; ++dw) {
                const int iw = w + dw;
                if (iw < 0 || iw >= W) continue;
                const float v = xs[(h * W + iw) * CG + c];
                if (first || v > mx || v != v) { mx = v; k = dw + 2; }
                first = false;
            }
            rm[e] = mx;
            rk[e] = uint8_t(k);
        }
        __syncthreads();
        for (int e = threadIdx.x; e < E; e += 256) {
            const int pix = e / CG, c = e % CG, h = pix / W, w = pix - h * W;
            float mx = 0.f;
            uint32_t cd = 0;
            bool first = true;
#pragma unroll
            for (int dh = -2; dh <= 2; ++dh) {
                const int ih = h + dh;
                if (ih < 0 || ih >= H) continue;
                const int q = (ih * W + w) * CG + c;
                const float v = rm[q];
                if (first || v > mx || v != v) { mx = v; cd = uint32_t((dh + 2) * 5) + rk[q]; }
                first = false;
            }
            const size_t o = (size_t(n) * HW + pix) * C + c0 + c;
            ys[e] = mx;
            code[j * plane + o] = uint8_t(cd);
            if (p_out) p_out[j * plane + o] = mx;
            yv[n * y_bs + int64_t(pix) * y_ld + c0 + c] = f2h(mx);
        }
        __syncthreads();
        float* t = xs; xs = ys; ys = t;
    }
}

template <int CG>
__global__ void __launch_bounds__(256) sppf_bwd_kernel(const uint8_t* __restrict__ code, int64_t plane,
                                                       const uint16_t* __restrict__ g1, const uint16_t* __restrict__ g2,
                                                       const uint16_t* __restrict__ g3, int64_t g_bs, int64_t g_ld,
                                                       uint16_t* __restrict__ dxv, int64_t v_bs, int64_t v_ld,
                                                       int accumulate, float* __restrict__ dx32, int H, int W, int C) {
    extern __shared__ float sm[];
    const int HW = H * W, E = HW * CG;
    float* gs = sm;                                            // routed gradient of the current pool output
    float* ns = sm + E;                                        // the next one
    uint8_t* ks = reinterpret_cast<uint8_t*>(sm + 2 * E);      // the current pool's codes
    const int n = blockIdx.y, c0 = blockIdx.x * CG;
    const size_t base = (size_t(n) * HW) * C + c0;
    for (int e = threadIdx.x; e < E; e += 256) {
        const int pix = e / CG, c = e % CG;
        gs[e] = bf2f(bf16_t(g3[n * g_bs + int64_t(pix) * g_ld + c0 + c]));
        ks[e] = code[2 * plane + base + size_t(pix) * C + c];
    }
    __syncthreads();
#pragma unroll 1
    for (int j = 2; j >= 0; --j) {
        const uint16_t* init = j == 2 ? g2 : j == 1 ? g1 : nullptr;
        for (int e = threadIdx.x; e < E; e += 256) {
            const int pix = e / CG, c = e % CG, h = pix / W, w = pix - h * W;
            float acc = 0.f;
            for (int qh = h - 2; qh <= h + 2; ++qh) {
                if (qh < 0 || qh >= H) continue;
#pragma unroll
                for (int dq = -2; dq <= 2; ++dq) {
                    const int qw = w + dq;
                    if (qw < 0 || qw >= W) continue;
                    const int q = (qh * W + qw) * CG + c;
                    if (ks[q] == uint8_t((h - qh + 2) * 5 + (w - qw + 2))) acc += gs[q];
                }
            }
            if (init) acc += bf2f(bf16_t(init[n * g_bs + int64_t(pix) * g_ld + c0 + c]));
            if (j > 0) {
                ns[e] = acc;
            } else {
                if (dx32) dx32[base + size_t(pix) * C + c] = acc;
                uint16_t* p = dxv + n * v_bs + int64_t(pix) * v_ld + c0 + c;
                if (accumulate) acc += bf2f(bf16_t(*p));
                *p = f2bf(acc);
            }
        }
        __syncthreads();
        if (j > 0) {
            float* t = gs; gs = ns; ns = t;
            for (int e = threadIdx.x; e < E; e += 256) ks[e] = code[(j - 1) * plane + base + size_t(e / CG) * C + (e % CG)];
            __syncthreads();
        }
    }
}

// channels per block of the fused chain (0: the map does not fit, use the per-pool launches): the
// forward on 8-channel blocks where they fit, the backward on 4-channel blocks (measured at s@640
// 64x20x20x256: 232 / 154 us on 8 / 4 channels — its three dependent gather levels per block want
// more blocks per CU; 2-channel blocks 175 us)
int sppf_cg(int h, int w, int c) {
    const int64_t hw = int64_t(h) * w;
    if (c % 8 == 0 && hw * 8 * 13 <= 96 * 1024) return 8;
    if (c % 4 == 0 && hw * 4 * 13 <= 96 * 1024) return 4;
    return 0;
}
int sppf_cg_bwd(int h, int w, int c) { return sppf_cg(h, w, c) ? 4 : 0; }
// the forward's channels per block for n images: narrower blocks until the grid holds ~256 of them (bs 1 at 20x20 x 256
// channels ran 32 blocks of 8: 37 us; every (pixel, channel) is computed alone, so the width changes no result)
static int sppf_cg_fwd(int n, int h, int w, int c) {
    int cg = sppf_cg(h, w, c);
    while (cg > 1 && int64_t(n) * (c / cg) < 256) cg >>= 1;
    return cg;
}

// channels per block of the LDS forms (0: the map does not fit, use the direct kernels)
int pool_cg(int h, int w, int c) {
    const int64_t hw = int64_t(h) * w;
    if (c % 8 == 0 && hw * 8 * 9 <= 64 * 1024) return 8;
    if (c % 4 == 0 && hw * 4 * 9 <= 64 * 1024) return 4;
    return 0;
}

// ------------------------------------------------------------------ nearest 2x upsample
__global__ void upsample2_fwd_kernel(const bf16_t* __restrict__ x, int64_t x_bs, int64_t x_ld, bf16_t* __restrict__ y,
                                     int64_t y_bs, int64_t y_ld, int N, int H, int W, int C) {
    const int cg = C / 8, OH = 2 * H, OW = 2 * W;
    const int64_t total = int64_t(N) * OH * OW * cg;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += int64_t(gridDim.x) * blockDim.x) {
        int g = int(i % cg);
        int64_t m = i / cg;
        int64_t n = m / (int64_t(OH) * OW), pix = m - n * OH * OW;
        int oh = int(pix / OW), ow = int(pix % OW);
        uint4 v = *reinterpret_cast<const uint4*>(x + n * x_bs + (int64_t(oh >> 1) * W + (ow >> 1)) * x_ld + g * 8);
        *reinterpret_cast<uint4*>(y + n * y_bs + pix * y_ld + g * 8) = v;
    }
}

__global__ void upsample2_bwd_kernel(const bf16_t* __restrict__ dy, int64_t d_bs, int64_t d_ld, bf16_t* __restrict__ dx,
                                     int64_t x_bs, int64_t x_ld, int N, int H, int W, int C, int accumulate) {
    const int cg = C / 8, OW = 2 * W;
    const int64_t total = int64_t(N) * H * W * cg;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += int64_t(gridDim.x) * blockDim.x) {
        int g = int(i % cg);
        int64_t m = i / cg;
        int64_t n = m / (int64_t(H) * W), pix = m - n * H * W;
        int h = int(pix / W), w = int(pix % W);
        float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int a = 0; a < 2; ++a)
            for (int b = 0; b < 2; ++b) {
                float v[8];
                unpack8(*reinterpret_cast<const uint4*>(dy + n * d_bs + (int64_t(2 * h + a) * OW + 2 * w + b) * d_ld + g * 8), v);
#pragma unroll
                for (int k = 0; k < 8; ++k) s[k] += v[k];
            }
        bf16_t* o = dx + n * x_bs + pix * x_ld + g * 8;
        if (accumulate) {
            float v[8];
            unpack8(*reinterpret_cast<const uint4*>(o), v);
#pragma unroll
            for (int k = 0; k < 8; ++k) s[k] += v[k];
        }
        *reinterpret_cast<uint4*>(o) = pack8(s);
    }
}

// ------------------------------------------------------------------ conversions
__global__ void view_to_f32_kernel(const bf16_t* __restrict__ x, int64_t bs, int64_t ld, float* __restrict__ y,
                                   int64_t M, int C, int HW) {
    const int cg = C / 8;
    const int64_t total = M * cg;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += int64_t(gridDim.x) * blockDim.x) {
        int g = int(i % cg);
        int64_t m = i / cg, n = m / HW, pix = m - n * HW;
        float v[8];
        unpack8(*reinterpret_cast<const uint4*>(x + n * bs + pix * ld + g * 8), v);
        float4* o = reinterpret_cast<float4*>(y + m * C + g * 8);
        o[0] = make_float4(v[0], v[1], v[2], v[3]);
        o[1] = make_float4(v[4], v[5], v[6], v[7]);
    }
}

__global__ void f32_to_view_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, int64_t bs, int64_t ld,
                                   int64_t M, int C, int HW, int accumulate) {
    const int cg = C / 8;
    const int64_t total = M * cg;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += int64_t(gridDim.x) * blockDim.x) {
        int g = int(i % cg);
        int64_t m = i / cg, n = m / HW, pix = m - n * HW;
        const float4* s = reinterpret_cast<const float4*>(x + m * C + g * 8);
        float4 a = s[0], b = s[1];
        float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        bf16_t* o = y + n * bs + pix * ld + g * 8;
        if (accumulate) {
            float u[8];
            unpack8(*reinterpret_cast<const uint4*>(o), u);
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] += u[k];
        }
        *reinterpret_cast<uint4*>(o) = pack8(v);
    }
}

// dst_view = src_view (+ dst_view); zero-fill when src is null
__global__ void view_axpy_kernel(const bf16_t* __restrict__ x, int64_t x_bs, int64_t x_ld, bf16_t* __restrict__ y,
                                 int64_t y_bs, int64_t y_ld, int64_t M, int C, int HW, int accumulate, int half) {
    const int cg = C / 8;
    const int64_t total = M * cg;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += int64_t(gridDim.x) * blockDim.x) {
        int g = int(i % cg);
        int64_t m = i / cg, n = m / HW, pix = m - n * HW;
        bf16_t* o = y + n * y_bs + pix * y_ld + g * 8;
        if (!x) { *reinterpret_cast<uint4*>(o) = make_uint4(0, 0, 0, 0); continue; }
        uint4 v = *reinterpret_cast<const uint4*>(x + n * x_bs + pix * x_ld + g * 8);
        if (accumulate) {
            float a[8], b[8];
            if (half) { unpack8h(v, a); unpack8h(*reinterpret_cast<const uint4*>(o), b); }
            else { unpack8(v, a); unpack8(*reinterpret_cast<const uint4*>(o), b); }
#pragma unroll
            for (int k = 0; k < 8; ++k) a[k] += b[k];
            v = half ? pack8h(a) : pack8(a);
        }
        *reinterpret_cast<uint4*>(o) = v;
    }
}

// ------------------------------------------------------------------ Detect head gradient split
// dhead (B, A, 64+nc) fp32 rows for one level (anchor offset `aoff`, HW anchors per image) ->
// dz_box bf16 [M][64], dz_cls bf16 [M][ncp] (ncp = nc rounded up to 8, zero padded), and per-block bias-gradient
// partials part[blockIdx.x][64 + ncp] (summed in a fixed order by colsum_kernel; no atomics).
// A pixel is G = 8 + ncp / 8 groups of 8 channels; thread t < S * G (S = 256 / G pixel slots per block pass) owns
// group t % G of slot t / G (nc <= 8: G 9, S 28).
__global__ void __launch_bounds__(256) head_grad_kernel(const float* __restrict__ dh, int64_t A, int64_t aoff, int HW,
                                                        int64_t M, int nc, bf16_t* __restrict__ dbox,
                                                        bf16_t* __restrict__ dcls, float* __restrict__ part) {
    __shared__ float red[256][9];            // [thread][8 sums] (+1 pad)
    const int ncp = (nc + 7) & ~7, G = 8 + ncp / 8, S = 256 / G, ncol = 64 + ncp;
    const int t = threadIdx.x, g = t % G, slot = t / G;
    const int no = 64 + nc;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (t < S * G) {
        for (int64_t m = int64_t(blockIdx.x) * S + slot; m < M; m += int64_t(gridDim.x) * S) {
            const int64_t n = m / HW, pix = m - n * HW;
            const float* row = dh + (n * A + aoff + pix) * no;
            float v[8];
            if (g < 8) {
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] = row[g * 8 + k];     // rows of 64+nc floats: 4-B aligned
                *reinterpret_cast<uint4*>(dbox + m * 64 + g * 8) = pack8(v);
            } else {
                const int c0 = (g - 8) * 8;
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] = c0 + k < nc ? row[64 + c0 + k] : 0.f;
                *reinterpret_cast<uint4*>(dcls + m * ncp + c0) = pack8(v);
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[k] += v[k];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) red[t][k] = acc[k];
    }
    __syncthreads();
    for (int col = t; col < ncol; col += blockDim.x) {     // column = group * 8 + k: sum the S slots in order
        const int gg = col >> 3, k = col & 7;
        float s = 0.f;
        for (int sl = 0; sl < S; ++sl) s += red[sl * G + gg][k];
        part[int64_t(blockIdx.x) * ncol + col] = s;
    }
}

// out[j] (+)= sum_r part[r * ld + j] (deterministic; fp32): a block takes 64 columns, its 4 waves
// the rows r = wave (mod 4) with 16 loads in flight per lane, then the 4 wave sums in wave order
__global__ void __launch_bounds__(256) colsum_kernel(const float* __restrict__ part, int rows, int n, int64_t ld,
                                                     float* __restrict__ out, int accumulate) {
    __shared__ float red[4][64];
    const int c = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int j = blockIdx.x * 64 + c;
    float s = 0.f;
    if (j < n) {
        int r = w;
        for (; r + 4 * 15 < rows; r += 4 * 16) {
            float v[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) v[u] = part[int64_t(r + 4 * u) * ld + j];
#pragma unroll
            for (int u = 0; u < 16; ++u) s += v[u];
        }
        for (; r < rows; r += 4) s += part[int64_t(r) * ld + j];
    }
    red[w][c] = s;
    __syncthreads();
    if (w == 0 && j < n) {
        const float t = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
        out[j] = accumulate ? out[j] + t : t;
    }
}

}  // namespace

int colsum_launch(const float* part, int rows, int n, int64_t ld, float* out, int accumulate, hipStream_t st) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(colsum_kernel, dim3((n + 63) / 64), dim3(256), 0, st, part, rows, n, ld, out, accumulate);
    return 0;
}

}  // namespace ym

using namespace ym;

#define VIEW_ALIGNED(bs, ld) ((bs) % 8 == 0 && (ld) % 8 == 0)

extern "C" int ym_maxpool5_f32_fwd(const float* x, float* y, uint8_t* code, uint16_t* yv, int64_t y_bs,
                                   int64_t y_ld, int n, int h, int w, int c, void* stream) {
    YM_CHECK_ARG(x && y && code && yv, "ym_maxpool5_f32_fwd: null argument");
    YM_CHECK_ARG(c % 4 == 0 && y_bs % 4 == 0 && y_ld % 4 == 0, "ym_maxpool5_f32_fwd: alignment");
    const int64_t t = int64_t(n) * h * w * (c / 4);
    YM_CHECK_ARG(int64_t(n) * h * w * c < (int64_t(1) << 31), "ym_maxpool5_f32_fwd: too large");
    if (t == 0) return YM_OK;
    const int cg = pool_cg(h, w, c);
    const size_t lds = size_t(h) * w * cg * 9;
    if (cg == 8)
        hipLaunchKernelGGL(maxpool5_lds_fwd_kernel<8>, dim3(unsigned(c / 8), unsigned(n)), dim3(256), lds,
                           as_stream(stream), x, y, code, yv, y_bs, y_ld, h, w, c);
    else if (cg == 4)
        hipLaunchKernelGGL(maxpool5_lds_fwd_kernel<4>, dim3(unsigned(c / 4), unsigned(n)), dim3(256), lds,
                           as_stream(stream), x, y, code, yv, y_bs, y_ld, h, w, c);
    else
        hipLaunchKernelGGL(maxpool5_f32_fwd_kernel, dim3(unsigned((t + 255) / 256)), dim3(256), 0, as_stream(stream),
                           x, y, code, yv, y_bs, y_ld, n, h, w, c);
    YM_LAUNCH_CHECK("ym_maxpool5_f32_fwd");
    return YM_OK;
}

extern "C" int ym_maxpool5_f32_bwd(const uint8_t* code, const float* dy, const uint16_t* init, int64_t i_bs,
                                   int64_t i_ld, float* dx, uint16_t* dxv, int64_t v_bs, int64_t v_ld, int accumulate,
                                   int n, int h, int w, int c, void* stream) {
    YM_CHECK_ARG(code && dy && (dx || dxv), "ym_maxpool5_f32_bwd: null argument");
    YM_CHECK_ARG(c % 4 == 0 && i_bs % 4 == 0 && i_ld % 4 == 0 && v_bs % 4 == 0 && v_ld % 4 == 0,
                 "ym_maxpool5_f32_bwd: alignment");
    const int64_t t = int64_t(n) * h * w * (c / 4);
    YM_CHECK_ARG(int64_t(n) * h * w * c < (int64_t(1) << 31), "ym_maxpool5_f32_bwd: too large");
    if (t == 0) return YM_OK;
    const int cg = pool_cg(h, w, c);
    const size_t lds = size_t(h) * w * cg * 5;
    if (cg == 8)
        hipLaunchKernelGGL(maxpool5_lds_bwd_kernel<8>, dim3(unsigned(c / 8), unsigned(n)), dim3(256), lds,
                           as_stream(stream), code, dy, init, i_bs, i_ld, dx, dxv, v_bs, v_ld, accumulate, h, w, c);
    else if (cg == 4)
        hipLaunchKernelGGL(maxpool5_lds_bwd_kernel<4>, dim3(unsigned(c / 4), unsigned(n)), dim3(256), lds,
                           as_stream(stream), code, dy, init, i_bs, i_ld, dx, dxv, v_bs, v_ld, accumulate, h, w, c);
    else
        hipLaunchKernelGGL(maxpool5_f32_bwd_kernel, dim3(unsigned((t + 255) / 256)), dim3(256), 0, as_stream(stream),
                           code, dy, init, i_bs, i_ld, dx, dxv, v_bs, v_ld, accumulate, n, h, w, c);
    YM_LAUNCH_CHECK("ym_maxpool5_f32_bwd");
    return YM_OK;
}

extern "C" int ym_sppf_supported(int h, int w, int c) { return sppf_cg(h, w, c) != 0; }

extern "C" int ym_sppf_fwd(const float* x, uint8_t* code, uint16_t* y1, uint16_t* y2, uint16_t* y3, int64_t y_bs,
                           int64_t y_ld, float* p_out, int n, int h, int w, int c, void* stream) {
    YM_CHECK_ARG(x && code && y1 && y2 && y3, "ym_sppf_fwd: null argument");
    const int cg = sppf_cg_fwd(n, h, w, c);
    YM_CHECK_ARG(cg != 0, "ym_sppf_fwd: map %dx%d x %d channels does not fit the fused kernel", h, w, c);
    YM_CHECK_ARG(int64_t(n) * h * w * c < (int64_t(1) << 31), "ym_sppf_fwd: too large");
    if (n == 0) return YM_OK;
    const int64_t plane = int64_t(n) * h * w * c;
    const size_t lds = size_t(h) * w * cg * 13;
    const dim3 grid(unsigned(c / cg), unsigned(n));
    if (cg == 8)
        hipLaunchKernelGGL(sppf_fwd_kernel<8>, grid, dim3(256), lds, as_stream(stream), x, code, plane, y1, y2, y3, y_bs,
                           y_ld, p_out, h, w, c);
    else if (cg == 4)
        hipLaunchKernelGGL(sppf_fwd_kernel<4>, grid, dim3(256), lds, as_stream(stream), x, code, plane, y1, y2, y3, y_bs,
                           y_ld, p_out, h, w, c);
    else if (cg == 2)
        hipLaunchKernelGGL(sppf_fwd_kernel<2>, grid, dim3(256), lds, as_stream(stream), x, code, plane, y1, y2, y3, y_bs,
                           y_ld, p_out, h, w, c);
    else
        hipLaunchKernelGGL(sppf_fwd_kernel<1>, grid, dim3(256), lds, as_stream(stream), x, code, plane, y1, y2, y3, y_bs,
                           y_ld, p_out, h, w, c);
    YM_LAUNCH_CHECK("ym_sppf_fwd");
    return YM_OK;
}

extern "C" int ym_sppf_bwd(const uint8_t* code, const uint16_t* g1, const uint16_t* g2, const uint16_t* g3,
                           int64_t g_bs, int64_t g_ld, uint16_t* dxv, int64_t v_bs, int64_t v_ld, int accumulate,
                           float* dx32, int n, int h, int w, int c, void* stream) {
    YM_CHECK_ARG(code && g1 && g2 && g3 && dxv, "ym_sppf_bwd: null argument");
    const int cg = sppf_cg_bwd(h, w, c);
    YM_CHECK_ARG(cg != 0, "ym_sppf_bwd: map %dx%d x %d channels does not fit the fused kernel", h, w, c);
    YM_CHECK_ARG(int64_t(n) * h * w * c < (int64_t(1) << 31), "ym_sppf_bwd: too large");
    if (n == 0) return YM_OK;
    const int64_t plane = int64_t(n) * h * w * c;
    const size_t lds = size_t(h) * w * cg * 9;
    hipLaunchKernelGGL(sppf_bwd_kernel<4>, dim3(unsigned(c / 4), unsigned(n)), dim3(256), lds, as_stream(stream), code,
                       plane, g1, g2, g3, g_bs, g_ld, dxv, v_bs, v_ld, accumulate, dx32, h, w, c);
    YM_LAUNCH_CHECK("ym_sppf_bwd");
    return YM_OK;
}

extern "C" int ym_upsample2_fwd(const uint16_t* x, int64_t x_bs, int64_t x_ld, uint16_t* y, int64_t y_bs, int64_t y_ld,
                                int n, int h, int w, int c, void* stream) {
    YM_CHECK_ARG(c % 8 == 0 && VIEW_ALIGNED(x_bs, x_ld) && VIEW_ALIGNED(y_bs, y_ld), "ym_upsample2_fwd: alignment");
    hipLaunchKernelGGL(upsample2_fwd_kernel, dim3(grid_for(int64_t(n) * 4 * h * w * (c / 8))), dim3(256), 0,
                       as_stream(stream), x, x_bs, x_ld, y, y_bs, y_ld, n, h, w, c);
    YM_LAUNCH_CHECK("ym_upsample2_fwd");
    return YM_OK;
}

extern "C" int ym_upsample2_bwd(const uint16_t* dy, int64_t d_bs, int64_t d_ld, uint16_t* dx, int64_t x_bs,
                                int64_t x_ld, int n, int h, int w, int c, int accumulate, void* stream) {
    YM_CHECK_ARG(c % 8 == 0 && VIEW_ALIGNED(d_bs, d_ld) && VIEW_ALIGNED(x_bs, x_ld), "ym_upsample2_bwd: alignment");
    hipLaunchKernelGGL(upsample2_bwd_kernel, dim3(grid_for(int64_t(n) * h * w * (c / 8))), dim3(256), 0,
                       as_stream(stream), dy, d_bs, d_ld, dx, x_bs, x_ld, n, h, w, c, accumulate);
    YM_LAUNCH_CHECK("ym_upsample2_bwd");
    return YM_OK;
}

extern "C" int ym_view_axpy(const uint16_t* x, int64_t x_bs, int64_t x_ld, uint16_t* y, int64_t y_bs, int64_t y_ld,
                            int64_t m, int c, int hw, int accumulate, int half, void* stream) {
    YM_CHECK_ARG(c % 8 == 0 && VIEW_ALIGNED(y_bs, y_ld) && (!x || VIEW_ALIGNED(x_bs, x_ld)), "ym_view_axpy: alignment");
    if (m == 0) return YM_OK;
    hipLaunchKernelGGL(view_axpy_kernel, dim3(grid_for(m * (c / 8))), dim3(256), 0, as_stream(stream), x, x_bs, x_ld, y,
                       y_bs, y_ld, m, c, hw, accumulate, half);
    YM_LAUNCH_CHECK("ym_view_axpy");
    return YM_OK;
}

extern "C" int ym_view_to_f32(const uint16_t* x, int64_t bs, int64_t ld, float* y, int64_t m, int c, int hw,
                              void* stream) {
    YM_CHECK_ARG(c % 8 == 0 && VIEW_ALIGNED(bs, ld), "ym_view_to_f32: alignment");
    hipLaunchKernelGGL(view_to_f32_kernel, dim3(grid_for(m * (c / 8))), dim3(256), 0, as_stream(stream), x, bs, ld, y, m,
                       c, hw);
    YM_LAUNCH_CHECK("ym_view_to_f32");
    return YM_OK;
}

extern "C" int ym_f32_to_view(const float* x, uint16_t* y, int64_t bs, int64_t ld, int64_t m, int c, int hw,
                              int accumulate, void* stream) {
    YM_CHECK_ARG(c % 8 == 0 && VIEW_ALIGNED(bs, ld), "ym_f32_to_view: alignment");
    hipLaunchKernelGGL(f32_to_view_kernel, dim3(grid_for(m * (c / 8))), dim3(256), 0, as_stream(stream), x, y, bs, ld, m,
                       c, hw, accumulate);
    YM_LAUNCH_CHECK("ym_f32_to_view");
    return YM_OK;
}

constexpr int HEAD_GRAD_MAX_NC = 1024;
// sized for the largest class count (512 x 1088 floats, 2.2 MB)
extern "C" size_t ym_head_grad_workspace_size(void) {
    return size_t(PARTIAL_BLOCKS) * (64 + HEAD_GRAD_MAX_NC) * sizeof(float);
}

extern "C" int ym_head_grad(const float* dhead, int64_t a_total, int64_t a_off, int hw, int64_t m, int nc,
                            uint16_t* dz_box, uint16_t* dz_cls, float* dbias_box, float* dbias_cls, float* workspace,
                            size_t workspace_bytes, void* stream) {
    YM_CHECK_ARG(nc >= 1 && nc <= HEAD_GRAD_MAX_NC, "ym_head_grad: nc=%d out of range (1..1024)", nc);
    YM_CHECK_ARG(workspace && workspace_bytes >= ym_head_grad_workspace_size(), "ym_head_grad: workspace too small");
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(head_grad_kernel, dim3(PARTIAL_BLOCKS), dim3(256), 0, st, dhead, a_total, a_off, hw, m, nc,
                       dz_box, dz_cls, workspace);
    const int ncol = 64 + ((nc + 7) & ~7);
    if (dbias_box) colsum_launch(workspace, PARTIAL_BLOCKS, 64, ncol, dbias_box, 1, st);
    if (dbias_cls) colsum_launch(workspace + 64, PARTIAL_BLOCKS, nc, ncol, dbias_cls, 1, st);
    YM_LAUNCH_CHECK("ym_head_grad");
    return YM_OK;
}


extern "C" int ym_copy2d(void* dst, int64_t dst_pitch, const void* src, int64_t src_pitch, int64_t width_bytes,
                         int64_t rows, void* stream) {
    YM_CHECK_ARG(width_bytes >= 0 && rows >= 0 && dst_pitch >= width_bytes && src_pitch >= width_bytes,
                 "ym_copy2d: bad pitches");
    if (width_bytes == 0 || rows == 0) return YM_OK;
    if (hipMemcpy2DAsync(dst, size_t(dst_pitch), src, size_t(src_pitch), size_t(width_bytes), size_t(rows),
                         hipMemcpyDeviceToDevice, as_stream(stream)) != hipSuccess)
    {
        ym::set_error("ym_copy2d: hipMemcpy2DAsync failed");
        return YM_ERR_HIP;
    }
    return YM_OK;
}
