// Training-mode BatchNorm2d + SiLU, forward and backward, NHWC bf16 (gfx950).
//
// Replaces BatchNorm2d (batch statistics, biased var for normalisation,
// unbiased var for the running estimate, eps 1e-3, momentum 0.03) and the
// shared in-place SiLU of Conv (/root/reference/yolo_scratch_cuda/models/
// yolo11_modules.py:24-33; eps/momentum set at yolo11_model.py:183-187).
//
// Forward (per Conv block): the conv epilogue emits per-block channel partial
// sums; bn_finalize reduces them in fp64 -> (scale, shift, mean, rstd) and
// updates running stats; bn_apply writes act(z*scale+shift) (+ residual) into
// the strided destination view (a concat slice).
// Backward: bn_bwd_reduce forms g = dy*act'(u) and per-block partials of
// sum(g), sum(g*xhat); bn_bwd_finalize -> dgamma, dbeta and the three apply
// coefficients; bn_bwd_apply writes dz = gamma*rstd*(g - mean(g) - xhat*mean(g*xhat)).
// Dtypes: z fp16, activations (out, residual) fp16, gradients (dy, dz) bf16.
#include <algorithm>

#include "common.h"

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
    for (int i = 0; i < 4; ++i) w[i] = uint32_t(f2h(f[2 * i])) | (uint32_t(f2h(f[2 * i + 1])) << 16);
    return make_uint4(w[0], w[1], w[2], w[3]);
}
__device__ __forceinline__ uint4 pack8(const float* f) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = uint32_t(f2bf(f[2 * i])) | (uint32_t(f2bf(f[2 * i + 1])) << 16);
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// grid: ceil(C/64) blocks of 1024 = 64 channels x 16 row groups
__global__ void __launch_bounds__(1024) bn_finalize_kernel(const float* __restrict__ ps, const float* __restrict__ pq,
                                                           int G, int C, double count, const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, float* running_mean,
                                                           float* running_var, int64_t* nbt, float momentum, float eps,
                                                           float* __restrict__ scale, float* __restrict__ shift,
                                                           float* __restrict__ mean_out, float* __restrict__ rstd_out) {
    __shared__ double sh[2][16][64];
    const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + cl;
    double s = 0.0, q = 0.0;
    if (c < C)
        for (int g = rg; g < G; g += 16) {
            s += ps[int64_t(g) * C + c];
            q += pq[int64_t(g) * C + c];
        }
    sh[0][rg][cl] = s;
    sh[1][rg][cl] = q;
    __syncthreads();
    if (rg == 0 && c < C) {
        for (int r = 1; r < 16; ++r) { s += sh[0][r][cl]; q += sh[1][r][cl]; }
        double mean = s / count;
        double var = q / count - mean * mean;
        if (var < 0) var = 0;
        double rstd = 1.0 / sqrt(var + double(eps));
        float sc = float(double(gamma[c]) * rstd);
        scale[c] = sc;
        shift[c] = float(double(beta[c]) - mean * double(sc));
        mean_out[c] = float(mean);
        rstd_out[c] = float(rstd);
        if (running_mean) {
            double unb = count > 1 ? var * count / (count - 1) : var;
            running_mean[c] = float((1.0 - momentum) * running_mean[c] + momentum * mean);
            running_var[c] = float((1.0 - momentum) * running_var[c] + momentum * unb);
        }
    }
    if (nbt && blockIdx.x == 0 && threadIdx.x == 0) *nbt += 1;
}

// eval: scale/shift from running stats
__global__ void bn_eval_coeff_kernel(int C, const float* gamma, const float* beta, const float* rm, const float* rv,
                                     float eps, float* scale, float* shift) {
    int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    float rstd = 1.0f / sqrtf(rv[c] + eps);
    float sc = gamma[c] * rstd;
    scale[c] = sc;
    shift[c] = beta[c] - rm[c] * sc;
}

// out[view] = act(z*scale + shift) (+ res[view]); z dense fp16 [M][C]; 8 channels per thread
__global__ void bn_apply_kernel(const bf16_t* __restrict__ z, int64_t M, int C, int HW, const float* __restrict__ scale,
                                const float* __restrict__ shift, int act, const bf16_t* __restrict__ res, int64_t r_bs,
                                int64_t r_ld, bf16_t* __restrict__ out, int64_t o_bs, int64_t o_ld,
                                float* __restrict__ out32) {
    const int cg = C / 8;
    const int64_t total = M * cg;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += int64_t(gridDim.x) * blockDim.x) {
        int g = int(i % cg);
        int64_t m = i / cg;
        int64_t n = m / HW, pix = m - n * HW;
        float v[8];
        unpack8h(*reinterpret_cast<const uint4*>(z + m * C + g * 8), v);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            float u = v[k] * scale[g * 8 + k] + shift[g * 8 + k];
            v[k] = act ? silu_f(u) : u;
        }
        if (res) {
            float r[8];
            unpack8h(*reinterpret_cast<const uint4*>(res + n * r_bs + pix * r_ld + g * 8), r);
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] += r[k];
        }
        *reinterpret_cast<uint4*>(out + n * o_bs + pix * o_ld + g * 8) = pack8h(v);
        if (out32) {
            float4* o = reinterpret_cast<float4*>(out32 + m * C + g * 8);
            o[0] = make_float4(v[0], v[1], v[2], v[3]);
            o[1] = make_float4(v[4], v[5], v[6], v[7]);
        }
    }
}

// per-block partials of sum(g) and sum(g*xhat); block = 256 threads = cg channel groups x rows
__global__ void __launch_bounds__(256) bn_bwd_reduce_kernel(const bf16_t* __restrict__ dy, int64_t d_bs, int64_t d_ld,
                                                            const bf16_t* __restrict__ z, int64_t M, int C, int HW,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ shift,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ rstd, int act,
                                                            float* __restrict__ ps, float* __restrict__ pg) {
    extern __shared__ float red[];   // [2][C]
    for (int i = threadIdx.x; i < 2 * C; i += blockDim.x) red[i] = 0.f;
    __syncthreads();
    const int cg = C / 8;
    const int rows = blockDim.x / cg;
    const int g = threadIdx.x % cg, r = threadIdx.x / cg;
    float s[8] = {0}, sx[8] = {0};
    if (r < rows) {
        float sc[8], sf[8], mu[8], rs[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            sc[k] = scale[g * 8 + k]; sf[k] = shift[g * 8 + k];
            mu[k] = mean[g * 8 + k]; rs[k] = rstd[g * 8 + k];
        }
        for (int64_t m = int64_t(blockIdx.x) * rows + r; m < M; m += int64_t(gridDim.x) * rows) {
            int64_t n = m / HW, pix = m - n * HW;
            float zv[8], dv[8];
            unpack8h(*reinterpret_cast<const uint4*>(z + m * C + g * 8), zv);
            unpack8(*reinterpret_cast<const uint4*>(dy + n * d_bs + pix * d_ld + g * 8), dv);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                float gg = dv[k];
                if (act) {
                    float u = zv[k] * sc[k] + sf[k];
                    float sg = 1.0f / (1.0f + __expf(-u));
                    gg *= sg * (1.0f + u * (1.0f - sg));
                }
                float xh = (zv[k] - mu[k]) * rs[k];
                s[k] += gg;
                sx[k] += gg * xh;
            }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            atomicAdd(&red[g * 8 + k], s[k]);
            atomicAdd(&red[C + g * 8 + k], sx[k]);
        }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        ps[int64_t(blockIdx.x) * C + c] = red[c];
        pg[int64_t(blockIdx.x) * C + c] = red[C + c];
    }
}

__global__ void __launch_bounds__(1024) bn_bwd_finalize_kernel(const float* __restrict__ ps, const float* __restrict__ pg,
                                                               int G, int C, double count,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ rstd, float* dgamma,
                                                               float* dbeta, int accumulate, float* __restrict__ coef) {
    __shared__ double sh[2][16][64];
    const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + cl;
    double s = 0.0, q = 0.0;
    if (c < C)
        for (int g = rg; g < G; g += 16) {
            s += ps[int64_t(g) * C + c];
            q += pg[int64_t(g) * C + c];
        }
    sh[0][rg][cl] = s;
    sh[1][rg][cl] = q;
    __syncthreads();
    if (rg == 0 && c < C) {
        for (int r = 1; r < 16; ++r) { s += sh[0][r][cl]; q += sh[1][r][cl]; }
        if (dgamma) dgamma[c] = float(accumulate ? dgamma[c] + q : q);
        if (dbeta) dbeta[c] = float(accumulate ? dbeta[c] + s : s);
        coef[c] = gamma[c] * rstd[c];               // k1
        coef[C + c] = float(s / count);             // k2 = mean(g)
        coef[2 * C + c] = float(q / count);         // k3 = mean(g * xhat)
    }
}

// dz[m][c] = k1*(g - k2 - xhat*k3), dz dense [M][C]
__global__ void bn_bwd_apply_kernel(const bf16_t* __restrict__ dy, int64_t d_bs, int64_t d_ld,
                                    const bf16_t* __restrict__ z, int64_t M, int C, int HW,
                                    const float* __restrict__ scale, const float* __restrict__ shift,
                                    const float* __restrict__ mean, const float* __restrict__ rstd, int act,
                                    const float* __restrict__ coef, bf16_t* __restrict__ dz) {
    const int cg = C / 8;
    const int64_t total = M * cg;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += int64_t(gridDim.x) * blockDim.x) {
        int g = int(i % cg);
        int64_t m = i / cg;
        int64_t n = m / HW, pix = m - n * HW;
        float zv[8], dv[8], o[8];
        unpack8h(*reinterpret_cast<const uint4*>(z + m * C + g * 8), zv);
        unpack8(*reinterpret_cast<const uint4*>(dy + n * d_bs + pix * d_ld + g * 8), dv);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            int c = g * 8 + k;
            float gg = dv[k];
            if (act) {
                float u = zv[k] * scale[c] + shift[c];
                float sg = 1.0f / (1.0f + __expf(-u));
                gg *= sg * (1.0f + u * (1.0f - sg));
            }
            float xh = (zv[k] - mean[c]) * rstd[c];
            o[k] = coef[c] * (gg - coef[C + c] - xh * coef[2 * C + c]);
        }
        *reinterpret_cast<uint4*>(dz + m * C + g * 8) = pack8(o);
    }
}

}  // namespace
}  // namespace ym

using namespace ym;

static int grid_for(int64_t work, int threads = 256, int cap = 4096) {
    int64_t g = (work + threads - 1) / threads;
    return int(std::max<int64_t>(1, std::min<int64_t>(g, cap)));
}

extern "C" int ym_bn_finalize(const float* part_sum, const float* part_sq, int parts, int c, double count,
                              const float* gamma, const float* beta, float* running_mean, float* running_var,
                              int64_t* num_batches_tracked, float momentum, float eps, float* scale, float* shift,
                              float* mean, float* rstd, void* stream) {
    YM_CHECK_ARG(count > 0, "ym_bn_finalize: count must be > 0");
    hipLaunchKernelGGL(bn_finalize_kernel, dim3((c + 63) / 64), dim3(1024), 0, as_stream(stream), part_sum, part_sq,
                       parts, c, count, gamma, beta, running_mean, running_var, num_batches_tracked, momentum, eps,
                       scale, shift, mean, rstd);
    YM_LAUNCH_CHECK("ym_bn_finalize");
    return YM_OK;
}

extern "C" int ym_bn_eval_coeff(int c, const float* gamma, const float* beta, const float* running_mean,
                                const float* running_var, float eps, float* scale, float* shift, void* stream) {
    hipLaunchKernelGGL(bn_eval_coeff_kernel, dim3((c + 255) / 256), dim3(256), 0, as_stream(stream), c, gamma, beta,
                       running_mean, running_var, eps, scale, shift);
    YM_LAUNCH_CHECK("ym_bn_eval_coeff");
    return YM_OK;
}

extern "C" int ym_bn_apply(const uint16_t* z, int64_t m, int c, int hw, const float* scale, const float* shift,
                           int act, const uint16_t* res, int64_t r_bs, int64_t r_ld, uint16_t* out, int64_t o_bs,
                           int64_t o_ld, float* out32, void* stream) {
    YM_CHECK_ARG(c % 8 == 0, "ym_bn_apply: C %% 8 != 0");
    YM_CHECK_ARG(o_ld % 8 == 0 && o_bs % 8 == 0 && (!res || (r_ld % 8 == 0 && r_bs % 8 == 0)),
                 "ym_bn_apply: views must be 16-byte aligned");
    if (m == 0) return YM_OK;
    hipLaunchKernelGGL(bn_apply_kernel, dim3(grid_for(m * (c / 8))), dim3(256), 0, as_stream(stream), z, m, c, hw,
                       scale, shift, act, res, r_bs, r_ld, out, o_bs, o_ld, out32);
    YM_LAUNCH_CHECK("ym_bn_apply");
    return YM_OK;
}

extern "C" int ym_bn_bwd_blocks(int64_t m, int c) {
    int rows = 256 / (c / 8);
    return grid_for((m + rows - 1) / rows, 1, 2048);
}

extern "C" int ym_bn_bwd_reduce(const uint16_t* dy, int64_t d_bs, int64_t d_ld, const uint16_t* z, int64_t m, int c,
                                int hw, const float* scale, const float* shift, const float* mean, const float* rstd,
                                int act, float* part_sum, float* part_dot, void* stream) {
    YM_CHECK_ARG(c % 8 == 0 && c / 8 <= 256, "ym_bn_bwd_reduce: C=%d unsupported", c);
    int blocks = ym_bn_bwd_blocks(m, c);
    hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(blocks), dim3(256), size_t(2 * c) * sizeof(float), as_stream(stream),
                       dy, d_bs, d_ld, z, m, c, hw, scale, shift, mean, rstd, act, part_sum, part_dot);
    YM_LAUNCH_CHECK("ym_bn_bwd_reduce");
    return YM_OK;
}

extern "C" int ym_bn_bwd_finalize(const float* part_sum, const float* part_dot, int parts, int c, double count,
                                  const float* gamma, const float* rstd, float* dgamma, float* dbeta, int accumulate,
                                  float* coef, void* stream) {
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((c + 63) / 64), dim3(1024), 0, as_stream(stream), part_sum,
                       part_dot, parts, c, count, gamma, rstd, dgamma, dbeta, accumulate, coef);
    YM_LAUNCH_CHECK("ym_bn_bwd_finalize");
    return YM_OK;
}

extern "C" int ym_bn_bwd_apply(const uint16_t* dy, int64_t d_bs, int64_t d_ld, const uint16_t* z, int64_t m, int c,
                               int hw, const float* scale, const float* shift, const float* mean, const float* rstd,
                               int act, const float* coef, uint16_t* dz, void* stream) {
    if (m == 0) return YM_OK;
    hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(grid_for(m * (c / 8))), dim3(256), 0, as_stream(stream), dy, d_bs,
                       d_ld, z, m, c, hw, scale, shift, mean, rstd, act, coef, dz);
    YM_LAUNCH_CHECK("ym_bn_bwd_apply");
    return YM_OK;
}
