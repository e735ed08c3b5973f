// Training-mode BatchNorm2d + SiLU, forward and backward, NHWC (gfx950).
//
// Replaces BatchNorm2d (batch statistics, biased var for normalisation,
// unbiased var for the running estimate, eps 1e-3, momentum 0.03) and the
// shared in-place SiLU of Conv (/root/reference/yolo_scratch_cuda/models/
// yolo11_modules.py:24-33; eps/momentum set at yolo11_model.py:183-187).
//
// Forward (per Conv block): the conv epilogue emits per-block channel partial
// sums; bn_finalize reduces them (fp64, two levels) -> (scale, shift, mean,
// rstd) and updates running stats; bn_apply writes act(z*scale+shift)
// (+ residual) into the strided destination view (a concat slice).
// Backward: bn_bwd_reduce forms g = dy*act'(u) and per-block partials of
// sum(g), sum(g*xhat); bn_bwd_finalize -> dgamma, dbeta and the three apply
// coefficients; bn_bwd_apply writes dz = gamma*rstd*(g - mean(g) - xhat*mean(g*xhat)).
// Dtypes: z fp16, activations (out, residual) fp16, gradients (dy, dz) bf16.
//
// Streaming kernels: a 256-thread block covers rows x (C/8) lanes, each thread
// owns 8 consecutive channels (16-B loads/stores) of one pixel per iteration
// and keeps its channels' parameters in registers; every activation view is a
// whole (B, H, W, ld) buffer, so pixel m lives at m*ld (no integer division).
#include <algorithm>
#include <cstdlib>

#include "common.h"

// The one-launch finalize's hand-off (below) rests on relaxed agent-scope atomics being lowered to
// `sc1` vector stores / loads and on vmcnt(0) + barrier + an agent fetch_add ordering them, as
// MI355X_MICROARCH.md's "valid forms" table records for gfx950 / ROCm 7.2; no other target was checked.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "bn.hip: the fence-free finalize hand-off is verified on gfx950 only"
#endif

namespace ym {
namespace {

// write-through store / L1-bypassing load of hand-off data (sc1 vector memory operations)
__device__ __forceinline__ void st_wt(double* p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_wt(const double* p) {
    return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

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
    for (int i = 0; i < 4; ++i) w[i] = pk2h(f[2 * i], f[2 * i + 1]);
    return make_uint4(w[0], w[1], w[2], w[3]);
}
__device__ __forceinline__ uint4 pack8(const float* f) {
    return make_uint4(pk2bf(f[0], f[1]), pk2bf(f[2], f[3]), pk2bf(f[4], f[5]), pk2bf(f[6], f[7]));
}
__device__ __forceinline__ void load8(const float* p, float* v) {
    float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ float dsilu(float u) {
    const float sg = __builtin_amdgcn_rcpf(1.0f + __expf(-u));
    return sg * (1.0f + u * (1.0f - sg));
}

// ---------------------------------------------------------------- one-launch finalize
// Level 1 of the partials reduction (grid (ceil(C/64), R)) and the finalize in ONE launch: every
// level-1 block publishes its fp64 row, takes a ticket on its channel group's counter, and the
// block drawing the last ticket folds the R rows and runs the finalize (forward: scale / shift /
// mean / rstd / running stats; backward: dgamma / dbeta / apply coefficients) and re-arms the
// counter.  Hand-off per MI355X_MICROARCH.md (inter-workgroup visibility, "valid forms"): the fp64
// rows stored write-through (sc1) -> every wave vmcnt(0) -> barrier -> lane 0 relaxed agent
// fetch_add; the last arriver: barrier -> sc1 loads.  (The earlier agent release + acquire fences
// cost ≈1.7 us each on this launch-latency-bound kernel, 154 launches per step.)
// Deterministic: the fold reads the rows in a fixed order whatever order the blocks finished in.
template <bool BWD>
__global__ void __launch_bounds__(256) bn_finalize_fused_kernel(
    const float* __restrict__ a, const float* __restrict__ bsq, int G, int C, int R, double count, double* p2,
    unsigned* counters, const float* __restrict__ gamma, const float* __restrict__ beta, float* running_mean,
    float* running_var, int64_t* nbt, float momentum, float eps, float* scale, float* shift, float* mean_out,
    float* rstd_out, const float* __restrict__ rstd_in, float* dgamma, float* dbeta, int accumulate, float* coef) {
    __shared__ double sh[2][4][64];
    __shared__ int last_sh;
    const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + cl;
    const int per = (G + R - 1) / R;
    const int g0 = blockIdx.y * per, g1 = min(G, g0 + per);
    double s = 0.0, q = 0.0;
    if (c < C) {
#pragma unroll 4
        for (int g = g0 + rg; g < g1; g += 4) {
            s += a[int64_t(g) * C + c];
            q += bsq[int64_t(g) * C + c];
        }
    }
    sh[0][rg][cl] = s;
    sh[1][rg][cl] = q;
    __syncthreads();
    if (rg == 0 && c < C) {
        st_wt(&p2[(int64_t(blockIdx.y) * 2 + 0) * C + c], sh[0][0][cl] + sh[0][1][cl] + sh[0][2][cl] + sh[0][3][cl]);
        st_wt(&p2[(int64_t(blockIdx.y) * 2 + 1) * C + c], sh[1][0][cl] + sh[1][1][cl] + sh[1][2][cl] + sh[1][3][cl]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned t = __hip_atomic_fetch_add(&counters[blockIdx.x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last_sh = t == unsigned(R - 1);
    }
    __syncthreads();
    if (!last_sh) return;
    // fold the R rows in a fixed order (as fold(): row groups over the 4 waves, then in order)
    s = 0.0;
    q = 0.0;
    if (c < C)
        for (int r = rg; r < R; r += 4) {
            s += ld_wt(&p2[(int64_t(r) * 2 + 0) * C + c]);
            q += ld_wt(&p2[(int64_t(r) * 2 + 1) * C + c]);
        }
    sh[0][rg][cl] = s;
    sh[1][rg][cl] = q;
    __syncthreads();
    if (threadIdx.x == 0) counters[blockIdx.x] = 0u;   // re-armed for the next launch (same stream)
    if (rg != 0 || c >= C) return;
    s = (sh[0][0][cl] + sh[0][1][cl]) + (sh[0][2][cl] + sh[0][3][cl]);
    q = (sh[1][0][cl] + sh[1][1][cl]) + (sh[1][2][cl] + sh[1][3][cl]);
    if constexpr (!BWD) {
        if (nbt && blockIdx.x == 0 && cl == 0) *nbt += 1;
        const double mu = s / count;
        double var = q / count - mu * mu;
        if (var < 0) var = 0;
        const double rstd = 1.0 / sqrt(var + double(eps));
        const float sc = float(double(gamma[c]) * rstd);
        scale[c] = sc;
        shift[c] = float(double(beta[c]) - mu * double(sc));
        mean_out[c] = float(mu);
        rstd_out[c] = float(rstd);
        if (running_mean) {
            const double unb = count > 1 ? var * count / (count - 1) : var;
            running_mean[c] = float((1.0 - momentum) * running_mean[c] + momentum * mu);
            running_var[c] = float((1.0 - momentum) * running_var[c] + momentum * unb);
        }
    } else {
        if (dgamma) dgamma[c] = float(accumulate ? dgamma[c] + q : q);
        if (dbeta) dbeta[c] = float(accumulate ? dbeta[c] + s : s);
        coef[c] = gamma[c] * rstd_in[c];
        coef[C + c] = float(s / count);
        coef[2 * C + c] = float(q / count);
    }
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

// eval: every layer of a table, block y = layer (bn_eval_coeff_kernel's arithmetic)
__global__ void bn_eval_coeff_batch_kernel(const ym_bn_eval_entry* __restrict__ tab) {
    const ym_bn_eval_entry e = tab[blockIdx.y];
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < e.c; c += gridDim.x * blockDim.x) {
        const float rstd = 1.0f / sqrtf(e.running_var[c] + e.eps);
        const float sc = e.gamma[c] * rstd;
        e.scale[c] = sc;
        e.shift[c] = e.beta[c] - e.running_mean[c] * sc;
    }
}

// ---------------------------------------------------------------- streaming kernels
// rows of one thread whose loads are in flight together in the streaming kernels
#ifndef BN_ROWS
#define BN_ROWS 2
#endif
struct Lanes {
    int g, r, rows;
    bool on;
};
__device__ __forceinline__ Lanes lanes(int C) {
    const int cg = C >> 3;
    Lanes L;
    L.rows = 256 / cg;
    L.g = threadIdx.x % cg;
    L.r = threadIdx.x / cg;
    L.on = L.r < L.rows;
    return L;
}

// out[m*o_ld + c] = act(z*scale + shift) (+ res[m*r_ld + c]);  optional fp32 dense copy
__global__ void __launch_bounds__(256) bn_apply_kernel(const bf16_t* __restrict__ z, int64_t M, int C,
                                                       const float* __restrict__ scale, const float* __restrict__ shift,
                                                       int act, const bf16_t* __restrict__ res, int64_t r_ld,
                                                       bf16_t* __restrict__ out, int64_t o_ld, float* __restrict__ out32) {
    const Lanes L = lanes(C);
    if (!L.on) return;
    const int c0 = L.g * 8;
    float sc[8], sf[8];
    load8(scale + c0, sc);
    load8(shift + c0, sf);
    const int64_t step = int64_t(gridDim.x) * L.rows;
    // BN_ROWS rows per iteration: every row's loads are in flight before any is used
    for (int64_t m = int64_t(blockIdx.x) * L.rows + L.r; m < M; m += BN_ROWS * step) {
        uint4 zr[BN_ROWS], rr[BN_ROWS];
#pragma unroll
        for (int u = 0; u < BN_ROWS; ++u) {
            const int64_t mm = m + u * step;
            if (mm < M) {
                zr[u] = *reinterpret_cast<const uint4*>(z + mm * C + c0);
                if (res) rr[u] = *reinterpret_cast<const uint4*>(res + mm * r_ld + c0);
            }
        }
#pragma unroll
        for (int u = 0; u < BN_ROWS; ++u) {
            const int64_t mm = m + u * step;
            if (mm >= M) break;
            float v[8];
            unpack8h(zr[u], v);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const float t = v[k] * sc[k] + sf[k];
                v[k] = act ? silu_f(t) : t;
            }
            if (res) {
                float r[8];
                unpack8h(rr[u], r);
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] += r[k];
            }
            *reinterpret_cast<uint4*>(out + mm * o_ld + c0) = pack8h(v);
            if (out32) {
                float4* o = reinterpret_cast<float4*>(out32 + mm * C + c0);
                o[0] = make_float4(v[0], v[1], v[2], v[3]);
                o[1] = make_float4(v[4], v[5], v[6], v[7]);
            }
        }
    }
}

// per-block partials of sum(g) and sum(g*xhat)
__global__ void __launch_bounds__(256) bn_bwd_reduce_kernel(const bf16_t* __restrict__ dy, int64_t d_ld,
                                                            const bf16_t* __restrict__ z, int64_t M, int C,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ shift,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ rstd, int act,
                                                            float* __restrict__ ps, float* __restrict__ pg) {
    extern __shared__ float red[];   // [2][rows][C]
    const Lanes L = lanes(C);
    const int c0 = L.g * 8;
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sx[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (L.on) {
        float sc[8], sf[8], mu[8], rs[8];
        load8(scale + c0, sc);
        load8(shift + c0, sf);
        load8(mean + c0, mu);
        load8(rstd + c0, rs);
        const int64_t step = int64_t(gridDim.x) * L.rows;
        for (int64_t m = int64_t(blockIdx.x) * L.rows + L.r; m < M; m += BN_ROWS * step) {
            uint4 zr[BN_ROWS], dr[BN_ROWS];
#pragma unroll
            for (int u = 0; u < BN_ROWS; ++u) {
                const int64_t mm = m + u * step;
                if (mm < M) {
                    zr[u] = *reinterpret_cast<const uint4*>(z + mm * C + c0);
                    dr[u] = *reinterpret_cast<const uint4*>(dy + mm * d_ld + c0);
                }
            }
#pragma unroll
            for (int u = 0; u < BN_ROWS; ++u) {
                if (m + u * step >= M) break;
                float zv[8], dv[8];
                unpack8h(zr[u], zv);
                unpack8(dr[u], dv);
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const float gg = act ? dv[k] * dsilu(zv[k] * sc[k] + sf[k]) : dv[k];
                    s[k] += gg;
                    sx[k] += gg * ((zv[k] - mu[k]) * rs[k]);
                }
            }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            red[L.r * C + c0 + k] = s[k];
            red[(L.rows + L.r) * C + c0 + k] = sx[k];
        }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        float a = 0.f, b = 0.f;
        for (int r = 0; r < L.rows; ++r) {
            a += red[r * C + c];
            b += red[(L.rows + r) * C + c];
        }
        ps[int64_t(blockIdx.x) * C + c] = a;
        pg[int64_t(blockIdx.x) * C + c] = b;
    }
}

// dz[m][c] = k1*(g - k2 - xhat*k3), dz dense [M][C] (may alias z)
// RES: also the residual branch's gradient, dres (+)= dy (the Bottleneck / Attention.pe shortcut),
// from the dy this kernel reads anyway (replaces a ym_view_axpy pass)
template <bool RES>
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(const bf16_t* __restrict__ dy, int64_t d_ld,
                                                           const bf16_t* z, int64_t M, int C,
                                                           const float* __restrict__ scale,
                                                           const float* __restrict__ shift,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ rstd, int act,
                                                           const float* __restrict__ coef, bf16_t* dz,
                                                           bf16_t* __restrict__ dres, int64_t r_ld, int r_acc) {
    const Lanes L = lanes(C);
    if (!L.on) return;
    const int c0 = L.g * 8;
    float sc[8], sf[8], mu[8], rs[8], k1[8], k2[8], k3[8];
    load8(scale + c0, sc);
    load8(shift + c0, sf);
    load8(mean + c0, mu);
    load8(rstd + c0, rs);
    load8(coef + c0, k1);
    load8(coef + C + c0, k2);
    load8(coef + 2 * C + c0, k3);
    const int64_t step = int64_t(gridDim.x) * L.rows;
    for (int64_t m = int64_t(blockIdx.x) * L.rows + L.r; m < M; m += BN_ROWS * step) {
        uint4 zr[BN_ROWS], dr[BN_ROWS];
#pragma unroll
        for (int u = 0; u < BN_ROWS; ++u) {
            const int64_t mm = m + u * step;
            if (mm < M) {
                zr[u] = *reinterpret_cast<const uint4*>(z + mm * C + c0);
                dr[u] = *reinterpret_cast<const uint4*>(dy + mm * d_ld + c0);
            }
        }
#pragma unroll
        for (int u = 0; u < BN_ROWS; ++u) {
            const int64_t mm = m + u * step;
            if (mm >= M) break;
            float zv[8], dv[8], o[8];
            unpack8h(zr[u], zv);
            unpack8(dr[u], dv);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const float gg = act ? dv[k] * dsilu(zv[k] * sc[k] + sf[k]) : dv[k];
                const float xh = (zv[k] - mu[k]) * rs[k];
                o[k] = k1[k] * (gg - k2[k] - xh * k3[k]);
            }
            *reinterpret_cast<uint4*>(dz + mm * C + c0) = pack8(o);
            if constexpr (RES) {
                uint4* rp = reinterpret_cast<uint4*>(dres + mm * r_ld + c0);
                if (r_acc) {
                    float rv[8];
                    unpack8(*rp, rv);
#pragma unroll
                    for (int k = 0; k < 8; ++k) rv[k] += dv[k];
                    *rp = pack8(rv);
                } else {
                    *rp = dr[u];
                }
            }
        }
    }
}

// BatchNorm backward statistics AND finalize in one launch for the small maps (ym_bn_bwd_reduce_fold): grid
// (G pixel blocks, C / 64 channel groups; fold_blocks), 256 threads = 8 lanes of 8 channels x 32 pixel rows.  Each
// workgroup reduces its rows for its 64 channels, publishes one partial row write-through, takes an agent-scope
// ticket of its channel group; the last workgroup of the group folds the group's G rows in fp64 in a fixed
// order (4 row subsets, 16 rows' loads in flight) and writes what ym_bn_bwd_finalize writes (dgamma, dbeta,
// the apply coefficients) for those channels, then re-arms the ticket.  The partial rows of a group are few
// (G = 64 on the 20x20 maps, <= 256 on 40x40): the fold is <= 4 rounds of loads, where one folding workgroup over
// the streaming kernel's 512 full-width rows would be latency-bound for tens of us.
constexpr int FOLD_GP = 64;

__global__ void __launch_bounds__(256) bn_bwd_reduce_fold_kernel(
    const bf16_t* __restrict__ dy, int64_t d_ld, const bf16_t* __restrict__ z, int64_t M, int C,
    const float* __restrict__ scale, const float* __restrict__ shift, const float* __restrict__ mean,
    const float* __restrict__ rstd, int act, float* ps, float* pg, const float* __restrict__ gamma, float* dgamma,
    float* dbeta, int accumulate, float* coef, unsigned* cnt, double count) {
    __shared__ float red[2][32][64];
    __shared__ double part[4][2][64];
    __shared__ int last_sh;
    const int tid = threadIdx.x, lg = tid & 7, r = tid >> 3;
    const int cg = blockIdx.y, c0 = cg * 64 + lg * 8;
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sx[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    {
        float sc[8], sf[8], mu[8], rs[8];
        load8(scale + c0, sc);
        load8(shift + c0, sf);
        load8(mean + c0, mu);
        load8(rstd + c0, rs);
        const int64_t step = int64_t(gridDim.x) * 32;
        for (int64_t m = int64_t(blockIdx.x) * 32 + r; m < M; m += 2 * step) {
            const int64_t m2 = m + step;
            const bool two = m2 < M;
            uint4 zr[2], dr[2];
            zr[0] = *reinterpret_cast<const uint4*>(z + m * C + c0);
            dr[0] = *reinterpret_cast<const uint4*>(dy + m * d_ld + c0);
            if (two) {
                zr[1] = *reinterpret_cast<const uint4*>(z + m2 * C + c0);
                dr[1] = *reinterpret_cast<const uint4*>(dy + m2 * d_ld + c0);
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                if (u == 1 && !two) break;
                float zv[8], dv[8];
                unpack8h(zr[u], zv);
                unpack8(dr[u], dv);
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const float gg = act ? dv[k] * dsilu(zv[k] * sc[k] + sf[k]) : dv[k];
                    s[k] += gg;
                    sx[k] += gg * ((zv[k] - mu[k]) * rs[k]);
                }
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        red[0][r][lg * 8 + k] = s[k];
        red[1][r][lg * 8 + k] = sx[k];
    }
    __syncthreads();
    if (tid < 64) {
        float a = 0.f, b = 0.f;
        for (int j = 0; j < 32; ++j) {
            a += red[0][j][tid];
            b += red[1][j][tid];
        }
        __hip_atomic_store(&ps[int64_t(blockIdx.x) * C + cg * 64 + tid], a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&pg[int64_t(blockIdx.x) * C + cg * 64 + tid], b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        const unsigned t = __hip_atomic_fetch_add(&cnt[cg], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last_sh = t == gridDim.x - 1;
    }
    __syncthreads();
    if (!last_sh) return;
    // fold: thread (k = tid / 64, cl = tid % 64) sums rows k, k + 4, ... with 8 rows' loads in flight
    const int cl = tid & 63, k = tid >> 6, ch = cg * 64 + cl;
    const int rows = int(gridDim.x);
    auto ld = [&](const float* p, int row) {
        return __hip_atomic_load(const_cast<float*>(p) + int64_t(row) * C + ch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    double fs = 0.0, fq = 0.0;
    int row = k;
    for (; row + 60 < rows; row += 64) {
        float vs[16], vq[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            vs[u] = ld(ps, row + 4 * u);
            vq[u] = ld(pg, row + 4 * u);
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            fs += double(vs[u]);
            fq += double(vq[u]);
        }
    }
    for (; row < rows; row += 4) {
        fs += double(ld(ps, row));
        fq += double(ld(pg, row));
    }
    part[k][0][cl] = fs;
    part[k][1][cl] = fq;
    __syncthreads();
    if (tid == 0) cnt[cg] = 0u;                    // re-armed for the next launch (same stream)
    if (k != 0) return;
    const double sum = (part[0][0][cl] + part[1][0][cl]) + (part[2][0][cl] + part[3][0][cl]);
    const double dot = (part[0][1][cl] + part[1][1][cl]) + (part[2][1][cl] + part[3][1][cl]);
    if (dgamma) dgamma[ch] = float(accumulate ? dgamma[ch] + dot : dot);
    if (dbeta) dbeta[ch] = float(accumulate ? dbeta[ch] + sum : sum);
    coef[ch] = gamma[ch] * rstd[ch];
    coef[C + ch] = float(sum / count);
    coef[2 * C + ch] = float(dot / count);
}

constexpr int RED_R = 32;   // level-1 row splits of the partials reduction

// grid caps of the streaming kernels (measured in the training step: 2048 / 512 with the conv forward's
// 1024 stat rows, +0.3 % over 4096 / 1024 / 2048)
constexpr int APPLY_CAP = 2048, REDUCE_CAP = 512;

int stream_blocks(int64_t M, int C, int cap) {
    int rows = 256 / (C / 8);
    int64_t g = (M + rows - 1) / rows;
    return int(std::max<int64_t>(1, std::min<int64_t>(g, cap)));
}

}  // namespace
}  // namespace ym

using namespace ym;

#define CHECK_C(c) YM_CHECK_ARG((c) % 8 == 0 && (c) / 8 <= 256, "BN: C=%d must be a multiple of 8 and <= 2048", (c))
#define CHECK_VIEW(bs, ld, hw) YM_CHECK_ARG((bs) == int64_t(hw) * (ld) && (ld) % 8 == 0, \
                                            "BN: views must be whole-image buffers with 16-B aligned rows")

// 256 B of ticket counters (one per 64-channel group, c <= 2048 -> at most 32) at a fixed offset,
// then the [RED_R][2][c] fp64 level-1 rows: calls with different c share one workspace safely
constexpr size_t BN_CNT_BYTES = 256;
extern "C" size_t ym_bn_workspace_size(int c) { return BN_CNT_BYTES + size_t(RED_R) * 2 * c * sizeof(double); }

extern "C" int ym_bn_finalize(const float* part_sum, const float* part_sq, int parts, int c, double count,
                              const float* gamma, const float* beta, float* running_mean, float* running_var,
                              int64_t* num_batches_tracked, float momentum, float eps, float* scale, float* shift,
                              float* mean, float* rstd, void* workspace, void* stream) {
    YM_CHECK_ARG(count > 0 && workspace, "ym_bn_finalize: count must be > 0, workspace required");
    hipStream_t st = as_stream(stream);
    double* p2 = reinterpret_cast<double*>(static_cast<char*>(workspace) + BN_CNT_BYTES);
    unsigned* cnt = static_cast<unsigned*>(workspace);
    hipLaunchKernelGGL((bn_finalize_fused_kernel<false>), dim3((c + 63) / 64, RED_R), dim3(256), 0, st, part_sum,
                       part_sq, parts, c, RED_R, count, p2, cnt, gamma, beta, running_mean, running_var,
                       num_batches_tracked, momentum, eps, scale, shift, mean, rstd, nullptr, nullptr, nullptr, 0,
                       nullptr);
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

extern "C" int ym_bn_eval_coeff_batch(const ym_bn_eval_entry* table_dev, int n_entries, void* stream) {
    YM_CHECK_ARG(n_entries >= 0 && (table_dev || n_entries == 0), "ym_bn_eval_coeff_batch: null table");
    if (n_entries == 0) return YM_OK;
    hipLaunchKernelGGL(bn_eval_coeff_batch_kernel, dim3(8, unsigned(n_entries)), dim3(256), 0, as_stream(stream),
                       table_dev);
    YM_LAUNCH_CHECK("ym_bn_eval_coeff_batch");
    return YM_OK;
}

extern "C" int ym_bn_apply(const uint16_t* z, int64_t m, int c, int hw, const float* scale, const float* shift,
                           int act, const uint16_t* res, int64_t r_bs, int64_t r_ld, uint16_t* out, int64_t o_bs,
                           int64_t o_ld, float* out32, void* stream) {
    CHECK_C(c);
    CHECK_VIEW(o_bs, o_ld, hw);
    if (res) CHECK_VIEW(r_bs, r_ld, hw);
    if (m == 0) return YM_OK;
    hipLaunchKernelGGL(bn_apply_kernel, dim3(stream_blocks(m, c, APPLY_CAP)), dim3(256), 0, as_stream(stream), z, m, c,
                       scale, shift, act, res, r_ld, out, o_ld, out32);
    YM_LAUNCH_CHECK("ym_bn_apply");
    return YM_OK;
}

// the largest maps (m * c >= 2^26: the stem, the 160x160 >= 64-channel and 80x80 256-channel layers) take twice the
// workgroups: the stem's statistics sit on the serial tail of the backward (+0.5-0.6 % step, bn_reduce_cap_ab.txt)
extern "C" int ym_bn_bwd_blocks(int64_t m, int c) {
    return stream_blocks(m, c, m * c >= (int64_t(1) << 26) ? 2 * REDUCE_CAP : REDUCE_CAP);
}

extern "C" int ym_bn_bwd_reduce(const uint16_t* dy, int64_t d_bs, int64_t d_ld, const uint16_t* z, int64_t m, int c,
                                int hw, const float* scale, const float* shift, const float* mean, const float* rstd,
                                int act, float* part_sum, float* part_dot, void* stream) {
    CHECK_C(c);
    CHECK_VIEW(d_bs, d_ld, hw);
    int blocks = ym_bn_bwd_blocks(m, c);
    int rows = 256 / (c / 8);
    hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(blocks), dim3(256), size_t(2) * rows * c * sizeof(float),
                       as_stream(stream), dy, d_ld, z, m, c, scale, shift, mean, rstd, act, part_sum, part_dot);
    YM_LAUNCH_CHECK("ym_bn_bwd_reduce");
    return YM_OK;
}

extern "C" int ym_bn_bwd_finalize(const float* part_sum, const float* part_dot, int parts, int c, double count,
                                  const float* gamma, const float* rstd, float* dgamma, float* dbeta, int accumulate,
                                  float* coef, void* workspace, void* stream) {
    YM_CHECK_ARG(workspace, "ym_bn_bwd_finalize: workspace required");
    hipStream_t st = as_stream(stream);
    double* p2 = reinterpret_cast<double*>(static_cast<char*>(workspace) + BN_CNT_BYTES);
    unsigned* cnt = static_cast<unsigned*>(workspace);
    hipLaunchKernelGGL((bn_finalize_fused_kernel<true>), dim3((c + 63) / 64, RED_R), dim3(256), 0, st, part_sum,
                       part_dot, parts, c, RED_R, count, p2, cnt, gamma, nullptr, nullptr, nullptr, nullptr, 0.f,
                       0.f, nullptr, nullptr, nullptr, nullptr, rstd, dgamma, dbeta, accumulate, coef);
    YM_LAUNCH_CHECK("ym_bn_bwd_finalize");
    return YM_OK;
}

// fused backward statistics + finalize policy (ym_bn_set_bwd_fold): -1 default (= 2), 0 off, 1 / 2 on (map size caps)
static Policy g_bwd_fold{-1};
// the maps it takes: whole 64-channel groups and at most 25600 pixels = 20x20 x 64 images on 64 workgroups per group
// (on larger maps 64 workgroups per group streamed the tensor slower than the streaming kernel's 512 full-width ones:
// 40x40 -0.5 %, profiles/r04/bn_bwd_fold_ab.txt); by default (round 5) it also takes <= 102400 pixels (40x40 x 64
// images) with 512 / groups workgroups per group (64..256): +0.0..+0.7 % img/s in three same-box pairs
// (profiles/r05/bn_bwd_fold40_ab.txt); mode 1 keeps the 20x20-only rule
static constexpr int64_t FOLD_MAX_M = 25600, FOLD_MAX_M2 = 102400;

static int fold_blocks(int64_t m, int c) {
    if (m <= FOLD_MAX_M) return FOLD_GP;
    return std::min(256, std::max(FOLD_GP, 512 / (c / 64)));
}

extern "C" int ym_bn_bwd_fold_ok(int64_t m, int c) {
    if (g_bwd_fold == 0) return 0;
    const int64_t cap = g_bwd_fold == 1 ? FOLD_MAX_M : FOLD_MAX_M2;
    return m > 0 && m <= cap && c % 64 == 0 && c <= 2048 && ym_bn_bwd_blocks(m, c) >= fold_blocks(m, c) ? 1 : 0;
}

extern "C" int ym_bn_set_bwd_fold(int mode) {
    // fused backward statistics + finalize: -1 default (= 2), 0 off, 1 on up to 25600 pixels, 2 up to 102400;
    // returns the previous setting
    return g_bwd_fold.set(mode < -1 || mode > 2 ? -1 : mode);
}

extern "C" int ym_bn_bwd_reduce_fold(const uint16_t* dy, int64_t d_bs, int64_t d_ld, const uint16_t* z, int64_t m, int c,
                                     int hw, const float* scale, const float* shift, const float* mean,
                                     const float* rstd, int act, float* part_sum, float* part_dot, const float* gamma,
                                     float* dgamma, float* dbeta, int accumulate, float* coef, void* workspace,
                                     void* stream) {
    CHECK_C(c);
    CHECK_VIEW(d_bs, d_ld, hw);
    YM_CHECK_ARG(workspace && gamma && coef, "ym_bn_bwd_reduce_fold: null argument");
    if (!ym_bn_bwd_fold_ok(m, c)) {
        // the streaming statistics kernel + the finalize launch (the same outputs)
        const int r = ym_bn_bwd_reduce(dy, d_bs, d_ld, z, m, c, hw, scale, shift, mean, rstd, act, part_sum, part_dot,
                                       stream);
        if (r != YM_OK) return r;
        return ym_bn_bwd_finalize(part_sum, part_dot, ym_bn_bwd_blocks(m, c), c, double(m), gamma, rstd, dgamma,
                                  dbeta, accumulate, coef, workspace, stream);
    }
    hipLaunchKernelGGL(bn_bwd_reduce_fold_kernel, dim3(fold_blocks(m, c), c / 64), dim3(256), 0, as_stream(stream), dy, d_ld, z,
                       m, c, scale, shift, mean, rstd, act, part_sum, part_dot, gamma, dgamma, dbeta, accumulate, coef,
                       static_cast<unsigned*>(workspace), double(m));
    YM_LAUNCH_CHECK("ym_bn_bwd_reduce_fold");
    return YM_OK;
}

extern "C" int ym_bn_bwd_apply(const uint16_t* dy, int64_t d_bs, int64_t d_ld, const uint16_t* z, int64_t m, int c,
                               int hw, const float* scale, const float* shift, const float* mean, const float* rstd,
                               int act, const float* coef, uint16_t* dz, void* stream) {
    CHECK_C(c);
    CHECK_VIEW(d_bs, d_ld, hw);
    if (m == 0) return YM_OK;
    hipLaunchKernelGGL(bn_bwd_apply_kernel<false>, dim3(stream_blocks(m, c, APPLY_CAP)), dim3(256), 0,
                       as_stream(stream), dy, d_ld, z, m, c, scale, shift, mean, rstd, act, coef, dz, nullptr, 0, 0);
    YM_LAUNCH_CHECK("ym_bn_bwd_apply");
    return YM_OK;
}

extern "C" int ym_bn_bwd_apply_res(const uint16_t* dy, int64_t d_bs, int64_t d_ld, const uint16_t* z, int64_t m,
                                   int c, int hw, const float* scale, const float* shift, const float* mean,
                                   const float* rstd, int act, const float* coef, uint16_t* dz, uint16_t* dres,
                                   int64_t r_bs, int64_t r_ld, int r_accumulate, void* stream) {
    CHECK_C(c);
    CHECK_VIEW(d_bs, d_ld, hw);
    CHECK_VIEW(r_bs, r_ld, hw);
    YM_CHECK_ARG(dres, "ym_bn_bwd_apply_res: null residual gradient");
    if (m == 0) return YM_OK;
    hipLaunchKernelGGL(bn_bwd_apply_kernel<true>, dim3(stream_blocks(m, c, APPLY_CAP)), dim3(256), 0,
                       as_stream(stream), dy, d_ld, z, m, c, scale, shift, mean, rstd, act, coef, dz, dres, r_ld,
                       r_accumulate);
    YM_LAUNCH_CHECK("ym_bn_bwd_apply_res");
    return YM_OK;
}
