// C2PSA attention core on CDNA4 MFMA (16x16x32; fp16 scores, bf16 gradients, fp32 accumulate).
//
// Replaces Attention.forward's matmuls/softmax (/root/reference/yolo_scratch_cuda/models/
// yolo11_modules.py:124-136): per (image b, head h), q/k/v are channel slices of the qkv conv
// output (NHWC view; head h owns channels h*(2KD+HD) + [q: 0..KD) [k: KD..2KD) [v: 2KD..2KD+HD)),
//   attn = softmax_j(q_i . k_j * scale),  out[i, h*HD + d] = sum_j attn[i][j] v[j][d].
// Flash-style: the N x N matrix never leaves the chip.  Forward keeps one row of softmax
// statistics (LSE) per query; the backward recomputes P from it and splits into a dK/dV kernel
// (a workgroup owns 64 keys, loops over queries) and a dQ kernel (owns 64 queries, loops over
// keys), so no gradient needs atomics.
//
// Fragment conventions (v_mfma_f32_16x16x32): A lane L holds A[L&15][k-slots of group g=L>>4],
// B lane L holds B[k-slots of g][L&15], D lane L holds D[4g + r][L&15].  Operands whose k axis
// runs along LDS rows are read with ds_read_b64_tr_b16 (tr_frag): group g's eight k-slots are
// rows {4g..4g+3, 16+4g..16+4g+3}, which is exactly how a D tile pair (rows 4g+r of two
// stacked 16-row tiles) lands in one lane — so P / dS go from accumulator to operand in place.
#include <algorithm>

#include "common.h"
#include "tile.h"

namespace ym {
namespace {

constexpr int KD = 32, HD = 64, HS = 2 * KD + HD;   // key dim, head dim, per-head qkv channels
constexpr int T = 64;                                // keys / queries per tile
constexpr int RK = KD * 2 + 16;                      // LDS row bytes of a 32-channel image (padded)
constexpr int RV = HD * 2 + 16;                      // LDS row bytes of a 64-channel image (padded)

typedef short s16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ s16x4 tr_read(const char* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}
// transposed operand: M index col0 + (lane&15) along the row, k slots = rows rb + {4g+q, 16+4g+q}
__device__ __forceinline__ s16x8 tr_frag(const char* img, int rs, int rb, int col0) {
    const int lane = threadIdx.x & 63, g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const char* a = img + (rb + 4 * g + q) * rs + (col0 + 4 * p) * 2;
    const s16x4 lo = tr_read(a), hi = tr_read(a + 16 * rs);
    return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
// row operand: row rb + (lane&15), 8 elements from element k0 + 8g
__device__ __forceinline__ s16x8 row_frag(const char* img, int rs, int rb, int k0) {
    const int lane = threadIdx.x & 63;
    return *reinterpret_cast<const s16x8*>(img + (rb + (lane & 15)) * rs + (k0 + 8 * (lane >> 4)) * 2);
}
__device__ __forceinline__ f32x4 mma_h(s16x8 a, s16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mma_b(s16x8 a, s16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                   0, 0);
}
__device__ __forceinline__ uint32_t pk2h(float a, float b) {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    h2 v = {(_Float16)a, (_Float16)b};
    return __builtin_bit_cast(uint32_t, v);
}
// two stacked D tiles (4 values each) -> one 8-slot operand
__device__ __forceinline__ s16x8 pack_bf(const float* lo, const float* hi) {
    uint4 u = make_uint4(pk2bf(lo[0], lo[1]), pk2bf(lo[2], lo[3]), pk2bf(hi[0], hi[1]), pk2bf(hi[2], hi[3]));
    return __builtin_bit_cast(s16x8, u);
}
__device__ __forceinline__ s16x8 pack_h(const float* lo, const float* hi) {
    uint4 u = make_uint4(pk2h(lo[0], lo[1]), pk2h(lo[2], lo[3]), pk2h(hi[0], hi[1]), pk2h(hi[2], hi[3]));
    return __builtin_bit_cast(s16x8, u);
}
__device__ __forceinline__ uint4 ld16(const uint16_t* p, bool ok) {
    return ok ? *reinterpret_cast<const uint4*>(p) : make_uint4(0, 0, 0, 0);
}

struct AttnArgs {
    const uint16_t* qkv; int64_t q_bs, q_ld;   // fp16 activations
    int N, heads;
    float scale;
};

// ------------------------------------------------------------------ forward
// block: 64 queries of one (b, h), 4 waves x 16 queries; S^T = K Q^T so P^T is already the
// B operand of O^T = V^T P^T
__global__ void __launch_bounds__(256) attn_fwd_kernel(AttnArgs a, uint16_t* __restrict__ out, int64_t o_bs,
                                                       int64_t o_ld, float* __restrict__ lse) {
    __shared__ __attribute__((aligned(16))) char Ks[T * RK];
    __shared__ __attribute__((aligned(16))) char Vs[T * RV];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
    const int h = blockIdx.y, b = blockIdx.z;
    const uint16_t* base = a.qkv + int64_t(b) * a.q_bs + h * HS;
    const int qi = blockIdx.x * T + wave * 16 + (lane & 15);      // this lane's query column
    const bool qok = qi < a.N;
    const s16x8 qb = __builtin_bit_cast(s16x8, ld16(base + int64_t(qi) * a.q_ld + 8 * g, qok));
    f32x4 o[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m = -INFINITY, l = 0.f;
    for (int k0 = 0; k0 < a.N; k0 += T) {
        {   // K: 64 rows x 4 chunks; V: 64 rows x 8 chunks
            const int r = tid >> 2, c = tid & 3;
            *reinterpret_cast<uint4*>(Ks + r * RK + c * 16) =
                ld16(base + int64_t(k0 + r) * a.q_ld + KD + c * 8, k0 + r < a.N);
#pragma unroll
            for (int it = 0; it < 2; ++it) {
                const int id = tid + 256 * it, rv = id >> 3, cv = id & 7;
                *reinterpret_cast<uint4*>(Vs + rv * RV + cv * 16) =
                    ld16(base + int64_t(k0 + rv) * a.q_ld + 2 * KD + cv * 8, k0 + rv < a.N);
            }
        }
        __syncthreads();
        float s[4][4];
        float tmax = -INFINITY;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
            const f32x4 st = mma_h(row_frag(Ks, RK, kt * 16, 0), qb, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int key = k0 + kt * 16 + 4 * g + r;
                s[kt][r] = key < a.N ? st[r] * a.scale : -INFINITY;
                tmax = fmaxf(tmax, s[kt][r]);
            }
        }
        tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
        tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
        const float mn = fmaxf(m, tmax);
        const float alpha = __expf(m - mn);
        float psum = 0.f;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                s[kt][r] = __expf(s[kt][r] - mn);
                psum += s[kt][r];
            }
        psum += __shfl_xor(psum, 16, 64);
        psum += __shfl_xor(psum, 32, 64);
        l = l * alpha + psum;
        m = mn;
#pragma unroll
        for (int d = 0; d < 4; ++d) o[d] *= alpha;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const s16x8 pb = pack_h(s[2 * ks], s[2 * ks + 1]);
#pragma unroll
            for (int d = 0; d < 4; ++d) o[d] = mma_h(tr_frag(Vs, RV, ks * 32, d * 16), pb, o[d]);
        }
        __syncthreads();
    }
    if (qok) {
        const float inv = 1.0f / l;
        uint16_t* op = out + int64_t(b) * o_bs + int64_t(qi) * o_ld + h * HD + 4 * g;
#pragma unroll
        for (int d = 0; d < 4; ++d)
            *reinterpret_cast<uint2*>(op + d * 16) = make_uint2(pk2h(o[d][0] * inv, o[d][1] * inv),
                                                                pk2h(o[d][2] * inv, o[d][3] * inv));
        if (g == 0) lse[(int64_t(b) * a.heads + h) * a.N + qi] = m + __logf(l);
    }
}

// D[b,h,i] = sum_d dO[i][h*HD+d] * O[i][h*HD+d]
__global__ void attn_bwd_pre_kernel(const uint16_t* __restrict__ o, int64_t o_bs, int64_t o_ld,
                                    const uint16_t* __restrict__ dout, int64_t d_bs, int64_t d_ld, int B, int heads,
                                    int N, float* __restrict__ D) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= B * heads * N) return;
    const int i = idx % N, h = (idx / N) % heads, b = idx / (N * heads);
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < HD / 8; ++c) {
        const uint4 x = *reinterpret_cast<const uint4*>(o + int64_t(b) * o_bs + int64_t(i) * o_ld + h * HD + c * 8);
        const uint4 y = *reinterpret_cast<const uint4*>(dout + int64_t(b) * d_bs + int64_t(i) * d_ld + h * HD + c * 8);
        const uint32_t xs[4] = {x.x, x.y, x.z, x.w}, ys[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
        for (int e = 0; e < 4; ++e)
            s += h2f(uint16_t(xs[e] & 0xffff)) * bf2f(bf16_t(ys[e] & 0xffff)) +
                 h2f(uint16_t(xs[e] >> 16)) * bf2f(bf16_t(ys[e] >> 16));
    }
    D[idx] = s;
}

__device__ __forceinline__ void store4(uint16_t* p, f32x4 v, float mul, int acc) {
    float f[4] = {v[0] * mul, v[1] * mul, v[2] * mul, v[3] * mul};
    if (acc) {
        const uint2 old = *reinterpret_cast<const uint2*>(p);
        f[0] += bf2f(bf16_t(old.x & 0xffff)); f[1] += bf2f(bf16_t(old.x >> 16));
        f[2] += bf2f(bf16_t(old.y & 0xffff)); f[3] += bf2f(bf16_t(old.y >> 16));
    }
    *reinterpret_cast<uint2*>(p) = make_uint2(pk2bf(f[0], f[1]), pk2bf(f[2], f[3]));
}

// ------------------------------------------------------------------ backward: dK, dV
// block: 64 keys of one (b, h), 4 waves x 16 keys; per 64-query tile:
//   S = Q K^T, P = exp(S*scale - LSE), dP = dO V^T, dS = P (dP - D),
//   dV^T += dO^T P,  dK^T += Q^T dS          (dK scaled at the end)
__global__ void __launch_bounds__(256) attn_bwd_kv_kernel(AttnArgs a, const uint16_t* __restrict__ dout, int64_t d_bs,
                                                          int64_t d_ld, const float* __restrict__ lse,
                                                          const float* __restrict__ D, uint16_t* __restrict__ dqkv,
                                                          int64_t g_bs, int64_t g_ld, int acc_k, int acc_v) {
    __shared__ __attribute__((aligned(16))) char Qh[T * RK];    // q fp16 (scores)
    __shared__ __attribute__((aligned(16))) char Qb[T * RK];    // q bf16 (dK operand)
    __shared__ __attribute__((aligned(16))) char Os[T * RV];    // dO bf16
    __shared__ float Ls[T], Ds[T];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
    const int h = blockIdx.y, b = blockIdx.z;
    const uint16_t* base = a.qkv + int64_t(b) * a.q_bs + h * HS;
    const uint16_t* dob = dout + int64_t(b) * d_bs + h * HD;
    const int kj = blockIdx.x * T + wave * 16 + (lane & 15);      // this lane's key column
    const bool kok = kj < a.N;
    const s16x8 kb = __builtin_bit_cast(s16x8, ld16(base + int64_t(kj) * a.q_ld + KD + 8 * g, kok));
    s16x8 vb[2];
#pragma unroll
    for (int kc = 0; kc < 2; ++kc)
        vb[kc] = __builtin_bit_cast(s16x8, h8_to_bf8(ld16(base + int64_t(kj) * a.q_ld + 2 * KD + 32 * kc + 8 * g, kok)));
    f32x4 dv[4], dk[2];
#pragma unroll
    for (int d = 0; d < 4; ++d) dv[d] = f32x4{0.f, 0.f, 0.f, 0.f};
    dk[0] = dk[1] = f32x4{0.f, 0.f, 0.f, 0.f};
    const float* lse_bh = lse + (int64_t(b) * a.heads + h) * a.N;
    const float* D_bh = D + (int64_t(b) * a.heads + h) * a.N;
    for (int q0 = 0; q0 < a.N; q0 += T) {
        {
            const int r = tid >> 2, c = tid & 3;
            const uint4 qv = ld16(base + int64_t(q0 + r) * a.q_ld + c * 8, q0 + r < a.N);
            *reinterpret_cast<uint4*>(Qh + r * RK + c * 16) = qv;
            *reinterpret_cast<uint4*>(Qb + r * RK + c * 16) = h8_to_bf8(qv);
#pragma unroll
            for (int it = 0; it < 2; ++it) {
                const int id = tid + 256 * it, ro = id >> 3, co = id & 7;
                *reinterpret_cast<uint4*>(Os + ro * RV + co * 16) =
                    ld16(dob + int64_t(q0 + ro) * d_ld + co * 8, q0 + ro < a.N);
            }
            if (tid < T) {
                const bool ok = q0 + tid < a.N;
                Ls[tid] = ok ? lse_bh[q0 + tid] : INFINITY;
                Ds[tid] = ok ? D_bh[q0 + tid] : 0.f;
            }
        }
        __syncthreads();
        float p[4][4], ds[4][4];
#pragma unroll
        for (int qt = 0; qt < 4; ++qt) {
            const f32x4 s = mma_h(row_frag(Qh, RK, qt * 16, 0), kb, f32x4{0.f, 0.f, 0.f, 0.f});
            f32x4 dp = mma_b(row_frag(Os, RV, qt * 16, 0), vb[0], f32x4{0.f, 0.f, 0.f, 0.f});
            dp = mma_b(row_frag(Os, RV, qt * 16, 32), vb[1], dp);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int qr = qt * 16 + 4 * g + r;
                p[qt][r] = kok ? __expf(s[r] * a.scale - Ls[qr]) : 0.f;
                ds[qt][r] = p[qt][r] * (dp[r] - Ds[qr]);
            }
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const s16x8 pb = pack_bf(p[2 * ks], p[2 * ks + 1]);
            const s16x8 sb = pack_bf(ds[2 * ks], ds[2 * ks + 1]);
#pragma unroll
            for (int d = 0; d < 4; ++d) dv[d] = mma_b(tr_frag(Os, RV, ks * 32, d * 16), pb, dv[d]);
#pragma unroll
            for (int d = 0; d < 2; ++d) dk[d] = mma_b(tr_frag(Qb, RK, ks * 32, d * 16), sb, dk[d]);
        }
        __syncthreads();
    }
    if (kok) {
        uint16_t* gp = dqkv + int64_t(b) * g_bs + int64_t(kj) * g_ld + h * HS + 4 * g;
#pragma unroll
        for (int d = 0; d < 2; ++d) store4(gp + KD + d * 16, dk[d], a.scale, acc_k);
#pragma unroll
        for (int d = 0; d < 4; ++d) store4(gp + 2 * KD + d * 16, dv[d], 1.f, acc_v);
    }
}

// ------------------------------------------------------------------ backward: dQ
// block: 64 queries of one (b, h), 4 waves x 16 queries; per 64-key tile:
//   S^T = K Q^T, P^T = exp(S^T*scale - LSE), dP^T = V dO^T, dS^T = P^T (dP^T - D),
//   dQ^T += K^T dS^T                          (scaled at the end)
__global__ void __launch_bounds__(256) attn_bwd_q_kernel(AttnArgs a, const uint16_t* __restrict__ dout, int64_t d_bs,
                                                         int64_t d_ld, const float* __restrict__ lse,
                                                         const float* __restrict__ D, uint16_t* __restrict__ dqkv,
                                                         int64_t g_bs, int64_t g_ld, int acc_q) {
    __shared__ __attribute__((aligned(16))) char Kh[T * RK];    // k fp16 (scores)
    __shared__ __attribute__((aligned(16))) char Kb[T * RK];    // k bf16 (dQ operand)
    __shared__ __attribute__((aligned(16))) char Vb[T * RV];    // v bf16 (dP operand)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
    const int h = blockIdx.y, b = blockIdx.z;
    const uint16_t* base = a.qkv + int64_t(b) * a.q_bs + h * HS;
    const int qi = blockIdx.x * T + wave * 16 + (lane & 15);
    const bool qok = qi < a.N;
    const s16x8 qb = __builtin_bit_cast(s16x8, ld16(base + int64_t(qi) * a.q_ld + 8 * g, qok));
    s16x8 ob[2];
#pragma unroll
    for (int kc = 0; kc < 2; ++kc)
        ob[kc] = __builtin_bit_cast(s16x8, ld16(dout + int64_t(b) * d_bs + int64_t(qi) * d_ld + h * HD + 32 * kc + 8 * g,
                                                qok));
    const float lq = qok ? lse[(int64_t(b) * a.heads + h) * a.N + qi] : INFINITY;
    const float dq_d = qok ? D[(int64_t(b) * a.heads + h) * a.N + qi] : 0.f;
    f32x4 dq[2];
    dq[0] = dq[1] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < a.N; k0 += T) {
        {
            const int r = tid >> 2, c = tid & 3;
            const uint4 kv = ld16(base + int64_t(k0 + r) * a.q_ld + KD + c * 8, k0 + r < a.N);
            *reinterpret_cast<uint4*>(Kh + r * RK + c * 16) = kv;
            *reinterpret_cast<uint4*>(Kb + r * RK + c * 16) = h8_to_bf8(kv);
#pragma unroll
            for (int it = 0; it < 2; ++it) {
                const int id = tid + 256 * it, rv = id >> 3, cv = id & 7;
                *reinterpret_cast<uint4*>(Vb + rv * RV + cv * 16) =
                    h8_to_bf8(ld16(base + int64_t(k0 + rv) * a.q_ld + 2 * KD + cv * 8, k0 + rv < a.N));
            }
        }
        __syncthreads();
        float ds[4][4];
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
            const f32x4 s = mma_h(row_frag(Kh, RK, kt * 16, 0), qb, f32x4{0.f, 0.f, 0.f, 0.f});
            f32x4 dp = mma_b(row_frag(Vb, RV, kt * 16, 0), ob[0], f32x4{0.f, 0.f, 0.f, 0.f});
            dp = mma_b(row_frag(Vb, RV, kt * 16, 32), ob[1], dp);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int key = k0 + kt * 16 + 4 * g + r;
                const float pv = key < a.N ? __expf(s[r] * a.scale - lq) : 0.f;
                ds[kt][r] = pv * (dp[r] - dq_d);
            }
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const s16x8 sb = pack_bf(ds[2 * ks], ds[2 * ks + 1]);
#pragma unroll
            for (int d = 0; d < 2; ++d) dq[d] = mma_b(tr_frag(Kb, RK, ks * 32, d * 16), sb, dq[d]);
        }
        __syncthreads();
    }
    if (qok) {
        uint16_t* gp = dqkv + int64_t(b) * g_bs + int64_t(qi) * g_ld + h * HS + 4 * g;
#pragma unroll
        for (int d = 0; d < 2; ++d) store4(gp + d * 16, dq[d], a.scale, acc_q);
    }
}

}  // namespace
}  // namespace ym

using namespace ym;

static bool attn_views_ok(int64_t bs, int64_t ld) { return bs % 8 == 0 && ld % 8 == 0; }

extern "C" int ym_attn_fwd(const uint16_t* qkv, int64_t q_bs, int64_t q_ld, int b, int heads, int n, int key_dim,
                           int head_dim, float scale, uint16_t* out, int64_t o_bs, int64_t o_ld, float* lse,
                           void* stream) {
    YM_CHECK_ARG(key_dim == KD && head_dim == HD, "ym_attn_fwd: only key_dim=32, head_dim=64 (got %d, %d)", key_dim,
                 head_dim);
    YM_CHECK_ARG(attn_views_ok(q_bs, q_ld) && o_bs % 4 == 0 && o_ld % 4 == 0, "ym_attn_fwd: view alignment");
    if (n == 0 || b == 0) return YM_OK;
    AttnArgs a{qkv, q_bs, q_ld, n, heads, scale};
    hipLaunchKernelGGL(attn_fwd_kernel, dim3((n + T - 1) / T, heads, b), dim3(256), 0, as_stream(stream), a, out, o_bs,
                       o_ld, lse);
    YM_LAUNCH_CHECK("ym_attn_fwd");
    return YM_OK;
}

extern "C" size_t ym_attn_workspace_size(int b, int heads, int n) { return size_t(b) * heads * n * sizeof(float); }

extern "C" int ym_attn_bwd(const uint16_t* qkv, int64_t q_bs, int64_t q_ld, const uint16_t* out, int64_t o_bs,
                           int64_t o_ld, const uint16_t* dout, int64_t d_bs, int64_t d_ld, const float* lse, int b,
                           int heads, int n, float scale, float* workspace, uint16_t* dqkv, int64_t g_bs, int64_t g_ld,
                           int acc_q, int acc_k, int acc_v, void* stream) {
    YM_CHECK_ARG(attn_views_ok(q_bs, q_ld) && attn_views_ok(o_bs, o_ld) && attn_views_ok(d_bs, d_ld) &&
                     g_bs % 4 == 0 && g_ld % 4 == 0,
                 "ym_attn_bwd: view alignment");
    YM_CHECK_ARG(int64_t(b) * heads * n < (int64_t(1) << 31), "ym_attn_bwd: too large");
    if (n == 0 || b == 0) return YM_OK;
    hipStream_t st = as_stream(stream);
    float* D = workspace;                   // [b][heads][n]
    const int nD = b * heads * n;
    hipLaunchKernelGGL(attn_bwd_pre_kernel, dim3(unsigned((nD + 255) / 256)), dim3(256), 0, st, out, o_bs, o_ld, dout,
                       d_bs, d_ld, b, heads, n, D);
    AttnArgs a{qkv, q_bs, q_ld, n, heads, scale};
    const dim3 grid((n + T - 1) / T, heads, b);
    hipLaunchKernelGGL(attn_bwd_kv_kernel, grid, dim3(256), 0, st, a, dout, d_bs, d_ld, lse, D, dqkv, g_bs, g_ld, acc_k,
                       acc_v);
    hipLaunchKernelGGL(attn_bwd_q_kernel, grid, dim3(256), 0, st, a, dout, d_bs, d_ld, lse, D, dqkv, g_bs, g_ld, acc_q);
    YM_LAUNCH_CHECK("ym_attn_bwd");
    return YM_OK;
}
