// NHWC convolutions on CDNA4 MFMA, fp32 accumulate: forward fp16 x fp16
// (v_mfma_f32_16x16x32_f16; activations are fp16), data/weight gradients bf16
// (v_mfma_f32_16x16x32_bf16; gradients are bf16, activations converted while staging).
//
// Replaces the reference's nn.Conv2d calls (and their autograd) inside
// Conv / Bottleneck / C2f / C3k / SPPF / PSA / Detect
// (/root/reference/yolo_scratch_cuda/models/yolo11_modules.py:21-33, 221-234).
//
// conv_gemm_kernel<MODE>  implicit GEMM, one kernel for forward (MODE_FWD) and
//   data-gradient (MODE_DGRAD).  GEMM rows = output pixels, cols = output
//   channels, K = taps x input channels.  Tiles BM pixels x BN channels x 32,
//   256 threads = 2x2 waves, register-staged double-buffered LDS.  LDS tiles
//   are stored chunk-major ([k-chunk of 8][row] x 16 B) with the row index
//   XOR-swizzled by 4*chunk, so both the 16-B fragment reads (one per lane per
//   MFMA operand) and the 16-B staging writes are bank-conflict free.
//   Epilogue: optional bias, bf16 or fp32 store into a strided NHWC view
//   (concat slices are free), optional accumulate (grad fan-in), and per-block
//   per-channel sum / sum-of-squares partials for training-mode BatchNorm.
// wgrad_kernel  dW[co][tap][ci] = sum_p dz[p][co] * x[src(p,tap)][ci]: K =
//   pixels, staged row-major and read TRANSPOSED with ds_read_b64_tr_b16 so the
//   pixel (reduction) axis lands in each lane's fragment; split-K over pixels
//   with fp32 atomics.
// conv_first_*  Cin = 1 stem (K = 9): direct fp32 VALU kernels.
// dw3x3_*       depthwise 3x3 (Attention.pe, yolo11_modules.py:122): direct.
#include <algorithm>

#include "common.h"

namespace ym {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr int MODE_FWD = 0;
constexpr int MODE_DGRAD = 1;
constexpr int BK = 32;   // k per LDS stage = one MFMA k-step
constexpr int NCH = BK / 8;

struct GemmArgs {
    const bf16_t* x; int64_t x_bs, x_ld;    // gathered activation view
    const bf16_t* w;                         // [Nout][KH][KW][Kin]
    void* y; int64_t y_bs, y_ld;             // output view
    const float* bias;                       // [Nout] or null
    float* st_sum; float* st_sq;             // [gridDim.x][Nout] or null
    int GH, GW, Kin;                         // gathered tensor spatial dims / channels
    int OH, OW, Nout;                        // output pixel grid and channels
    int KH, KW, stride, pad;
    int64_t M;                               // N*OH*OW
    int mtiles;
    int out_f32, accumulate;
};

__device__ __forceinline__ int swz(int row, int c) { return row ^ (c << 2); }

template <int BM, int BN, int MODE>
__global__ void __launch_bounds__(256) conv_gemm_kernel(GemmArgs a) {
    constexpr int TM = BN / 32;          // 16-channel subtiles per wave
    constexpr int TN = BM / 32;          // 16-pixel subtiles per wave
    constexpr int A_ITEMS = (BN * NCH + 255) / 256;
    constexpr int B_ITEMS = (BM * NCH + 255) / 256;
    __shared__ uint4 As[2][NCH][BN];
    __shared__ uint4 Bs[2][NCH][BM];
    __shared__ float red[2][2][BN];      // [sum|sq][wave pixel half][channel]

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 1, wc = wave & 1;
    const int fc = lane >> 4, fr = lane & 15;
    const int n0 = blockIdx.y * BN;
    const int kc = (a.Kin + BK - 1) / BK;
    const int nk = a.KH * a.KW * kc;
    const int64_t OHW = int64_t(a.OH) * a.OW;
    const int64_t wrow = int64_t(a.KH) * a.KW * a.Kin;

    float ssum[TM][4], ssq[TM][4];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) ssum[i][r] = ssq[i][r] = 0.f;

    for (int mt = blockIdx.x; mt < a.mtiles; mt += gridDim.x) {
        const int64_t m0 = int64_t(mt) * BM;
        // per-item pixel decomposition of the B tile rows this thread stages
        int64_t b_img[B_ITEMS];
        int b_oh[B_ITEMS], b_ow[B_ITEMS];
        bool b_ok[B_ITEMS];
#pragma unroll
        for (int it = 0; it < B_ITEMS; ++it) {
            int id = tid + it * 256;
            int row = id / NCH;
            int64_t m = m0 + row;
            b_ok[it] = (id < BM * NCH) && (m < a.M);
            const uint32_t um = b_ok[it] ? uint32_t(m) : 0u;
            const uint32_t n = um / uint32_t(OHW), pix = um - n * uint32_t(OHW);
            b_img[it] = int64_t(n) * a.x_bs;
            b_oh[it] = int(pix / uint32_t(a.OW));
            b_ow[it] = int(pix - uint32_t(b_oh[it]) * uint32_t(a.OW));
        }
        uint4 ra[A_ITEMS], rb[B_ITEMS];
        auto load = [&](int k) {
            const int tap = k / kc, k0 = (k - tap * kc) * BK;
            const int kh = tap / a.KW, kw = tap - kh * a.KW;
#pragma unroll
            for (int it = 0; it < A_ITEMS; ++it) {
                int id = tid + it * 256;
                int row = id / NCH, c = id % NCH;
                int ch = n0 + row, kk = k0 + 8 * c;
                uint4 v = make_uint4(0, 0, 0, 0);
                if (id < BN * NCH && ch < a.Nout && kk < a.Kin)
                    v = *reinterpret_cast<const uint4*>(a.w + int64_t(ch) * wrow + int64_t(tap) * a.Kin + kk);
                ra[it] = v;
            }
#pragma unroll
            for (int it = 0; it < B_ITEMS; ++it) {
                int id = tid + it * 256;
                int c = id % NCH, kk = k0 + 8 * c;
                uint4 v = make_uint4(0, 0, 0, 0);
                if (b_ok[it] && kk < a.Kin) {
                    int gh, gw;
                    bool ok;
                    if (MODE == MODE_FWD) {
                        gh = b_oh[it] * a.stride - a.pad + kh;
                        gw = b_ow[it] * a.stride - a.pad + kw;
                        ok = gh >= 0 && gh < a.GH && gw >= 0 && gw < a.GW;
                    } else {
                        int th = b_oh[it] + a.pad - kh, tw = b_ow[it] + a.pad - kw;
                        ok = th >= 0 && tw >= 0 && (th % a.stride) == 0 && (tw % a.stride) == 0;
                        gh = th / a.stride;
                        gw = tw / a.stride;
                        ok = ok && gh < a.GH && gw < a.GW;
                    }
                    if (ok)
                        v = *reinterpret_cast<const uint4*>(a.x + b_img[it] + (int64_t(gh) * a.GW + gw) * a.x_ld + kk);
                }
                rb[it] = v;
            }
        };
        auto store = [&](int buf) {
#pragma unroll
            for (int it = 0; it < A_ITEMS; ++it) {
                int id = tid + it * 256;
                if (id < BN * NCH) {
                    int row = id / NCH, c = id % NCH;
                    As[buf][c][swz(row, c)] = ra[it];
                }
            }
#pragma unroll
            for (int it = 0; it < B_ITEMS; ++it) {
                int id = tid + it * 256;
                if (id < BM * NCH) {
                    int row = id / NCH, c = id % NCH;
                    Bs[buf][c][swz(row, c)] = rb[it];
                }
            }
        };

        f32x4 acc[TM][TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

        load(0);
        __syncthreads();     // previous tile's readers are done with both buffers
        store(0);
        __syncthreads();
        for (int k = 0; k < nk; ++k) {
            const int buf = k & 1;
            if (k + 1 < nk) load(k + 1);
            bf16x8 af[TM], bfr[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                int row = wr * (BN / 2) + i * 16 + fr;
                af[i] = __builtin_bit_cast(bf16x8, As[buf][fc][swz(row, fc)]);
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                int row = wc * (BM / 2) + j * 16 + fr;
                bfr[j] = __builtin_bit_cast(bf16x8, Bs[buf][fc][swz(row, fc)]);
            }
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    if constexpr (MODE == MODE_FWD)   // fp16 activations x fp16 weights
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, af[i]),
                                                                           __builtin_bit_cast(f16x8, bfr[j]),
                                                                           acc[i][j], 0, 0, 0);
                    else                              // bf16 gradients x bf16 weights
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
                }
            if (k + 1 < nk) store(buf ^ 1);
            __syncthreads();
        }

        // epilogue: D[channel][pixel]; lane holds 4 consecutive channels of one pixel
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int64_t m = m0 + wc * (BM / 2) + j * 16 + fr;
            if (m >= a.M) continue;
            const uint32_t n = uint32_t(m) / uint32_t(OHW), pix = uint32_t(m) - n * uint32_t(OHW);
            const int64_t obase = int64_t(n) * a.y_bs + int64_t(pix) * a.y_ld;
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int cb = n0 + wr * (BN / 2) + i * 16 + fc * 4;
                float v[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    v[r] = acc[i][j][r];
                    if (a.bias && cb + r < a.Nout) v[r] += a.bias[cb + r];
                }
                if (a.st_sum) {
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (cb + r < a.Nout) { ssum[i][r] += v[r]; ssq[i][r] += v[r] * v[r]; }
                }
                if (a.out_f32 == 2) {
                    uint16_t* yp = reinterpret_cast<uint16_t*>(a.y) + obase + cb;
                    if (cb + 3 < a.Nout) {
                        uint2 o;
                        o.x = uint32_t(f2h(v[0])) | (uint32_t(f2h(v[1])) << 16);
                        o.y = uint32_t(f2h(v[2])) | (uint32_t(f2h(v[3])) << 16);
                        *reinterpret_cast<uint2*>(yp) = o;
                    } else {
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            if (cb + r < a.Nout) yp[r] = f2h(v[r]);
                    }
                } else if (a.out_f32) {
                    float* yp = reinterpret_cast<float*>(a.y) + obase + cb;
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (cb + r < a.Nout) yp[r] = a.accumulate ? yp[r] + v[r] : v[r];
                } else {
                    bf16_t* yp = reinterpret_cast<bf16_t*>(a.y) + obase + cb;
                    if (cb + 3 < a.Nout) {
                        if (a.accumulate) {
                            uint2 o = *reinterpret_cast<const uint2*>(yp);
                            v[0] += bf2f(bf16_t(o.x & 0xffff)); v[1] += bf2f(bf16_t(o.x >> 16));
                            v[2] += bf2f(bf16_t(o.y & 0xffff)); v[3] += bf2f(bf16_t(o.y >> 16));
                        }
                        uint2 o;
                        o.x = uint32_t(f2bf(v[0])) | (uint32_t(f2bf(v[1])) << 16);
                        o.y = uint32_t(f2bf(v[2])) | (uint32_t(f2bf(v[3])) << 16);
                        *reinterpret_cast<uint2*>(yp) = o;
                    } else {
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            if (cb + r < a.Nout) yp[r] = f2bf(a.accumulate ? bf2f(yp[r]) + v[r] : v[r]);
                    }
                }
            }
        }
    }

    if (a.st_sum) {
        // reduce over the 16 pixel lanes, then over the two pixel-half waves
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float s = ssum[i][r], q = ssq[i][r];
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) {
                    s += __shfl_xor(s, o, 64);
                    q += __shfl_xor(q, o, 64);
                }
                if (fr == 0) {
                    int cl = wr * (BN / 2) + i * 16 + (lane >> 4) * 4 + r;
                    red[0][wc][cl] = s;
                    red[1][wc][cl] = q;
                }
            }
        __syncthreads();
        for (int c = tid; c < BN; c += 256) {
            int ch = n0 + c;
            if (ch < a.Nout) {
                a.st_sum[int64_t(blockIdx.x) * a.Nout + ch] = red[0][0][c] + red[0][1][c];
                a.st_sq[int64_t(blockIdx.x) * a.Nout + ch] = red[1][0][c] + red[1][1][c];
            }
        }
    }
}

// ------------------------------------------------------------------ wgrad
struct WgradArgs {
    const bf16_t* dz; int64_t dz_bs, dz_ld;  // (N, OH, OW, Cout) view
    const bf16_t* x; int64_t x_bs, x_ld;     // (N, IH, IW, Cin) view
    float* dw;                               // [Cout][KH*KW][Cin] fp32, accumulated atomically
    int IH, IW, Cin, OH, OW, Cout, KH, KW, stride, pad;
    int64_t M;                               // N*OH*OW
    int64_t chunk;                           // pixels per split (multiple of 32)
    int ci_tiles;
};

constexpr int WG_T = 64;                      // tile: 64 co x 64 ci
constexpr int WG_RS = WG_T * 2 + 32;          // LDS row stride in bytes (bank-conflict-free tr reads)

__global__ void __launch_bounds__(256) wgrad_kernel(WgradArgs a) {
    __shared__ __attribute__((aligned(16))) char As[2][32 * WG_RS];   // dz rows (pixels) x 64 co
    __shared__ __attribute__((aligned(16))) char Bs[2][32 * WG_RS];   // x rows (pixels) x 64 ci
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 1, wc = wave & 1;
    const int co0 = blockIdx.x * WG_T;
    const int tap = blockIdx.y / a.ci_tiles;
    const int ci0 = (blockIdx.y - tap * a.ci_tiles) * WG_T;
    const int kh = tap / a.KW, kw = tap - kh * a.KW;
    const int64_t p_begin = int64_t(blockIdx.z) * a.chunk;
    const int64_t p_end = min(a.M, p_begin + a.chunk);
    if (p_begin >= p_end) return;
    const int64_t OHW = int64_t(a.OH) * a.OW;
    const int srow = tid >> 3, sc = tid & 7;      // staging: one 16-B chunk per thread per tile

    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    uint4 ra, rb;
    const uint32_t uOHW = uint32_t(OHW), uOW = uint32_t(a.OW);
    auto load = [&](int64_t p0) {
        int64_t p = p0 + srow;
        ra = make_uint4(0, 0, 0, 0);
        rb = make_uint4(0, 0, 0, 0);
        if (p < p_end) {
            const uint32_t up = uint32_t(p);                  // M < 2^31 (checked on the host)
            const uint32_t n = up / uOHW, pix = up - n * uOHW;
            const int oh = int(pix / uOW), ow = int(pix - uint32_t(oh) * uOW);
            int co = co0 + sc * 8;
            if (co < a.Cout) ra = *reinterpret_cast<const uint4*>(a.dz + int64_t(n) * a.dz_bs + int64_t(pix) * a.dz_ld + co);
            int ih = oh * a.stride - a.pad + kh, iw = ow * a.stride - a.pad + kw;
            int ci = ci0 + sc * 8;
            if (ci < a.Cin && ih >= 0 && ih < a.IH && iw >= 0 && iw < a.IW) {
                uint4 h = *reinterpret_cast<const uint4*>(a.x + int64_t(n) * a.x_bs + (int64_t(ih) * a.IW + iw) * a.x_ld + ci);
                uint32_t w4[4] = {h.x, h.y, h.z, h.w};
#pragma unroll
                for (int e = 0; e < 4; ++e)   // fp16 activation -> bf16 MFMA operand
                    w4[e] = uint32_t(f2bf(h2f(uint16_t(w4[e] & 0xffff)))) | (uint32_t(f2bf(h2f(uint16_t(w4[e] >> 16)))) << 16);
                rb = make_uint4(w4[0], w4[1], w4[2], w4[3]);
            }
        }
    };
    auto store = [&](int buf) {
        *reinterpret_cast<uint4*>(&As[buf][srow * WG_RS + sc * 16]) = ra;
        *reinterpret_cast<uint4*>(&Bs[buf][srow * WG_RS + sc * 16]) = rb;
    };

    // transposed fragment read: group g = lane>>4 owns k rows {4g..4g+3} and {16+4g..16+4g+3};
    // lane 4q+p of the group addresses row (4g+q [+16]), columns col0 + 4p .. +3
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
    auto frag = [&](const char* base, int col0) -> bf16x8 {
        const char* p1 = base + (4 * g + q) * WG_RS + (col0 + 4 * pp) * 2;
        const char* p2 = p1 + 16 * WG_RS;
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(p1));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(p2));
        typedef short s16x8 __attribute__((ext_vector_type(8)));
        s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        return __builtin_bit_cast(bf16x8, v);
    };

    load(p_begin);
    store(0);
    __syncthreads();
    int buf = 0;
    for (int64_t p0 = p_begin; p0 < p_end; p0 += 32) {
        const bool more = p0 + 32 < p_end;
        if (more) load(p0 + 32);
        bf16x8 af[2], bf[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i] = frag(As[buf], wr * 32 + i * 16);
#pragma unroll
        for (int j = 0; j < 2; ++j) bf[j] = frag(Bs[buf], wc * 32 + j * 16);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
        if (more) store(buf ^ 1);
        __syncthreads();
        buf ^= 1;
    }
    // D[co][ci]: lane holds co rows (lane>>4)*4 + r, ci column lane&15
    const int64_t trow = int64_t(a.KH) * a.KW * a.Cin;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            int ci = ci0 + wc * 32 + j * 16 + (lane & 15);
            if (ci >= a.Cin) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                int co = co0 + wr * 32 + i * 16 + (lane >> 4) * 4 + r;
                if (co < a.Cout) atomicAdd(a.dw + co * trow + int64_t(tap) * a.Cin + ci, acc[i][j][r]);
            }
        }
}

// [Cout][KH*KW][Cin] fp32 -> [Cout][Cin][KH][KW] fp32 (PyTorch OIHW), optionally accumulating
__global__ void ohwi_to_oihw_kernel(const float* __restrict__ src, float* __restrict__ dst, int Cout, int Cin,
                                    int T, int accumulate) {
    int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    int64_t total = int64_t(Cout) * Cin * T;
    if (i >= total) return;
    int t = int(i % T);
    int64_t r = i / T;
    int ci = int(r % Cin);
    int co = int(r / Cin);
    float v = src[(int64_t(co) * T + t) * Cin + ci];
    dst[i] = accumulate ? dst[i] + v : v;
}

// ------------------------------------------------------------------ stem conv (Cin = 1), fp32 image input
// y[n,oh,ow,co] = sum_t w[co][t] * img[n, oh*s-p+kh, ow*s-p+kw]; stats partials per block
__global__ void __launch_bounds__(256) conv_first_fwd_kernel(const float* __restrict__ img, const float* __restrict__ w,
                                                             bf16_t* __restrict__ y, float* __restrict__ st_sum,
                                                             float* __restrict__ st_sq, int N, int H, int W, int OH,
                                                             int OW, int Cout, int K, int stride, int pad) {
    // block: 256 threads = 8 channel-groups of 4... generic: thread -> (pixel, 4 channels)
    extern __shared__ float smem[];
    float* ws = smem;                        // Cout*K
    float* red = smem + Cout * K;            // 2 * Cout
    for (int i = threadIdx.x; i < Cout * K; i += blockDim.x) ws[i] = w[i];
    for (int i = threadIdx.x; i < 2 * Cout; i += blockDim.x) red[i] = 0.f;
    __syncthreads();
    const int cg = Cout / 4;                 // channel groups per pixel
    const int64_t M = int64_t(N) * OH * OW;
    const int64_t total = M * cg;
    float ls[4] = {0, 0, 0, 0}, lq[4] = {0, 0, 0, 0};
    int my_cg = -1;
    for (int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; idx < total;
         idx += int64_t(gridDim.x) * blockDim.x) {
        int g4 = int(idx % cg);
        int64_t m = idx / cg;
        my_cg = g4;   // blockDim multiple of cg keeps g4 fixed per thread
        int64_t n = m / (int64_t(OH) * OW);
        int64_t pix = m - n * OH * OW;
        int oh = int(pix / OW), ow = int(pix % OW);
        float patch[9];
        for (int kh = 0, t = 0; kh < 3; ++kh)
            for (int kw = 0; kw < 3; ++kw, ++t) {
                int ih = oh * stride - pad + kh, iw = ow * stride - pad + kw;
                patch[t] = (ih >= 0 && ih < H && iw >= 0 && iw < W) ? img[(n * H + ih) * W + iw] : 0.f;
            }
        uint2 o;
        float v[4];
        for (int r = 0; r < 4; ++r) {
            const float* wr_ = ws + (g4 * 4 + r) * K;
            float s = 0.f;
            for (int t = 0; t < K; ++t) s += wr_[t] * patch[t];
            v[r] = s;
            ls[r] += s;
            lq[r] += s * s;
        }
        o.x = uint32_t(f2h(v[0])) | (uint32_t(f2h(v[1])) << 16);
        o.y = uint32_t(f2h(v[2])) | (uint32_t(f2h(v[3])) << 16);
        *reinterpret_cast<uint2*>(y + m * Cout + g4 * 4) = o;
    }
    if (my_cg >= 0)
        for (int r = 0; r < 4; ++r) {
            atomicAdd(&red[my_cg * 4 + r], ls[r]);
            atomicAdd(&red[Cout + my_cg * 4 + r], lq[r]);
        }
    __syncthreads();
    for (int c = threadIdx.x; c < Cout; c += blockDim.x) {
        st_sum[int64_t(blockIdx.x) * Cout + c] = red[c];
        st_sq[int64_t(blockIdx.x) * Cout + c] = red[Cout + c];
    }
}

// dW[co][t] += sum_p dz[p][co] * patch(p)[t]   (no dgrad: the image needs no gradient)
__global__ void __launch_bounds__(256) conv_first_wgrad_kernel(const bf16_t* __restrict__ dz, const float* __restrict__ img,
                                                               float* __restrict__ dw, int N, int H, int W, int OH,
                                                               int OW, int Cout, int stride, int pad) {
    extern __shared__ float sred[];          // Cout*9
    for (int i = threadIdx.x; i < Cout * 9; i += blockDim.x) sred[i] = 0.f;
    __syncthreads();
    const int cg = Cout / 4;
    const int64_t M = int64_t(N) * OH * OW;
    const int64_t total = M * cg;
    float acc[4][9];
    for (int r = 0; r < 4; ++r)
        for (int t = 0; t < 9; ++t) acc[r][t] = 0.f;
    int my_cg = -1;
    for (int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; idx < total;
         idx += int64_t(gridDim.x) * blockDim.x) {
        int g4 = int(idx % cg);
        int64_t m = idx / cg;
        my_cg = g4;
        int64_t n = m / (int64_t(OH) * OW);
        int64_t pix = m - n * OH * OW;
        int oh = int(pix / OW), ow = int(pix % OW);
        uint2 d = *reinterpret_cast<const uint2*>(dz + m * Cout + g4 * 4);
        float g[4] = {bf2f(bf16_t(d.x & 0xffff)), bf2f(bf16_t(d.x >> 16)), bf2f(bf16_t(d.y & 0xffff)),
                      bf2f(bf16_t(d.y >> 16))};
        for (int kh = 0, t = 0; kh < 3; ++kh)
            for (int kw = 0; kw < 3; ++kw, ++t) {
                int ih = oh * stride - pad + kh, iw = ow * stride - pad + kw;
                float xv = (ih >= 0 && ih < H && iw >= 0 && iw < W) ? img[(n * H + ih) * W + iw] : 0.f;
                for (int r = 0; r < 4; ++r) acc[r][t] += g[r] * xv;
            }
    }
    if (my_cg >= 0)
        for (int r = 0; r < 4; ++r)
            for (int t = 0; t < 9; ++t) atomicAdd(&sred[(my_cg * 4 + r) * 9 + t], acc[r][t]);
    __syncthreads();
    for (int i = threadIdx.x; i < Cout * 9; i += blockDim.x) atomicAdd(&dw[i], sred[i]);
}

// ------------------------------------------------------------------ depthwise 3x3, stride 1, pad 1
// input channel c of the conv reads source channel map(c) = (c / gsz) * gstride + goff + c % gsz
// (Attention.pe consumes v.reshape(B, C, H, W), i.e. the v slice of every head of qkv)
struct DwArgs {
    const bf16_t* x; int64_t x_bs, x_ld; int gsz, gstride, goff;
    const float* w;            // fp32 [C][9]
    bf16_t* y;                 // dense (N, H, W, C) (fwd) / dx view (bwd)
    int64_t y_bs, y_ld;
    int N, H, W, C;
};

__global__ void dw3x3_fwd_kernel(DwArgs a, float* st_sum, float* st_sq) {
    // one thread per (pixel, channel); block = 256 channels-major threads
    extern __shared__ float sh[];           // 2*C partials
    for (int i = threadIdx.x; i < 2 * a.C; i += blockDim.x) sh[i] = 0.f;
    __syncthreads();
    const int64_t total = int64_t(a.N) * a.H * a.W * a.C;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += int64_t(gridDim.x) * blockDim.x) {
        int c = int(i % a.C);
        int64_t m = i / a.C;
        int64_t n = m / (int64_t(a.H) * a.W);
        int64_t pix = m - n * a.H * a.W;
        int h = int(pix / a.W), wcol = int(pix % a.W);
        int sc = (c / a.gsz) * a.gstride + a.goff + c % a.gsz;
        float s = 0.f;
        for (int kh = 0; kh < 3; ++kh)
            for (int kw = 0; kw < 3; ++kw) {
                int ih = h - 1 + kh, iw = wcol - 1 + kw;
                if (ih >= 0 && ih < a.H && iw >= 0 && iw < a.W)
                    s += a.w[c * 9 + kh * 3 + kw] * h2f(a.x[n * a.x_bs + (int64_t(ih) * a.W + iw) * a.x_ld + sc]);
            }
        a.y[m * a.C + c] = f2h(s);
        atomicAdd(&sh[c], s);
        atomicAdd(&sh[a.C + c], s * s);
    }
    __syncthreads();
    for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
        st_sum[int64_t(blockIdx.x) * a.C + c] = sh[c];
        st_sq[int64_t(blockIdx.x) * a.C + c] = sh[a.C + c];
    }
}

// dx (mapped channels, accumulate into view) and dW (atomic) from dense dz (N,H,W,C)
__global__ void dw3x3_bwd_kernel(DwArgs a, const bf16_t* __restrict__ dz, float* __restrict__ dw, int accumulate) {
    extern __shared__ float sh[];           // 9*C
    for (int i = threadIdx.x; i < 9 * a.C; i += blockDim.x) sh[i] = 0.f;
    __syncthreads();
    const int64_t total = int64_t(a.N) * a.H * a.W * a.C;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += int64_t(gridDim.x) * blockDim.x) {
        int c = int(i % a.C);
        int64_t m = i / a.C;
        int64_t n = m / (int64_t(a.H) * a.W);
        int64_t pix = m - n * a.H * a.W;
        int h = int(pix / a.W), wcol = int(pix % a.W);
        int sc = (c / a.gsz) * a.gstride + a.goff + c % a.gsz;
        float gx = 0.f;
        for (int kh = 0; kh < 3; ++kh)
            for (int kw = 0; kw < 3; ++kw) {
                // dx[h,w] += dz[h+1-kh, w+1-kw] * w[kh,kw]
                int oh = h + 1 - kh, ow = wcol + 1 - kw;
                if (oh >= 0 && oh < a.H && ow >= 0 && ow < a.W)
                    gx += a.w[c * 9 + kh * 3 + kw] * bf2f(dz[(n * a.H * a.W + int64_t(oh) * a.W + ow) * a.C + c]);
                // dW[kh,kw] += dz[h,w] * x[h-1+kh, w-1+kw]
                int ih = h - 1 + kh, iw = wcol - 1 + kw;
                if (ih >= 0 && ih < a.H && iw >= 0 && iw < a.W)
                    atomicAdd(&sh[c * 9 + kh * 3 + kw],
                              bf2f(dz[m * a.C + c]) * h2f(a.x[n * a.x_bs + (int64_t(ih) * a.W + iw) * a.x_ld + sc]));
            }
        bf16_t* yp = a.y + n * a.y_bs + pix * a.y_ld + sc;
        *yp = f2bf(accumulate ? bf2f(*yp) + gx : gx);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 9 * a.C; i += blockDim.x) atomicAdd(&dw[i], sh[i]);
}

// ------------------------------------------------------------------ weight preparation
// fp32 OIHW master weights -> fp16 [Cout][KH][KW][Cin] (fwd) and bf16 [Cin][KH][KW][Cout] (dgrad)
__global__ void prep_weights_kernel(const ym_wprep_entry* __restrict__ tab, int n_entries, int64_t total) {
    int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= total) return;
    int e = 0;
    while (e + 1 < n_entries && tab[e + 1].elem_offset <= i) ++e;
    const ym_wprep_entry t = tab[e];
    int64_t j = i - t.elem_offset;                 // index in OIHW
    int T = t.kh * t.kw;
    int tap = int(j % T);
    int64_t r = j / T;
    int ci = int(r % t.cin);
    int co = int(r / t.cin);
    const float v = t.src[j];
    if (t.dst_fwd) t.dst_fwd[(int64_t(co) * T + tap) * t.cin + ci] = f2h(v);     // fp16 (forward operand)
    if (t.dst_t) t.dst_t[(int64_t(ci) * T + tap) * t.cout_t + co] = f2bf(v);     // bf16 (dgrad operand)
}

template <int BM, int BN, int MODE>
int launch_gemm(const GemmArgs& a0, int max_blocks, hipStream_t st) {
    GemmArgs a = a0;
    a.mtiles = int((a.M + BM - 1) / BM);
    int ntiles = (a.Nout + BN - 1) / BN;
    int gx = a.mtiles;
    if (a.st_sum) {
        // stats partials are per grid-x block: bound the grid, keep it a multiple of 8 (XCD grouping)
        int cap = max(8, (max_blocks / ntiles) & ~7);
        gx = min(gx, cap);
    }
    hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, MODE>), dim3(gx, ntiles), dim3(256), 0, st, a);
    return gx;
}

}  // namespace
}  // namespace ym

using namespace ym;

static int pick_and_launch(GemmArgs a, int mode, int max_blocks, hipStream_t st) {
    // channel tile from the output channel count
    if (mode == MODE_FWD) {
        if (a.Nout >= 128) return launch_gemm<128, 128, MODE_FWD>(a, max_blocks, st);
        if (a.Nout >= 64) return launch_gemm<128, 64, MODE_FWD>(a, max_blocks, st);
        return launch_gemm<128, 32, MODE_FWD>(a, max_blocks, st);
    }
    if (a.Nout >= 128) return launch_gemm<128, 128, MODE_DGRAD>(a, max_blocks, st);
    if (a.Nout >= 64) return launch_gemm<128, 64, MODE_DGRAD>(a, max_blocks, st);
    return launch_gemm<128, 32, MODE_DGRAD>(a, max_blocks, st);
}

extern "C" int ym_conv_stat_blocks(int64_t M, int Cout) {
    // grid-x used for the stats partials by ym_conv_fwd (callers size the partial buffers with it)
    int BN = Cout >= 128 ? 128 : (Cout >= 64 ? 64 : 32);
    int ntiles = (Cout + BN - 1) / BN;
    int mtiles = int((M + 127) / 128);
    int cap = std::max(8, (2048 / ntiles) & ~7);
    return std::min(mtiles, cap);
}

extern "C" int ym_conv_fwd(const ym_conv_desc* d, const uint16_t* x, const uint16_t* w, void* y, const float* bias,
                           float* stat_sum, float* stat_sq, void* stream) {
    YM_CHECK_ARG(d && x && w && y, "ym_conv_fwd: null argument");
    YM_CHECK_ARG(d->cin % 8 == 0, "ym_conv_fwd: Cin %% 8 != 0 (Cin=%d)", d->cin);
    YM_CHECK_ARG(d->x_ld % 8 == 0 && d->x_bs % 8 == 0, "ym_conv_fwd: input view not 16-byte aligned");
    YM_CHECK_ARG(d->out_f32 == 1 || (d->y_ld % 4 == 0 && d->y_bs % 4 == 0), "ym_conv_fwd: output view not 8-byte aligned");
    YM_CHECK_ARG((stat_sum == nullptr) == (stat_sq == nullptr), "ym_conv_fwd: stats pointers");
    GemmArgs a{};
    a.x = x; a.x_bs = d->x_bs; a.x_ld = d->x_ld;
    a.w = w;
    a.y = y; a.y_bs = d->y_bs; a.y_ld = d->y_ld;
    a.bias = bias; a.st_sum = stat_sum; a.st_sq = stat_sq;
    a.GH = d->h; a.GW = d->w; a.Kin = d->cin;
    a.OH = d->oh; a.OW = d->ow; a.Nout = d->cout;
    a.KH = d->k; a.KW = d->k; a.stride = d->stride; a.pad = d->pad;
    a.M = int64_t(d->n) * d->oh * d->ow;
    a.out_f32 = d->out_f32; a.accumulate = d->accumulate;
    if (a.M == 0) return YM_OK;
    YM_CHECK_ARG(a.M < (int64_t(1) << 31), "ym_conv_fwd: too many pixels");
    pick_and_launch(a, MODE_FWD, 2048, as_stream(stream));
    YM_LAUNCH_CHECK("ym_conv_fwd");
    return YM_OK;
}

extern "C" int ym_conv_dgrad(const ym_conv_desc* d, const uint16_t* dz, const uint16_t* wt, uint16_t* dx, void* stream) {
    // d describes the FORWARD conv; dz is (n, oh, ow, cout) with the y_* view, dx is (n, h, w, cin) with the x_* view
    YM_CHECK_ARG(d && dz && wt && dx, "ym_conv_dgrad: null argument");
    YM_CHECK_ARG(d->cout % 8 == 0, "ym_conv_dgrad: Cout %% 8 != 0 (Cout=%d)", d->cout);
    YM_CHECK_ARG(d->y_ld % 8 == 0 && d->y_bs % 8 == 0, "ym_conv_dgrad: dz view not 16-byte aligned");
    YM_CHECK_ARG(d->x_ld % 4 == 0 && d->x_bs % 4 == 0, "ym_conv_dgrad: dx view not 8-byte aligned");
    GemmArgs a{};
    a.x = dz; a.x_bs = d->y_bs; a.x_ld = d->y_ld;
    a.w = wt;
    a.y = dx; a.y_bs = d->x_bs; a.y_ld = d->x_ld;
    a.GH = d->oh; a.GW = d->ow; a.Kin = d->cout;
    a.OH = d->h; a.OW = d->w; a.Nout = d->cin;
    a.KH = d->k; a.KW = d->k; a.stride = d->stride; a.pad = d->pad;
    a.M = int64_t(d->n) * d->h * d->w;
    a.accumulate = d->accumulate;
    if (a.M == 0) return YM_OK;
    YM_CHECK_ARG(a.M < (int64_t(1) << 31), "ym_conv_dgrad: too many pixels");
    pick_and_launch(a, MODE_DGRAD, 4096, as_stream(stream));
    YM_LAUNCH_CHECK("ym_conv_dgrad");
    return YM_OK;
}

extern "C" int ym_conv_wgrad(const ym_conv_desc* d, const uint16_t* dz, const uint16_t* x, float* dw_ohwi, void* stream) {
    // dw_ohwi [cout][k*k][cin] fp32 must be zeroed (or hold a partial sum) by the caller
    YM_CHECK_ARG(d && dz && x && dw_ohwi, "ym_conv_wgrad: null argument");
    YM_CHECK_ARG(d->cin % 8 == 0 && d->cout % 8 == 0, "ym_conv_wgrad: channels %% 8 != 0");
    YM_CHECK_ARG(d->x_ld % 8 == 0 && d->y_ld % 8 == 0 && d->x_bs % 8 == 0 && d->y_bs % 8 == 0,
                 "ym_conv_wgrad: views not 16-byte aligned");
    WgradArgs a{};
    a.dz = dz; a.dz_bs = d->y_bs; a.dz_ld = d->y_ld;
    a.x = x; a.x_bs = d->x_bs; a.x_ld = d->x_ld;
    a.dw = dw_ohwi;
    a.IH = d->h; a.IW = d->w; a.Cin = d->cin; a.OH = d->oh; a.OW = d->ow; a.Cout = d->cout;
    a.KH = d->k; a.KW = d->k; a.stride = d->stride; a.pad = d->pad;
    a.M = int64_t(d->n) * d->oh * d->ow;
    if (a.M == 0) return YM_OK;
    YM_CHECK_ARG(a.M < (int64_t(1) << 31), "ym_conv_wgrad: too many pixels");
    int co_t = (a.Cout + WG_T - 1) / WG_T;
    a.ci_tiles = (a.Cin + WG_T - 1) / WG_T;
    int cols = a.ci_tiles * a.KH * a.KW;
    int64_t steps = (a.M + 31) / 32;
    int64_t splits = std::max<int64_t>(1, std::min<int64_t>(2048 / (co_t * cols), steps / 8));
    splits = std::min<int64_t>(splits, 65535);
    a.chunk = ((steps + splits - 1) / splits) * 32;
    splits = (a.M + a.chunk - 1) / a.chunk;
    hipLaunchKernelGGL(wgrad_kernel, dim3(co_t, cols, unsigned(splits)), dim3(256), 0, as_stream(stream), a);
    YM_LAUNCH_CHECK("ym_conv_wgrad");
    return YM_OK;
}

extern "C" int ym_wgrad_to_oihw(const float* src, float* dst, int cout, int cin, int taps, int accumulate, void* stream) {
    int64_t total = int64_t(cout) * cin * taps;
    if (total == 0) return YM_OK;
    hipLaunchKernelGGL(ohwi_to_oihw_kernel, dim3(unsigned((total + 255) / 256)), dim3(256), 0, as_stream(stream), src,
                       dst, cout, cin, taps, accumulate);
    YM_LAUNCH_CHECK("ym_wgrad_to_oihw");
    return YM_OK;
}

extern "C" int ym_conv_first_fwd(const float* img, const float* w_oihw, uint16_t* y, float* stat_sum, float* stat_sq,
                                 int n, int h, int w, int oh, int ow, int cout, int stride, int pad, int blocks,
                                 void* stream) {
    YM_CHECK_ARG(cout % 4 == 0 && 256 % (cout / 4) == 0, "ym_conv_first_fwd: cout=%d unsupported", cout);
    size_t lds = (size_t(cout) * 9 + 2 * cout) * sizeof(float);
    hipLaunchKernelGGL(conv_first_fwd_kernel, dim3(blocks), dim3(256), lds, as_stream(stream), img, w_oihw, y,
                       stat_sum, stat_sq, n, h, w, oh, ow, cout, 9, stride, pad);
    YM_LAUNCH_CHECK("ym_conv_first_fwd");
    return YM_OK;
}

extern "C" int ym_conv_first_wgrad(const uint16_t* dz, const float* img, float* dw_oihw, int n, int h, int w, int oh,
                                   int ow, int cout, int stride, int pad, void* stream) {
    YM_CHECK_ARG(cout % 4 == 0 && 256 % (cout / 4) == 0, "ym_conv_first_wgrad: cout=%d unsupported", cout);
    hipLaunchKernelGGL(conv_first_wgrad_kernel, dim3(1024), dim3(256), size_t(cout) * 9 * sizeof(float),
                       as_stream(stream), dz, img, dw_oihw, n, h, w, oh, ow, cout, stride, pad);
    YM_LAUNCH_CHECK("ym_conv_first_wgrad");
    return YM_OK;
}

extern "C" int ym_dw3x3_fwd(const uint16_t* x, int64_t x_bs, int64_t x_ld, int gsz, int gstride, int goff,
                            const float* w, uint16_t* y, float* stat_sum, float* stat_sq, int n, int h, int wd, int c,
                            int blocks, void* stream) {
    DwArgs a{x, x_bs, x_ld, gsz, gstride, goff, w, y, 0, 0, n, h, wd, c};
    hipLaunchKernelGGL(dw3x3_fwd_kernel, dim3(blocks), dim3(256), size_t(2 * c) * sizeof(float), as_stream(stream), a,
                       stat_sum, stat_sq);
    YM_LAUNCH_CHECK("ym_dw3x3_fwd");
    return YM_OK;
}

extern "C" int ym_dw3x3_bwd(const uint16_t* x, int64_t x_bs, int64_t x_ld, int gsz, int gstride, int goff,
                            const float* w, const uint16_t* dz, uint16_t* dx, int64_t dx_bs, int64_t dx_ld, float* dw,
                            int n, int h, int wd, int c, int accumulate, void* stream) {
    DwArgs a{x, x_bs, x_ld, gsz, gstride, goff, w, dx, dx_bs, dx_ld, n, h, wd, c};
    hipLaunchKernelGGL(dw3x3_bwd_kernel, dim3(256), dim3(256), size_t(9 * c) * sizeof(float), as_stream(stream), a, dz,
                       dw, accumulate);
    YM_LAUNCH_CHECK("ym_dw3x3_bwd");
    return YM_OK;
}

extern "C" int ym_prep_weights(const ym_wprep_entry* table_dev, int n_entries, int64_t total_elems, void* stream) {
    if (total_elems == 0) return YM_OK;
    hipLaunchKernelGGL(prep_weights_kernel, dim3(unsigned((total_elems + 255) / 256)), dim3(256), 0, as_stream(stream),
                       table_dev, n_entries, total_elems);
    YM_LAUNCH_CHECK("ym_prep_weights");
    return YM_OK;
}
