// Direct MFMA convolution for the high-resolution, few-channel layers of the YOLOv11 graph
// (the 320x320 / 160x160 maps of the stem stage: 32-128 channels), fp16 forward / bf16 data
// gradient, fp32 accumulate.
//
// Replaces nn.Conv2d forward / input-gradient inside Conv (/root/reference/yolo_scratch_cuda/
// models/yolo11_modules.py:21-33) where the implicit GEMMs (conv.hip, conv_pipe.hip) are
// latency-bound: with 32-96 input channels a 128-pixel tile has only 5-9 K steps, each one a full
// LDS-DMA round trip, and the 3x3 taps re-stage the input nine times through LDS (measured
// 0.22-0.26 ms for a 32->32 3x3 160x160 layer whose HBM roof is 0.03 ms).
//
// Here the whole weight tensor of the layer lives in registers (at most 144 VGPRs: Cout/16 x taps x
// Cin/32 MFMA A-fragments per lane) and every wave streams pixels: each 16-pixel MFMA B-fragment
// is ONE 16-byte load per lane straight from the NHWC activation (8 consecutive channels of one
// pixel; the 3x3 neighbours' re-reads hit L1/L2), out-of-image taps read zero through out-of-range
// buffer offsets.  No LDS on the main path, no barriers; the only reduction is the BatchNorm
// statistics (xor shuffles, then the waves in order through LDS: one partial row per workgroup).
// Data gradients: stride 1 as a conv of dz with the transposed weight copy (taps mirrored by the
// index formula), stride 2 over 2x2-pixel quads (all four output-parity classes of a dz pixel's
// neighbourhood in one task, conv_direct_quad_kernel).
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "conv_direct.h"
#include "conv_epi.h"
#include "tile.h"

namespace ym {

Policy g_direct_force{-1};

namespace {

struct DirArgs {
    const uint16_t* x; int64_t x_bs, x_ld;    // gathered input view (fwd: x fp16, dgrad: dz bf16)
    const uint16_t* w;                         // [Nout][KS][KS][Kin] (fwd: fp16 w, dgrad: bf16 transposed copy)
    void* y; int64_t y_bs, y_ld;               // output view
    float* st_sum; float* st_sq;               // [gridDim.x][Nout] or null
    int GH, GW, OH, OW, N;                     // gathered map, output map
    int Kin, Nout, pad;
    int accumulate;
    int OHc, OWc;                              // class map (dgrad stride 2: ceil(O/2); else O)
    int64_t tpc;                               // tasks (16 x TP pixels, or 2x2-pixel quads, per lane group)
};

template <int MODE>
using frag_t = typename std::conditional<MODE == 0, f16x8, bf16x8>::type;

__device__ __forceinline__ f32x4 mma(f16x8 a, f16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mma(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// pixel coordinates of the lane's pixel in each 16-pixel group of task `tl` (class (PY, PX) of a
// stride-2 data gradient: every other row / column)
template <int TP, int CS>
struct TaskPix {
    int n[TP], oh[TP], ow[TP];
    bool ok[TP];
    __device__ __forceinline__ void decode(const DirArgs& a, int64_t tl, int fr, int py, int px) {
        const uint32_t chw = uint32_t(a.OHc) * uint32_t(a.OWc);
#pragma unroll
        for (int g = 0; g < TP; ++g) {
            const int64_t m = tl * (16 * TP) + g * 16 + fr;
            const uint32_t nn = uint32_t(m / chw), r = uint32_t(m - int64_t(nn) * chw);
            const uint32_t i = r / uint32_t(a.OWc), j = r - i * uint32_t(a.OWc);
            n[g] = int(nn);
            oh[g] = int(i) * CS + py;
            ow[g] = int(j) * CS + px;
            ok[g] = int(nn) < a.N && oh[g] < a.OH && ow[g] < a.OW;
        }
    }
};

// NT: 16-channel output tiles (Nout <= 16 NT), KC: 32-channel input chunks (Kin = 32 KC), KS kernel
// size, S stride, MODE 0 forward (fp16 out + statistics) / 1 data gradient (bf16 out), TP 16-pixel
// groups per wave task, (PY, PX) the output-parity class of a stride-2 data gradient (else 0, 0).
// All of a task's input fragments are loaded before its first MFMA (one memory latency per task, not
// one per tap); the 1x1 forms also load the NEXT task's fragments before this task's MFMAs.
template <int NT, int KC, int KS, int S, int MODE, int TP, int PY, int PX>
__device__ __forceinline__ void direct_body(const DirArgs& a, float (&ssum)[NT][4], float (&ssq)[NT][4], int64_t first,
                                            int64_t step, int64_t ntask, char* ep) {
    using F = frag_t<MODE>;
    constexpr int TAPS = KS * KS;
    constexpr bool CLS = S == 2 && MODE == 1;
    constexpr int CS = CLS ? 2 : 1;
    const int lane = threadIdx.x & 63, fr = lane & 15, fc = lane >> 4;
    // taps that reach this class (all taps otherwise)
    auto live = [&](int t) constexpr -> bool {
        const int kh = t / KS, kw = t % KS;
        return !CLS || (((PY + 1 - kh) & 1) == 0 && ((PX + 1 - kw) & 1) == 0);
    };
    F wa[TAPS][KC][NT];
    {
        const __amdgpu_buffer_rsrc_t wr = make_rsrc(a.w, int64_t(a.Nout) * TAPS * a.Kin * 2);
#pragma unroll
        for (int t = 0; t < TAPS; ++t) {
            if (!live(t)) continue;
#pragma unroll
            for (int kc = 0; kc < KC; ++kc)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) {
                    const int co = nt * 16 + fr;
                    const uint32_t off =
                        co < a.Nout ? uint32_t(((co * TAPS + t) * a.Kin + kc * 32 + fc * 8) * 2) : OOB;
                    wa[t][kc][nt] = __builtin_bit_cast(F, buf_load16(wr, off));
                }
        }
    }
    const __amdgpu_buffer_rsrc_t xr = make_rsrc(a.x, int64_t(a.N) * a.x_bs * 2);
    const __amdgpu_buffer_rsrc_t yres = make_rsrc(a.y, int64_t(a.N) * a.y_bs * 2);
    auto load = [&](const TaskPix<TP, CS>& P, F (&b)[TAPS][TP][KC]) {
#pragma unroll
        for (int t = 0; t < TAPS; ++t) {
            if (!live(t)) continue;
            const int kh = t / KS, kw = t % KS;
#pragma unroll
            for (int g = 0; g < TP; ++g) {
                int ih, iw;
                if constexpr (MODE == 0) {
                    ih = P.oh[g] * S - a.pad + kh;
                    iw = P.ow[g] * S - a.pad + kw;
                } else {
                    ih = (P.oh[g] + a.pad - kh) >> (S - 1);     // exact for the taps this class keeps
                    iw = (P.ow[g] + a.pad - kw) >> (S - 1);
                }
                const bool in = P.ok[g] && unsigned(ih) < unsigned(a.GH) && unsigned(iw) < unsigned(a.GW);
                const uint32_t base =
                    in ? uint32_t((int64_t(P.n[g]) * a.x_bs + (int64_t(ih) * a.GW + iw) * a.x_ld + fc * 8) * 2) : OOB;
#pragma unroll
                for (int kc = 0; kc < KC; ++kc)
                    b[t][g][kc] = __builtin_bit_cast(F, buf_load16(xr, base == OOB ? OOB : base + kc * 64));
            }
        }
    };
    TaskPix<TP, CS> P;
    F b[TAPS][TP][KC];
    int64_t task = first;
    if (task < ntask) {
        P.decode(a, task, fr, PY, PX);
        load(P, b);
    }
    for (; task < ntask; task += step) {
        f32x4 acc[TP][NT];
#pragma unroll
        for (int g = 0; g < TP; ++g)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) acc[g][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        TaskPix<TP, CS> Q = P;
        if constexpr (KS == 1) {
            // the next task's fragments in flight during this task's MFMAs and stores
            F bn[TAPS][TP][KC];
            const bool more = task + step < ntask;
            if (more) {
                P.decode(a, task + step, fr, PY, PX);
                load(P, bn);
            }
#pragma unroll
            for (int g = 0; g < TP; ++g)
#pragma unroll
                for (int kc = 0; kc < KC; ++kc)
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt) acc[g][nt] = mma(wa[0][kc][nt], b[0][g][kc], acc[g][nt]);
#pragma unroll
            for (int g = 0; g < TP; ++g)
#pragma unroll
                for (int kc = 0; kc < KC; ++kc) b[0][g][kc] = bn[0][g][kc];
        } else {
#pragma unroll
            for (int t = 0; t < TAPS; ++t) {
                if (!live(t)) continue;
#pragma unroll
                for (int g = 0; g < TP; ++g)
#pragma unroll
                    for (int kc = 0; kc < KC; ++kc)
#pragma unroll
                        for (int nt = 0; nt < NT; ++nt) acc[g][nt] = mma(wa[t][kc][nt], b[t][g][kc], acc[g][nt]);
            }
            if (task + step < ntask) {
                P.decode(a, task + step, fr, PY, PX);
                load(P, b);
            }
        }
        if constexpr (NT == 2 || NT == 4) {
            // transposed through this wave's LDS area and stored as 16-B pieces of each pixel's channel
            // run (conv_epi.h): 8-B fragment stores strided by the pixel pitch were the epilogue's cost.
            // Pixel q's output offset comes from the lane that owns it (lane q % 16 decoded pixel q of
            // its group for the loads) by a lane shuffle, not by decoding q again.
            f32x4 accT[NT][TP];
            uint32_t own[TP];
#pragma unroll
            for (int g = 0; g < TP; ++g) {
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) accT[nt][g] = acc[g][nt];
                own[g] = Q.ok[g] ? uint32_t((int64_t(Q.n[g]) * a.y_bs + (int64_t(Q.oh[g]) * a.OW + Q.ow[g]) * a.y_ld) * 2)
                                 : OOB;
            }
            auto pix_off = [&](int q) -> uint32_t {
                uint32_t v = 0;
#pragma unroll
                for (int g = 0; g < TP; ++g)
                    if ((q >> 4) == g) v = own[g];
                return uint32_t(__shfl(int(v), q & 15, 64));
            };
            epilogue_store<NT, TP>(accT, ssum, ssq, MODE == 0, ep, lane, 0, a.Nout, yres, MODE == 0,
                                   MODE == 1 && a.accumulate, pix_off);
            continue;
        }
        // epilogue: lane holds channels nt*16 + fc*4 + r of pixel fr of group g
#pragma unroll
        for (int g = 0; g < TP; ++g) {
            if (!Q.ok[g]) continue;
            const int64_t ob = int64_t(Q.n[g]) * a.y_bs + (int64_t(Q.oh[g]) * a.OW + Q.ow[g]) * a.y_ld;
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                const int cb = nt * 16 + fc * 4;
                if (cb >= a.Nout) continue;                 // Nout % 8 == 0: 4-channel groups are whole
                const f32x4 v = acc[g][nt];
                uint2 o;
                if constexpr (MODE == 0) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        ssum[nt][r] += v[r];
                        ssq[nt][r] += v[r] * v[r];
                    }
                    o.x = pk2h(v[0], v[1]);
                    o.y = pk2h(v[2], v[3]);
                } else {
                    float w4[4] = {v[0], v[1], v[2], v[3]};
                    if (a.accumulate) {
                        const uint2 old = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16_t*>(a.y) + ob + cb);
                        w4[0] += bf2f(bf16_t(old.x & 0xffff)); w4[1] += bf2f(bf16_t(old.x >> 16));
                        w4[2] += bf2f(bf16_t(old.y & 0xffff)); w4[3] += bf2f(bf16_t(old.y >> 16));
                    }
                    o.x = pk2bf(w4[0], w4[1]);
                    o.y = pk2bf(w4[2], w4[3]);
                }
                *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(a.y) + ob + cb) = o;
            }
        }
    }
}

// Stride-2 3x3 data gradient, all four output-parity classes in one task: a lane owns the 2x2 dx
// pixels (2i + py, 2j + px) of one (image, i, j) and loads the 2x2 dz pixels (i + dh, j + dw) they
// read ONCE — each of the nine taps maps one dz pixel (dh = kh == 0, dw = kw == 0) onto one class
// (py = kh != 1, px = kw != 1); the epilogue stores the quad's two rows as back-to-back column pairs,
// so each 128-B line of dx (two 32-channel bf16 pixels) is completed by one wave at one time.
// Round 3: the row-parity tasks it replaces (one launch row per row class, column pairs per task) read
// every dz row twice, and the two classes (3 vs 6 taps) drifted apart so the second read missed L2:
// s@640 model.1 data gradient 255 -> 188 us, bit-identical (same tap / chunk order per pixel).
template <int NT, int KC, int TP>
__device__ __forceinline__ void direct_body_s2dg_quad(const DirArgs& a, int64_t first, int64_t step, int64_t ntask,
                                                      char* ep) {
    using F = bf16x8;
    const int lane = threadIdx.x & 63, fr = lane & 15, fc = lane >> 4;
    F wa[9][KC][NT];
    {
        const __amdgpu_buffer_rsrc_t wr = make_rsrc(a.w, int64_t(a.Nout) * 9 * a.Kin * 2);
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
            for (int kc = 0; kc < KC; ++kc)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) {
                    const int co = nt * 16 + fr;
                    const uint32_t off = co < a.Nout ? uint32_t(((co * 9 + t) * a.Kin + kc * 32 + fc * 8) * 2) : OOB;
                    wa[t][kc][nt] = __builtin_bit_cast(F, buf_load16(wr, off));
                }
    }
    const __amdgpu_buffer_rsrc_t xr = make_rsrc(a.x, int64_t(a.N) * a.x_bs * 2);
    const __amdgpu_buffer_rsrc_t yres = make_rsrc(a.y, int64_t(a.N) * a.y_bs * 2);
    struct Quads {
        int n[TP], i[TP], j[TP];
        bool ok[TP];
    };
    auto decode = [&](int64_t tl, Quads& P) {
        const uint32_t chw = uint32_t(a.OHc) * uint32_t(a.OWc);
#pragma unroll
        for (int g = 0; g < TP; ++g) {
            const int64_t m = tl * (16 * TP) + g * 16 + fr;
            const uint32_t nn = uint32_t(m / chw), r = uint32_t(m - int64_t(nn) * chw);
            const uint32_t i = r / uint32_t(a.OWc), j = r - i * uint32_t(a.OWc);
            P.n[g] = int(nn);
            P.i[g] = int(i);
            P.j[g] = int(j);
            P.ok[g] = int(nn) < a.N;
        }
    };
    // b[g][dh][dw][kc]: dz pixel (i + dh, j + dw) of group g (zero outside the dz map)
    auto load = [&](const Quads& P, F (&b)[TP][2][2][KC]) {
#pragma unroll
        for (int g = 0; g < TP; ++g)
#pragma unroll
            for (int dh = 0; dh < 2; ++dh)
#pragma unroll
                for (int dw = 0; dw < 2; ++dw) {
                    const int ih = P.i[g] + dh, iw = P.j[g] + dw;
                    const bool in = P.ok[g] && ih < a.GH && iw < a.GW;
                    const uint32_t base =
                        in ? uint32_t((int64_t(P.n[g]) * a.x_bs + (int64_t(ih) * a.GW + iw) * a.x_ld + fc * 8) * 2) : OOB;
#pragma unroll
                    for (int kc = 0; kc < KC; ++kc)
                        b[g][dh][dw][kc] = __builtin_bit_cast(F, buf_load16(xr, base == OOB ? OOB : base + kc * 64));
                }
    };
    Quads P;
    F b[TP][2][2][KC];
    int64_t task = first;
    if (task < ntask) {
        decode(task, P);
        load(P, b);
    }
    float ssum[NT][4], ssq[NT][4];     // unused (no statistics in a data gradient)
    for (; task < ntask; task += step) {
        // accT[4g + 2 py + px]: the quad's rows as two back-to-back column pairs
        f32x4 accT[NT][4 * TP];
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int q = 0; q < 4 * TP; ++q) accT[nt][q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const int kh = t / 3, kw = t % 3;
            const int py = kh != 1, px = kw != 1, dh = kh == 0, dw = kw == 0;
#pragma unroll
            for (int g = 0; g < TP; ++g)
#pragma unroll
                for (int kc = 0; kc < KC; ++kc)
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt)
                        accT[nt][4 * g + 2 * py + px] = mma(wa[t][kc][nt], b[g][dh][dw][kc], accT[nt][4 * g + 2 * py + px]);
        }
        const Quads Q = P;
        if (task + step < ntask) {
            decode(task + step, P);
            load(P, b);
        }
        uint32_t own[4 * TP];
#pragma unroll
        for (int g = 0; g < TP; ++g)
#pragma unroll
            for (int py = 0; py < 2; ++py)
#pragma unroll
                for (int px = 0; px < 2; ++px) {
                    const int oh = 2 * Q.i[g] + py, ow = 2 * Q.j[g] + px;
                    own[4 * g + 2 * py + px] =
                        Q.ok[g] && oh < a.OH && ow < a.OW
                            ? uint32_t((int64_t(Q.n[g]) * a.y_bs + (int64_t(oh) * a.OW + ow) * a.y_ld) * 2)
                            : OOB;
                }
        auto pix_off = [&](int q) -> uint32_t {
            uint32_t v = 0;
#pragma unroll
            for (int k = 0; k < 4 * TP; ++k)
                if ((q >> 4) == k) v = own[k];
            return uint32_t(__shfl(int(v), q & 15, 64));
        };
        epilogue_store<NT, 4 * TP>(accT, ssum, ssq, false, ep, lane, 0, a.Nout, yres, false, a.accumulate != 0,
                                   pix_off);
    }
}

// forward / stride-1 data gradient (the stride-2 data gradient is conv_direct_quad_kernel)
template <int NT, int KC, int KS, int S, int MODE, int TP>
__global__ void __launch_bounds__(256) conv_direct_kernel(DirArgs a) {
    __shared__ float red[2][4][16 * NT];
    __shared__ __attribute__((aligned(16))) char epl[4][16 * 16 * NT * 2];   // per-wave epilogue transpose
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int fr = lane & 15, fc = lane >> 4;
    float ssum[NT][4], ssq[NT][4];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) ssum[nt][r] = ssq[nt][r] = 0.f;
    // XCD-contiguous task ranges (gridDim.x is a multiple of 8; block b runs on XCD b % 8): the 3x3
    // neighbour rows of a task, and for a stride-2 data gradient the other three parity classes of
    // the same pixels, are read by the same XCD at about the same time — from its L2, not from HBM
    const int xcd = blockIdx.x & 7, q = blockIdx.x >> 3, nq = gridDim.x >> 3;
    const int64_t lo = a.tpc * xcd / 8, hi = a.tpc * (xcd + 1) / 8;
    const int64_t first = lo + int64_t(q) * 4 + wave, step = int64_t(nq) * 4;
    static_assert(!(S == 2 && MODE == 1), "the stride-2 data gradient runs conv_direct_quad_kernel");
    direct_body<NT, KC, KS, S, MODE, TP, 0, 0>(a, ssum, ssq, first, step, hi, epl[wave]);
    if constexpr (MODE == 0) {
        if (!a.st_sum) return;
        // 16 pixel lanes per channel group, then the 4 waves in order
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float s = ssum[nt][r], q = ssq[nt][r];
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) {
                    s += __shfl_xor(s, o, 64);
                    q += __shfl_xor(q, o, 64);
                }
                if (fr == 0) {
                    red[0][wave][nt * 16 + fc * 4 + r] = s;
                    red[1][wave][nt * 16 + fc * 4 + r] = q;
                }
            }
        __syncthreads();
        for (int c = threadIdx.x; c < a.Nout; c += 256) {
            a.st_sum[int64_t(blockIdx.x) * a.Nout + c] = (red[0][0][c] + red[0][1][c]) + (red[0][2][c] + red[0][3][c]);
            a.st_sq[int64_t(blockIdx.x) * a.Nout + c] = (red[1][0][c] + red[1][1][c]) + (red[1][2][c] + red[1][3][c]);
        }
    }
}

// the four-class stride-2 data gradient: 2 workgroups per CU (256 VGPRs per lane at most; one quad group per
// task — two, at one workgroup per CU, measured 6 % slower)
template <int NT, int KC, int TP>
__global__ void __launch_bounds__(256, 2) conv_direct_quad_kernel(DirArgs a) {
    __shared__ __attribute__((aligned(16))) char epl[4][16 * 16 * NT * 2];
    const int wave = threadIdx.x >> 6;
    const int xcd = blockIdx.x & 7, q = blockIdx.x >> 3, nq = gridDim.x >> 3;
    const int64_t lo = a.tpc * xcd / 8, hi = a.tpc * (xcd + 1) / 8;
    const int64_t first = lo + int64_t(q) * 4 + wave, step = int64_t(nq) * 4;
    direct_body_s2dg_quad<NT, KC, TP>(a, first, step, hi, epl[wave]);
}

using KernFn = void (*)(DirArgs);

struct Variant {
    int nt, kc, ks, s, mode, tp;
    KernFn fn;
};

#define DIR_VARIANT(NT, KC, KS, S, MODE, TP) {NT, KC, KS, S, MODE, TP, conv_direct_kernel<NT, KC, KS, S, MODE, TP>}
// the YOLOv11 stem-stage layers (s@640: stem 1->32 s2 has its own kernel; model.1 32->64 3x3 s2,
// C3k2 64->64 1x1 / 32->32 3x3 / 96->128 1x1) in both directions (an 80x80 128->128 1x1 variant
// measured slower than the implicit GEMM: 0.083 vs 0.076 ms)
const Variant kVariants[] = {
    DIR_VARIANT(4, 1, 3, 2, 0, 2),   // fwd 32 -> 64, 3x3 s2 (two 16-pixel groups per task: 204 -> 191 us vs one)
    {2, 2, 3, 2, 1, 1, conv_direct_quad_kernel<2, 2, 1>},   // dgrad of it: dz 64 -> dx 32, 2x2-pixel quads
    DIR_VARIANT(2, 1, 3, 1, 0, 2),   // fwd 32 -> 32, 3x3 s1
    DIR_VARIANT(2, 1, 3, 1, 1, 2),   // dgrad 32 -> 32, 3x3 s1
    DIR_VARIANT(4, 2, 1, 1, 0, 4),   // 64 -> 64 1x1 (fwd and dgrad)
    DIR_VARIANT(4, 2, 1, 1, 1, 4),
    DIR_VARIANT(8, 3, 1, 1, 0, 2),   // fwd 96 -> 128 1x1
    DIR_VARIANT(6, 4, 1, 1, 1, 4),   // dgrad: dz 128 -> dx 96 (four groups per task: 176 -> 164 us vs two)
};
#undef DIR_VARIANT

// default 1 (>= 1 M output pixels).  Round 5: mode 3 (>= 200 k) measured the s@640 inference at bs 8 / 32 +0-2 / +3-4 %
// and the bs64 step unchanged in sum, but it moves the 80x80 layers of the bs64 step to this kernel and the largest
// of them (128 -> 128 3x3 s2, the bench line's probe) ran 0.174 -> 0.203 ms: kept at 1
// (profiles/r05/direct_threshold_ab.txt)
int direct_mode() { return g_direct_force >= 0 ? g_direct_force : 1; }

// workgroups of variant i the whole chip holds at once (CUs x the kernel's occupancy), cached per device and
// variant; the cache entries are atomics, so concurrent planners at worst compute the same value twice
constexpr int kMaxDev = 64;
int resident_blocks(int i) {
    static std::atomic<int> cache[kMaxDev][16];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) dev = 0;
    int v = cache[dev][i].load(std::memory_order_relaxed);
    if (v == 0) {
        int cus = 256, per = 1;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void*>(kVariants[i].fn), 256, 0) !=
                hipSuccess || per < 1)
            per = 1;
        v = std::max(8, (cus * per) & ~7);
        cache[dev][i].store(v, std::memory_order_relaxed);
    }
    return v;
}

}  // namespace

DirectPlan direct_plan(const ym_conv_desc* d, int dgrad, bool inference) {
    DirectPlan p{};
    int mode = direct_mode();
    // the inference forward (no statistics): mode 3's threshold under the default policy (s@640 bs 8 / 32 +0-2 / +3-4 %,
    // profiles/r05/direct_threshold_ab.txt; the training step keeps 1 M: its 80x80 layers ran slower here)
    if (inference && !dgrad && mode == 1 && g_direct_force < 0) mode = 3;
    if (!d || mode == 0) return p;
    if (d->k != 1 && d->k != 3) return p;
    if (d->pad != d->k / 2 || (d->stride != 1 && d->stride != 2)) return p;
    if (dgrad && d->k == 1 && d->stride != 1) return p;
    const int kin = dgrad ? d->cout : d->cin, nout = dgrad ? d->cin : d->cout;
    if (kin % 32 || nout % 8) return p;
    if (!dgrad && d->out_f32 != 2) return p;          // z (fp16) of a Conv block only
    const int64_t in_ld = dgrad ? d->y_ld : d->x_ld, in_bs = dgrad ? d->y_bs : d->x_bs;
    const int64_t out_ld = dgrad ? d->x_ld : d->y_ld, out_bs = dgrad ? d->x_bs : d->y_bs;
    if (in_ld % 8 || in_bs % 8 || out_ld % 4 || out_bs % 4) return p;
    if (int64_t(d->n) * in_bs * 2 >= (int64_t(1) << 31) || int64_t(d->n) * out_bs * 2 >= (int64_t(1) << 31)) return p;
    // high-resolution maps only (where the implicit GEMMs are latency-bound): >= 1 M output pixels
    const int OH = dgrad ? d->h : d->oh, OW = dgrad ? d->w : d->ow;
    const int64_t M = select_n(d) * OH * OW;
    if (mode == 1 && M < (int64_t(1) << 20)) return p;
    if (mode == 3 && M < 200000) return p;          // >= 200 k: the 160x160 stage from 8 images up
    for (int i = 0; i < int(sizeof(kVariants) / sizeof(kVariants[0])); ++i) {
        const Variant& v = kVariants[i];
        if (v.mode != dgrad || v.ks != d->k || v.s != d->stride || v.kc * 32 != kin) continue;
        if (v.nt * 16 < nout || (v.nt - 1) * 16 >= nout) continue;
        p.ok = 1;
        p.variant = i;
        const int os = dgrad ? d->stride : 1;
        const int64_t OHc = (OH + os - 1) / os, OWc = (OW + os - 1) / os;
        const int64_t tpc = (int64_t(d->n) * OHc * OWc + 16 * v.tp - 1) / (16 * v.tp);
        // persistent: as many workgroups as the chip holds at once (1024 before: model.1 forward -12 %, its data
        // gradient -5.5 %, the other stem-stage layers -1..-10 %, profiles/r03/direct_grid_ab.txt)
        const int64_t GCAP = resident_blocks(i);
        p.grid = int(std::max<int64_t>(8, std::min<int64_t>(GCAP, (tpc + 3) / 4)) & ~int64_t(7));
        return p;
    }
    return p;
}

int direct_launch(const DirectPlan& p, const ym_conv_desc* d, int dgrad, const uint16_t* x, const uint16_t* w,
                  void* y, float* st_sum, float* st_sq, hipStream_t st) {
    const Variant& v = kVariants[p.variant];
    DirArgs a{};
    a.x = x; a.w = w; a.y = y;
    if (!dgrad) {
        a.x_bs = d->x_bs; a.x_ld = d->x_ld; a.y_bs = d->y_bs; a.y_ld = d->y_ld;
        a.GH = d->h; a.GW = d->w; a.OH = d->oh; a.OW = d->ow; a.Kin = d->cin; a.Nout = d->cout;
        a.st_sum = st_sum; a.st_sq = st_sq;
    } else {
        a.x_bs = d->y_bs; a.x_ld = d->y_ld; a.y_bs = d->x_bs; a.y_ld = d->x_ld;
        a.GH = d->oh; a.GW = d->ow; a.OH = d->h; a.OW = d->w; a.Kin = d->cout; a.Nout = d->cin;
    }
    a.N = d->n; a.pad = d->pad; a.accumulate = d->accumulate;
    const int os = dgrad ? d->stride : 1;
    a.OHc = (a.OH + os - 1) / os; a.OWc = (a.OW + os - 1) / os;   // (stride 2: quad rows / columns)
    a.tpc = (int64_t(a.N) * a.OHc * a.OWc + 16 * v.tp - 1) / (16 * v.tp);
    hipLaunchKernelGGL(v.fn, dim3(p.grid), dim3(256), 0, st, a);
    return 0;
}

}  // namespace ym
