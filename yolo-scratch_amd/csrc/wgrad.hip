// Convolution weight gradients on CDNA4 MFMA (bf16 x bf16, fp32 accumulate).
//
// Replaces the weight half of nn.Conv2d's autograd inside Conv / Detect
// (/root/reference/yolo_scratch_cuda/models/yolo11_modules.py:21-33, 221-234):
// dW[co][ci][kh][kw] = sum over output pixels p of dz[p][co] * x[src(p, kh, kw)][ci].
// K of this GEMM is the pixel axis (N*OH*OW, up to 1.6 M at s@640 bs64), so every kernel
// splits it over grid.z and writes fp32 partials [split][Cout][taps][Cin]; wgrad_reduce_kernel
// sums the splits and writes the PyTorch OIHW gradient (overwrite or accumulate) — no atomics,
// no zero-fill by the caller.
//
// wgrad3_kernel<S>  3x3, pad 1, stride S in {1, 2}: one workgroup owns a 64co x 64ci tile for
//   ALL nine taps (144 fp32 accumulators per lane).  Per unit of <= 64 output pixels (an 8x8 block,
//   or whole rows of a narrow map) it stages dz (64 pixels x 64 co) and the input halo ((7S+3)^2
//   pixels x 64 ci for 8x8) once — fp16
//   activations converted to bf16 once — and every tap reads its shifted window out of the same
//   halo with transposed LDS reads (ds_read_b64_tr_b16) whose tap offsets are immediates.
// wgrad1_kernel<T>  1x1 stride 1 over whole-image views: pixels are a flat axis, so each lane's
//   staging offsets are fixed for the whole K loop; T x T tiles, 64 pixels per stage.
// wgrad_generic_kernel<T>  any other geometry (per-tap columns, fp32 atomics into split 0).
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "tile.h"

namespace ym {
namespace {

typedef short s16x8 __attribute__((ext_vector_type(8)));

struct WgArgs {
    const bf16_t* dz; int64_t dz_bs, dz_ld;   // (N, OH, OW, Cout) bf16 view
    const uint16_t* x; int64_t x_bs, x_ld;    // (N, IH, IW, Cin) fp16 view
    float* part;                              // [splits][Cout][taps][Cin] fp32
    int N, IH, IW, Cin, OH, OW, Cout, KH, KW, stride, pad;
    int64_t M;                                // N*OH*OW
    int64_t units;                            // K units: 64-pixel stages (1x1), tw x th rectangles (3x3), 32-pixel steps
    int64_t chunk;                            // units per split
    int ci_tiles;                             // generic kernel: channel tiles per tap column
    int co_t, ci_t, splits;                   // wgrad3 / wgrad1: tile grid (1-D launch, see wg_tile)
    int xcd_map;                              // splits % 8 == 0: one split's tiles all on one XCD
};

// (co tile, ci tile, split) of this workgroup of a 1-D launch of co_t * ci_t * splits blocks.  With
// xcd_map the blocks of one split — the (co, ci) tiles that read the SAME pixel range of dz and x —
// are the consecutive blocks of one XCD (block b runs on XCD b % 8), so that range comes from HBM
// once and from the XCD's L2 for the other tiles; in plain order the co tiles of one split landed on
// 8 different XCDs and the weight gradients fetched 2.2x their algorithmic bytes (profiles/r02).
__device__ __forceinline__ void wg_tile(const WgArgs& a, int& co, int& ci, int& split) {
    const int b = blockIdx.x, nt = a.co_t * a.ci_t;
    int t;
    if (a.xcd_map) {
        const int xcd = b & 7, q = b >> 3;
        t = q % nt;
        split = (q / nt) * 8 + xcd;
    } else {
        t = b % nt;
        split = b / nt;
    }
    co = t % a.co_t;
    ci = t / a.co_t;
}

// transposed 16x(32 k) fragment: two ds_read_b64_tr_b16, k rows {4g..4g+3} from p_lo and
// {16+4g..} from p_hi (g = lane>>4); the same k permutation on both operands cancels
__device__ __forceinline__ bf16x8 tr_frag(const char* p_lo, const char* p_hi) {
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p_lo));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p_hi));
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
}

// ------------------------------------------------------------------ 3x3
// TCO x TCI (64 or 32) channel tiles; a wave owns WCO co x WCI ci of the tile for all 9 taps
// ((TCO/WCO) x (TCI/WCI) waves).  Per 32-pixel k step a wave reads its co fragments once and every
// tap's ci fragments once, so LDS bytes per MFMA = 1 KB / (WCO/16) + (WCO/16) KB / (9 WCI/16): the
// 64 x 16 waves of the stride-1 64x64 tiles (4 waves) read 0.36 KB per MFMA where 32 x 16 waves
// (8 waves) read 0.61 — 152 B/clk per CU against LDS's 128, which bounded the kernel.  32-channel
// tiles serve the 32-channel layers of the stem stage, which a 64x64 tile ran three-quarters empty.
// A K unit is a tw x th rectangle of output pixels (tw * th <= 64; the plan picks 8x8, or whole
// rows — 20 x 3 — on the 20-wide maps, where 8x8 tiles cover 24x24 = 1.44x the pixels).  The units
// of a split are staged through two register sets: while unit t is multiplied, the loads of units
// t + 1 and t + 2 are in flight.
// DB: two LDS buffers — the next unit is written into the other buffer while this one is multiplied, one
// barrier per unit (single buffer: the store between two barriers, every wave off the MFMA pipe meanwhile).
// LA: tap lookahead in the multiply (round 6).  0: each tap's ci fragments are read right before its TI x TJ MFMAs (hipcc
// keeps one fragment set live: every tap waits lgkmcnt(0) for its own reads, 18 exposed LDS round trips per unit);
// 1: tap t+1's fragments are read ahead of tap t's MFMAs into a second set (TJ x 4 more VGPRs), so each read has one
// tap of MFMAs to land behind
template <int S, int TCO, int TCI, int WCO, int WCI, int TW, int TH, bool DEEP, bool DB = false, int LA = 0>
__global__ void __launch_bounds__((TCO / WCO) * (TCI / WCI) * 64) wgrad3_kernel(WgArgs a) {
    constexpr int NWC = TCI / WCI;            // waves along ci
    constexpr int NWV = (TCO / WCO) * NWC;
    constexpr int NT = NWV * 64;
    constexpr int TI = WCO / 16;              // 16-co subtiles per wave
    constexpr int TJ = WCI / 16;              // 16-ci subtiles per wave
    static_assert(TI >= 1 && TJ >= 1, "wgrad3 tile geometry");
    constexpr int CPD = TCO / 8, CPX = TCI / 8;       // 16-B chunks per dz / halo row
    constexpr int RPD = NT / CPD, RPX = NT / CPX;     // rows staged per pass
    constexpr int DI = (64 + RPD - 1) / RPD;  // dz chunks per thread (threads past row 63 idle)
    constexpr int RSD = TCO * 2 + 32;         // dz rows: consecutive-row tr reads conflict free
    constexpr int RSX = TCI * 2 + (S == 1 ? 32 : 16);   // halo rows: reads step S rows
    constexpr int TP = TW * TH;               // pixels of a unit (<= 64)
    constexpr int HW = (TW - 1) * S + 3, HR = ((TH - 1) * S + 3) * HW;   // halo width / rows
    constexpr int XI = (HR + RPX - 1) / RPX;  // 16-B halo chunks per thread
    static_assert(TP <= 64, "wgrad3 unit");
    constexpr int NB = DB ? 2 : 1;
    __shared__ __attribute__((aligned(16))) char Dzb[NB][64 * RSD];
    __shared__ __attribute__((aligned(16))) char Xhb[NB][HR * RSX];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave / NWC, wc = wave % NWC;
    int cot, cit, split;
    wg_tile(a, cot, cit, split);
    const int co0 = cot * TCO, ci0 = cit * TCI;
    const int dsc = tid % CPD, dsrow = tid / CPD;     // staging: chunk of rows row + RP*it
    const int xsc = tid % CPX, xsrow = tid / CPX;
    const bool co_ok = co0 + dsc * 8 < a.Cout, ci_ok = ci0 + xsc * 8 < a.Cin;
    int d_py[DI], d_px[DI], x_hy[XI], x_hx[XI];
#pragma unroll
    for (int it = 0; it < DI; ++it) {
        const int p = dsrow + RPD * it;
        d_py[it] = p < TP ? p / TW : 1 << 20;         // pixel slots past the unit stage zeros
        d_px[it] = p < TP ? p - (p / TW) * TW : 0;
    }
#pragma unroll
    for (int it = 0; it < XI; ++it) {
        const int r = xsrow + RPX * it;
        x_hy[it] = r / HW;
        x_hx[it] = r - x_hy[it] * HW;
    }
    const int ntw = (a.OW + TW - 1) / TW, nth = (a.OH + TH - 1) / TH;
    const int64_t t_begin = int64_t(split) * a.chunk;
    const int64_t t_end = std::min<int64_t>(a.units, t_begin + a.chunk);
    // the unit the next load() stages, stepped from one call to the next (every call site loads units in order, one
    // per call): round 5, in place of four runtime divisions per load (precomputing the chunks' offsets as well cost
    // 17 VGPRs, one workgroup per CU on the 8-wave tiles)
    int64_t l_t = t_begin;
    int l_tw, l_th, l_n;
    {
        const int u = int(t_begin < t_end ? t_begin : 0), r = u / ntw;
        l_tw = u - r * ntw;
        l_th = r % nth;
        l_n = r / nth;
    }

    // fragment-read geometry: lane's k rows (pixels of the unit) for the two 32-pixel halves; pixel
    // slots past the unit read halo row 0 (always staged, finite) against their zero dz rows
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
    int hb_lo[2], hb_hi[2];                   // halo row of (pixel, tap 0,0)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
        const int plo = kk * 32 + 4 * g + q, phi = plo + 16;
        hb_lo[kk] = plo < TP ? (plo / TW) * S * HW + (plo % TW) * S : 0;
        hb_hi[kk] = phi < TP ? (phi / TW) * S * HW + (phi % TW) * S : 0;
    }

    f32x4 acc[9][TI][TJ];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j) acc[t][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    uint4 da[DI], xa[XI], db[DI], xb[XI];
    // stages unit l_t and steps it: no unit argument, so a call site cannot look as if it chose the unit (a reordered
    // or prefetched call would stage the wrong unit silently) — units go in stream order, one per call
    auto load = [&](uint4 (&rdz)[DI], uint4 (&rx)[XI]) {
        const bool live = l_t < t_end;             // past the split: zeros, no branch around the loads
        const int tw = l_tw, th = l_th, n = l_n;
        if (live) {
            ++l_t;
            if (++l_tw == ntw) {
                l_tw = 0;
                if (++l_th == nth) { l_th = 0; ++l_n; }
            }
        }
        const int oh0 = th * TH, ow0 = tw * TW;
        const __amdgpu_buffer_rsrc_t rd = make_rsrc(a.dz + int64_t(n) * a.dz_bs, a.dz_bs * 2);
        const __amdgpu_buffer_rsrc_t rxs = make_rsrc(a.x + int64_t(n) * a.x_bs, a.x_bs * 2);
#pragma unroll
        for (int it = 0; it < DI; ++it) {
            const int oh = oh0 + d_py[it], ow = ow0 + d_px[it];
            const bool ok = live && co_ok && dsrow + RPD * it < 64 && oh < a.OH && ow < a.OW;
            rdz[it] = buf_load16(rd, ok ? uint32_t(((oh * a.OW + ow) * int(a.dz_ld) + co0 + dsc * 8) * 2) : OOB);
        }
        const int ih0 = oh0 * S - 1, iw0 = ow0 * S - 1;
#pragma unroll
        for (int it = 0; it < XI; ++it) {
            const int ih = ih0 + x_hy[it], iw = iw0 + x_hx[it];
            const bool ok = live && ci_ok && xsrow + RPX * it < HR && unsigned(ih) < unsigned(a.IH) && unsigned(iw) < unsigned(a.IW);
            rx[it] = buf_load16(rxs, ok ? uint32_t(((ih * a.IW + iw) * int(a.x_ld) + ci0 + xsc * 8) * 2) : OOB);
        }
    };
    auto store = [&](int buf, const uint4 (&rdz)[DI], const uint4 (&rx)[XI]) {
        char* Dz = Dzb[buf];
        char* Xh = Xhb[buf];
#pragma unroll
        for (int it = 0; it < DI; ++it)
            if (dsrow + RPD * it < 64) *reinterpret_cast<uint4*>(Dz + (dsrow + RPD * it) * RSD + dsc * 16) = rdz[it];
#pragma unroll
        for (int it = 0; it < XI; ++it)
            if (xsrow + RPX * it < HR)
                *reinterpret_cast<uint4*>(Xh + (xsrow + RPX * it) * RSX + xsc * 16) = h8_to_bf8(rx[it]);
    };
    auto compute = [&](int buf) {
        const char* Dz = Dzb[buf];
        const char* Xh = Xhb[buf];
        int hl[2] = {hb_lo[0], hb_lo[1]}, hh[2] = {hb_hi[0], hb_hi[1]};
        asm volatile("" : "+v"(hl[0]), "+v"(hl[1]), "+v"(hh[0]), "+v"(hh[1]));
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            bf16x8 af[TI];
#pragma unroll
            for (int i = 0; i < TI; ++i) {
                const int col = (wr * WCO + i * 16 + 4 * pp) * 2;
                af[i] = tr_frag(Dz + (kk * 32 + 4 * g + q) * RSD + col, Dz + (kk * 32 + 16 + 4 * g + q) * RSD + col);
            }
            if constexpr (LA == 1) {
                auto read_tap = [&](bf16x8 (&bfr)[TJ], int tap) {
                    const int toff = (tap / 3) * HW + tap % 3;
#pragma unroll
                    for (int j = 0; j < TJ; ++j) {
                        const int col = (wc * WCI + j * 16 + 4 * pp) * 2;
                        bfr[j] = tr_frag(Xh + (hl[kk] + toff) * RSX + col, Xh + (hh[kk] + toff) * RSX + col);
                    }
                };
                bf16x8 bq[2][TJ];
                read_tap(bq[0], 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 2 * TI + 2 * TJ, 0);  // the co fragments and tap 0's
#pragma unroll
                for (int tap = 0; tap < 9; ++tap) {
                    if (tap + 1 < 9) read_tap(bq[(tap + 1) & 1], tap + 1);
#pragma unroll
                    for (int i = 0; i < TI; ++i)
#pragma unroll
                        for (int j = 0; j < TJ; ++j)
                            acc[tap][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bq[tap & 1][j], acc[tap][i][j],
                                                                                      0, 0, 0);
                    // the next tap's reads go out ahead of this tap's MFMAs
                    if (tap + 1 < 9) __builtin_amdgcn_sched_group_barrier(0x100, 2 * TJ, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, TI * TJ, 0);
                }
                continue;
            }
#pragma unroll
            for (int kh = 0; kh < 3; ++kh)
#pragma unroll
                for (int kw = 0; kw < 3; ++kw) {
                    const int toff = kh * HW + kw;
                    bf16x8 bfr[TJ];
#pragma unroll
                    for (int j = 0; j < TJ; ++j) {
                        const int col = (wc * WCI + j * 16 + 4 * pp) * 2;
                        bfr[j] = tr_frag(Xh + (hl[kk] + toff) * RSX + col, Xh + (hh[kk] + toff) * RSX + col);
                    }
#pragma unroll
                    for (int i = 0; i < TI; ++i)
#pragma unroll
                        for (int j = 0; j < TJ; ++j)
                            acc[kh * 3 + kw][i][j] =
                                __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[kh * 3 + kw][i][j], 0, 0, 0);
                }
        }
    };

    if constexpr (DB && DEEP) {
        // units in pairs over the two register sets and the two LDS buffers: unit t + 1 is written into the
        // other buffer (its loads issued a unit ago) while unit t is multiplied, then unit t + 3's loads go out
        if (t_begin < t_end) {
            load(da, xa);
            load(db, xb);
            store(0, da, xa);
            __syncthreads();
            load(da, xa);
        }
        for (int64_t t = t_begin; t < t_end; t += 2) {
            compute(0);                       // unit t
            store(1, db, xb);                 // unit t + 1 into the other buffer (read two barriers ago)
            load(db, xb);
            __syncthreads();
            compute(1);                       // unit t + 1
            store(0, da, xa);                 // unit t + 2
            load(da, xa);
            __syncthreads();
        }
    } else if constexpr (DB) {
        if (t_begin < t_end) {
            load(da, xa);
            store(0, da, xa);
            __syncthreads();
            load(da, xa);
        }
        int buf = 0;
        for (int64_t t = t_begin; t < t_end; ++t) {
            compute(buf);
            if (t + 1 < t_end) {
                store(buf ^ 1, da, xa);
                load(da, xa);
            }
            __syncthreads();
            buf ^= 1;
        }
    } else if constexpr (DEEP) {
        // units go in pairs, one per register set (static indexing; a split with an odd count multiplies
        // one unit of zeros at its end): the loop has one exit, so the accumulators are not copied
        // between the two bodies' register assignments
        if (t_begin < t_end) {
            load(da, xa);
            load(db, xb);
            store(0, da, xa);
            __syncthreads();
            load(da, xa);
        }
        for (int64_t t = t_begin; t < t_end; t += 2) {
            compute(0);                       // unit t (set a's, staged)
            __syncthreads();
            store(0, db, xb);
            __syncthreads();
            load(db, xb);
            compute(0);                       // unit t + 1
            __syncthreads();
            store(0, da, xa);
            __syncthreads();
            load(da, xa);
        }
    } else {
        // one register set: unit t + 1 in flight while unit t is multiplied
        if (t_begin < t_end) {
            load(da, xa);
            store(0, da, xa);
            __syncthreads();
            load(da, xa);
        }
        for (int64_t t = t_begin; t < t_end; ++t) {
            compute(0);
            __syncthreads();
            if (t + 1 >= t_end) break;
            store(0, da, xa);
            __syncthreads();
            load(da, xa);
        }
    }

    // partials: D[co][ci], lane holds co rows (lane>>4)*4 + r, ci column lane&15
    float* base = a.part + int64_t(split) * a.Cout * 9 * a.Cin;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j) {
                const int ci = ci0 + wc * WCI + j * 16 + (lane & 15);
                if (ci >= a.Cin) continue;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int co = co0 + wr * WCO + i * 16 + (lane >> 4) * 4 + r;
                    if (co < a.Cout) base[(int64_t(co) * 9 + t) * a.Cin + ci] = acc[t][i][j][r];
                }
            }
}

// ------------------------------------------------------------------ 1x1, whole-image views
template <int T>
__global__ void __launch_bounds__(256, 2) wgrad1_kernel(WgArgs a) {
    constexpr int KP = 64;                    // pixels per stage (2 MFMA k-steps)
    constexpr int RS = T * 2 + 32;
    constexpr int CPR = T / 8;                // 16-B chunks per row
    constexpr int RPP = 256 / CPR;            // rows staged per pass
    constexpr int ITEMS = KP / RPP;
    constexpr int TS = T / 32;
    __shared__ __attribute__((aligned(16))) char As[2][KP * RS];   // dz rows x T co
    __shared__ __attribute__((aligned(16))) char Bs[2][KP * RS];   // x rows x T ci (bf16)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 1, wc = wave & 1;
    int cot, cit, split;
    wg_tile(a, cot, cit, split);
    const int co0 = cot * T, ci0 = cit * T;
    const int sc = tid % CPR, srow = tid / CPR;
    const int64_t p_begin = (int64_t(split) * a.chunk) * KP;
    const int64_t p_end = std::min<int64_t>(a.M, p_begin + a.chunk * KP);
    uint32_t dz_off[ITEMS], x_off[ITEMS];
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
        const int r = srow + RPP * it;
        dz_off[it] = co0 + sc * 8 < a.Cout ? uint32_t((r * int(a.dz_ld) + co0 + sc * 8) * 2) : OOB;
        x_off[it] = ci0 + sc * 8 < a.Cin ? uint32_t((r * int(a.x_ld) + ci0 + sc * 8) * 2) : OOB;
    }

    f32x4 acc[TS][TS];
#pragma unroll
    for (int i = 0; i < TS; ++i)
#pragma unroll
        for (int j = 0; j < TS; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // two register sets (units t + 1 and t + 2 in flight while unit t is multiplied; one unit of
    // look-ahead left the kernel waiting on its loads two thirds of its cycles — SQ_WAIT_ANY 66 %,
    // profiles/r03/pmc73_summary.txt); units go in pairs, a split with an odd count multiplies zeros
    uint4 ra0[ITEMS], rb0[ITEMS], ra1[ITEMS], rb1[ITEMS];
    auto load = [&](int64_t p0, uint4 (&ra)[ITEMS], uint4 (&rb)[ITEMS]) {
        // records end at p_end: rows past it (and whole units past it) read as zero
        const int64_t left = std::max<int64_t>(0, p_end - p0);
        const __amdgpu_buffer_rsrc_t rd = make_rsrc(a.dz + p0 * a.dz_ld, left * a.dz_ld * 2);
        const __amdgpu_buffer_rsrc_t rx = make_rsrc(a.x + p0 * a.x_ld, left * a.x_ld * 2);
#pragma unroll
        for (int it = 0; it < ITEMS; ++it) {
            ra[it] = buf_load16(rd, dz_off[it]);
            rb[it] = buf_load16(rx, x_off[it]);
        }
    };
    auto store = [&](int buf, const uint4 (&ra)[ITEMS], const uint4 (&rb)[ITEMS]) {
#pragma unroll
        for (int it = 0; it < ITEMS; ++it) {
            const int r = srow + RPP * it;
            *reinterpret_cast<uint4*>(&As[buf][r * RS + sc * 16]) = ra[it];
            *reinterpret_cast<uint4*>(&Bs[buf][r * RS + sc * 16]) = h8_to_bf8(rb[it]);
        }
    };
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
    auto compute = [&](int buf) {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const char* A0 = As[buf] + (kk * 32 + 4 * g + q) * RS;
            const char* B0 = Bs[buf] + (kk * 32 + 4 * g + q) * RS;
            bf16x8 af[TS], bfr[TS];
#pragma unroll
            for (int i = 0; i < TS; ++i) {
                const int col = (wr * (T / 2) + i * 16 + 4 * pp) * 2;
                af[i] = tr_frag(A0 + col, A0 + 16 * RS + col);
            }
#pragma unroll
            for (int j = 0; j < TS; ++j) {
                const int col = (wc * (T / 2) + j * 16 + 4 * pp) * 2;
                bfr[j] = tr_frag(B0 + col, B0 + 16 * RS + col);
            }
#pragma unroll
            for (int i = 0; i < TS; ++i)
#pragma unroll
                for (int j = 0; j < TS; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
    };

    if (p_begin < p_end) {
        load(p_begin, ra0, rb0);
        load(p_begin + KP, ra1, rb1);
        store(0, ra0, rb0);
        __syncthreads();
        load(p_begin + 2 * KP, ra0, rb0);
    }
    for (int64_t p0 = p_begin; p0 < p_end; p0 += 2 * KP) {
        compute(0);                           // unit at p0
        store(1, ra1, rb1);
        __syncthreads();
        load(p0 + 3 * KP, ra1, rb1);
        compute(1);                           // unit at p0 + KP (zeros past the split)
        store(0, ra0, rb0);
        __syncthreads();
        load(p0 + 4 * KP, ra0, rb0);
    }
    float* base = a.part + int64_t(split) * a.Cout * a.Cin;
#pragma unroll
    for (int i = 0; i < TS; ++i)
#pragma unroll
        for (int j = 0; j < TS; ++j) {
            const int ci = ci0 + wc * (T / 2) + j * 16 + (lane & 15);
            if (ci >= a.Cin) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int co = co0 + wr * (T / 2) + i * 16 + (lane >> 4) * 4 + r;
                if (co < a.Cout) base[int64_t(co) * a.Cin + ci] = acc[i][j][r];
            }
        }
}

// ------------------------------------------------------------------ generic (any k, stride, pad, view)
// one (co tile, tap, ci tile) per block, 32 pixels per step, fp32 atomics into split 0
template <int T>
__global__ void __launch_bounds__(256) wgrad_generic_kernel(WgArgs a) {
    constexpr int RS = T * 2 + 32;
    constexpr int CPR = T / 8;
    constexpr int ITEMS = 32 * CPR / 256;
    constexpr int TS = T / 32;
    __shared__ __attribute__((aligned(16))) char As[2][32 * RS];
    __shared__ __attribute__((aligned(16))) char Bs[2][32 * RS];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 1, wc = wave & 1;
    const int co0 = blockIdx.x * T;
    const int tap = blockIdx.y / a.ci_tiles;
    const int ci0 = (blockIdx.y - tap * a.ci_tiles) * T;
    const int kh = tap / a.KW, kw = tap - kh * a.KW;
    const int64_t p_begin = int64_t(blockIdx.z) * a.chunk * 32;
    const int64_t p_end = std::min<int64_t>(a.M, p_begin + a.chunk * 32);
    if (p_begin >= p_end) return;
    const uint32_t uOHW = uint32_t(a.OH) * uint32_t(a.OW), uOW = uint32_t(a.OW);

    f32x4 acc[TS][TS];
#pragma unroll
    for (int i = 0; i < TS; ++i)
#pragma unroll
        for (int j = 0; j < TS; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    uint4 ra[ITEMS], rb[ITEMS];
    auto load = [&](int64_t p0) {
#pragma unroll
        for (int it = 0; it < ITEMS; ++it) {
            const int id = tid + it * 256, srow = id / CPR, sc = id % CPR;
            const int64_t p = p0 + srow;
            ra[it] = make_uint4(0, 0, 0, 0);
            rb[it] = make_uint4(0, 0, 0, 0);
            if (p < p_end) {
                const uint32_t up = uint32_t(p);
                const uint32_t n = up / uOHW, pix = up - n * uOHW;
                const int oh = int(pix / uOW), ow = int(pix - uint32_t(oh) * uOW);
                const int co = co0 + sc * 8;
                if (co < a.Cout)
                    ra[it] = *reinterpret_cast<const uint4*>(a.dz + int64_t(n) * a.dz_bs + int64_t(pix) * a.dz_ld + co);
                const int ih = oh * a.stride - a.pad + kh, iw = ow * a.stride - a.pad + kw;
                const int ci = ci0 + sc * 8;
                if (ci < a.Cin && ih >= 0 && ih < a.IH && iw >= 0 && iw < a.IW)
                    rb[it] = h8_to_bf8(*reinterpret_cast<const uint4*>(a.x + int64_t(n) * a.x_bs +
                                                                       (int64_t(ih) * a.IW + iw) * a.x_ld + ci));
            }
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int it = 0; it < ITEMS; ++it) {
            const int id = tid + it * 256, srow = id / CPR, sc = id % CPR;
            *reinterpret_cast<uint4*>(&As[buf][srow * RS + sc * 16]) = ra[it];
            *reinterpret_cast<uint4*>(&Bs[buf][srow * RS + sc * 16]) = rb[it];
        }
    };
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
    load(p_begin);
    store(0);
    __syncthreads();
    int buf = 0;
    for (int64_t p0 = p_begin; p0 < p_end; p0 += 32) {
        const bool more = p0 + 32 < p_end;
        if (more) load(p0 + 32);
        const char* A0 = As[buf] + (4 * g + q) * RS;
        const char* B0 = Bs[buf] + (4 * g + q) * RS;
        bf16x8 af[TS], bfr[TS];
#pragma unroll
        for (int i = 0; i < TS; ++i) {
            const int col = (wr * (T / 2) + i * 16 + 4 * pp) * 2;
            af[i] = tr_frag(A0 + col, A0 + 16 * RS + col);
        }
#pragma unroll
        for (int j = 0; j < TS; ++j) {
            const int col = (wc * (T / 2) + j * 16 + 4 * pp) * 2;
            bfr[j] = tr_frag(B0 + col, B0 + 16 * RS + col);
        }
#pragma unroll
        for (int i = 0; i < TS; ++i)
#pragma unroll
            for (int j = 0; j < TS; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        if (more) store(buf ^ 1);
        __syncthreads();
        buf ^= 1;
    }
    const int taps = a.KH * a.KW;
#pragma unroll
    for (int i = 0; i < TS; ++i)
#pragma unroll
        for (int j = 0; j < TS; ++j) {
            const int ci = ci0 + wc * (T / 2) + j * 16 + (lane & 15);
            if (ci >= a.Cin) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int co = co0 + wr * (T / 2) + i * 16 + (lane >> 4) * 4 + r;
                if (co < a.Cout) atomicAdd(a.part + (int64_t(co) * taps + tap) * a.Cin + ci, acc[i][j][r]);
            }
        }
}

// ------------------------------------------------------------------ split reduction -> OIHW
// block: 64 consecutive (co, tap, ci) elements x 4 split lanes; dst[co][ci][tap] (+)= sum
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* __restrict__ part, int64_t splits,
                                                           int Cout, int taps, int Cin, float* __restrict__ dst,
                                                           int accumulate) {
    __shared__ float red[4][64];
    const int64_t E = int64_t(Cout) * taps * Cin;
    const int64_t e = int64_t(blockIdx.x) * 64 + (threadIdx.x & 63);
    const int zl = threadIdx.x >> 6;
    float s = 0.f;
    if (e < E) {
        int64_t z = zl;
        for (; z + 12 < splits; z += 16) {
            const float v0 = part[z * E + e], v1 = part[(z + 4) * E + e];
            const float v2 = part[(z + 8) * E + e], v3 = part[(z + 12) * E + e];
            s += (v0 + v1) + (v2 + v3);
        }
        for (; z < splits; z += 4) s += part[z * E + e];
    }
    red[zl][threadIdx.x & 63] = s;
    __syncthreads();
    if (zl == 0 && e < E) {
        const float v = (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
        const int ci = int(e % Cin);
        const int64_t r = e / Cin;
        const int t = int(r % taps), co = int(r / taps);
        float* d = dst + (int64_t(co) * Cin + ci) * taps + t;
        *d = accumulate ? *d + v : v;
    }
}

// ------------------------------------------------------------------ launch plan
struct WgPlan {
    int kind;          // 3: wgrad3, 1: wgrad1, 0: generic
    int T;             // wgrad1 / generic tile; wgrad3: co tile (ci tile in T2)
    int T2;
    int co_t, ci_t;
    int64_t units, chunk, splits;
    int tw, th;        // wgrad3 unit rectangle
    bool deep;         // wgrad3: two register sets (units t + 1, t + 2 in flight)
};

// workgroups per weight-gradient launch (ym_wgrad_set_target; the stride-1 3x3 rule's doubled target scales with it).
// Round 5: 160 measured +0.2 % img/s in the step (three same-box pairs, profiles/r05/wgrad_target_streams_ab.txt) but
// each launch ran longer alone (the 3x3 family's single-stream roofline fraction 0.2107 -> 0.1974, wgrad 0.199 ->
// 0.161, profiles/r05/at_589d336): kept at 256, the gain inside the run-to-run spread
Policy g_wg_target{256};

// tap lookahead of the shipped wgrad3 instances (wgrad3_kernel LA)
constexpr int kWgLA = 0;
#ifdef YM_EXPERIMENTS
Policy g_wg_la{kWgLA};
#endif

WgPlan wg_plan(const ym_conv_desc* d) {
    WgPlan p{};
    const int64_t M = int64_t(d->n) * d->oh * d->ow;
    const bool whole = d->x_bs == int64_t(d->h) * d->w * d->x_ld && d->y_bs == int64_t(d->oh) * d->ow * d->y_ld;
    if (d->k == 3 && d->pad == 1 && (d->stride == 1 || d->stride == 2)) {
        p.kind = 3;
        p.T = d->cout <= 32 ? 32 : 64;
        p.T2 = d->cin <= 32 ? 32 : 64;
        p.tw = p.th = 8;
        p.units = int64_t(d->n) * ((d->oh + 7) / 8) * ((d->ow + 7) / 8);
        // whole-row units on the narrow maps 8x8 tiles pad (a 20-wide map: 20 x 3 rows, 448 units per
        // 64 images instead of 576 covering 24x24; 10 wide: 10 x 6) — 64x64 channel tiles only
        if ((d->ow == 20 || d->ow == 10) && p.T == 64 && p.T2 == 64) {
            p.tw = d->ow; p.th = 64 / d->ow;
            p.units = int64_t(d->n) * ((d->oh + p.th - 1) / p.th);
        }
    } else if (d->k == 1 && d->stride == 1 && d->pad == 0 && whole) {
        p.kind = 1;
        // 128-wide tiles once both channel counts reach 96: fewer tiles re-read dz and x fewer times, at
        // the cost of padding a channel count below 128 — the 96 -> 128 1x1 at 160x160 measured 0.357 ms
        // on 64-wide tiles (x and dz read twice each from HBM), 0.142 ms on one padded 128-wide tile
        p.T = (d->cout >= 96 && d->cin >= 96) ? 128 : 64;
        p.units = (M + 63) / 64;
    } else {
        p.kind = 0;
        p.T = (d->cout >= 128 && d->cin >= 128) ? 128 : 64;
        p.units = (M + 31) / 32;
    }
    p.co_t = (d->cout + p.T - 1) / p.T;
    p.ci_t = (d->cin + (p.kind == 3 ? p.T2 : p.T) - 1) / (p.kind == 3 ? p.T2 : p.T);
    const int64_t cols = int64_t(p.co_t) * p.ci_t * (p.kind == 0 ? d->k * d->k : 1);
    // enough K units per workgroup to amortise writing its fp32 partial tile (64x64x9 floats for
    // 3x3: 147 KB, about the input an 8x8-pixel unit moves 12 times)
    int64_t min_units = p.kind == 3 ? 12 : 8;
    // workgroups per launch (g_wg_target above; round 1: 256 vs 512 / 1024 in the step)
    int64_t target = g_wg_target;
    // stride-1 3x3 layers with few units per channel tile (20x20 maps, 256-channel 40x40): twice the target (512 when it
    // was 256) in workgroups of >= 6 units — the larger partials cost less than half the CUs idling (s@640 bs64, same-process A/B:
    // 128->128 20x20 34.7 -> 30.2 us, 256->128 40x40 84.8 -> 76.1 us; the stride-2 20x20 layers and
    // 128-channel 40x40 ones measured slower, so they keep 256)
    if (p.kind == 3 && d->stride == 1 && p.units / cols < 256) { target = 2 * g_wg_target; min_units = 6; }
    // the second register set pays where a split runs many units (maps >= 64 wide: 80x80 128->128
    // 152.8 -> 147.6 us); below that the extra VGPRs (120 -> 166: one workgroup per CU) cost as much
    p.deep = p.kind == 3 && d->ow >= 64;
    int64_t splits = std::max<int64_t>(1, std::min<int64_t>(target / cols, p.units / min_units));
    splits = std::min<int64_t>(splits, p.kind == 0 ? 65535 : 256);
    if (p.kind != 0 && splits >= 8) splits &= ~int64_t(7);      // whole XCD groups (wg_tile)
    p.chunk = (p.units + splits - 1) / splits;
    p.splits = std::max<int64_t>(1, (p.units + p.chunk - 1) / p.chunk);
    return p;
}

}  // namespace

#ifdef YM_EXPERIMENTS
extern "C" int ym_wgrad_set_lookahead(int la) {
    // wgrad3_kernel LA: 0 each tap's fragments read right before its MFMAs, 1 one tap ahead; out of range restores the
    // shipped setting; returns the previous one
    return g_wg_la.set(la < 0 || la > 1 ? kWgLA : la);
}
#endif

extern "C" int ym_wgrad_set_target(int wgs) {
    // workgroups per weight-gradient launch the split-K plan aims for (default 256; <= 0 restores it); returns the
    // previous setting
    return g_wg_target.set(wgs <= 0 ? 256 : wgs);
}

template <int LA>
void wg3_launch(const ym_conv_desc* d, const WgPlan& p, const WgArgs& a, dim3 grid, hipStream_t st) {
    const int tc = (p.T == 32 ? 1 : 0) | (p.T2 == 32 ? 2 : 0);     // bit 0: 32-co, bit 1: 32-ci tile
#define WG3_LAUNCH(S_, D_, B_)                                                                                    \
        if (p.tw == 20) {                                                                                   \
            hipLaunchKernelGGL((wgrad3_kernel<S_, 64, 64, 32, 16, 20, 3, false, B_, LA>), grid, dim3(512), 0, st, a); \
        } else if (p.tw == 10) {                                                                            \
            hipLaunchKernelGGL((wgrad3_kernel<S_, 64, 64, 32, 16, 10, 6, false, B_, LA>), grid, dim3(512), 0, st, a); \
        } else {                                                                                            \
            switch (tc) {                                                                                   \
                case 0: hipLaunchKernelGGL((wgrad3_kernel<S_, 64, 64, 32, 16, 8, 8, D_, B_, LA>), grid, dim3(512), 0, st, a); break; \
                case 1: hipLaunchKernelGGL((wgrad3_kernel<S_, 32, 64, 16, 16, 8, 8, D_, B_, LA>), grid, dim3(512), 0, st, a); break; \
                case 2: hipLaunchKernelGGL((wgrad3_kernel<S_, 64, 32, 32, 16, 8, 8, D_, B_, LA>), grid, dim3(256), 0, st, a); break; \
                default: hipLaunchKernelGGL((wgrad3_kernel<S_, 32, 32, 16, 16, 8, 8, D_, B_, LA>), grid, dim3(256), 0, st, a); break; \
            }                                                                                               \
        }
    // two LDS buffers on the stride-1 layers and the deep stride-2 ones (same-process A/B: -4..-10 % on the
    // 80x80 / 160x160 layers, +3.5..+4.8 % on the narrow stride-2 maps; profiles/r04/wgrad3_db_ab.txt)
    if (d->stride == 1 || p.deep) {
        if (d->stride == 1) {
            if (p.deep) { WG3_LAUNCH(1, true, true) } else { WG3_LAUNCH(1, false, true) }
        } else {
            if (p.deep) { WG3_LAUNCH(2, true, true) } else { WG3_LAUNCH(2, false, true) }
        }
    } else {
        if (d->stride == 1) {
            if (p.deep) { WG3_LAUNCH(1, true, false) } else { WG3_LAUNCH(1, false, false) }
        } else {
            if (p.deep) { WG3_LAUNCH(2, true, false) } else { WG3_LAUNCH(2, false, false) }
        }
    }
#undef WG3_LAUNCH
}

int wgrad_kernel(const ym_conv_desc* d, char* name, size_t len) {
    const WgPlan p = wg_plan(d);
    if (p.kind == 3) {
        const int tc = (p.T == 32 ? 1 : 0) | (p.T2 == 32 ? 2 : 0);
        const bool db = d->stride == 1 || p.deep;        // two LDS buffers (ym_conv_wgrad)
        snprintf(name, len, "wgrad3 s%d %dx%d %dx%d%s%s", d->stride, p.T, p.T2, p.tw, p.th, p.deep ? " deep" : "",
                 db ? " db" : "");
        return 13000 + (d->stride == 2 ? 500 : 0) + 100 * tc + (p.tw == 20 ? 10 : p.tw == 10 ? 20 : 0) + (p.deep ? 1 : 0) +
               (db ? 2 : 0);
    }
    if (p.kind == 1) {
        snprintf(name, len, "wgrad1 %d", p.T);
        return 11000 + p.T;
    }
    snprintf(name, len, "wgrad generic %d", p.T);
    return 10000 + p.T;
}

}  // namespace ym

using namespace ym;

extern "C" size_t ym_conv_wgrad_workspace_size(const ym_conv_desc* d) {
    if (!d) return 0;
    const WgPlan p = wg_plan(d);
    const int64_t E = int64_t(d->cout) * d->k * d->k * d->cin;
    return size_t((p.kind == 0 ? 1 : p.splits) * E) * sizeof(float);
}

extern "C" int ym_conv_wgrad(const ym_conv_desc* d, const uint16_t* dz, const uint16_t* x, void* workspace,
                             size_t workspace_bytes, float* dw_oihw, int accumulate, void* stream) {
    YM_CHECK_ARG(d && dz && x && dw_oihw, "ym_conv_wgrad: null argument");
    YM_CHECK_ARG(d->cin % 8 == 0 && d->cout % 8 == 0, "ym_conv_wgrad: channels %% 8 != 0");
    YM_CHECK_ARG(d->x_ld % 8 == 0 && d->y_ld % 8 == 0 && d->x_bs % 8 == 0 && d->y_bs % 8 == 0,
                 "ym_conv_wgrad: views not 16-byte aligned");
    const WgPlan p = wg_plan(d);
    const int taps = d->k * d->k;
    const int64_t E = int64_t(d->cout) * taps * d->cin;
    const size_t need = size_t((p.kind == 0 ? 1 : p.splits) * E) * sizeof(float);
    YM_CHECK_ARG(workspace && workspace_bytes >= need, "ym_conv_wgrad: workspace %zu < %zu bytes", workspace_bytes,
                 need);
    const int64_t M = int64_t(d->n) * d->oh * d->ow;
    YM_CHECK_ARG(M < (int64_t(1) << 31), "ym_conv_wgrad: too many pixels");
    YM_CHECK_ARG(d->x_bs * 2 < (int64_t(1) << 31) && d->y_bs * 2 < (int64_t(1) << 31),
                 "ym_conv_wgrad: image stride too large");
    hipStream_t st = as_stream(stream);
    WgArgs a{};
    a.dz = dz; a.dz_bs = d->y_bs; a.dz_ld = d->y_ld;
    a.x = x; a.x_bs = d->x_bs; a.x_ld = d->x_ld;
    a.part = static_cast<float*>(workspace);
    a.N = d->n; a.IH = d->h; a.IW = d->w; a.Cin = d->cin; a.OH = d->oh; a.OW = d->ow; a.Cout = d->cout;
    a.KH = d->k; a.KW = d->k; a.stride = d->stride; a.pad = d->pad;
    a.M = M; a.units = p.units; a.chunk = p.chunk;
    int64_t splits = p.splits;
    a.co_t = p.co_t; a.ci_t = p.ci_t; a.splits = int(splits);
    a.xcd_map = splits % 8 == 0;
    if (M == 0) {
        // no pixels: the gradient is zero
        splits = 0;
    } else if (p.kind == 3) {
        YM_CHECK_ARG(int64_t(d->h) * d->w * d->x_ld * 2 < (int64_t(1) << 31), "ym_conv_wgrad: image too large");
        const dim3 grid(unsigned(p.co_t * p.ci_t * splits));
#ifdef YM_EXPERIMENTS
        if (g_wg_la == 0) wg3_launch<0>(d, p, a, grid, st);
        else wg3_launch<1>(d, p, a, grid, st);
#else
        wg3_launch<kWgLA>(d, p, a, grid, st);
#endif
    } else if (p.kind == 1) {
        const dim3 grid(unsigned(p.co_t * p.ci_t * splits));
        if (p.T == 128)
            hipLaunchKernelGGL(wgrad1_kernel<128>, grid, dim3(256), 0, st, a);
        else
            hipLaunchKernelGGL(wgrad1_kernel<64>, grid, dim3(256), 0, st, a);
    } else {
        if (hipMemsetAsync(workspace, 0, size_t(E) * sizeof(float), st) != hipSuccess) {
            set_error("ym_conv_wgrad: memset failed");
            return YM_ERR_HIP;
        }
        a.ci_tiles = p.ci_t;
        const dim3 grid(p.co_t, p.ci_t * taps, unsigned(splits));
        if (p.T == 128)
            hipLaunchKernelGGL(wgrad_generic_kernel<128>, grid, dim3(256), 0, st, a);
        else
            hipLaunchKernelGGL(wgrad_generic_kernel<64>, grid, dim3(256), 0, st, a);
        splits = 1;
    }
    YM_LAUNCH_CHECK("ym_conv_wgrad");
    if (splits == 0) {
        if (!accumulate && hipMemsetAsync(dw_oihw, 0, size_t(E) * sizeof(float), st) != hipSuccess) {
            set_error("ym_conv_wgrad: memset failed");
            return YM_ERR_HIP;
        }
        return YM_OK;
    }
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(unsigned((E + 63) / 64)), dim3(256), 0, st,
                       static_cast<const float*>(workspace), splits, d->cout, taps, d->cin, dw_oihw, accumulate);
    YM_LAUNCH_CHECK("ym_conv_wgrad(reduce)");
    return YM_OK;
}

