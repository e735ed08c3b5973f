// Persistent software-pipelined implicit-GEMM convolution for gfx950 (fp16 forward, bf16 data
// gradient, fp32 accumulate) — the large 3x3 / 1x1 layers of the YOLOv11 graph.
//
// Replaces nn.Conv2d forward / input-gradient inside Conv (/root/reference/yolo_scratch_cuda/
// models/yolo11_modules.py:21-33, Detect :221-234) where the GEMM is big enough to fill the chip.
//
// Why a second implicit GEMM (conv.hip keeps the 2-stage one for small / odd shapes): its
// 128 x 128 tiles, one K stage in flight and one barrier + read burst per K step leave the MFMA
// pipes 77 % idle (profiles/r01/pmc_op6): every K step opens with the LDS latency of its fragment
// reads, and 64 B/cycle of staging per CU at peak is more than the TA delivers.  Here:
//  * 256 pixels x 128 channels per tile, 16 waves of 32 x 64 (64-channel tiles: 8 waves of 64 x 32),
//    K steps of 64 (two 32-deep halves):
//    a third fewer staged bytes per FLOP than 128 x 128;
//  * a 3-stage LDS ring filled by LDS-DMA (buffer_load ... lds) with TWO stages in flight, counted
//    vmcnt waits and raw s_barrier (no vmcnt(0) drain in the loop);
//  * the barrier sits in the MIDDLE of a K step: a step reads its second-half fragments, runs the
//    first half's 16 MFMAs, waits for the next stage, barriers, issues the DMA into the buffer it
//    has just finished with, reads the next stage's first-half fragments and runs the second half's
//    16 MFMAs — every LDS read has 16 MFMAs to hide behind, the pipe never waits on a fresh read;
//  * the K offset rides in the buffer instruction's SGPR soffset (channel counts are multiples of
//    64): one DMA costs no VALU inside a tap;
//  * persistent workgroups (one per CU) stream their tiles back to back: the next tile's first
//    stages are in flight during the current tile's epilogue; tiles are grouped per XCD, the
//    channel tiles of one pixel tile on the same XCD (input rows reused from its L2);
//  * BatchNorm statistics accumulate in registers across a workgroup's tiles and are written as
//    one partial row per workgroup (no atomics, fixed order: bit-reproducible).
// The stride-2 data gradient runs as 4 output-parity classes inside the same tile stream, each
// with only the taps that land (as conv.hip).
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "conv_epi.h"
#include "conv_pipe.h"
#include "bn_fold.h"
#include "tile.h"

namespace ym {

// selection policy (ym_conv_set_pipe): -1 default (3); 0 never; 1 layers of >= 1024 tiles with >= 128
// output channels, no stride-2 data gradient; 2 every eligible layer of >= 256 tiles; 3 (default) the
// wider rule of pipe_plan (s@640 bs64 step: 2940 img/s vs 2902 for rule 1)
Policy g_pipe_force{-1};
// experiments (ym_pipe_set_exp, yolomi_experimental.h; tools/pipe_ab.py): 0 shipped; 1 the 8-wave 256 x 128 tile;
// 10-13 ablations of the 16-wave tile (conv_pipe_kernel ABL 1, 2, 4, 8: wrong results by design); 20 the generic
// (class-search) control path.  Built only into the measurement library (make exp: -DYM_EXPERIMENTS,
// libyolomi_exp.so); the shipping libyolomi.so has neither the setter nor the ablation instances.
// Measured and rejected in round 6, built into the measurement library only (profiles/r06/pipe_mfma_order_ab.txt):
// the MFMA shape (ym_conv_set_pipe_mfma: 0 16x16x32 shipped; 1 32x32x16 on the same tiles, +8..+23 % per layer;
// 2 32x32x16 on 8 waves of 64 x 64, +1..+14 %) and the K-step issue order (ym_conv_set_pipe_order / conv_pipe_kernel
// RO: 1 pins every fragment read ahead of the MFMAs it covers, -3..+7 %)
#ifdef YM_EXPERIMENTS
Policy g_pipe_mfma{0};
Policy g_pipe_order{0};   // also conv_hpipe.hip (conv_pipe.h)
Policy g_pipe_loop{2};    // conv_pipe_kernel LP of the single-class path (2 shipped)
Policy g_pipe_eval_loop{0};  // conv_pipe_kernel LP of the eval instance (0 shipped, 2 the nested loop)
Policy g_pipe_taporder{-1};  // conv_pipe_kernel TO of the single-class forward: -1 the shipped rule (tap_inner), 0 / 1 forced
Policy g_pipe_exp{0};
#else
constexpr int g_pipe_exp = 0;
#endif

namespace {

constexpr int PF = 0;   // forward: fp16 x fp16
constexpr int PD = 1;   // data gradient: bf16 x bf16

struct PipeArgs {
    const bf16_t* x; int64_t x_bs, x_ld;     // gathered tensor view (elements)
    const bf16_t* w;                          // [Nout][KH][KW][Kin]
    void* y; int64_t y_bs, y_ld;              // output view
    const float* bias;                        // [Nout] or null
    float* st_sum; float* st_sq;              // [rows][Nout] or null
    int GH, GW, Kin;
    int OH, OW, Nout;
    int KH, KW, stride, pad, N;
    int out_f32, accumulate;
    int os;                                   // 2: stride-2 data gradient (4 parity classes)
    int ntiles;                               // channel tiles
    int mt_pre[5];                            // first m-tile of each class (prefix), mt_pre[ncls] = total
    int ncls;
    BnFoldArgs fold;                          // BatchNorm finalize as the tail (ym_conv_fwd_bn); gamma null = off
};

struct Cls {
    int py, px, OWc, kh0, kw0, nkw, ntap;
    uint32_t OHW;
    int64_t Mc;
};

__device__ __forceinline__ Cls cls_of(const PipeArgs& a, int c) {
    Cls k;
    const int os = a.os;
    k.py = os == 2 ? (c >> 1) : 0;
    k.px = os == 2 ? (c & 1) : 0;
    const int OHc = (a.OH - k.py + os - 1) / os;
    k.OWc = (a.OW - k.px + os - 1) / os;
    k.kh0 = os == 2 ? ((k.py + a.pad) & 1) : 0;
    k.kw0 = os == 2 ? ((k.px + a.pad) & 1) : 0;
    k.nkw = (a.KW - k.kw0 + os - 1) / os;
    k.ntap = ((a.KH - k.kh0 + os - 1) / os) * k.nkw;
    k.OHW = uint32_t(OHc) * uint32_t(k.OWc);
    k.Mc = int64_t(a.N) * k.OHW;
    return k;
}

__device__ __forceinline__ int cls_find(const PipeArgs& a, int mt) {
    int c = 0;
    while (c + 1 < a.ncls && mt >= a.mt_pre[c + 1]) ++c;
    return c;
}

__device__ __forceinline__ int fsw128(int r) { return (r >> 1) & 7; }

// (image, in-image index, row) of pixel m0 + r, r < 256, given the tile's (tn, tp) = divmod(m0, ohw) (computed
// once per tile): one wrap for the image, the row by the float reciprocal of the row width with one
// correction (x < 2^24) — the generic 32-bit divisions these replace cost ~30 VALU each and ran per pixel
// in every tile's setup and epilogue (12 per lane and tile)
__device__ __forceinline__ void split_pix(uint32_t tn, uint32_t tp, uint32_t r, uint32_t ohw, uint32_t w, float inv_w,
                                          uint32_t& n, uint32_t& pix, uint32_t& row) {
    pix = tp + r;
    n = tn;
    while (pix >= ohw) { pix -= ohw; ++n; }
    uint32_t q = uint32_t(float(pix) * inv_w);
    const int rem = int(pix) - int(q * w);
    q = rem < 0 ? q - 1 : (rem >= int(w) ? q + 1 : q);
    row = q;
}

// one 1-KiB LDS-DMA piece: lane l's 16 bytes from rsrc + voff + soff land at lds + 16 l
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* lds, uint32_t voff, uint32_t soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}

template <int N>
__device__ __forceinline__ void vm_wait() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
    asm volatile("" ::: "memory");
}

// every ds_read issued so far has returned, then the workgroup barrier (no vmcnt drain); the
// sched_barriers keep the compiler from moving MFMAs / LDS reads across it
__device__ __forceinline__ void step_barrier() {
    __builtin_amdgcn_sched_barrier(0);
    // the builtin, not inline asm: the compiler's wait-count pass sees this wait, so the MFMAs after the
    // barrier do not wait again for the fragments read before it (with an asm wait they stalled on the
    // next stage's freshly issued reads: lgkmcnt(3..0) ahead of the first four MFMAs of every step)
    __builtin_amdgcn_s_waitcnt(0xC07F);       // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}

// issue side of the stage stream: which tile / tap / 64-channel chunk the next LDS-DMA stage
// stages, and the per-lane gather offsets of the current tile and tap.  All control state is
// wave-uniform (scalar registers); per stage the DMAs cost one M0 write each, per tap one
// bounds select per gather row, per tile one pixel decomposition.
// C1 (every launch pipe_plan makes by default: one output class, maps of >= BM pixels): no class search, no
// per-tile divisions — the tile's (image, in-image offset) advance by a constant step with one wrap, the
// buffer resource over the tile's images is built once per tile.  (Round 5: the generic form spent ~3.8 SALU
// and ~3.5 VALU per MFMA, SQ_INSTS_* over op 73, much of it the per-tile class search and 32-bit divisions of
// both the issue and the compute side; its no-MFMA ablation alone ran 107 of the layer's 145 us.)
// TO (round 6, single-class path only): K order of the stage stream.  0: channel chunk innermost — (tap 0, chunk 0),
// (tap 0, chunk 1), .., (tap 1, chunk 0), ..; 1: tap innermost — every tap of channel chunk 0, then of chunk 1, so
// the taps that re-read the same input pixels run back to back and their overlap comes from L2 (one 64-channel
// chunk's footprint per tile instead of every chunk's)
template <int BM, int BN, int NW, int MODE, int ABL = 0, bool C1 = false, int TO = 0>
struct Issuer {
    static constexpr int AI = BN / 8 / NW, BI = BM / 8 / NW, RB = 128;
    const PipeArgs& a;
    int wave, lrow, lslot, kc;
    uint32_t xld_b;
    int mt_lo, qstride, ntile;
    // stream position
    int i = 0, ti = 0, tj = 0, kci = 0;
    // current tile
    int nrows = 0, nkw = 1, kh0 = 0, kw0 = 0;
    const bf16_t* x_tile = nullptr;
    int x_bytes = 0;
    int bh[BI], bw[BI];
    uint32_t bc[BI], b_off[BI];
    uint32_t a_tap = 0;
    // C1: the staged tile's first pixel (image, in-image offset, flat index) and the per-tile step
    int tn = 0, m0 = 0, step_n = 0, m_step = 0;
    uint32_t tp = 0, step_p = 0, ohw = 1;
    float inv_w = 1.f;
    __amdgpu_buffer_rsrc_t xres_t;

    __device__ Issuer(const PipeArgs& a_, int wave_, int lane, int mt_lo_, int qstride_, int ntile_)
        : a(a_), wave(wave_), lrow(lane >> 3), lslot(lane & 7), kc(a_.Kin >> 6), xld_b(uint32_t(a_.x_ld) * 2u),
          mt_lo(mt_lo_), qstride(qstride_), ntile(ntile_) {
        if constexpr (C1) {
            // a zero-record resource until the first tile_setup: a workgroup without tiles still issues its prologue's
            // (out-of-range) DMAs through it, and an uninitialised descriptor made them real loads (a memory fault at
            // s@640 bs2 under ym_conv_set_select_batch(64), where most of the grid has no tile)
            xres_t = make_rsrc(a.x, 0);
            ohw = uint32_t(a.OH) * uint32_t(a.OW);
            m0 = mt_lo * BM;
            tn = int(uint32_t(m0) / ohw);
            tp = uint32_t(m0) - uint32_t(tn) * ohw;
            m_step = qstride * BM;
            step_n = int(uint32_t(m_step) / ohw);
            step_p = uint32_t(m_step) - uint32_t(step_n) * ohw;
            inv_w = 1.0f / float(a.OW);
            nkw = a.KW;
            nrows = a.KH;
        }
    }

    __device__ __forceinline__ void tile_setup() {
        if constexpr (C1) {
            x_tile = a.x + int64_t(tn) * a.x_bs;
            const int64_t xb = (int64_t(a.N) - tn) * a.x_bs * 2;
            x_bytes = int(xb < 0x7fffffff ? xb : 0x7fffffff);
            const uint64_t xp = reinterpret_cast<uint64_t>(x_tile);
            const uint32_t xlo = uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(xp))));
            const uint32_t xhi = uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(xp >> 32))));
            xres_t = make_rsrc(reinterpret_cast<const void*>((uint64_t(xhi) << 32) | xlo),
                               __builtin_amdgcn_readfirstlane(x_bytes));
            const int M = a.N * int(ohw);
#pragma unroll
            for (int j = 0; j < BI; ++j) {
                const int r = (wave * BI + j) * 8 + lrow;
                if (m0 + r < M) {
                    uint32_t pix = tp + uint32_t(r), n = 0;
                    if (pix >= ohw) { pix -= ohw; n = 1; }              // ohw >= BM: at most one wrap
                    uint32_t q = uint32_t(float(pix) * inv_w);
                    const int rem = int(pix) - int(q * uint32_t(a.OW));
                    q = rem < 0 ? q - 1 : (rem >= a.OW ? q + 1 : q);
                    const int oh = int(q), ow = int(pix - q * uint32_t(a.OW));
                    if (MODE == PF) {
                        bh[j] = oh * a.stride - a.pad;
                        bw[j] = ow * a.stride - a.pad;
                    } else {                        // stride-1 data gradient
                        bh[j] = oh + a.pad;
                        bw[j] = ow + a.pad;
                    }
                    bc[j] = n * uint32_t(a.x_bs) * 2u + uint32_t(bh[j] * a.GW + bw[j]) * xld_b +
                            uint32_t(lslot ^ fsw128(r)) * 16u;
                } else {
                    bh[j] = -(1 << 20);             // no tap is in range
                    bw[j] = 0;
                    bc[j] = 0;
                }
            }
            return;
        }
        const int mt = mt_lo + i * qstride;
        const int c = cls_find(a, mt);
        const Cls k = cls_of(a, c);
        nkw = k.nkw;
        nrows = k.ntap / k.nkw;
        kh0 = k.kh0;
        kw0 = k.kw0;
        const int64_t m0l = int64_t(mt - a.mt_pre[c]) * BM;
        const uint32_t nfirst = uint32_t(m0l) / k.OHW, tpl = uint32_t(m0l) - nfirst * k.OHW;
        const float inv_wl = 1.0f / float(k.OWc);
        x_tile = a.x + int64_t(nfirst) * a.x_bs;
        const int64_t xb = (int64_t(a.N) - nfirst) * a.x_bs * 2;
        x_bytes = int(xb < 0x7fffffff ? xb : 0x7fffffff);
#pragma unroll
        for (int j = 0; j < BI; ++j) {
            const int r = (wave * BI + j) * 8 + lrow;
            const int64_t m = m0l + r;
            if (m < k.Mc) {
                uint32_t n, pix, ii;
                split_pix(nfirst, tpl, uint32_t(r), k.OHW, uint32_t(k.OWc), inv_wl, n, pix, ii);
                const int oh = int(ii) * a.os + k.py, ow = int(pix - ii * uint32_t(k.OWc)) * a.os + k.px;
                if (MODE == PF) {
                    bh[j] = oh * a.stride - a.pad;
                    bw[j] = ow * a.stride - a.pad;
                } else {                        // the class's first tap lands on whole pixels
                    bh[j] = (oh + a.pad - k.kh0) >> (a.stride - 1);
                    bw[j] = (ow + a.pad - k.kw0) >> (a.stride - 1);
                }
                bc[j] = (n - nfirst) * uint32_t(a.x_bs) * 2u + uint32_t(bh[j] * a.GW + bw[j]) * xld_b +
                        uint32_t(lslot ^ fsw128(r)) * 16u;
            } else {
                bh[j] = -(1 << 20);             // no tap is in range
                bw[j] = 0;
                bc[j] = 0;
            }
        }
    }

    __device__ __forceinline__ void tap_setup() {
        const int dir = MODE == PF ? 1 : -1;
        const int ost = MODE == PF ? 1 : a.stride;
        const uint32_t delta = uint32_t(dir * (ti * a.GW + tj)) * xld_b;
#pragma unroll
        for (int j = 0; j < BI; ++j) {
            const int gh = bh[j] + dir * ti, gw = bw[j] + dir * tj;
            const bool ok = uint32_t(gh) < uint32_t(a.GH) && uint32_t(gw) < uint32_t(a.GW);
            b_off[j] = ok ? bc[j] + delta : OOB;
        }
        a_tap = C1 ? uint32_t((ti * a.KW + tj) * a.Kin) * 2u
                   : uint32_t(((kh0 + ti * ost) * a.KW + (kw0 + tj * ost)) * a.Kin) * 2u;
    }

    __device__ __forceinline__ void start() {
        if (ntile > 0) {
            tile_setup();
            tap_setup();
        }
    }

    // the DMAs of the stage at the stream position into `st` (straight-line code: the caller interleaves
    // them with MFMAs); `live` false = past the stream's end: out-of-range offsets, nothing is fetched and
    // every step keeps the same DMA count (the counted vmcnt waits stay constant)
    __device__ __forceinline__ void issue_dma(char* st, __amdgpu_buffer_rsrc_t wres, const uint32_t* a_off, bool live) {
        const uint32_t kb = uint32_t(kci) * 128u;
        __amdgpu_buffer_rsrc_t xres;
        if constexpr (C1) {
            xres = xres_t;
        } else {
            // wave-uniform base / size (readfirstlane: else hipcc waterfalls every DMA over the resource)
            const uint64_t xb = reinterpret_cast<uint64_t>(x_tile);
            const uint32_t xlo = uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(xb))));
            const uint32_t xhi = uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(xb >> 32))));
            xres = make_rsrc(reinterpret_cast<const void*>((uint64_t(xhi) << 32) | xlo),
                             __builtin_amdgcn_readfirstlane(x_bytes));
        }
#pragma unroll
        for (int j = 0; j < AI; ++j)
            dma16(wres, st + (wave * AI + j) * 1024, live && !(ABL & 9) ? a_off[j] : OOB, a_tap + kb);
#pragma unroll
        for (int j = 0; j < BI; ++j)
            dma16(xres, st + BN * RB + (wave * BI + j) * 1024, live && !(ABL & 5) ? b_off[j] : OOB, kb);
    }

    // advance the stream position by one stage (new tap: its gather offsets; new tile: its pixels)
    __device__ __forceinline__ void advance() {
        if constexpr (TO == 1) {
            static_assert(C1, "tap-innermost order: single-class path");
            if (++tj == nkw) {
                tj = 0;
                if (++ti == nrows) {
                    ti = 0;
                    if (++kci == kc) {
                        kci = 0;
                        if (++i < ntile) {
                            m0 += m_step;
                            tn += step_n;
                            tp += step_p;
                            if (tp >= ohw) { tp -= ohw; ++tn; }
                            tile_setup();
                        }
                    }
                }
            }
            tap_setup();
            return;
        }
        if (++kci == kc) {
            kci = 0;
            if (++tj == nkw) {
                tj = 0;
                if (++ti == nrows) {
                    ti = 0;
                    if (++i < ntile) {
                        if constexpr (C1) {
                            m0 += m_step;
                            tn += step_n;
                            tp += step_p;
                            if (tp >= ohw) { tp -= ohw; ++tn; }
                        }
                        tile_setup();
                    }
                }
            }
            tap_setup();
        }
    }
};

// EPI 2: the register-only epilogue (epilogue_regs: no LDS, so hipcc does not drain the in-flight stages in front of
// it) whose stores the next step's wait leaves in flight — both directions since round 4 (the LDS-transposed form
// measured 2-7 % slower on every forward, profiles/r04/pipe_fwd_reg_epilogue_ab.txt)
// ABL (ablations for measurement only, never selected by pipe_plan): 1 every stage DMA out of range (issued, nothing
// fetched), 2 no MFMAs (fragments still read), 4 only the gathered input's DMAs out of range, 8 only the weights'
// C1: one output class on maps of >= BM pixels (Issuer's fast path; the stride-2 data gradient's four classes and tiny
// maps take the generic one)
// EV: the eval-mode Conv block instance (ym_conv_fwd_eval at large batches: running-statistics BatchNorm / SiLU /
// residual in the register epilogue, conv_epi.h EvalEpi; a C1 forward without statistics; e is not read otherwise)
// MF: the MFMA shape — 16 (v_mfma_f32_16x16x32: 16x16 subtiles, one MFMA per 32-deep half and subtile pair) or 32
// (v_mfma_f32_32x32x16, round 6: 32x32 subtiles, two 16-deep MFMAs per half; half the MFMA instructions for the same
// FLOPs, a 32-cycle issue window per MFMA instead of 16, the same LDS fragment bytes; conv_epi.h epilogue_regs32_x)
// RO: issue order inside a K step (round 6).  0: after the barrier the stage DMAs go out between the second half's MFMAs
// and the next stage's first-half fragments are read two MFMAs before the end of the step (the compiler also floats the
// second-half reads into the middle of the first half); 1: every fragment read is pinned ahead of the MFMAs it covers —
// the second-half reads at the top of the step, the next stage's first-half reads right after the barrier, ahead of
// the DMAs — so each read has a whole half (TM * TN * KS MFMAs per wave) of cover
// LP: loop form of the single-class path (round 6).  0: one flat loop over the workgroup's K steps whose body tests for
// a tile's first step (accumulator reset, the wait that leaves the previous epilogue's stores in flight) and last step
// (epilogue) every iteration; 1: tiles x K steps as two nested loops — the tile's first step peeled with its own wait,
// the inner loop a bare K step; 2 (shipped for the training instances since round 6): as 1 with the ring slot carried as
// a byte offset (an add instead of a multiply) and the stream-end test against a hoisted limit.  ~22 instead of ~33
// scalar instructions per common K step; same-process layer A/B (profiles/r06/pipe_loop_ab.txt) -1..-5 % on most
// pipelined layers (op 71 fwd -11.6 %), op 73 fwd +1.5 %; the whole step within +-0.2 % (the launches overlap other
// streams' work there).  The eval instance keeps 0 (not measured)
template <int BM, int BN, int WM, int WN, int MODE, int EPI = 2, int NS = 3, int ABL = 0, bool C1 = false,
          bool EV = false, int MF = 16, int RO = 0, int LP = 0, int TO = 0>
__global__ void __launch_bounds__(WM * WN * 64, 1) conv_pipe_kernel(PipeArgs a, EvalArgs e) {
    static_assert(!EV || (C1 && MODE == PF && ABL == 0), "the eval instance is a single-class forward");
    static_assert(MF == 16 || MF == 32, "MFMA shape");
    // NS: LDS ring of K stages — stage g computing, g+1 .. g+NS-1 in flight (3; 2 for the 64-KB+ stages of the
    // 256-channel / 512-pixel tiles)
    static_assert(NS == 2 || NS == 3, "ring depth");
    static_assert(LP == 0 || C1, "the nested loop form is the single-class path's");
    constexpr int RB = 128;                   // 64 K x 2 B per LDS row
    constexpr int NW = WM * WN;
    constexpr int AI = BN / 8 / NW;           // weight DMA instructions per wave per stage
    constexpr int BI = BM / 8 / NW;           // activation DMA instructions per wave per stage
    constexpr int DPS = AI + BI;              // DMAs per wave per stage (the vmcnt unit)
    constexpr int TM = BN / WM / MF;          // MF-channel subtiles per wave
    constexpr int TN = BM / WN / MF;          // MF-pixel subtiles per wave
    constexpr int KS = MF == 16 ? 1 : 2;      // MFMA K slices per 32-deep half (and fragment reads per subtile)
    constexpr int NR = MF == 16 ? 4 : 16;     // accumulator registers per subtile and lane
    typedef float AccT __attribute__((ext_vector_type(NR)));
    constexpr int STAGE = (BM + BN) * RB;
    static_assert(AI >= 1 && BI >= 1 && TM >= 1 && TN >= 1, "tile too small for 8-row DMA pieces");
    static_assert(EPI == 2, "register-only epilogue");
    constexpr int WCH = BN / WM;                          // channels per wave
    constexpr int EPS = MF == 16 ? TM * TN / 2 : TM * TN * 2;   // epilogue stores per lane
    // the ring; the statistics' cross-wave reduction reuses its first bytes after the last tile
    static_assert(NS * STAGE <= 160 * 1024 && 2 * (BM / (BM / WN)) * BN * 4 <= NS * STAGE, "LDS budget");
    __shared__ __attribute__((aligned(16))) char smem[NS * STAGE];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave / WN, wc = wave % WN;
    const int fc = lane >> 4, fr = lane & 15;
    const int kc = a.Kin >> 6;                // 64-deep K chunks per tap

    // ---- this workgroup's tiles: channel tile fixed per workgroup, m-tiles of its XCD's range
    const int G8 = int(gridDim.x) >> 3;
    const int xcd = int(blockIdx.x) & 7, q = int(blockIdx.x) >> 3;
    const int nt = q % a.ntiles, qq = q / a.ntiles, qstride = G8 / a.ntiles;
    const int mt_total = a.mt_pre[a.ncls];
    const int per = (mt_total + 7) >> 3;
    const int mt_lo = xcd * per + qq, mt_hi = min(xcd * per + per, mt_total);
    const int ntile = mt_lo < mt_hi ? (mt_hi - mt_lo + qstride - 1) / qstride : 0;
    const int n0 = nt * BN;
    int total = 0;                            // K steps of this workgroup's whole stream
    if (C1) total = ntile * a.KH * a.KW * kc;
    else if (a.ncls == 1) total = ntile * cls_of(a, 0).ntap * kc;
    else
        for (int t = 0; t < ntile; ++t) total += cls_of(a, cls_find(a, mt_lo + t * qstride)).ntap * kc;

    // weight DMA rows (fixed): row r of the A image = output channel n0 + r
    const uint32_t wrow_b = uint32_t(a.KH * a.KW * a.Kin) * 2u;
    const __amdgpu_buffer_rsrc_t wres = make_rsrc(a.w, int64_t(a.Nout) * wrow_b);
    uint32_t a_off[AI];
#pragma unroll
    for (int j = 0; j < AI; ++j) {
        const int r = (wave * AI + j) * 8 + (lane >> 3);
        const int ch = n0 + r;
        a_off[j] = ch < a.Nout ? uint32_t(ch) * wrow_b + uint32_t((lane & 7) ^ fsw128(r)) * 16u : OOB;
    }

    // per-lane fragment read offsets inside a stage (subtile i / j adds MF * RB * i: fsw128 is 16-periodic).
    // 16x16x32: lane (fc, fr) reads row fr of the subtile, 16-B chunk kk * 4 + fc of the 128-B row; 32x32x16: lane
    // (h, p) reads row p, chunk kk * 4 + 2 s + h for K slice s (the operand layout of cdna_hip_programming.md §3)
    uint32_t offA[2 * KS], offB[2 * KS];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int lr = MF == 16 ? fr : (lane & 31);
            const int ch = MF == 16 ? kk * 4 + fc : kk * 4 + 2 * s + (lane >> 5);
            const int ra = wr * (BN / WM) + lr, rb = wc * (BM / WN) + lr;
            offA[kk * KS + s] = uint32_t(ra * RB + ((ch ^ fsw128(ra)) << 4));
            offB[kk * KS + s] = uint32_t(BN * RB + rb * RB + ((ch ^ fsw128(rb)) << 4));
        }
    bf16x8 f0a[TM * KS], f0b[TN * KS], f1a[TM * KS], f1b[TN * KS];
    auto read_frags = [&](bf16x8* fa, bf16x8* fb, int slot_off, int kk) {     // slot_off: the ring slot's byte offset
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const char* As = smem + slot_off + offA[kk * KS + s];
            const char* Bs = smem + slot_off + offB[kk * KS + s];
#pragma unroll
            for (int i = 0; i < TM; ++i) fa[i * KS + s] = *reinterpret_cast<const bf16x8*>(As + i * MF * RB);
#pragma unroll
            for (int j = 0; j < TN; ++j) fb[j * KS + s] = *reinterpret_cast<const bf16x8*>(Bs + j * MF * RB);
        }
    };
    AccT acc[TM][TN];
    auto mma = [&](const bf16x8* fa, const bf16x8* fb) {
        if constexpr ((ABL & 2) != 0) {
#pragma unroll
            for (int i = 0; i < TM * KS; ++i) asm volatile("" ::"v"(fa[i]));
#pragma unroll
            for (int j = 0; j < TN * KS; ++j) asm volatile("" ::"v"(fb[j]));
            return;
        }
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const bf16x8 av = fa[i * KS + s], bv = fb[j * KS + s];
                    if constexpr (MF == 16) {
                        if constexpr (MODE == PF)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, av),
                                                                                __builtin_bit_cast(f16x8, bv), acc[i][j],
                                                                                0, 0, 0);
                        else
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc[i][j], 0, 0, 0);
                    } else {
                        if constexpr (MODE == PF)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, av),
                                                                                __builtin_bit_cast(f16x8, bv), acc[i][j],
                                                                                0, 0, 0);
                        else
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc[i][j], 0, 0, 0);
                    }
                }
    };
    auto zero_acc = [&]() {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < NR; ++r) acc[i][j][r] = 0.f;
    };

    float ssum[TM][NR], ssq[TM][NR];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < NR; ++r) ssum[i][r] = ssq[i][r] = 0.f;

    Issuer<BM, BN, NW, MODE, ABL, C1, TO> is(a, wave, lane, mt_lo, qstride, ntile);
    is.start();

    // prologue: stages 0..2 in flight (stages past the stream's end fetch nothing); stage 0 landed
    // everywhere; its first-half fragments read
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        is.issue_dma(smem + s * STAGE, wres, a_off, s < total);
        is.advance();
    }
    vm_wait<(NS - 1) * DPS>();
    step_barrier();
    if (total > 0) read_frags(f0a, f0b, 0, 0);
    int boff = 0;                             // LP 2: the computing slot's byte offset (buf * STAGE)

    // compute side: one K step per iteration; tiles end inside the stream
    int ct = 0, ck = 0, cnk = C1 ? a.KH * a.KW * kc : 0, buf = 0;
    int64_t m0 = 0;
    Cls cc{};
    uint32_t t_n = 0, t_p = 0;                // divmod(m0, OHW) of the computing tile
    float inv_owc = 1.f;
    // C1: the computing tile's first pixel, advanced per tile as the issuer's
    int c_m0 = 0, c_tn = 0;
    uint32_t c_tp = 0;
    if constexpr (C1) {
        c_m0 = mt_lo * BM;
        c_tn = int(uint32_t(c_m0) / is.ohw);
        c_tp = uint32_t(c_m0) - uint32_t(c_tn) * is.ohw;
    }
    const int Mtot = a.N * int(is.ohw);
    // one K step: the second half's fragments read and the first half's MFMAs; the wait and barrier; stage g+NS's DMAs
    // into the freed slot between the second half's MFMAs; the next stage's first-half reads.  keep_epi: a tile's
    // first step after an epilogue, whose stores may stay in flight across the wait; live: stage g+NS is in the stream
    auto kstep = [&](bool keep_epi, bool live) __attribute__((always_inline)) {
        const int cur = LP == 2 ? boff : buf * STAGE;
        read_frags(f1a, f1b, cur, 1);
        mma(f0a, f0b);
        constexpr int MH = TM * TN * KS;                                            // MFMAs per half
        if constexpr (RO == 1) {
            __builtin_amdgcn_sched_group_barrier(0x100, (TM + TN) * KS, 0);        // this step's second-half reads
            __builtin_amdgcn_sched_group_barrier(0x008, MH, 0);                     // first-half MFMAs
        }
        // stage g+1 must have landed (own DMAs); stage g+2 may stay in flight (every step issues DPS DMAs,
        // live or not, so the count is constant); in a tile's first step the previous tile's epilogue stores,
        // issued after stage g+2's pieces, may stay in flight too
        if (keep_epi) vm_wait<(NS - 2) * DPS + EPS>();
        else vm_wait<(NS - 2) * DPS>();
        step_barrier();
        // the slot of stage g is free again (every wave's reads of it returned before the barrier): stage
        // g+3's DMAs go out one at a time between the second half's MFMAs (issued in a burst they held both
        // waves of a SIMD off the MFMA pipe for the whole burst), then the next stage's first-half reads
        const int nbuf = buf == NS - 1 ? 0 : buf + 1;
        const int nboff = boff == (NS - 1) * STAGE ? 0 : boff + STAGE;
        is.issue_dma(smem + cur, wres, a_off, live);
        read_frags(f0a, f0b, LP == 2 ? nboff : nbuf * STAGE, 0);
        mma(f1a, f1b);
        if constexpr (RO == 1) {
            __builtin_amdgcn_sched_group_barrier(0x100, (TM + TN) * KS, 0);        // next-stage reads first
#pragma unroll
            for (int d = 0; d < DPS; ++d) {
                __builtin_amdgcn_sched_group_barrier(0x008, MH / (DPS + 1), 0);     // MFMAs
                __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                 // one DMA
            }
            __builtin_amdgcn_sched_group_barrier(0x008, MH - DPS * (MH / (DPS + 1)), 0);
        } else {
#pragma unroll
            for (int d = 0; d < DPS; ++d) {
                __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                 // one DMA
                __builtin_amdgcn_sched_group_barrier(0x008, MH / (DPS + 1), 0);     // MFMAs
            }
            __builtin_amdgcn_sched_group_barrier(0x100, (TM + TN) * KS, 0);        // next-stage reads
            __builtin_amdgcn_sched_group_barrier(0x008, MH - DPS * (MH / (DPS + 1)), 0);
        }
        is.advance();
        if constexpr (LP == 2) boff = nboff;
        else buf = nbuf;
    };
    // the tile's epilogue
    auto epilogue = [&]() __attribute__((always_inline)) {
        // epilogue: D[channel][pixel] (a lane holds 4 consecutive channels of one pixel per subtile) is
        // transposed in registers (conv_epi.h epilogue_regs: pairs of 16-pixel subtiles exchanged with
        // v_permlane16_swap), so every store is a 16-B piece of a pixel's contiguous channel run, issued as
        // buffer stores whose out-of-tile pixels fall out of range (no branches, a fixed count per tile)
        {
            const int wch0 = n0 + wr * WCH;
            const int64_t ybytes = (int64_t(a.N - 1) * a.y_bs + int64_t(a.OH) * a.OW * a.y_ld) * 2;
            const __amdgpu_buffer_rsrc_t yres = make_rsrc(a.y, ybytes);
            auto pix_off = [&](int qp) -> uint32_t {
                if constexpr (C1) {
                    // one class, stride-1 output: the output pixel IS the in-image offset (one wrap: ohw >= BM)
                    const int q = wc * (BM / WN) + qp;
                    if (c_m0 + q >= Mtot) return OOB;
                    uint32_t pix = c_tp + uint32_t(q);
                    int n = c_tn;
                    if (pix >= is.ohw) { pix -= is.ohw; ++n; }
                    return uint32_t((int64_t(n) * a.y_bs + int64_t(pix) * a.y_ld + wch0) * 2);
                }
                const int64_t m = m0 + wc * (BM / WN) + qp;
                if (m >= cc.Mc) return OOB;
                uint32_t n, pix, ci_;
                split_pix(t_n, t_p, uint32_t(wc * (BM / WN) + qp), cc.OHW, uint32_t(cc.OWc), inv_owc, n, pix, ci_);
                const int64_t opix = int64_t(ci_ * a.os + cc.py) * a.OW + int64_t(pix - ci_ * uint32_t(cc.OWc)) * a.os + cc.px;
                return uint32_t((int64_t(n) * a.y_bs + opix * a.y_ld + wch0) * 2);
            };
            auto pix_ok = [&](int qp) -> bool {
                if constexpr (C1) return c_m0 + wc * (BM / WN) + qp < Mtot;
                return m0 + wc * (BM / WN) + qp < cc.Mc;
            };
            if constexpr (EV) {
                const EvalEpi ee{e.sc, e.sh, e.act, make_rsrc(e.res, e.res ? e.res_bytes : 0), e.res != nullptr};
                auto res_off = [&](int qp) -> uint32_t {     // pix_off's C1 pixel walk on the residual view's strides
                    const int q = wc * (BM / WN) + qp;
                    if (c_m0 + q >= Mtot) return OOB;
                    uint32_t pix = c_tp + uint32_t(q);
                    int n = c_tn;
                    if (pix >= is.ohw) { pix -= is.ohw; ++n; }
                    return uint32_t((int64_t(n) * e.r_bs + int64_t(pix) * e.r_ld + wch0) * 2);
                };
                if constexpr (MF == 16)
                    epilogue_regs_x<TM, TN>(acc, ssum, ssq, false, lane, wch0, a.Nout, yres, true, false, pix_off, pix_ok,
                                            &ee, res_off);
                else
                    epilogue_regs32_x<TM, TN>(acc, ssum, ssq, false, lane, wch0, a.Nout, yres, true, false, pix_off,
                                              pix_ok, &ee, res_off);
            } else {
                if constexpr (MF == 16)
                    epilogue_regs<TM, TN>(acc, ssum, ssq, a.st_sum != nullptr, lane, wch0, a.Nout, yres,
                                          a.out_f32 == 2, a.accumulate != 0, pix_off, pix_ok);
                else
                    epilogue_regs32_x<TM, TN>(acc, ssum, ssq, a.st_sum != nullptr, lane, wch0, a.Nout, yres,
                                              a.out_f32 == 2, a.accumulate != 0, pix_off, pix_ok, nullptr, pix_off);
            }
        }
    };
    if constexpr (LP >= 1) {
        int g = 0;
        for (int t = 0; t < ntile; ++t) {
            if (t > 0) {
                c_m0 += is.m_step;
                c_tn += is.step_n;
                c_tp += is.step_p;
                if (c_tp >= is.ohw) { c_tp -= is.ohw; ++c_tn; }
            }
            zero_acc();
            kstep(EPI == 2 && t > 0, g + NS < total);
            ++g;
            if constexpr (LP == 2) {
                // the stream's last NS stages fetch nothing: live while g < glim
                const int glim = total - NS;
                for (int k = 1; k < cnk; ++k, ++g) kstep(false, g < glim);
            } else {
                for (int k = 1; k < cnk; ++k, ++g) kstep(false, g + NS < total);
            }
            epilogue();
        }
    } else {
        for (int g = 0; g < total; ++g) {
            if (C1 && ck == 0) {
                if (ct > 0) {
                    c_m0 += is.m_step;
                    c_tn += is.step_n;
                    c_tp += is.step_p;
                    if (c_tp >= is.ohw) { c_tp -= is.ohw; ++c_tn; }
                }
                zero_acc();
            } else if (ck == 0) {
                const int mt = mt_lo + ct * qstride;
                const int c = cls_find(a, mt);
                cc = cls_of(a, c);
                m0 = int64_t(mt - a.mt_pre[c]) * BM;
                t_n = uint32_t(m0) / cc.OHW;
                t_p = uint32_t(m0) - t_n * cc.OHW;
                inv_owc = 1.0f / float(cc.OWc);
                cnk = cc.ntap * kc;
                zero_acc();
            }
            kstep(EPI == 2 && ck == 0 && ct > 0, g + NS < total);
            if (++ck < cnk) continue;
            ck = 0;
            ++ct;

            epilogue();
        }
    }

    if (a.st_sum) {
        // one partial row per workgroup of this channel tile: row = xcd + 8 * qq
        vm_wait<0>();
        __syncthreads();
        float (*red)[WN][BN] = reinterpret_cast<float (*)[WN][BN]>(smem);   // [sum|sq][pixel wave][channel]
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                float s = ssum[i][r], sq = ssq[i][r];
                // over the lanes holding other pixels of the same channel: 16 (16x16 layout) or 32 (32x32)
#pragma unroll
                for (int o = 1; o < MF; o <<= 1) {
                    s += __shfl_xor(s, o, 64);
                    sq += __shfl_xor(sq, o, 64);
                }
                if ((lane & (MF - 1)) == 0) {
                    const int cl = MF == 16 ? wr * (BN / WM) + i * 16 + fc * 4 + r
                                            : wr * (BN / WM) + i * 32 + 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3);
                    red[0][wc][cl] = s;
                    red[1][wc][cl] = sq;
                }
            }
        __syncthreads();
        const int row = xcd + 8 * qq;
        for (int cl = tid; cl < BN; cl += NW * 64) {
            const int ch = n0 + cl;
            if (ch < a.Nout) {
                float ps = 0.f, pq = 0.f;
#pragma unroll
                for (int w = 0; w < WN; ++w) { ps += red[0][w][cl]; pq += red[1][w][cl]; }
                stat_store(&a.st_sum[int64_t(row) * a.Nout + ch], ps, a.fold.gamma != nullptr);
                stat_store(&a.st_sq[int64_t(row) * a.Nout + ch], pq, a.fold.gamma != nullptr);
            }
        }
        if (a.fold.gamma) bn_fold_tail<BN, NW * 64>(a.fold, a.st_sum, a.st_sq, a.Nout, nt, int(gridDim.x) / a.ntiles, smem);
    }
}

// tile configurations: 0 / 1 the shipped 16-wave 256 x 128 and 8-wave 256 x 64 tiles; 2 experimental
// (ym_pipe_set_exp 1): 256 x 128 on 8 waves of 64 x 64 — round 5, same process: within +-3.5 % of the 16-wave tile
// on every layer with 31 % fewer LDS-array cycles (profiles/r05/pipe_wave_tile_ab.txt), so the LDS array does not
// bound it.  (256 x 256 / 512 x 128 tiles on 8 waves of 128 x 64 need 128 accumulator registers per lane and
// spilled 213-439 VGPRs at the 256-register cap of two waves per SIMD: not kept.)
struct Cfg {
    int bm, bn;
};
constexpr Cfg kCfg[] = {{256, 128}, {256, 64}, {256, 128}};

// 256 x 128 tiles run on 16 waves of 32 x 64 (four per SIMD, 127 VGPRs): same staging and LDS as 8 waves
// of 64 x 64, 1.5x the fragment reads, but while some waves of a SIMD issue their DMA pieces or wait at
// the barrier others issue MFMAs — same-process A/B against 8 waves: fwd / dgrad 0-7 % faster on every
// layer measured (1x1 80x80 192->256 -6.8 / -6.2 %, 3x3 40x40 128->128 -3.3 / -6.7 %, stride-2 80x80 equal)
// cfg 0 / 1 / 2 tiles (kCfg) of one control path (C1), MFMA shape (MF) and issue order (RO)
template <int MODE, bool C1, int MF, int RO, int LP = 0, int TO = 0>
void launch_tiles(int cfg, const PipeArgs& a, int grid, hipStream_t st) {
    switch (cfg) {
        case 0: conv_pipe_kernel<256, 128, 4, 4, MODE, 2, 3, 0, C1, false, MF, RO, LP, TO><<<dim3(grid), dim3(1024), 0, st>>>(a, EvalArgs{}); break;
        case 1: conv_pipe_kernel<256, 64, 1, 8, MODE, 2, 3, 0, C1, false, MF, RO, LP, TO><<<dim3(grid), dim3(512), 0, st>>>(a, EvalArgs{}); break;
        default: conv_pipe_kernel<256, 128, 2, 4, MODE, 2, 3, 0, C1, false, MF, RO, LP, TO><<<dim3(grid), dim3(512), 0, st>>>(a, EvalArgs{}); break;
    }
}

// the tap-innermost K order (Issuer TO 1) where it measured faster: stride-2 3x3 forwards reading maps >= 128 wide (op 6,
// 128 -> 128 at 160x160 -> 80x80: -12 % time, -27 % HBM fetch; profiles/r06/pipe_taporder_ab.txt) — there one tile's
// input over every channel chunk overflows its share of the XCD's L2, one chunk's does not.  Elsewhere it measured
// 0..+5 % slower (a tap_setup per K step, and the footprint fits L2 either way)
inline bool tap_inner(const PipeArgs& a) { return a.stride == 2 && a.KH == 3 && a.GW >= 128; }

template <int MODE>
void launch_mode(int cfg, const PipeArgs& a, int grid, hipStream_t st) {
    const bool c1 = a.ncls == 1 && int64_t(a.OH) * a.OW >= kCfg[cfg].bm && g_pipe_exp != 20;
#ifdef YM_EXPERIMENTS
    if (cfg == 0 && g_pipe_exp >= 10 && g_pipe_exp < 20) {
        switch (g_pipe_exp) {
            case 10: conv_pipe_kernel<256, 128, 4, 4, MODE, 2, 3, 1, true><<<dim3(grid), dim3(1024), 0, st>>>(a, EvalArgs{}); return;
            case 11: conv_pipe_kernel<256, 128, 4, 4, MODE, 2, 3, 2, true><<<dim3(grid), dim3(1024), 0, st>>>(a, EvalArgs{}); return;
            case 12: conv_pipe_kernel<256, 128, 4, 4, MODE, 2, 3, 4, true><<<dim3(grid), dim3(1024), 0, st>>>(a, EvalArgs{}); return;
            default: conv_pipe_kernel<256, 128, 4, 4, MODE, 2, 3, 8, true><<<dim3(grid), dim3(1024), 0, st>>>(a, EvalArgs{}); return;
        }
    }
#endif
#ifdef YM_EXPERIMENTS
    const int mf = g_pipe_mfma, ro = g_pipe_order;
    const int c = mf == 2 && cfg == 0 ? 2 : cfg;
    if (c1) {
        if (mf != 0) {
            if (ro) launch_tiles<MODE, true, 32, 1>(c, a, grid, st);
            else launch_tiles<MODE, true, 32, 0>(c, a, grid, st);
        } else {
            if (ro) launch_tiles<MODE, true, 16, 1>(c, a, grid, st);
            else if (MODE == PF && (g_pipe_taporder == 1 || (g_pipe_taporder < 0 && tap_inner(a)))) {
                if constexpr (MODE == PF) launch_tiles<MODE, true, 16, 0, 2, 1>(c, a, grid, st);
            }
            else if (g_pipe_loop == 0) launch_tiles<MODE, true, 16, 0, 0>(c, a, grid, st);
            else if (g_pipe_loop == 1) launch_tiles<MODE, true, 16, 0, 1>(c, a, grid, st);
            else launch_tiles<MODE, true, 16, 0, 2>(c, a, grid, st);
        }
        return;
    }
    if (mf != 0) launch_tiles<MODE, false, 32, 0>(c, a, grid, st);
    else launch_tiles<MODE, false, 16, 0>(c, a, grid, st);
#else
    if (c1) {
        if constexpr (MODE == PF) {
            if (tap_inner(a)) {
                launch_tiles<MODE, true, 16, 0, 2, 1>(cfg, a, grid, st);
                return;
            }
        }
        launch_tiles<MODE, true, 16, 0, 2>(cfg, a, grid, st);
    } else {
        launch_tiles<MODE, false, 16, 0>(cfg, a, grid, st);
    }
#endif
}

// the eval instance (EV): cfg 1 / 2 tiles on 8 waves (the 16-wave 256 x 128 tile's 127 VGPRs leave no room for the
// eval epilogue at four waves per SIMD; cfg 0 runs as the 8-wave cfg 2)
void launch_eval(int cfg, const PipeArgs& a, const EvalArgs& e, int grid, hipStream_t st) {
#ifdef YM_EXPERIMENTS
    if (g_pipe_mfma != 0) {
        if (cfg == 1) conv_pipe_kernel<256, 64, 1, 8, PF, 2, 3, 0, true, true, 32><<<dim3(grid), dim3(512), 0, st>>>(a, e);
        else conv_pipe_kernel<256, 128, 2, 4, PF, 2, 3, 0, true, true, 32><<<dim3(grid), dim3(512), 0, st>>>(a, e);
        return;
    }
    if (g_pipe_eval_loop == 2) {
        // the nested loop form of the training instances: inference bs 1 / 8 / 128 within the run-to-run spread of the
        // flat form (profiles/r06/pipe_eval_loop_ab.txt), so the eval instance keeps the flat loop
        if (cfg == 1) conv_pipe_kernel<256, 64, 1, 8, PF, 2, 3, 0, true, true, 16, 0, 2><<<dim3(grid), dim3(512), 0, st>>>(a, e);
        else conv_pipe_kernel<256, 128, 2, 4, PF, 2, 3, 0, true, true, 16, 0, 2><<<dim3(grid), dim3(512), 0, st>>>(a, e);
        return;
    }
#endif
    if (cfg == 1) conv_pipe_kernel<256, 64, 1, 8, PF, 2, 3, 0, true, true><<<dim3(grid), dim3(512), 0, st>>>(a, e);
    else conv_pipe_kernel<256, 128, 2, 4, PF, 2, 3, 0, true, true><<<dim3(grid), dim3(512), 0, st>>>(a, e);
}

void launch_cfg(int mode, int cfg, const PipeArgs& a, int grid, hipStream_t st) {
    // both directions: the register-only epilogue (round 4 for the forward, with the statistics masked by a compare:
    // same-process A/B 2-7 % faster on every pipelined forward, profiles/r04/pipe_fwd_reg_epilogue_ab.txt)
    if (mode == PF) launch_mode<PF>(cfg, a, grid, st);
    else launch_mode<PD>(cfg, a, grid, st);
}

}  // namespace

PipePlan pipe_plan(const ym_conv_desc* d, int dgrad) {
    PipePlan p{};
    const int mode = g_pipe_force >= 0 ? g_pipe_force : 3;
    if (!d || mode == 0) return p;
    const int kin = dgrad ? d->cout : d->cin, nout = dgrad ? d->cin : d->cout;
    if (kin % 64 != 0 || nout % 8 != 0) return p;
    if (d->k != 3 && d->k != 1) return p;
    if (d->stride != 1 && d->stride != 2) return p;
    if (dgrad && d->k == 1 && d->stride == 2) return p;
    const int64_t in_ld = dgrad ? d->y_ld : d->x_ld, in_bs = dgrad ? d->y_bs : d->x_bs;
    const int64_t out_ld = dgrad ? d->x_ld : d->y_ld, out_bs = dgrad ? d->x_bs : d->y_bs;
    if (in_ld % 8 || in_bs % 8 || out_ld % 4 || out_bs % 4) return p;
    if (!dgrad && d->out_f32 == 1) return p;       // Detect's fp32 bias convs stay on conv.hip
    const int os = dgrad ? d->stride : 1;
    // rule 1: only where it measured faster in isolation (tools/pipe_check.py): >= 128 output channels
    // (the 256 x 128 tile) and no stride-2 data gradient
    if (mode == 1 && (nout < 128 || os == 2)) return p;
    // 3: the wider rule (A/B runs): every 1x1, and 3x3 with >= 128 output channels or (forward) >= 128
    // input channels, at >= 256 tiles; never the stride-2 data gradient
    if (mode == 3 && (os == 2 || (d->k == 3 && nout < 128 && (dgrad || kin < 128)))) return p;
    const int OH = dgrad ? d->h : d->oh, OW = dgrad ? d->w : d->ow;
    // split_pix: in-image pixel indices as exact floats, row estimates within one of the truth
    if (int64_t(OH) * OW >= (int64_t(1) << 24) || OH >= (1 << 16)) return p;
    const int64_t M = select_n(d) * ((OH + os - 1) / os) * ((OW + os - 1) / os) * os * os;
    p.cfg = nout >= 128 ? 0 : 1;
    if (g_pipe_exp == 1 && nout >= 128) p.cfg = 2;
    const int bm = kCfg[p.cfg].bm, bn = kCfg[p.cfg].bn;
    const int ntiles = (nout + bn - 1) / bn;
    const int64_t tiles = (M / bm) * ntiles;
    // enough tiles to keep every CU busy for several tiles (tail imbalance), else conv.hip's kernels
    if (tiles < int64_t(mode >= 2 ? 256 : 1024)) return p;
    // 32-bit buffer offsets relative to a tile's first image
    if (in_bs * 2 * (256 / std::max<int64_t>(int64_t(OH / os) * (OW / os), 1) + 2) >= (int64_t(1) << 31)) return p;
    int grid = 256;
    const int unit = 8 * ntiles;
    grid = (grid / unit) * unit;
    if (grid < unit) return p;
    p.grid = grid;
    p.rows = grid / ntiles;
    p.ok = 1;
    return p;
}

#ifdef YM_EXPERIMENTS
extern "C" int ym_conv_set_pipe_order(int mode) {
    // K-step issue order of the pipelined kernel (conv_pipe_kernel RO: 0 default, 1 fragment reads pinned first)
    return g_pipe_order.set(mode < 0 || mode > 1 ? 0 : mode);
}

extern "C" int ym_conv_set_pipe_loop(int mode) {
    // loop form of the pipelined kernel's single-class path (conv_pipe_kernel LP: 0 flat, 1 nested tiles x K steps,
    // 2 nested with the slot offset carried)
    return g_pipe_loop.set(mode < 0 || mode > 2 ? 2 : mode);
}

extern "C" int ym_conv_set_pipe_eval_loop(int mode) {
    // loop form of the pipelined kernel's eval instance (conv_pipe_kernel LP: 0 flat, 2 nested); returns the previous
    return g_pipe_eval_loop.set(mode == 2 ? 2 : 0);
}

extern "C" int ym_conv_set_pipe_taporder(int mode) {
    // K order of the pipelined kernel's single-class forward (conv_pipe_kernel TO): 0 chunk innermost, 1 tap innermost,
    // anything else the shipped rule (tap_inner)
    return g_pipe_taporder.set(mode < 0 || mode > 1 ? -1 : mode);
}

extern "C" int ym_conv_set_pipe_mfma(int mode) {
    // MFMA shape of the pipelined implicit GEMM (see g_pipe_mfma); out of range restores the default 0
    return g_pipe_mfma.set(mode < 0 || mode > 2 ? 0 : mode);
}

extern "C" int ym_pipe_set_exp(int v) {
    return g_pipe_exp.set(v);
}
#endif

int pipe_launch(const PipePlan& p, const ym_conv_desc* d, int dgrad, const uint16_t* x, const uint16_t* w, void* y,
                const float* bias, float* st_sum, float* st_sq, hipStream_t st, const ym_bn_fold* fold) {
    PipeArgs a{};
    const int bm = kCfg[p.cfg].bm, bn = kCfg[p.cfg].bn;
    if (!dgrad) {
        a.x = x; a.x_bs = d->x_bs; a.x_ld = d->x_ld;
        a.y = y; a.y_bs = d->y_bs; a.y_ld = d->y_ld;
        a.GH = d->h; a.GW = d->w; a.Kin = d->cin;
        a.OH = d->oh; a.OW = d->ow; a.Nout = d->cout;
        a.os = 1;
        a.out_f32 = d->out_f32;
    } else {
        a.x = x; a.x_bs = d->y_bs; a.x_ld = d->y_ld;
        a.y = y; a.y_bs = d->x_bs; a.y_ld = d->x_ld;
        a.GH = d->oh; a.GW = d->ow; a.Kin = d->cout;
        a.OH = d->h; a.OW = d->w; a.Nout = d->cin;
        a.os = d->stride;
        a.out_f32 = 0;
    }
    a.w = w;
    a.bias = bias; a.st_sum = st_sum; a.st_sq = st_sq;
    a.KH = d->k; a.KW = d->k; a.stride = d->stride; a.pad = d->pad; a.N = d->n;
    a.accumulate = d->accumulate;
    a.ntiles = (a.Nout + bn - 1) / bn;
    a.ncls = a.os == 2 ? 4 : 1;
    int acc = 0;
    for (int c = 0; c < a.ncls; ++c) {
        const int py = a.os == 2 ? (c >> 1) : 0, px = a.os == 2 ? (c & 1) : 0;
        const int64_t ohc = (a.OH - py + a.os - 1) / a.os, owc = (a.OW - px + a.os - 1) / a.os;
        a.mt_pre[c] = acc;
        acc += int((int64_t(a.N) * ohc * owc + bm - 1) / bm);
    }
    a.mt_pre[a.ncls] = acc;
    if (!dgrad && st_sum) a.fold = bn_fold_args(fold);
    launch_cfg(dgrad ? PD : PF, p.cfg, a, p.grid, st);
    return YM_OK;
}

bool pipe_eval_ok(const PipePlan& p, const ym_conv_desc* d) {
    // the eval instance is the single-class (C1) forward: maps of >= BM pixels, the shipped control path
    return p.ok && int64_t(d->oh) * d->ow >= kCfg[p.cfg].bm && g_pipe_exp != 20 && d->out_f32 == 2 && !d->accumulate;
}

int pipe_launch_eval(const PipePlan& p, const ym_conv_desc* d, const uint16_t* x, const uint16_t* w, uint16_t* y,
                     const EvalArgs& e, hipStream_t st) {
    if (!pipe_eval_ok(p, d)) return 1;
    PipeArgs a{};
    a.x = x; a.x_bs = d->x_bs; a.x_ld = d->x_ld;
    a.y = y; a.y_bs = d->y_bs; a.y_ld = d->y_ld;
    a.GH = d->h; a.GW = d->w; a.Kin = d->cin;
    a.OH = d->oh; a.OW = d->ow; a.Nout = d->cout;
    a.os = 1;
    a.out_f32 = 2;
    a.w = w;
    a.KH = d->k; a.KW = d->k; a.stride = d->stride; a.pad = d->pad; a.N = d->n;
    // cfg 0 runs as the 8-wave 256 x 128 instance (same tile, grid and rows)
    const int cfg = p.cfg == 1 ? 1 : 2;
    const int bm = kCfg[cfg].bm, bn = kCfg[cfg].bn;
    a.ntiles = (a.Nout + bn - 1) / bn;
    a.ncls = 1;
    a.mt_pre[0] = 0;
    a.mt_pre[1] = int((int64_t(a.N) * a.OH * a.OW + bm - 1) / bm);
    launch_eval(cfg, a, e, p.grid, st);
    return 0;
}

}  // namespace ym
