// NHWC convolutions on CDNA4 MFMA, fp32 accumulate: forward fp16 x fp16
// (v_mfma_f32_16x16x32_f16; activations are fp16), data gradients bf16
// (v_mfma_f32_16x16x32_bf16; gradients are bf16).
//
// Replaces the reference's nn.Conv2d calls (and their autograd) inside
// Conv / Bottleneck / C2f / C3k / SPPF / PSA / Detect
// (/root/reference/yolo_scratch_cuda/models/yolo11_modules.py:21-33, 221-234).
//
// conv_gemm_kernel<MODE>  implicit GEMM, one kernel for forward (MODE_FWD) and
//   data-gradient (MODE_DGRAD).  GEMM rows = output pixels, cols = output
//   channels, K = taps x input channels.  Tiles BM pixels x BN channels x 64,
//   256 threads = 2x2 waves, register-staged double-buffered LDS, operands
//   fetched with raw buffer loads (out-of-image taps and channel tails read as
//   zero through an out-of-range offset, no branches).  LDS tiles are stored
//   chunk-major ([k-chunk of 8][row] x 16 B) with swizzled rows (swz below) so
//   the 16-B fragment reads and the 16-B staging writes are conflict free.
//   The K loop runs tap-major: per-row source offsets are set up once per tap.
//   m-tiles are grouped per XCD.  The stride-2 data gradient runs as four
//   output-parity classes (blockIdx.z), each with only the taps that land.
//   Epilogue: optional bias, bf16 or fp32 store into a strided NHWC view
//   (concat slices are free), optional accumulate (grad fan-in), and per-block
//   per-channel sum / sum-of-squares partials for training-mode BatchNorm.
// (weight gradients: wgrad.hip)
// conv_first_*  Cin = 1 stem (K = 9): direct fp32 VALU kernels.
// dw3x3_*       depthwise 3x3 (Attention.pe, yolo11_modules.py:122): direct.
#include <algorithm>
#include <cstdlib>
#include <string>

#include "common.h"
#include "conv_direct.h"
#include "conv_epi.h"
#include "conv_halo.h"
#include "conv_hpipe.h"
#include "conv_pipe.h"
#include "bn_fold.h"
#include "reduce.h"
#include "tile.h"

namespace ym {
Policy g_select_n{0};
std::atomic<unsigned> g_policy_gen{0};

namespace {

constexpr int MODE_FWD = 0;
constexpr int MODE_DGRAD = 1;

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
    int N;                                   // images
    int ostep;                               // 2: dgrad of a stride-2 conv, one output parity class per blockIdx.z
    int ntl;                                 // channel tiles interleaved into grid x (0: they are grid y)
    int ep_lds;                              // data gradient: LDS-transposed 16-B epilogue (conv_epi.h)
    BnFoldArgs fold;                         // BatchNorm finalize as the tail (ym_conv_fwd_bn); gamma null = off
};

// LDS images are lane-linear (LDS-DMA writes lane l of a wave-instruction at base + 16*l): 128-B
// rows of 8 16-B slots, row r's chunk c stored in slot c ^ f(r), f(r) = (r >> 1) & 7.  The swizzle
// lives on the global (source) side: a DMA lane that fills slot s of row r loads chunk s ^ f(r), so
// each 8-lane group still reads one whole 128-B row.  A ds_read_b128 lane group (rows {0-3,12-15}
// at chunk c, rows {4-11} at chunk c^1) then covers 16 distinct (row parity, slot) bank quads.
// 64-B rows (32-deep K stages, 4 slots): slot c ^ F(r), F(r) = 2 * ((r >> 2) & 1) — measured
// conflict-free (SQ_LDS_BANK_CONFLICT 0; the earlier F = {0, 3, 2, 1}[(r >> 2) & 3] cost 45-50 %
// extra LDS cycles in the 128x64 tiles, tools/pmc_conv.sh).
template <int RB>
__device__ __forceinline__ int fsw(int r) {
    if constexpr (RB == 128) return (r >> 1) & 7;
    else return ((r >> 2) & 1) << 1;                    // F(r) = 2 * ((r >> 2) & 1)
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
    asm volatile("" ::: "memory");
}

// workgroup barrier without the vmcnt(0) drain __syncthreads() implies; LDS-DMA ordering is
// the caller's (counted wait_vmcnt before it), the asm clobbers keep LDS accesses on their side
__device__ __forceinline__ void raw_barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// WM x WN waves: wave (wr, wc) owns BN/WM channels x BM/WN pixels of the tile; KB-deep K stages
// (rows of KB*2 bytes), an NS-stage LDS ring with NS-1 stages in flight
// EV: the eval-mode Conv block instance (ym_conv_fwd_eval: BatchNorm / SiLU / residual in the register epilogue; e is
// not read by the other instances)
template <int BM, int BN, int WM, int WN, int KB, int NS, int MODE, bool EV = false>
__global__ void __launch_bounds__(WM * WN * 64, (WM * WN == 4 && NS * (BM + BN) * KB * 2 <= 72 * 1024) ? 2 : 1)
conv_gemm_kernel(GemmArgs a, EvalArgs e) {
    constexpr int BK = KB;
    constexpr int RB = KB * 2;           // LDS row bytes
    constexpr int CPR = KB / 8;          // 16-B chunks per row
    constexpr int RPI = 1024 / RB;       // rows per DMA wave-instruction
    constexpr int NW = WM * WN, NT = NW * 64;
    constexpr int TM = BN / WM / 16;     // 16-channel subtiles per wave
    constexpr int TN = BM / WN / 16;     // 16-pixel subtiles per wave
    constexpr int AI = BN / RPI / NW;    // A (weight) DMA instructions per wave per stage
    constexpr int BI = BM / RPI / NW;    // B (activation) DMA instructions per wave per stage
    constexpr int STAGE = (BM + BN) * RB;
    constexpr int NSTAGE = NS;
    static_assert(AI >= 1 && BI >= 1, "tile too small for the staging map");
    // one LDS array (a second __shared__ object can de-pipeline LDS-DMA, cdna_hip_programming.md §5)
    __shared__ __attribute__((aligned(16))) char smem[NSTAGE * STAGE];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave / WN, wc = wave % WN;
    const int fc = lane >> 4, fr = lane & 15;
    // block -> (grid-x slot bx, channel tile): with ntl > 0 the channel tiles of one m-tile sequence
    // are adjacent launches on the same XCD (linear ids 8 apart), so the input rows one of them
    // stages are still in that XCD's L2 when the others stage them; bx keeps the stats row layout
    int bx = blockIdx.x, gxx = gridDim.x, nt = blockIdx.y;
    if (a.ntl > 0) {
        const int s = int(blockIdx.x) >> 3;
        nt = s % a.ntl;
        bx = (s / a.ntl) * 8 + (int(blockIdx.x) & 7);
        gxx = gridDim.x / a.ntl;
    }
    const int n0 = nt * BN;
    const int kc = (a.Kin + BK - 1) / BK;
    // output pixel mapping: oh = i*os + py, ow = j*os + px over a class grid OHc x OWc;
    // for the stride-2 data gradient only the taps kh = kh0 + 2i, kw = kw0 + 2j reach whole pixels
    const int os = a.ostep;
    const int py = os == 2 ? int(blockIdx.z >> 1) : 0, px = os == 2 ? int(blockIdx.z & 1) : 0;
    const int OHc = (a.OH - py + os - 1) / os, OWc = (a.OW - px + os - 1) / os;
    const int kh0 = os == 2 ? ((py + a.pad) & 1) : 0, kw0 = os == 2 ? ((px + a.pad) & 1) : 0;
    const int nkw = (a.KW - kw0 + os - 1) / os;
    const int ntap = ((a.KH - kh0 + os - 1) / os) * nkw;
    const int nk = ntap * kc;
    const uint32_t OHW = uint32_t(OHc) * uint32_t(OWc);
    const int64_t Mc = int64_t(a.N) * OHW;
    // pixel decompositions by float reciprocals where every flat pixel index is exact as a float (round 5: the per-tile
    // 64-bit division and per-row 32-bit divisions of the tile setup and the epilogue were most of this kernel's
    // 7 VALU per MFMA on the short-K layers); larger maps keep the integer divisions
    const bool fdiv = Mc < (int64_t(1) << 24);
    const float inv_ohw = 1.0f / float(OHW), inv_owc = 1.0f / float(OWc);
    auto dm_ohw = [&](uint32_t x, uint32_t& q, uint32_t& r) {
        if (fdiv) fdivmod(x, OHW, inv_ohw, q, r);
        else { q = x / OHW; r = x - q * OHW; }
    };
    auto dm_owc = [&](uint32_t x, uint32_t& q, uint32_t& r) {
        if (fdiv) fdivmod(x, uint32_t(OWc), inv_owc, q, r);
        else { q = x / uint32_t(OWc); r = x - q * uint32_t(OWc); }
    };
    const int mtiles = int((Mc + BM - 1) / BM);
    const uint32_t wrow_b = uint32_t(a.KH * a.KW * a.Kin) * 2u;
    const uint32_t xld_b = uint32_t(a.x_ld) * 2u;

    // DMA geometry: instruction j of this wave fills rows (wave*I + j)*RPI + lane/CPR, slot lane%CPR
    const int lrow = lane / CPR, lslot = lane % CPR;
    const __amdgpu_buffer_rsrc_t wres = make_rsrc(a.w, int64_t(a.Nout) * wrow_b);
    uint32_t a_off[AI], a_chk[AI];
#pragma unroll
    for (int j = 0; j < AI; ++j) {
        const int r = (wave * AI + j) * RPI + lrow;
        const int ch = n0 + r;
        a_chk[j] = uint32_t(lslot ^ fsw<RB>(r)) * 8u;      // chunk (in elements) this lane loads
        a_off[j] = ch < a.Nout ? uint32_t(ch) * wrow_b : OOB;
    }

    float ssum[TM][4], ssq[TM][4];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) ssum[i][r] = ssq[i][r] = 0.f;

    // m-tiles grouped per XCD (workgroups go to XCDs round-robin by linear id; gridDim.x % 8 == 0):
    // neighbouring tiles share input halo rows in that XCD's L2
    const int xcd = bx & 7, lstride = gxx >> 3;
    const int per_xcd = (mtiles + 7) >> 3;
    const int mt_end = min((xcd + 1) * per_xcd, mtiles);
    // K steps this workgroup walks: all nk, or the eval K-split's slice blockIdx.z of e.ks (k_lo .. k_lo + nkl)
    int k_lo = 0, nkl = nk;
    if constexpr (EV) {
        if (e.ks > 1) {
            k_lo = int(blockIdx.z) * nk / e.ks;
            nkl = (int(blockIdx.z) + 1) * nk / e.ks - k_lo;
        }
    }
    for (int mt = xcd * per_xcd + (bx >> 3); mt < mt_end; mt += lstride) {
        const int64_t m0 = int64_t(mt) * BM;
        const uint32_t nfirst = uint32_t(m0) / OHW;          // Mc < 2^31 (host check): one 32-bit scalar division
        const __amdgpu_buffer_rsrc_t xres =
            make_rsrc(a.x + int64_t(nfirst) * a.x_bs, (int64_t(a.N) - nfirst) * a.x_bs * 2);
        int b_oh[BI], b_ow[BI];
        uint32_t b_img[BI], b_off[BI], b_chk[BI];
#pragma unroll
        for (int j = 0; j < BI; ++j) {
            const int r = (wave * BI + j) * RPI + lrow;
            const int64_t m = m0 + r;
            const uint32_t um = m < Mc ? uint32_t(m) : 0u;
            uint32_t n, pix, i, col;
            dm_ohw(um, n, pix);
            dm_owc(pix, i, col);
            b_chk[j] = uint32_t(lslot ^ fsw<RB>(r)) * 8u;
            b_img[j] = m < Mc ? (n - nfirst) * uint32_t(a.x_bs) * 2u : OOB;
            b_oh[j] = int(i) * os + py;
            b_ow[j] = int(col) * os + px;
        }
        int t_i = 0, t_j = 0;                // (row, column) of the next staged tap among the class's taps
        auto tap_setup = [&]() {
            const int kh = kh0 + t_i * os, kw = kw0 + t_j * os;
            if (++t_j == nkw) { t_j = 0; ++t_i; }
#pragma unroll
            for (int j = 0; j < BI; ++j) {
                int gh, gw;
                if (MODE == MODE_FWD) {
                    gh = b_oh[j] * a.stride - a.pad + kh;
                    gw = b_ow[j] * a.stride - a.pad + kw;
                } else {                       // th, tw are multiples of the stride here
                    gh = (b_oh[j] + a.pad - kh) >> (a.stride - 1);
                    gw = (b_ow[j] + a.pad - kw) >> (a.stride - 1);
                }
                const bool ok = b_img[j] != OOB && gh >= 0 && gh < a.GH && gw >= 0 && gw < a.GW;
                b_off[j] = ok ? b_img[j] + uint32_t(gh * a.GW + gw) * xld_b : OOB;
            }
            return uint32_t((kh * a.KW + kw) * a.Kin) * 2u;
        };
        int c_next = 0;
        uint32_t a_tap = 0;
        if constexpr (EV) {
            if (k_lo) {                    // a K slice starting at tap k_lo / kc, chunk k_lo % kc
                const int tap = k_lo / kc;
                t_i = tap / nkw;
                t_j = tap - t_i * nkw;
                c_next = k_lo - tap * kc;
                if (c_next) a_tap = tap_setup();
            }
        }
        // issue one stage of LDS-DMA: AI + BI buffer_load_dwordx4 ... lds per wave
        auto issue = [&](int buf) {
            if (c_next == 0) a_tap = tap_setup();
            const int k0 = c_next * BK;
            char* st = smem + buf * STAGE;
#pragma unroll
            for (int j = 0; j < AI; ++j) {
                const uint32_t kk = uint32_t(k0) + a_chk[j];
                const uint32_t off = (kk < uint32_t(a.Kin) && a_off[j] != OOB) ? a_off[j] + a_tap + kk * 2u : OOB;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    wres, (__attribute__((address_space(3))) void*)(st + (wave * AI + j) * 1024), 16, off, 0, 0, 0);
            }
#pragma unroll
            for (int j = 0; j < BI; ++j) {
                const uint32_t kk = uint32_t(k0) + b_chk[j];
                const uint32_t off = (kk < uint32_t(a.Kin) && b_off[j] != OOB) ? b_off[j] + kk * 2u : OOB;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    xres, (__attribute__((address_space(3))) void*)(st + BN * RB + (wave * BI + j) * 1024), 16, off,
                    0, 0, 0);
            }
            if (++c_next == kc) c_next = 0;
        };

        f32x4 acc[TM][TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

        // nk == 0: a parity class no tap reaches (1x1 stride-2): zero gradient
        raw_barrier();                     // previous tile's readers are done with every stage
#pragma unroll
        for (int s0 = 0; s0 < NSTAGE - 1; ++s0)
            if (s0 < nkl) issue(s0);
        for (int k = 0; k < nkl; ++k) {
            const int buf = k % NSTAGE;
            // this wave's DMAs of stage k have landed (the later stages may stay in flight)
            const int ahead = min(NSTAGE - 2, nkl - 1 - k);
            if (NSTAGE >= 4 && ahead >= 2) wait_vmcnt<(NSTAGE >= 4 ? 2 : 0) * (AI + BI)>();
            else if (NSTAGE >= 3 && ahead >= 1) wait_vmcnt<(NSTAGE >= 3 ? 1 : 0) * (AI + BI)>();
            else wait_vmcnt<0>();
            raw_barrier();                 // ... everyone's, and everyone finished reading stage k-1
            if (k + NSTAGE - 1 < nkl) issue((k + NSTAGE - 1) % NSTAGE);
            const char* As = smem + buf * STAGE;
            const char* Bs = As + BN * RB;
            // fragments of both 32-deep halves first, then the MFMAs (two register sets; the order is
            // pinned with sched_group_barrier: left to itself the compiler re-reads one A fragment at a
            // time behind an lgkmcnt(0), exposing the LDS latency every 4 MFMAs)
            constexpr int KS = BK / 32;
            bf16x8 af[KS][TM], bfr[KS][TN];
#pragma unroll
            for (int kk = 0; kk < KS; ++kk) {
                const int cch = kk * 4 + fc;
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const int r = wr * (BN / WM) + i * 16 + fr;
                    af[kk][i] = *reinterpret_cast<const bf16x8*>(As + r * RB + ((cch ^ fsw<RB>(r)) << 4));
                }
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int r = wc * (BM / WN) + j * 16 + fr;
                    bfr[kk][j] = *reinterpret_cast<const bf16x8*>(Bs + r * RB + ((cch ^ fsw<RB>(r)) << 4));
                }
            }
#pragma unroll
            for (int kk = 0; kk < KS; ++kk) {
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j) {
                        if constexpr (MODE == MODE_FWD)   // fp16 activations x fp16 weights
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                                __builtin_bit_cast(f16x8, af[kk][i]), __builtin_bit_cast(f16x8, bfr[kk][j]), acc[i][j],
                                0, 0, 0);
                        else                              // bf16 gradients x bf16 weights
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kk][i], bfr[kk][j], acc[i][j], 0,
                                                                               0, 0);
                    }
            }
#pragma unroll
            for (int kk = 0; kk < KS; ++kk) __builtin_amdgcn_sched_group_barrier(0x100, TM + TN, 0);
#pragma unroll
            for (int kk = 0; kk < KS; ++kk) __builtin_amdgcn_sched_group_barrier(0x008, TM * TN, 0);
        }

        if constexpr (BN / WM >= 32) {
            if (a.ep_lds) {
                // 16-bit output (fp16 z + statistics, or the bf16 data gradient + fan-in accumulate): transposed in
                // registers (conv_epi.h epilogue_regs) and stored as 16-B pieces of each pixel's channel run
                const __amdgpu_buffer_rsrc_t yres = make_rsrc(a.y, int64_t(a.N) * a.y_bs * 2);
                const int wch0 = n0 + wr * (BN / WM);
                auto pix_off = [&](int q) -> uint32_t {
                    const int64_t m = m0 + wc * (BM / WN) + q;
                    if (m >= Mc) return OOB;
                    uint32_t n, pix, ci_, col;
                    dm_ohw(uint32_t(m), n, pix);
                    dm_owc(pix, ci_, col);
                    const int64_t opix = int64_t(ci_ * os + py) * a.OW + int64_t(col) * os + px;
                    return uint32_t((int64_t(n) * a.y_bs + opix * a.y_ld + wch0) * 2);
                };
                auto pix_ok = [&](int q) -> bool { return m0 + wc * (BM / WN) + q < Mc; };
                if constexpr (EV) {
                    if (e.ks > 1) {        // K slice: fp32 partial sums, 4 channels of one pixel per lane (Nout % 8 == 0)
#pragma unroll
                        for (int j = 0; j < TN; ++j) {
                            const int64_t m = m0 + wc * (BM / WN) + j * 16 + fr;
                            if (m >= Mc) continue;
                            float* pp = e.part + (int64_t(blockIdx.z) * Mc + m) * a.Nout;
#pragma unroll
                            for (int i = 0; i < TM; ++i) {
                                const int cb = wch0 + i * 16 + fc * 4;
                                if (cb < a.Nout)
                                    *reinterpret_cast<float4*>(pp + cb) =
                                        make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
                            }
                        }
                        continue;
                    }
                    const EvalEpi ee{e.sc, e.sh, e.act, make_rsrc(e.res, e.res ? e.res_bytes : 0), e.res != nullptr};
                    auto res_off = [&](int q) -> uint32_t {        // the forward: one class, stride-1 output grid
                        const int64_t m = m0 + wc * (BM / WN) + q;
                        if (m >= Mc) return OOB;
                        uint32_t n, pix;
                        dm_ohw(uint32_t(m), n, pix);
                        return uint32_t((int64_t(n) * e.r_bs + int64_t(pix) * e.r_ld + wch0) * 2);
                    };
                    epilogue_regs_x<TM, TN>(acc, ssum, ssq, false, lane, wch0, a.Nout, yres, true, false, pix_off,
                                            pix_ok, &ee, res_off);
                } else {
                    epilogue_regs<TM, TN>(acc, ssum, ssq, MODE == MODE_FWD && a.st_sum != nullptr, lane, wch0, a.Nout,
                                          yres, MODE == MODE_FWD, MODE == MODE_DGRAD && a.accumulate != 0, pix_off,
                                          pix_ok);
                }
                continue;
            }
        }
        // epilogue: D[channel][pixel]; lane holds 4 consecutive channels of one pixel
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int64_t m = m0 + wc * (BM / WN) + j * 16 + fr;
            if (m >= Mc) continue;
            const uint32_t n = uint32_t(m) / OHW, pix = uint32_t(m) - n * OHW;
            const uint32_t ci_ = pix / uint32_t(OWc);
            const int64_t opix = int64_t(ci_ * os + py) * a.OW + int64_t(pix - ci_ * uint32_t(OWc)) * os + px;
            const int64_t obase = int64_t(n) * a.y_bs + opix * a.y_ld;
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int cb = n0 + wr * (BN / WM) + i * 16 + fc * 4;
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
                        o.x = pk2h(v[0], v[1]);
                        o.y = pk2h(v[2], v[3]);
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
                        o.x = pk2bf(v[0], v[1]);
                        o.y = pk2bf(v[2], v[3]);
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
        float (*red)[WN][BN] = reinterpret_cast<float (*)[WN][BN]>(smem);   // [sum|sq][pixel wave][channel]
        raw_barrier();                     // staging LDS is free again
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
                    int cl = wr * (BN / WM) + i * 16 + (lane >> 4) * 4 + r;
                    red[0][wc][cl] = s;
                    red[1][wc][cl] = q;
                }
            }
        __syncthreads();
        for (int c = tid; c < BN; c += NT) {
            int ch = n0 + c;
            if (ch < a.Nout) {
                float ps = 0.f, pq = 0.f;
#pragma unroll
                for (int w = 0; w < WN; ++w) { ps += red[0][w][c]; pq += red[1][w][c]; }
                stat_store(&a.st_sum[int64_t(bx) * a.Nout + ch], ps, a.fold.gamma != nullptr);
                stat_store(&a.st_sq[int64_t(bx) * a.Nout + ch], pq, a.fold.gamma != nullptr);
            }
        }
        if (a.fold.gamma) bn_fold_tail<BN, NT>(a.fold, a.st_sum, a.st_sq, a.Nout, nt, gxx, smem);
    }
}

// ------------------------------------------------------------------ stem conv (Cin = CH image planes), fp32 image input
// one thread per (output pixel, 8 channels), the 8 x 9CH weights in registers, 32-bit index math
// (N*OH*OW and N*CH*H*W < 2^31, checked on the host).  HBM-bound: writes the fp16 z (2 B/elem).
// The image is the reference's NCHW (B, CH, H, W) fp32 tensor; tap t = ci * 9 + kh * 3 + kw is the OIHW weight order,
// and the sum runs over t in that order (CH = 1: the crater config's single plane).
// Channel pieces (these small VALU kernels): a launch covers channels c_base .. c_base + Cout of a Ct-channel layer,
// Cout / 8 a power of two <= 64 (the lane-group reductions); a width like the x-scale stem's 96 runs as pieces 64 + 32
// (ch_pieces below), rows / partial rows strided by Ct.
template <int CH>
__device__ __forceinline__ void stem_patch(const float* __restrict__ img, int n, int H, int W, int oh, int ow,
                                           int stride, int pad, float* patch) {
#pragma unroll
    for (int ci = 0; ci < CH; ++ci)
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
                const int ih = oh * stride - pad + kh, iw = ow * stride - pad + kw;
                patch[ci * 9 + kh * 3 + kw] = (unsigned(ih) < unsigned(H) && unsigned(iw) < unsigned(W))
                                                  ? img[((n * CH + ci) * H + ih) * W + iw] : 0.f;
            }
}

template <int CH>
__global__ void __launch_bounds__(256) conv_first_fwd_kernel(const float* __restrict__ img, const float* __restrict__ w,
                                                             uint16_t* __restrict__ y, float* __restrict__ st_sum,
                                                             float* __restrict__ st_sq, int N, int H, int W, int OH,
                                                             int OW, int Cout, int stride, int pad, int c_base,
                                                             int Ct) {
    constexpr int T = 9 * CH;
    __shared__ float red[2][512];
    const int G = Cout >> 3;                 // channel groups (divides 64)
    const int g = threadIdx.x % G;
    float wr[8][T];
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int t = 0; t < T; ++t) wr[r][t] = w[(c_base + g * 8 + r) * T + t];
    float ls[8], lq[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) ls[r] = lq[r] = 0.f;
    const int M = N * OH * OW, OHW = OH * OW;
    const int step = gridDim.x * (256 / G);
    for (int m = (blockIdx.x * 256 + threadIdx.x) / G; m < M; m += step) {
        const int n = m / OHW, pix = m - n * OHW, oh = pix / OW, ow = pix - oh * OW;
        float patch[T];
        stem_patch<CH>(img, n, H, W, oh, ow, stride, pad, patch);
        float v[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            float s = 0.f;
#pragma unroll
            for (int t = 0; t < T; ++t) s += wr[r][t] * patch[t];
            v[r] = s;
            ls[r] += s;
            lq[r] += s * s;
        }
        uint4 o;
        o.x = pk2h(v[0], v[1]);
        o.y = pk2h(v[2], v[3]);
        o.z = pk2h(v[4], v[5]);
        o.w = pk2h(v[6], v[7]);
        if (y) *reinterpret_cast<uint4*>(y + size_t(m) * Ct + c_base + g * 8) = o;   // null: statistics only
    }
    // lanes with the same channel group: xor-reduce over the other lane bits, then the waves in order
#pragma unroll
    for (int r = 0; r < 8; ++r)
        for (int o = G; o < 64; o <<= 1) {
            ls[r] += __shfl_xor(ls[r], o, 64);
            lq[r] += __shfl_xor(lq[r], o, 64);
        }
    ordered_wave_add8(red[0], red[1], ls, lq, g, G);
    for (int c = threadIdx.x; c < Cout; c += 256) {
        st_sum[int64_t(blockIdx.x) * Ct + c_base + c] = red[0][c];
        st_sq[int64_t(blockIdx.x) * Ct + c_base + c] = red[1][c];
    }
}

// eval-mode stem Conv block in one launch (ym_conv_first_fwd_eval): one thread per output pixel and ALL its channels
// (the weights, scale and shift broadcast from LDS), the running-statistics BatchNorm + SiLU on the fp32 sums
// (EvalEpi's arithmetic, the training kernel's summation order) and 16-B stores of the pixel's contiguous channel
// run — a wave writes 64 whole pixel rows; the 9 CH image reads are made once per pixel, not once per 8 channels.
// No statistics, no fp16 z, no apply launch.  Cout % 8 == 0, Cout <= 512 (CH = 1, 2), <= 256 (CH = 3, 4).
template <int CH>
__global__ void __launch_bounds__(256) conv_first_eval_kernel(const float* __restrict__ img, const float* __restrict__ w,
                                                              const float* __restrict__ sc, const float* __restrict__ sh,
                                                              int act, uint16_t* __restrict__ y, int64_t y_bs,
                                                              int64_t y_ld, int N, int H, int W, int OH, int OW,
                                                              int Cout, int stride, int pad) {
    constexpr int T = 9 * CH;
    // weights tap-major in LDS ([t][c]: 8 channels of one tap = two 16-B broadcast reads)
    __shared__ __attribute__((aligned(16))) float wl[(CH <= 2 ? 512 : 256) * T];
    __shared__ __attribute__((aligned(16))) float sl[512], hl[512];
    for (int i = threadIdx.x; i < Cout * T; i += 256) {
        const int c = i / T, t = i - c * T;
        wl[t * Cout + c] = w[i];
    }
    for (int i = threadIdx.x; i < Cout; i += 256) {
        sl[i] = sc[i];
        hl[i] = sh[i];
    }
    __syncthreads();
    const int M = N * OH * OW, OHW = OH * OW;
    for (int m = blockIdx.x * 256 + threadIdx.x; m < M; m += gridDim.x * 256) {
        const int n = m / OHW, pix = m - n * OHW, oh = pix / OW, ow = pix - oh * OW;
        float patch[T];
        stem_patch<CH>(img, n, H, W, oh, ow, stride, pad, patch);
        uint16_t* yp = y + int64_t(n) * y_bs + int64_t(pix) * y_ld;
        for (int c0 = 0; c0 < Cout; c0 += 8) {
            float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int t = 0; t < T; ++t) {                        // tap order per channel: the training kernel's sum
                const float4 w0 = *reinterpret_cast<const float4*>(wl + t * Cout + c0);
                const float4 w1 = *reinterpret_cast<const float4*>(wl + t * Cout + c0 + 4);
                const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
                for (int r = 0; r < 8; ++r) v[r] += wv[r] * patch[t];
            }
            const float4 s0 = *reinterpret_cast<const float4*>(sl + c0), s1 = *reinterpret_cast<const float4*>(sl + c0 + 4);
            const float4 h0 = *reinterpret_cast<const float4*>(hl + c0), h1 = *reinterpret_cast<const float4*>(hl + c0 + 4);
            const float sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
            const float hv[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const float u = fmaf(v[r], sv[r], hv[r]);
                v[r] = act ? silu_f(u) : u;
            }
            uint4 o;
            o.x = pk2h(v[0], v[1]);
            o.y = pk2h(v[2], v[3]);
            o.z = pk2h(v[4], v[5]);
            o.w = pk2h(v[6], v[7]);
            *reinterpret_cast<uint4*>(yp + c0) = o;
        }
    }
}

// part[block][co*9 + t] = sum over the block's pixels p of dz[p][co] * patch(p)[t]  (no dgrad: the
// image needs no gradient); dW += the rows summed in order (colsum_kernel)
template <int CH>
__global__ void __launch_bounds__(256) conv_first_wgrad_kernel(const bf16_t* __restrict__ dz, const float* __restrict__ img,
                                                               float* __restrict__ part, int N, int H, int W, int OH,
                                                               int OW, int Cout, int stride, int pad, int c_base,
                                                               int Ct) {
    constexpr int T = 9 * CH;
    __shared__ float red[128 * T];
    const int G = Cout >> 3;
    const int g = threadIdx.x % G;
    float acc[8][T];
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int t = 0; t < T; ++t) acc[r][t] = 0.f;
    const int M = N * OH * OW, OHW = OH * OW;
    const int step = gridDim.x * (256 / G);
    // two pixels per iteration (loads of both first); accumulation order unchanged (m, m + step, ...)
    for (int m0 = (blockIdx.x * 256 + threadIdx.x) / G; m0 < M; m0 += 2 * step) {
        uint4 d[2];
        float xv[2][T];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int m = m0 + u * step < M ? m0 + u * step : m0;
            const int n = m / OHW, pix = m - n * OHW, oh = pix / OW, ow = pix - oh * OW;
            d[u] = *reinterpret_cast<const uint4*>(dz + size_t(m) * Ct + c_base + g * 8);
            stem_patch<CH>(img, n, H, W, oh, ow, stride, pad, xv[u]);
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            if (m0 + u * step >= M) break;
            const uint32_t dd[4] = {d[u].x, d[u].y, d[u].z, d[u].w};
            float gv[8];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                gv[2 * e] = bf2f(bf16_t(dd[e] & 0xffff));
                gv[2 * e + 1] = bf2f(bf16_t(dd[e] >> 16));
            }
#pragma unroll
            for (int t = 0; t < T; ++t)
#pragma unroll
                for (int r = 0; r < 8; ++r) acc[r][t] += gv[r] * xv[u][t];
        }
    }
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int t = 0; t < T; ++t)
            for (int o = G; o < 64; o <<= 1) acc[r][t] += __shfl_xor(acc[r][t], o, 64);
    ordered_wave_add_taps<T>(red, acc, g, G);
    for (int i = threadIdx.x; i < Cout * T; i += 256) part[int64_t(blockIdx.x) * Ct * T + c_base * T + i] = red[i];
}

// ------------------------------------------------------------------ depthwise 3x3, stride 1, pad 1
// input channel c of the conv reads source channel map(c) = (c / gsz) * gstride + goff + c % gsz
// (Attention.pe consumes v.reshape(B, C, H, W), i.e. the v slice of every head of qkv)
struct DwArgs {
    const bf16_t* x; int64_t x_bs, x_ld; int gsz, gstride, goff;
    const float* w;            // fp32 [C][9]
    bf16_t* y;                 // dense (N, H, W, Ct) (fwd) / dx view (bwd)
    int64_t y_bs, y_ld;
    int N, H, W, C;            // C: this launch's channels (a piece of Ct, from c_base; see conv_first_fwd_kernel)
    int c_base, Ct;
};

// one thread per (pixel, 8 channels): 16-B loads, the 8x9 weights in registers, statistics and
// weight-gradient partials in registers, reduced once per thread (xor shuffles over the lanes
// with the same channel group, then LDS) — no per-element atomics.  C/8 divides 256.
__device__ __forceinline__ void unpack8(uint4 u, float* f, bool half) {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        f[2 * e] = half ? h2f(uint16_t(w[e] & 0xffff)) : bf2f(bf16_t(w[e] & 0xffff));
        f[2 * e + 1] = half ? h2f(uint16_t(w[e] >> 16)) : bf2f(bf16_t(w[e] >> 16));
    }
}

__global__ void __launch_bounds__(256) dw3x3_fwd_kernel(DwArgs a, float* st_sum, float* st_sq) {
    __shared__ float red[2][512];
    const int G = a.C >> 3, g = threadIdx.x % G;
    const int c0 = a.c_base + g * 8, sc0 = (c0 / a.gsz) * a.gstride + a.goff + c0 % a.gsz;
    float wr[8][9];
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int t = 0; t < 9; ++t) wr[r][t] = a.w[(c0 + r) * 9 + t];
    float ls[8], lq[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) ls[r] = lq[r] = 0.f;
    const int HW = a.H * a.W, M = a.N * HW;
    const int step = gridDim.x * (256 / G);
    for (int m = (blockIdx.x * 256 + threadIdx.x) / G; m < M; m += step) {
        const int n = m / HW, pix = m - n * HW, h = pix / a.W, wc = pix - h * a.W;
        float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
                const int ih = h - 1 + kh, iw = wc - 1 + kw;
                if (unsigned(ih) < unsigned(a.H) && unsigned(iw) < unsigned(a.W)) {
                    float xv[8];
                    unpack8(*reinterpret_cast<const uint4*>(a.x + n * a.x_bs + int64_t(ih * a.W + iw) * a.x_ld + sc0),
                            xv, true);
#pragma unroll
                    for (int r = 0; r < 8; ++r) s[r] += wr[r][kh * 3 + kw] * xv[r];
                }
            }
        uint4 o;
        o.x = pk2h(s[0], s[1]);
        o.y = pk2h(s[2], s[3]);
        o.z = pk2h(s[4], s[5]);
        o.w = pk2h(s[6], s[7]);
        *reinterpret_cast<uint4*>(a.y + size_t(m) * a.Ct + c0) = o;
#pragma unroll
        for (int r = 0; r < 8; ++r) { ls[r] += s[r]; lq[r] += s[r] * s[r]; }
    }
#pragma unroll
    for (int r = 0; r < 8; ++r)
        for (int o = G; o < 64; o <<= 1) {
            ls[r] += __shfl_xor(ls[r], o, 64);
            lq[r] += __shfl_xor(lq[r], o, 64);
        }
    ordered_wave_add8(red[0], red[1], ls, lq, g, G);
    for (int c = threadIdx.x; c < a.C; c += 256) {
        st_sum[int64_t(blockIdx.x) * a.Ct + a.c_base + c] = red[0][c];
        st_sq[int64_t(blockIdx.x) * a.Ct + a.c_base + c] = red[1][c];
    }
}

// eval-mode depthwise Conv block in one launch (ym_dw3x3_fwd_eval, Attention.pe in eval mode): the same per-(pixel,
// 8 channels) depthwise conv, then the running-statistics BatchNorm (+ SiLU if act) and + the fp16 residual view in
// fp32, one fp16 rounding (ym_bn_apply's arithmetic on the fp32 sum), one 16-B store into the y view (a.y_bs / a.y_ld)
__global__ void __launch_bounds__(256) dw3x3_fwd_eval_kernel(DwArgs a, const float* __restrict__ sc,
                                                             const float* __restrict__ sh, int act,
                                                             const uint16_t* __restrict__ res, int64_t r_bs,
                                                             int64_t r_ld) {
    const int G = a.C >> 3, g = threadIdx.x % G;
    const int c0 = a.c_base + g * 8, sc0 = (c0 / a.gsz) * a.gstride + a.goff + c0 % a.gsz;
    float wr[8][9], s8[8], h8[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
#pragma unroll
        for (int t = 0; t < 9; ++t) wr[r][t] = a.w[(c0 + r) * 9 + t];
        s8[r] = sc[c0 + r];
        h8[r] = sh[c0 + r];
    }
    const int HW = a.H * a.W, M = a.N * HW;
    const int step = gridDim.x * (256 / G);
    for (int m = (blockIdx.x * 256 + threadIdx.x) / G; m < M; m += step) {
        const int n = m / HW, pix = m - n * HW, h = pix / a.W, wc = pix - h * a.W;
        float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
                const int ih = h - 1 + kh, iw = wc - 1 + kw;
                if (unsigned(ih) < unsigned(a.H) && unsigned(iw) < unsigned(a.W)) {
                    float xv[8];
                    unpack8(*reinterpret_cast<const uint4*>(a.x + n * a.x_bs + int64_t(ih * a.W + iw) * a.x_ld + sc0),
                            xv, true);
#pragma unroll
                    for (int r = 0; r < 8; ++r) s[r] += wr[r][kh * 3 + kw] * xv[r];
                }
            }
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const float t = fmaf(s[r], s8[r], h8[r]);
            s[r] = act ? silu_f(t) : t;
        }
        if (res) {                                               // 8-B aligned residual rows
            const uint2* rp = reinterpret_cast<const uint2*>(res + int64_t(n) * r_bs + int64_t(pix) * r_ld + c0);
            const uint2 r0 = rp[0], r1 = rp[1];
            const uint32_t rw[4] = {r0.x, r0.y, r1.x, r1.y};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                s[2 * k] += h2f(uint16_t(rw[k] & 0xffff));
                s[2 * k + 1] += h2f(uint16_t(rw[k] >> 16));
            }
        }
        uint4 o;
        o.x = pk2h(s[0], s[1]);
        o.y = pk2h(s[2], s[3]);
        o.z = pk2h(s[4], s[5]);
        o.w = pk2h(s[6], s[7]);
        *reinterpret_cast<uint4*>(a.y + int64_t(n) * a.y_bs + int64_t(pix) * a.y_ld + c0) = o;
    }
}

// dx (mapped channels, overwrite or accumulate into the view) and dW (+=) from dense dz (N,H,W,C)
__global__ void __launch_bounds__(256) dw3x3_bwd_kernel(DwArgs a, const bf16_t* __restrict__ dz, float* __restrict__ part,
                                                        int accumulate) {
    __shared__ float red[512 * 9];
    const int G = a.C >> 3, g = threadIdx.x % G;
    const int c0 = a.c_base + g * 8, sc0 = (c0 / a.gsz) * a.gstride + a.goff + c0 % a.gsz;
    float wr[8][9], acc[8][9];
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            wr[r][t] = a.w[(c0 + r) * 9 + t];
            acc[r][t] = 0.f;
        }
    const int HW = a.H * a.W, M = a.N * HW;
    const int step = gridDim.x * (256 / G);
    for (int m = (blockIdx.x * 256 + threadIdx.x) / G; m < M; m += step) {
        const int n = m / HW, pix = m - n * HW, h = pix / a.W, wc = pix - h * a.W;
        float d0[8], gx[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        unpack8(*reinterpret_cast<const uint4*>(dz + size_t(m) * a.Ct + c0), d0, false);
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
                // dx[h,w] += dz[h+1-kh, w+1-kw] * w[kh,kw]
                const int oh = h + 1 - kh, ow = wc + 1 - kw;
                if (unsigned(oh) < unsigned(a.H) && unsigned(ow) < unsigned(a.W)) {
                    float dv[8];
                    unpack8(*reinterpret_cast<const uint4*>(dz + size_t(n * HW + oh * a.W + ow) * a.Ct + c0), dv, false);
#pragma unroll
                    for (int r = 0; r < 8; ++r) gx[r] += wr[r][kh * 3 + kw] * dv[r];
                }
                // dW[kh,kw] += dz[h,w] * x[h-1+kh, w-1+kw]
                const int ih = h - 1 + kh, iw = wc - 1 + kw;
                if (unsigned(ih) < unsigned(a.H) && unsigned(iw) < unsigned(a.W)) {
                    float xv[8];
                    unpack8(*reinterpret_cast<const uint4*>(a.x + n * a.x_bs + int64_t(ih * a.W + iw) * a.x_ld + sc0),
                            xv, true);
#pragma unroll
                    for (int r = 0; r < 8; ++r) acc[r][kh * 3 + kw] += d0[r] * xv[r];
                }
            }
        bf16_t* yp = a.y + n * a.y_bs + int64_t(pix) * a.y_ld + sc0;
        if (accumulate) {
            float old[8];
            unpack8(*reinterpret_cast<const uint4*>(yp), old, false);
#pragma unroll
            for (int r = 0; r < 8; ++r) gx[r] += old[r];
        }
        *reinterpret_cast<uint4*>(yp) = make_uint4(pk2bf(gx[0], gx[1]), pk2bf(gx[2], gx[3]), pk2bf(gx[4], gx[5]),
                                                   pk2bf(gx[6], gx[7]));
    }
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int t = 0; t < 9; ++t)
            for (int o = G; o < 64; o <<= 1) acc[r][t] += __shfl_xor(acc[r][t], o, 64);
    ordered_wave_add_taps<9>(red, acc, g, G);
    for (int i = threadIdx.x; i < 9 * a.C; i += 256) part[int64_t(blockIdx.x) * 9 * a.Ct + 9 * a.c_base + i] = red[i];
}

// ------------------------------------------------------------------ weight preparation
// fp32 OIHW master weights -> fp16 [Cout][KH][KW][Cin] (fwd, blockIdx.y 0) and bf16
// [Cin][KH][KW][Cout_t] (dgrad, blockIdx.y 1).  A thread owns DESTINATION elements (coalesced 2-B
// stores; the fp32 gathers hit L2).  A block owns PREP_CHUNK consecutive elements of the concatenated
// index space: one block-uniform binary search finds the chunk's first entry; a chunk inside one entry
// (nearly all of them) runs PREP_PER independent gathers per thread before its stores, a chunk that
// crosses entries walks the table element by element.  (Round 3's one-element-per-thread kernel with a
// binary search per element: 168 us per step on s@640.)
constexpr int PREP_PER = 16, PREP_CHUNK = 256 * PREP_PER;
// the forward-only launch (ym_prep_weights_fwd): smaller chunks — more workgroups in flight; round 5, s@640's table:
// 16 / 8 elements per thread 32.8 / 27.1 us (the two-pass launch keeps 16: 8 measured 66.5 -> 72.4 us)
#ifndef YM_PREP_PER_FWD
#define YM_PREP_PER_FWD 8
#endif
constexpr int PREP_PER_FWD = YM_PREP_PER_FWD;
constexpr int PREP_LDS = 8192;                               // floats of the transposed pass's tile

__device__ __forceinline__ void prep_one(const ym_wprep_entry& t, int j, int pass) {
    const int T = t.kh * t.kw;
    if (pass == 0) {
        if (!t.dst_fwd) return;
        const int ci = j % t.cin, r = j / t.cin;
        const int tap = r % T, co = r / T;
        t.dst_fwd[j] = f2h(t.src[(int64_t(co) * t.cin + ci) * T + tap]);
    } else {
        if (!t.dst_t) return;
        const int co = j % t.cout, r = j / t.cout;
        const int tap = r % T, ci = r / T;
        t.dst_t[(int64_t(ci) * T + tap) * t.cout_t + co] = f2bf(t.src[(int64_t(co) * t.cin + ci) * T + tap]);
    }
}

// FWD_ONLY: the forward copies alone (ym_prep_weights_fwd: tables without transposed copies, e.g. an eval plan's) —
// no LDS tile, so twice the resident workgroups per CU, and no second grid row of workgroups that find nothing to do
template <bool FWD_ONLY>
__global__ void __launch_bounds__(256) prep_weights_kernel(const ym_wprep_entry* __restrict__ tab, int n_entries,
                                                           int64_t total) {
    constexpr int PER = FWD_ONLY ? PREP_PER_FWD : PREP_PER, CHUNK = 256 * PER;
    const int64_t c0 = int64_t(blockIdx.x) * CHUNK, c1 = min(c0 + CHUNK, total);
    const int pass = FWD_ONLY ? 0 : int(blockIdx.y);
    // the chunk's first entry (the last with elem_offset <= c0; offsets ascending): a two-level 64-ary search, each level
    // one load per lane + a ballot (every wave repeats it: no LDS, no barrier) — 2 memory round trips for <= 4096
    // entries where a binary search chains ~log2(entries) dependent loads (~7 x ~0.8 us per workgroup on s@640, most
    // of this launch's time: 5.5 k short workgroups); larger tables continue with the binary search
    const int lane = threadIdx.x & 63;
    const int s1 = (n_entries + 63) >> 6;
    int lo = 0, hi = n_entries - 1;
    {
        const int i1 = min(lane * s1, n_entries - 1);
        const uint64_t m1 = __ballot(lane * s1 < n_entries && tab[i1].elem_offset <= c0);
        lo = (__popcll(m1) - 1) * s1;                            // lane 0 (offset 0) always qualifies
        hi = min(lo + s1 - 1, n_entries - 1);
        if (s1 > 1 && s1 <= 64) {
            const int i2 = min(lo + lane, hi);
            const uint64_t m2 = __ballot(lane < s1 && lo + lane <= hi && tab[i2].elem_offset <= c0);
            lo += __popcll(m2) - 1;
            hi = lo;
        }
    }
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (tab[mid].elem_offset <= c0) lo = mid;
        else hi = mid - 1;
    }
    const ym_wprep_entry t = tab[lo];
    const int64_t t_end = lo + 1 < n_entries ? tab[lo + 1].elem_offset : total;
    if (c1 <= t_end) {
        uint16_t* dst = pass == 0 ? t.dst_fwd : t.dst_t;
        if (!dst) return;
        const int T = t.kh * t.kw;
        const int jb = int(c0 - t.elem_offset) + threadIdx.x, nj = int(c1 - t.elem_offset);
        // data-gradient copy: the chunk is rows fs..fe of the [F = cin*T][cout] space; their sources are the
        // column run src[co][fs..fe] of EVERY co — staged through LDS (runs of contiguous floats in, whole
        // destination rows out) instead of one lane per row-strided 4-B gather (round 4: 160 -> 74 us per step
        // with the gather, the transposed pass the larger part of it)
        const int F = t.cin * T;
        const int j0 = int(c0 - t.elem_offset);
        const int fs = j0 / t.cout, fe = (nj - 1) / t.cout, nf = fe - fs + 1;
        const int ld = nf | 1;                                   // odd row stride: conflict-free column reads
        if constexpr (!FWD_ONLY) {
            if (pass == 1 && t.cout * ld <= PREP_LDS) {
                __shared__ float tile[PREP_LDS];
                for (int idx = threadIdx.x; idx < t.cout * nf; idx += 256) {
                    const int co = idx / nf, fi = idx - co * nf;
                    tile[co * ld + fi] = t.src[int64_t(co) * F + fs + fi];
                }
                __syncthreads();
                for (int j = jb; j < nj; j += 256) {
                    const int f = j / t.cout, co = j - f * t.cout;
                    dst[int64_t(f) * t.cout_t + co] = f2bf(tile[co * ld + (f - fs)]);
                }
                return;
            }
        }
        float v[PER];
        int64_t di[PER];
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int j = min(jb + k * 256, nj - 1);
            int64_t si;
            if (pass == 0) {
                const int ci = j % t.cin, r = j / t.cin;
                const int tap = r % T, co = r / T;
                si = (int64_t(co) * t.cin + ci) * T + tap;
                di[k] = j;
            } else {
                const int co = j % t.cout, r = j / t.cout;
                const int tap = r % T, ci = r / T;
                si = (int64_t(co) * t.cin + ci) * T + tap;
                di[k] = (int64_t(ci) * T + tap) * t.cout_t + co;
            }
            v[k] = t.src[si];
        }
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            if (jb + k * 256 >= nj) break;
            dst[di[k]] = pass == 0 ? f2h(v[k]) : f2bf(v[k]);
        }
        return;
    }
    // the chunk crosses entries: walk the table per element (entries are sorted by offset)
    int e = lo;
    for (int64_t i = c0 + threadIdx.x; i < c1; i += 256) {
        while (e + 1 < n_entries && tab[e + 1].elem_offset <= i) ++e;
        prep_one(tab[e], int(i - tab[e].elem_offset), pass);
    }
}

// grid x: a multiple of 8 (the kernel groups m-tiles per XCD); with BatchNorm statistics the
// partials are one row per grid-x block, so the grid is bounded and blocks loop over tiles
// grid-x bound of the forward with BN statistics (rows of its partials)
constexpr int FWD_STAT_BLOCKS = 1024;

static int grid_x(int mtiles, int ntiles, bool stats, int max_blocks) {
    int gx = (mtiles + 7) & ~7;
    if (stats) gx = std::min(gx, std::max(8, (max_blocks / ntiles) & ~7));
    return gx;
}

// the kernel's buffer offsets are 32-bit, relative to the first image of a tile
static bool offsets_fit(int64_t bs, int64_t class_pixels) {
    const int64_t images = 256 / std::max<int64_t>(class_pixels, 1) + 2;
    return bs * 2 * images < (int64_t(1) << 31);
}

// the eval K-split's second launch (ym_conv_fwd_eval with ks > 1): y = act(sum_z part[z] * scale + shift) (+ res),
// the register epilogue's arithmetic (EvalEpi) on the slices' fp32 sum, summed in slice order (deterministic);
// one thread per (pixel, 8 channels), C % 8 == 0, M * C / 8 < 2^31 and M < 2^32 (host checks)
__global__ void __launch_bounds__(256) eval_fold_kernel(const float* __restrict__ part, int ks, int64_t M, int C,
                                                        uint32_t OHW, const float* __restrict__ sc,
                                                        const float* __restrict__ sh, int act,
                                                        const uint16_t* __restrict__ res, int64_t r_bs, int64_t r_ld,
                                                        uint16_t* __restrict__ y, int64_t y_bs, int64_t y_ld) {
    const int G = C >> 3;
    const int64_t idx = int64_t(blockIdx.x) * 256 + threadIdx.x;
    if (idx >= M * G) return;
    const int64_t m = idx / G;
    const int c0 = int(idx - m * G) * 8;
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int z = 0; z < ks; ++z) {
        const float4* p = reinterpret_cast<const float4*>(part + (int64_t(z) * M + m) * C + c0);
        const float4 a = p[0], b = p[1];
        v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
        v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
    }
    const float4 s0 = *reinterpret_cast<const float4*>(sc + c0), s1 = *reinterpret_cast<const float4*>(sc + c0 + 4);
    const float4 h0 = *reinterpret_cast<const float4*>(sh + c0), h1 = *reinterpret_cast<const float4*>(sh + c0 + 4);
    const float s[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    const float h[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const float t = fmaf(v[k], s[k], h[k]);
        v[k] = act ? silu_f(t) : t;
    }
    const uint32_t n = uint32_t(m) / OHW, pix = uint32_t(m) - n * OHW;
    if (res) {                                                   // 8-B aligned residual rows (r_ld % 4 == 0)
        const uint2* rp = reinterpret_cast<const uint2*>(res + int64_t(n) * r_bs + int64_t(pix) * r_ld + c0);
        const uint2 r0 = rp[0], r1 = rp[1];
        const uint32_t rw[4] = {r0.x, r0.y, r1.x, r1.y};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            v[2 * k] += h2f(uint16_t(rw[k] & 0xffff));
            v[2 * k + 1] += h2f(uint16_t(rw[k] >> 16));
        }
    }
    uint4 o;
    o.x = pk2h(v[0], v[1]);
    o.y = pk2h(v[2], v[3]);
    o.z = pk2h(v[4], v[5]);
    o.w = pk2h(v[6], v[7]);
    *reinterpret_cast<uint4*>(y + int64_t(n) * y_bs + int64_t(pix) * y_ld + c0) = o;
}

template <int BM, int BN, int WM, int WN, int KB, int NS, int MODE, bool EV = false>
int launch_gemm(const GemmArgs& a0, int max_blocks, hipStream_t st, const EvalArgs& e = EvalArgs{}) {
    GemmArgs a = a0;
    const int os = a.ostep;
    const int64_t Mc = int64_t(a.N) * ((a.OH + os - 1) / os) * ((a.OW + os - 1) / os);   // largest class
    a.mtiles = int((Mc + BM - 1) / BM);
    int ntiles = (a.Nout + BN - 1) / BN;
    int gx = grid_x(a.mtiles, ntiles, a.st_sum != nullptr, max_blocks);
    // channel tiles of one m-tile sequence interleaved into grid x (dispatched together)
    a.ntl = ntiles > 1 ? ntiles : 0;
    const int gz = os == 2 ? 4 : (EV && e.ks > 1 ? e.ks : 1);   // parity classes / eval K slices
    const dim3 grid(a.ntl ? gx * ntiles : gx, a.ntl ? 1 : ntiles, gz), block(WM * WN * 64);
    hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, WM, WN, KB, NS, MODE, EV>), grid, block, 0, st, a, e);
    return gx;
}

}  // namespace
}  // namespace ym

using namespace ym;

struct Tile {
    int bm, bn;
};

// 128-pixel tiles with the widest channel tile that still gives >= 1.5 workgroups per CU (small late
// layers: 20x20 maps).  The large layers' 256 x 128 tiles live in conv_pipe.hip (persistent,
// 3-stage LDS-DMA ring): at this kernel's pipeline depth they measured 9 % slower in sum than
// 128 x 128 (tools/layer_bench.py, s@640 bs64), so the former opt-in here is gone.
static Tile pick_tile(int64_t Mc, int classes, int nout) {
    const int64_t blocks_per_ntile = ((Mc + 127) / 128) * classes;
    int bn = nout >= 128 ? 128 : (nout >= 64 ? 64 : 32);
    while (bn > 32 && blocks_per_ntile * ((nout + bn - 1) / bn) < 384) bn >>= 1;
    return {128, bn};
}

template <int KB, int NS, int MODE>
static int launch_tile_k(const GemmArgs& a, Tile t, int max_blocks, hipStream_t st) {
    if (t.bn == 128) return launch_gemm<128, 128, 2, 2, KB, NS, MODE>(a, max_blocks, st);
    if (t.bn == 64) return launch_gemm<128, 64, 2, 2, KB, NS, MODE>(a, max_blocks, st);
    // 32-channel tiles need 64-deep stages (one 8-row DMA instruction per wave)
    return launch_gemm<128, 32, 2, 2, 64, (KB == 64 ? NS : 2), MODE>(a, max_blocks, st);
}

// K-stage depth x ring depth, measured per layer (tools/layer_bench.py): 64-channel tiles prefer 32-deep stages
template <int MODE>
static int launch_tile(const GemmArgs& a, Tile t, int max_blocks, hipStream_t st) {
    return t.bm == 128 && t.bn == 64 ? launch_tile_k<32, 3, MODE>(a, t, max_blocks, st)
                                     : launch_tile_k<64, 2, MODE>(a, t, max_blocks, st);
}

// nsel: the batch the tile choice is made for (select_n: the real batch unless a parity test pins the
// selection of a larger one)
static int pick_and_launch(GemmArgs a, int mode, int max_blocks, int64_t nsel, hipStream_t st) {
    const int os = a.ostep;
    const int64_t Mc = nsel * ((a.OH + os - 1) / os) * ((a.OW + os - 1) / os);
    const Tile t = pick_tile(Mc, os == 2 ? 4 : 1, a.Nout);
    return mode == MODE_FWD ? launch_tile<MODE_FWD>(a, t, max_blocks, st) : launch_tile<MODE_DGRAD>(a, t, max_blocks, st);
}

// rows of the BN statistics partials of the 2-stage implicit GEMM's forward: M output pixels, the tile
// chosen for Msel of them
static int gemm_stat_rows(int64_t M, int64_t Msel, int Cout) {
    const Tile t = pick_tile(Msel, 1, Cout);
    const int mtiles = int((M + t.bm - 1) / t.bm);
    return grid_x(mtiles, (Cout + t.bn - 1) / t.bn, true, FWD_STAT_BLOCKS);
}

extern "C" int ym_conv_stat_blocks(int64_t M, int Cout) {
    // grid-x of the 2-stage implicit GEMM's statistics partials (the generic kernel only; the row count of
    // any conv forward is ym_conv_fwd_stat_rows)
    return gemm_stat_rows(M, M, Cout);
}

extern "C" int ym_conv_set_select_batch(int n) {
    // kernel selection as if the batch held n images (0: the real batch); returns the previous setting
    return g_select_n.set(n > 0 ? n : 0);
}

extern "C" int ym_conv_set_halo(int mode) {
    // selection policy of the halo-staged 3x3 kernel: -1 default, 0 never, 1 wherever it applies,
    // 2 where it measured faster in the step (the default), 3 the wider per-layer rule; returns the
    // previous setting
    return g_halo_force.set(mode < -1 || mode > 3 ? -1 : mode);
}

extern "C" int ym_conv_set_pipe(int mode) {
    // selection policy of the pipelined implicit GEMM: -1 default, 0 never, 1 layers of >= 1024
    // tiles (default), 2 >= 256 tiles; returns the previous setting
    return g_pipe_force.set(mode < -1 || mode > 3 ? -1 : mode);
}

extern "C" int ym_conv_set_direct(int mode) {
    // selection policy of the direct register-weight kernel: -1 default, 0 never, 1 maps of
    // >= 1 M output pixels (default), 2 any size, 3 >= 200 k output pixels; returns the previous setting
    return g_direct_force.set(mode < -1 || mode > 3 ? -1 : mode);
}

extern "C" int ym_conv_set_hpipe(int mode) {
    // selection policy of the halo-staged pipelined 3x3 kernel: -1 default, 0 never, 1 eligible layers of
    // >= 512 tiles (default), 2 every eligible layer; returns the previous setting
    return g_hpipe_force.set(mode < -1 || mode > 2 ? -1 : mode);
}

extern "C" int ym_conv_algo(const ym_conv_desc* d, int dgrad) {
    // 4: halo-staged pipelined 3x3 kernel (conv_hpipe.hip), 3: direct register-weight kernel
    // (conv_direct.hip), 2: persistent pipelined implicit GEMM (conv_pipe.hip), 1: halo-staged 3x3 kernel
    // (conv_halo.hip), 0: 2-stage implicit GEMM
    if (d && direct_plan(d, dgrad ? 1 : 0).ok) return 3;
    if (d && hpipe_plan(d, dgrad ? 1 : 0).ok) return 4;
    if (d && pipe_plan(d, dgrad ? 1 : 0).ok) return 2;
    return d && halo_plan(d, dgrad ? 1 : 0).ok ? 1 : 0;
}

extern "C" int ym_conv_kernel(const ym_conv_desc* d, int dir, char* name, int name_len) {
    // the kernel instance a bias-free forward (dir 0), data gradient (1) or weight gradient (2) of this conv
    // runs: an id (algo x 1000 + template instance; weight gradients 10000 + ...) and, when name is given,
    // its name, e.g. "direct v3", "pipe 256x128", "wgrad3 s2 64x64 8x8 deep"
    char buf[96];
    int id = -1;
    if (!d || dir < 0 || dir > 2) {
        snprintf(buf, sizeof buf, "invalid");
    } else if (dir == 2) {
        id = wgrad_kernel(d, buf, sizeof buf);
    } else {
        const DirectPlan dp = direct_plan(d, dir);
        const HPipePlan hq = hpipe_plan(d, dir);
        const PipePlan pp = pipe_plan(d, dir);
        const HaloPlan hp = halo_plan(d, dir);
        if (dp.ok) {
            id = 3000 + dp.variant;
            snprintf(buf, sizeof buf, "direct v%d", dp.variant);
        } else if (hq.ok) {
            id = 4000 + hq.cfg;
            snprintf(buf, sizeof buf, "hpipe %s", hq.cfg == 0 ? "16x16px x 128" : hq.cfg == 1 ? "16x16px x 64" : "16x16px x 64 wres");
        } else if (pp.ok) {
            id = 2000 + pp.cfg;
            static const char* const pipe_names[] = {"256x128", "256x64", "256x128 8w"};
            snprintf(buf, sizeof buf, "pipe %s", pipe_names[pp.cfg]);
        } else if (hp.ok) {
            id = 1000 + 100 * hp.cfg + std::min(hp.TW, 99);
            snprintf(buf, sizeof buf, "halo %s %dx%d", hp.cfg == 0 ? "C8" : "C4", hp.TH, hp.TW);
        } else {
            const int os = dir ? d->stride : 1;
            const int OH = dir ? d->h : d->oh, OW = dir ? d->w : d->ow, nout = dir ? d->cin : d->cout;
            const Tile t = pick_tile(select_n(d) * ((OH + os - 1) / os) * ((OW + os - 1) / os), os == 2 ? 4 : 1, nout);
            id = t.bn;
            snprintf(buf, sizeof buf, "gemm %dx%d%s", t.bm, t.bn, os == 2 ? " 4-class" : "");
        }
    }
    if (name && name_len > 0) snprintf(name, size_t(name_len), "%s", buf);
    return id;
}

extern "C" int ym_conv_fwd_stat_rows(const ym_conv_desc* d) {
    // rows of the BN statistics partials ym_conv_fwd writes for this conv (halo or implicit-GEMM grid)
    if (!d) return 0;
    const DirectPlan dp = direct_plan(d, 0);
    if (dp.ok) return dp.grid;
    const HPipePlan hq = hpipe_plan(d, 0);
    if (hq.ok) return hq.rows;
    const PipePlan pp = pipe_plan(d, 0);
    if (pp.ok) return pp.rows;
    const HaloPlan hp = halo_plan(d, 0);
    if (hp.ok) return hp.gx;
    return gemm_stat_rows(int64_t(d->n) * d->oh * d->ow, select_n(d) * d->oh * d->ow, d->cout);
}

// ym_conv_fwd_bn's fold policy (ym_conv_set_fold): -1 default (on), 0 off, 1 on
static Policy g_fold_mode{-1};

// fold: the BatchNorm finalize as the pipelined kernel's tail (ym_conv_fwd_bn), null elsewhere
static int conv_fwd_impl(const ym_conv_desc* d, const uint16_t* x, const uint16_t* w, void* y, const float* bias,
                         float* stat_sum, float* stat_sq, void* stream, const ym_bn_fold* fold = nullptr) {
    YM_CHECK_ARG(d && x && w && y, "ym_conv_fwd: null argument");
    YM_CHECK_ARG(d->cin % 8 == 0, "ym_conv_fwd: Cin %% 8 != 0 (Cin=%d)", d->cin);
    YM_CHECK_ARG(d->k >= 1 && d->k <= 3, "ym_conv_fwd: kernel size %d unsupported (1..3)", d->k);
    YM_CHECK_ARG(d->x_ld % 8 == 0 && d->x_bs % 8 == 0, "ym_conv_fwd: input view not 16-byte aligned");
    YM_CHECK_ARG(d->out_f32 == 1 || (d->y_ld % 4 == 0 && d->y_bs % 4 == 0), "ym_conv_fwd: output view not 8-byte aligned");
    YM_CHECK_ARG((stat_sum == nullptr) == (stat_sq == nullptr), "ym_conv_fwd: stats pointers");
    // the statistics row count (ym_conv_fwd_stat_rows) describes the bias-free forward of a Conv block
    YM_CHECK_ARG(!(bias && stat_sum), "ym_conv_fwd: BN statistics of a conv with bias are not supported");
    YM_CHECK_ARG(!(d->accumulate && d->out_f32 == 2), "ym_conv_fwd: accumulate into an fp16 output is not supported");
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
    a.N = d->n;
    a.ostep = 1;
    // fp16 z: the register-transposed epilogue with 16-B row stores (round 4; fp32 / bias outputs: fragment stores)
    a.ep_lds = d->out_f32 == 2 && !bias && d->y_ld % 8 == 0 && d->y_bs % 8 == 0 &&
               int64_t(d->n) * d->y_bs * 2 < (int64_t(1) << 31) && reinterpret_cast<uintptr_t>(y) % 16 == 0;
    if (a.M == 0) return YM_OK;
    // the direct and halo-pipelined kernels have no bias term: a conv with bias takes the kernels below
    const DirectPlan dp = bias ? DirectPlan{} : direct_plan(d, 0, stat_sum == nullptr);
    if (dp.ok) {
        direct_launch(dp, d, 0, x, w, y, stat_sum, stat_sq, as_stream(stream));
        YM_LAUNCH_CHECK("ym_conv_fwd (direct)");
        return YM_OK;
    }
    YM_CHECK_ARG(a.M < (int64_t(1) << 31), "ym_conv_fwd: too many pixels");
    const HPipePlan hq = bias ? HPipePlan{} : hpipe_plan(d, 0);
    if (hq.ok) {
        hpipe_launch(hq, d, 0, x, w, y, stat_sum, stat_sq, as_stream(stream));
        YM_LAUNCH_CHECK("ym_conv_fwd (hpipe)");
        return YM_OK;
    }
    YM_CHECK_ARG(offsets_fit(d->x_bs, int64_t(d->oh) * d->ow), "ym_conv_fwd: input image stride too large");
    const PipePlan pp = pipe_plan(d, 0);
    if (pp.ok) {
        pipe_launch(pp, d, 0, x, w, y, bias, stat_sum, stat_sq, as_stream(stream), fold);
        YM_LAUNCH_CHECK("ym_conv_fwd (pipe)");
        return YM_OK;
    }
    const HaloPlan hp = halo_plan(d, 0);
    if (hp.ok) {
        halo_launch(hp, d, 0, x, w, y, bias, stat_sum, stat_sq, as_stream(stream), fold);
        YM_LAUNCH_CHECK("ym_conv_fwd (halo)");
        return YM_OK;
    }
    if (stat_sum) a.fold = bn_fold_args(fold);
    pick_and_launch(a, MODE_FWD, FWD_STAT_BLOCKS, select_n(d), as_stream(stream));
    YM_LAUNCH_CHECK("ym_conv_fwd");
    return YM_OK;
}

extern "C" int ym_conv_fwd(const ym_conv_desc* d, const uint16_t* x, const uint16_t* w, void* y, const float* bias,
                           float* stat_sum, float* stat_sq, void* stream) {
    return conv_fwd_impl(d, x, w, y, bias, stat_sum, stat_sq, stream);
}

extern "C" int ym_conv_fwd_bn_fused(const ym_conv_desc* d) {
    // the pipelined, halo-staged and 2-stage GEMM forwards (bias-free, with statistics) fold the finalize into
    // their tail; the direct and halo-pipelined forwards run conv + ym_bn_finalize
    if (!d || g_fold_mode == 0) return 0;
    if (direct_plan(d, 0).ok || hpipe_plan(d, 0).ok) return 0;
    return 1;
}

extern "C" int ym_conv_fwd_bn(const ym_conv_desc* d, const uint16_t* x, const uint16_t* w, void* y, float* stat_sum,
                              float* stat_sq, const ym_bn_fold* bn, void* stream) {
    YM_CHECK_ARG(d && bn && stat_sum && stat_sq, "ym_conv_fwd_bn: null argument");
    YM_CHECK_ARG(bn->gamma && bn->beta && bn->scale && bn->shift && bn->mean && bn->rstd && bn->workspace,
                 "ym_conv_fwd_bn: null BatchNorm argument");
    YM_CHECK_ARG(bn->count > 0, "ym_conv_fwd_bn: count must be > 0");
    YM_CHECK_ARG(d->cout <= 2048, "ym_conv_fwd_bn: Cout=%d > 2048", d->cout);
    if (ym_conv_fwd_bn_fused(d)) return conv_fwd_impl(d, x, w, y, nullptr, stat_sum, stat_sq, stream, bn);
    const int r = conv_fwd_impl(d, x, w, y, nullptr, stat_sum, stat_sq, stream);
    if (r != YM_OK) return r;
    return ym_bn_finalize(stat_sum, stat_sq, ym_conv_fwd_stat_rows(d), d->cout, bn->count, bn->gamma, bn->beta,
                          bn->running_mean, bn->running_var, bn->num_batches_tracked, bn->momentum, bn->eps,
                          bn->scale, bn->shift, bn->mean, bn->rstd, bn->workspace, stream);
}

// ------------------------------------------------------------------ eval-mode Conv block in one launch
// (inference: conv -> BatchNorm with the running statistics -> SiLU -> + residual, yolo11_modules.py:21-33 in eval mode):
// where the forward runs the halo-staged kernel or the 2-stage implicit GEMM, the BatchNorm / SiLU / residual are
// applied by their register epilogue (conv_epi.h EvalEpi) and the launch writes the activation view; the fp16 z and
// ym_bn_apply's launch go (a bs-1 s@640 eval forward is ~75 conv blocks, each ~4 us of apply launch).
// The eval GEMM tile is 128x64 (the register epilogue needs >= 32 channels per wave; the 128x128 instance spills with
// it); the halo kernel's eval instance is its 4-wave C4 tile (C8 spills).
// the eval GEMM's K stage x ring (ym_conv_set_eval_cfg): 0: 32-deep stages, 3-stage ring (the training 128x64 tile's),
// 1: 64-deep x 3, 2: 64-deep x 4 — at bs 1 a launch covers a few tiles and walks its whole K serially, so deeper
// stages halve its DMA round trips (128-deep x 3, one workgroup per CU, measured slower: profiles/r05/eval_split_ab.txt)
static Policy g_eval_cfg{1};
static Policy g_eval_narrow{1};

extern "C" int ym_conv_set_eval_narrow(int on) {
    // eval GEMM outputs of <= 32 channels on the 128 x 32 tile (1, default; <0 restores it) or the 128 x 64 (0);
    // returns the previous setting
    return g_eval_narrow.set(on < 0 ? 1 : (on ? 1 : 0));
}

extern "C" int ym_conv_set_eval_cfg(int cfg) {
    // the eval GEMM's stage / ring configuration (0..2, -1 default 1); returns the previous setting
    return g_eval_cfg.set(cfg < 0 || cfg > 2 ? 1 : cfg);
}

// K-split on small grids (ym_conv_set_eval_split): a bs-1 late layer is a few dozen 128x64 tiles, each walking a K of
// up to 72 stages serially (~0.6 us a stage); with ks > 1 the launch's blockIdx.z walks K slice z of ks into an fp32
// partial slab (EvalArgs.part) and eval_fold_kernel applies BatchNorm / SiLU / residual to the slices' sum — one
// extra launch (~4 us) for a K walk ks times shorter.  Split where the layer has <= g_eval_split tiles and >= 12 K
// stages: ks = min(stages / 4, 256 / tiles, 16) (>= 4 stages a slice, <= ~one workgroup per CU).
static Policy g_eval_split{64}, g_eval_split_nk{12}, g_eval_gemm_tiles{0};

extern "C" int ym_conv_set_eval_split(int max_tiles) {
    // the eval K-split's tile threshold (0: never split, -1: default 64); returns the previous setting
    return g_eval_split.set(max_tiles < 0 ? 64 : max_tiles);
}

extern "C" int ym_conv_set_eval_split_nk(int min_stages) {
    // the eval K-split's K-stage threshold (-1: default 12); returns the previous setting
    return g_eval_split_nk.set(min_stages < 0 ? 12 : min_stages);
}

extern "C" int ym_conv_set_eval_gemm_tiles(int max_tiles) {
    // eval convs of <= max_tiles 128x64 tiles take the 2-stage GEMM where the halo kernel would run (0: never,
    // -1: default 0); returns the previous setting
    return g_eval_gemm_tiles.set(max_tiles < 0 ? 0 : max_tiles);
}

static int64_t eval_tiles(const ym_conv_desc* d) {
    const int64_t M = int64_t(d->n) * d->oh * d->ow;
    return ((M + 127) / 128) * ((d->cout + 63) / 64);
}

static bool eval_gemm_fits(const ym_conv_desc* d) {
    const int64_t M = int64_t(d->n) * d->oh * d->ow;
    return M < (int64_t(1) << 31) && offsets_fit(d->x_bs, int64_t(d->oh) * d->ow);
}

// K slices of d's eval forward (1: no split); d passed ym_conv_fwd_eval_ok's layout checks
static int eval_ks(const ym_conv_desc* d) {
    if (g_eval_split == 0 || !eval_gemm_fits(d)) return 1;
    const int64_t M = int64_t(d->n) * d->oh * d->ow;
    const int64_t tiles = ((M + 127) / 128) * ((d->cout + 63) / 64);
    // K stages of the instance ym_conv_fwd_eval launches: the narrow (<= 32-channel) 128 x 32 tile always runs
    // 64-deep stages, the 128 x 64 one 32-deep under eval cfg 0
    const int KB = (g_eval_narrow && d->cout <= 32) || g_eval_cfg != 0 ? 64 : 32;
    const int nk = d->k * d->k * ((d->cin + KB - 1) / KB);
    if (tiles > g_eval_split || nk < g_eval_split_nk) return 1;
    const int64_t ks = std::min<int64_t>(std::min<int64_t>(nk / 4, std::max<int64_t>(1, 256 / tiles)), 16);
    return ks >= 2 && M * (d->cout / 8) < (int64_t(1) << 31) ? int(ks) : 1;
}

// the pipelined forward's eval instance for layers of >= 256 tiles (ym_conv_set_eval_pipe; 0: those layers run
// ym_conv_fwd + ym_bn_apply)
static Policy g_eval_pipe{1};

extern "C" int ym_conv_set_eval_pipe(int on) {
    // the pipelined forward's eval instance on (1, default; -1 restores it) or off (0); returns the previous setting
    return g_eval_pipe.set(on < 0 ? 1 : (on ? 1 : 0));
}

// layers whose training kernel has no eval instance, routed to an eval instance anyway (ym_conv_set_eval_route):
// bit 0 the halo kernel's 8-wave tile (C8: its eval instance spills) -> the 2-stage GEMM's; bit 1 the halo-pipelined
// 3x3 kernel -> the halo C4 / GEMM eval instances
static Policy g_eval_route{0};

extern "C" int ym_conv_set_eval_route(int mask) {
    // see g_eval_route (-1: default 0); returns the previous setting
    return g_eval_route.set(mask < 0 ? 0 : (mask & 3));
}

static bool eval_layout_ok(const ym_conv_desc* d) {
    if (!d || d->cin % 8 || d->cout % 8 || d->k < 1 || d->k > 3 || d->out_f32 != 2 || d->accumulate) return false;
    if (d->x_ld % 8 || d->x_bs % 8 || d->y_ld % 8 || d->y_bs % 8) return false;
    if (int64_t(d->n) * d->y_bs * 2 >= (int64_t(1) << 31)) return false;
    if (direct_plan(d, 0, true).ok) return false;                    // no eval epilogue there
    if (hpipe_plan(d, 0).ok && !((g_eval_route & 2) && eval_gemm_fits(d))) return false;
    const PipePlan pp = pipe_plan(d, 0);
    return !pp.ok || (g_eval_pipe && pipe_eval_ok(pp, d));          // the pipelined forward's eval instance
}

// the eval forward runs the halo kernel's eval instance (not the GEMM) for d
static bool eval_halo(const ym_conv_desc* d, const HaloPlan& hp) {
    return hp.ok && hp.cfg == 1 && !(eval_tiles(d) <= g_eval_gemm_tiles && eval_gemm_fits(d));
}

extern "C" int ym_conv_fwd_eval_ok(const ym_conv_desc* d) {
    if (!eval_layout_ok(d)) return 0;
    if (pipe_plan(d, 0).ok) return 1;
    if (eval_ks(d) > 1 || (eval_tiles(d) <= g_eval_gemm_tiles && eval_gemm_fits(d))) return 1;
    const HaloPlan hp = halo_plan(d, 0);
    if (hp.ok) return hp.cfg == 1 ? 1 : ((g_eval_route & 1) && eval_gemm_fits(d) ? 1 : 0);
    return eval_gemm_fits(d) ? 1 : 0;
}

extern "C" size_t ym_conv_fwd_eval_workspace_size(const ym_conv_desc* d) {
    // bytes of the fp32 slice partials ym_conv_fwd_eval's K-split takes for d (0: one launch, no workspace)
    if (!eval_layout_ok(d)) return 0;
    const int ks = eval_ks(d);
    return ks > 1 ? size_t(ks) * size_t(int64_t(d->n) * d->oh * d->ow) * size_t(d->cout) * sizeof(float) : 0;
}

extern "C" int ym_conv_fwd_eval(const ym_conv_desc* d, const uint16_t* x, const uint16_t* w, const float* scale,
                                const float* shift, int act, const uint16_t* res, int64_t r_bs, int64_t r_ld,
                                uint16_t* y, void* workspace, size_t workspace_bytes, void* stream) {
    YM_CHECK_ARG(d && x && w && scale && shift && y, "ym_conv_fwd_eval: null argument");
    YM_CHECK_ARG(ym_conv_fwd_eval_ok(d), "ym_conv_fwd_eval: not an eval-epilogue case (ym_conv_fwd_eval_ok = 0)");
    YM_CHECK_ARG(reinterpret_cast<uintptr_t>(y) % 16 == 0 && reinterpret_cast<uintptr_t>(res) % 8 == 0 &&
                 reinterpret_cast<uintptr_t>(scale) % 16 == 0 && reinterpret_cast<uintptr_t>(shift) % 16 == 0,
                 "ym_conv_fwd_eval: misaligned output / residual / coefficient pointer");
    YM_CHECK_ARG(!res || (r_ld % 4 == 0 && r_bs % 4 == 0 && r_ld >= d->cout && r_bs >= int64_t(d->oh) * d->ow * r_ld &&
                          int64_t(d->n) * r_bs * 2 < (int64_t(1) << 31)),
                 "ym_conv_fwd_eval: residual view strides");
    if (int64_t(d->n) * d->oh * d->ow == 0) return YM_OK;
    // the K-split where it applies and the caller gave its workspace (null / too small: one launch)
    const size_t need = ym_conv_fwd_eval_workspace_size(d);
    const int ks = need && workspace && workspace_bytes >= need && reinterpret_cast<uintptr_t>(workspace) % 16 == 0
                       ? eval_ks(d) : 1;
    EvalArgs ev{scale, shift, act, res, int64_t(d->n) * r_bs * 2, r_bs, r_ld};
    if (ks > 1) {
        ev.ks = ks;
        ev.part = static_cast<float*>(workspace);
    }
    hipStream_t st = as_stream(stream);
    const PipePlan pp = pipe_plan(d, 0);
    if (pp.ok) {                                  // large maps (>= 256 tiles): the pipelined forward's eval instance
        YM_CHECK_ARG(pipe_launch_eval(pp, d, x, w, y, ev, st) == 0, "ym_conv_fwd_eval: pipelined launch refused");
        YM_LAUNCH_CHECK("ym_conv_fwd_eval (pipe)");
        return YM_OK;
    }
    const HaloPlan hp = halo_plan(d, 0);
    if (ks == 1 && eval_halo(d, hp)) {
        YM_CHECK_ARG(halo_launch(hp, d, 0, x, w, y, nullptr, nullptr, nullptr, st, nullptr, &ev) == 0,
                     "ym_conv_fwd_eval: halo launch refused");
        YM_LAUNCH_CHECK("ym_conv_fwd_eval (halo)");
        return YM_OK;
    }
    GemmArgs a{};
    a.x = x; a.x_bs = d->x_bs; a.x_ld = d->x_ld;
    a.w = w;
    a.y = y; a.y_bs = d->y_bs; a.y_ld = d->y_ld;
    a.GH = d->h; a.GW = d->w; a.Kin = d->cin;
    a.OH = d->oh; a.OW = d->ow; a.Nout = d->cout;
    a.KH = d->k; a.KW = d->k; a.stride = d->stride; a.pad = d->pad;
    a.M = int64_t(d->n) * d->oh * d->ow;
    a.out_f32 = 2;
    a.N = d->n;
    a.ostep = 1;
    a.ep_lds = 1;
    // outputs of <= 32 channels: the 128 x 32 tile on 4 waves along the pixels (1 x 4: 32 channels per wave, the
    // register epilogue's minimum) instead of half-masking the 128 x 64 tile (ym_conv_set_eval_narrow)
    if (g_eval_narrow && d->cout <= 32) launch_gemm<128, 32, 1, 4, 64, 3, MODE_FWD, true>(a, FWD_STAT_BLOCKS, st, ev);
    else if (g_eval_cfg == 0) launch_gemm<128, 64, 2, 2, 32, 3, MODE_FWD, true>(a, FWD_STAT_BLOCKS, st, ev);
    else if (g_eval_cfg == 1) launch_gemm<128, 64, 2, 2, 64, 3, MODE_FWD, true>(a, FWD_STAT_BLOCKS, st, ev);
    else launch_gemm<128, 64, 2, 2, 64, 4, MODE_FWD, true>(a, FWD_STAT_BLOCKS, st, ev);
    if (ks > 1) {
        const int64_t threads = a.M * (d->cout / 8);
        hipLaunchKernelGGL(eval_fold_kernel, dim3(unsigned((threads + 255) / 256)), dim3(256), 0, st, ev.part, ks, a.M,
                           d->cout, uint32_t(d->oh) * uint32_t(d->ow), scale, shift, act, res, r_bs, r_ld, y, d->y_bs,
                           d->y_ld);
    }
    YM_LAUNCH_CHECK("ym_conv_fwd_eval");
    return YM_OK;
}

extern "C" int ym_conv_set_fold(int mode) {
    // ym_conv_fwd_bn's fold policy: -1 default (on), 0 off, 1 on; returns the previous setting
    return g_fold_mode.set(mode < -1 || mode > 1 ? -1 : mode);
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
    a.N = d->n;
    // stride-2: one launch over the 4 output parity classes, each with only its valid taps
    YM_CHECK_ARG(d->k >= 1 && d->k <= 3, "ym_conv_dgrad: kernel size %d unsupported (1..3)", d->k);
    YM_CHECK_ARG(d->stride == 1 || d->stride == 2, "ym_conv_dgrad: stride %d unsupported (1, 2)", d->stride);
    a.ostep = d->stride;
    a.ep_lds = int64_t(d->n) * d->x_bs * 2 < (int64_t(1) << 31) && d->x_ld % 8 == 0 && d->x_bs % 8 == 0 &&
               reinterpret_cast<uintptr_t>(dx) % 16 == 0;     // 16-B stores of whole 8-channel runs
    if (a.M == 0) return YM_OK;
    YM_CHECK_ARG(a.M < (int64_t(1) << 31), "ym_conv_dgrad: too many pixels");
    YM_CHECK_ARG(offsets_fit(d->y_bs, int64_t(d->h / d->stride) * (d->w / d->stride)),
                 "ym_conv_dgrad: gradient image stride too large");
    const DirectPlan dp = direct_plan(d, 1);
    if (dp.ok) {
        direct_launch(dp, d, 1, dz, wt, dx, nullptr, nullptr, as_stream(stream));
        YM_LAUNCH_CHECK("ym_conv_dgrad (direct)");
        return YM_OK;
    }
    const HPipePlan hq = hpipe_plan(d, 1);
    if (hq.ok) {
        hpipe_launch(hq, d, 1, dz, wt, dx, nullptr, nullptr, as_stream(stream));
        YM_LAUNCH_CHECK("ym_conv_dgrad (hpipe)");
        return YM_OK;
    }
    const PipePlan pp = pipe_plan(d, 1);
    if (pp.ok) {
        pipe_launch(pp, d, 1, dz, wt, dx, nullptr, nullptr, nullptr, as_stream(stream));
        YM_LAUNCH_CHECK("ym_conv_dgrad (pipe)");
        return YM_OK;
    }
    const HaloPlan hp = halo_plan(d, 1);
    if (hp.ok) {
        halo_launch(hp, d, 1, dz, wt, dx, nullptr, nullptr, nullptr, as_stream(stream));
        YM_LAUNCH_CHECK("ym_conv_dgrad (halo)");
        return YM_OK;
    }
    pick_and_launch(a, MODE_DGRAD, 4096, select_n(d), as_stream(stream));
    YM_LAUNCH_CHECK("ym_conv_dgrad");
    return YM_OK;
}

// channel pieces of a c-channel layer for the lane-group kernels (stem, depthwise): powers of two of 8-channel groups,
// largest first, at most max_groups each — f(c_base, channels) per launch (64 + 32 for the x-scale stem's 96)
template <class F>
static void ch_pieces(int c, int max_groups, F f) {
    int base = 0, groups = c / 8;
    while (groups > 0) {
        int p = 1;
        while (p * 2 <= groups && p * 2 <= max_groups) p *= 2;
        f(base * 8, p * 8);
        base += p;
        groups -= p;
    }
}

// the stem kernels' instance for `ch` image planes (1..4: the reference builds ch = 1 for its crater config and any
// ch through build_yolo11(ch=...), models/yolo11_model.py:23, 258; RGB is 3)
#define YM_STEM_CH_SWITCH(ch, KERNEL, ...)                                                                         \
    switch (ch) {                                                                                                  \
        case 1: hipLaunchKernelGGL(KERNEL<1>, __VA_ARGS__); break;                                                 \
        case 2: hipLaunchKernelGGL(KERNEL<2>, __VA_ARGS__); break;                                                 \
        case 3: hipLaunchKernelGGL(KERNEL<3>, __VA_ARGS__); break;                                                 \
        default: hipLaunchKernelGGL(KERNEL<4>, __VA_ARGS__); break;                                                \
    }

extern "C" int ym_conv_first_fwd(const float* img, const float* w_oihw, uint16_t* y, float* stat_sum, float* stat_sq,
                                 int n, int h, int w, int oh, int ow, int cout, int stride, int pad, int ch, int blocks,
                                 void* stream) {
    YM_CHECK_ARG(cout % 8 == 0 && cout > 0 && cout <= 4096, "ym_conv_first_fwd: cout=%d unsupported", cout);
    YM_CHECK_ARG(ch >= 1 && ch <= 4, "ym_conv_first_fwd: ch=%d image planes unsupported (1..4)", ch);
    YM_CHECK_ARG(int64_t(n) * oh * ow < (int64_t(1) << 31) && int64_t(n) * ch * h * w < (int64_t(1) << 31),
                 "ym_conv_first_fwd: too many pixels");
    YM_CHECK_ARG(blocks >= 1 && stat_sum && stat_sq, "ym_conv_first_fwd: statistics buffers / blocks");
    ch_pieces(cout, 64, [&](int c_base, int c) {
        YM_STEM_CH_SWITCH(ch, conv_first_fwd_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), img, w_oihw, y,
                          stat_sum, stat_sq, n, h, w, oh, ow, c, stride, pad, c_base, cout)
    });
    YM_LAUNCH_CHECK("ym_conv_first_fwd");
    return YM_OK;
}

extern "C" int ym_conv_first_fwd_eval(const float* img, const float* w_oihw, const float* scale, const float* shift,
                                      int act, uint16_t* y, int64_t y_bs, int64_t y_ld, int n, int h, int w, int oh,
                                      int ow, int cout, int stride, int pad, int ch, void* stream) {
    YM_CHECK_ARG(img && w_oihw && scale && shift && y, "ym_conv_first_fwd_eval: null argument");
    YM_CHECK_ARG(ch >= 1 && ch <= 4, "ym_conv_first_fwd_eval: ch=%d image planes unsupported (1..4)", ch);
    YM_CHECK_ARG(cout % 8 == 0 && cout <= (ch <= 2 ? 512 : 256), "ym_conv_first_fwd_eval: cout=%d unsupported", cout);
    YM_CHECK_ARG(int64_t(n) * oh * ow < (int64_t(1) << 31) && int64_t(n) * ch * h * w < (int64_t(1) << 31),
                 "ym_conv_first_fwd_eval: too many pixels");
    YM_CHECK_ARG(y_ld % 8 == 0 && y_bs % 8 == 0 && y_ld >= cout && y_bs >= int64_t(oh) * ow * y_ld &&
                     reinterpret_cast<uintptr_t>(y) % 16 == 0,
                 "ym_conv_first_fwd_eval: output view not 16-byte aligned");
    const int64_t threads = int64_t(n) * oh * ow;                 // one per output pixel
    if (threads == 0) return YM_OK;
    const int blocks = int(std::min<int64_t>((threads + 255) / 256, 8192));
    YM_STEM_CH_SWITCH(ch, conv_first_eval_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), img, w_oihw, scale,
                      shift, act, y, y_bs, y_ld, n, h, w, oh, ow, cout, stride, pad)
    YM_LAUNCH_CHECK("ym_conv_first_fwd_eval");
    return YM_OK;
}

extern "C" size_t ym_conv_first_wgrad_workspace_size(int cout, int ch) {
    return size_t(PARTIAL_BLOCKS) * size_t(cout > 0 ? cout : 0) * 9 * size_t(ch > 0 ? ch : 0) * sizeof(float);
}

extern "C" int ym_conv_first_wgrad(const uint16_t* dz, const float* img, float* dw_oihw, int n, int h, int w, int oh,
                                   int ow, int cout, int stride, int pad, int ch, float* workspace,
                                   size_t workspace_bytes, void* stream) {
    YM_CHECK_ARG(cout % 8 == 0 && cout > 0 && cout <= 4096, "ym_conv_first_wgrad: cout=%d unsupported", cout);
    YM_CHECK_ARG(ch >= 1 && ch <= 4, "ym_conv_first_wgrad: ch=%d image planes unsupported (1..4)", ch);
    YM_CHECK_ARG(int64_t(n) * oh * ow < (int64_t(1) << 31) && int64_t(n) * ch * h * w < (int64_t(1) << 31),
                 "ym_conv_first_wgrad: too many pixels");
    YM_CHECK_ARG(workspace && workspace_bytes >= ym_conv_first_wgrad_workspace_size(cout, ch),
                 "ym_conv_first_wgrad: workspace too small");
    hipStream_t st = as_stream(stream);
    ch_pieces(cout, 16, [&](int c_base, int c) {             // <= 128 channels a piece (the kernel's LDS rows)
        YM_STEM_CH_SWITCH(ch, conv_first_wgrad_kernel, dim3(PARTIAL_BLOCKS), dim3(256), 0, st, dz, img, workspace, n, h,
                          w, oh, ow, c, stride, pad, c_base, cout)
    });
    colsum_launch(workspace, PARTIAL_BLOCKS, cout * 9 * ch, int64_t(cout) * 9 * ch, dw_oihw, 1, st);
    YM_LAUNCH_CHECK("ym_conv_first_wgrad");
    return YM_OK;
}

// any C % 8 == 0 (run as ch_pieces of <= 512 channels); 8-channel aligned channel map and views
static bool dw_shape_ok(int64_t x_bs, int64_t x_ld, int gsz, int gstride, int goff, int c) {
    return c % 8 == 0 && c > 0 && c <= 8192 && gsz % 8 == 0 && gstride % 8 == 0 && goff % 8 == 0 && x_bs % 8 == 0 &&
           x_ld % 8 == 0;
}

extern "C" int ym_dw3x3_fwd(const uint16_t* x, int64_t x_bs, int64_t x_ld, int gsz, int gstride, int goff,
                            const float* w, uint16_t* y, float* stat_sum, float* stat_sq, int n, int h, int wd, int c,
                            int blocks, void* stream) {
    YM_CHECK_ARG(dw_shape_ok(x_bs, x_ld, gsz, gstride, goff, c) && int64_t(n) * h * wd < (int64_t(1) << 31),
                 "ym_dw3x3_fwd: unsupported shape (C %% 8 != 0 or channel map / views not 8-channel aligned)");
    YM_CHECK_ARG(blocks >= 1 && stat_sum && stat_sq, "ym_dw3x3_fwd: statistics buffers / blocks");
    ch_pieces(c, 64, [&](int c_base, int cp) {
        const DwArgs a{x, x_bs, x_ld, gsz, gstride, goff, w, y, 0, 0, n, h, wd, cp, c_base, c};
        hipLaunchKernelGGL(dw3x3_fwd_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), a, stat_sum, stat_sq);
    });
    YM_LAUNCH_CHECK("ym_dw3x3_fwd");
    return YM_OK;
}

extern "C" int ym_dw3x3_fwd_eval(const uint16_t* x, int64_t x_bs, int64_t x_ld, int gsz, int gstride, int goff,
                                 const float* w, const float* scale, const float* shift, int act, const uint16_t* res,
                                 int64_t r_bs, int64_t r_ld, uint16_t* y, int64_t y_bs, int64_t y_ld, int n, int h,
                                 int wd, int c, void* stream) {
    YM_CHECK_ARG(x && w && scale && shift && y, "ym_dw3x3_fwd_eval: null argument");
    YM_CHECK_ARG(dw_shape_ok(x_bs, x_ld, gsz, gstride, goff, c) && int64_t(n) * h * wd < (int64_t(1) << 31),
                 "ym_dw3x3_fwd_eval: unsupported shape (C %% 8 != 0 or channel map / views not 8-channel aligned)");
    YM_CHECK_ARG(y_bs % 8 == 0 && y_ld % 8 == 0 && reinterpret_cast<uintptr_t>(y) % 16 == 0 &&
                     (!res || (r_bs % 4 == 0 && r_ld % 4 == 0 && reinterpret_cast<uintptr_t>(res) % 8 == 0)),
                 "ym_dw3x3_fwd_eval: output / residual view alignment");
    if (int64_t(n) * h * wd == 0) return YM_OK;
    ch_pieces(c, 64, [&](int c_base, int cp) {
        const int64_t threads = int64_t(n) * h * wd * (cp / 8);
        const DwArgs a{x, x_bs, x_ld, gsz, gstride, goff, w, y, y_bs, y_ld, n, h, wd, cp, c_base, c};
        hipLaunchKernelGGL(dw3x3_fwd_eval_kernel, dim3(unsigned(std::min<int64_t>((threads + 255) / 256, 4096))),
                           dim3(256), 0, as_stream(stream), a, scale, shift, act, res, r_bs, r_ld);
    });
    YM_LAUNCH_CHECK("ym_dw3x3_fwd_eval");
    return YM_OK;
}

extern "C" size_t ym_dw3x3_bwd_workspace_size(int c) {
    return size_t(PARTIAL_BLOCKS) * size_t(c > 0 ? c : 0) * 9 * sizeof(float);
}

extern "C" int ym_dw3x3_bwd(const uint16_t* x, int64_t x_bs, int64_t x_ld, int gsz, int gstride, int goff,
                            const float* w, const uint16_t* dz, uint16_t* dx, int64_t dx_bs, int64_t dx_ld, float* dw,
                            int n, int h, int wd, int c, int accumulate, float* workspace, size_t workspace_bytes,
                            void* stream) {
    YM_CHECK_ARG(dw_shape_ok(x_bs, x_ld, gsz, gstride, goff, c) && dx_bs % 8 == 0 && dx_ld % 8 == 0 &&
                     int64_t(n) * h * wd < (int64_t(1) << 31),
                 "ym_dw3x3_bwd: unsupported shape (C %% 8 != 0 or channel map / views not 8-channel aligned)");
    YM_CHECK_ARG(workspace && workspace_bytes >= ym_dw3x3_bwd_workspace_size(c), "ym_dw3x3_bwd: workspace too small");
    hipStream_t st = as_stream(stream);
    ch_pieces(c, 64, [&](int c_base, int cp) {
        const DwArgs a{x, x_bs, x_ld, gsz, gstride, goff, w, dx, dx_bs, dx_ld, n, h, wd, cp, c_base, c};
        hipLaunchKernelGGL(dw3x3_bwd_kernel, dim3(PARTIAL_BLOCKS), dim3(256), 0, st, a, dz, workspace, accumulate);
    });
    colsum_launch(workspace, PARTIAL_BLOCKS, c * 9, int64_t(c) * 9, dw, 1, st);
    YM_LAUNCH_CHECK("ym_dw3x3_bwd");
    return YM_OK;
}

extern "C" int ym_prep_weights(const ym_wprep_entry* table_dev, int n_entries, int64_t total_elems, void* stream) {
    if (total_elems == 0) return YM_OK;
    hipLaunchKernelGGL(prep_weights_kernel<false>, dim3(unsigned((total_elems + PREP_CHUNK - 1) / PREP_CHUNK), 2),
                       dim3(256), 0, as_stream(stream), table_dev, n_entries, total_elems);
    YM_LAUNCH_CHECK("ym_prep_weights");
    return YM_OK;
}

extern "C" int ym_prep_weights_fwd(const ym_wprep_entry* table_dev, int n_entries, int64_t total_elems, void* stream) {
    if (total_elems == 0) return YM_OK;
    constexpr int CHUNK = 256 * PREP_PER_FWD;
    hipLaunchKernelGGL(prep_weights_kernel<true>, dim3(unsigned((total_elems + CHUNK - 1) / CHUNK)), dim3(256),
                       0, as_stream(stream), table_dev, n_entries, total_elems);
    YM_LAUNCH_CHECK("ym_prep_weights_fwd");
    return YM_OK;
}
