// Halo-staged persistent pipelined 3x3 stride-1 convolution for gfx950 (fp16 forward, bf16 data
// gradient, fp32 accumulate) — the 3x3 layers on maps whose sides are multiples of 16 (80x80, 160x160
// at s@640; 160x160 / 320x320 at m@1280).
//
// Replaces nn.Conv2d (k=3, s=1, p=1) forward / input-gradient inside Conv and Bottleneck
// (/root/reference/yolo_scratch_cuda/models/yolo11_modules.py:21-47, Detect :221-234).
//
// Why: conv_pipe.hip's implicit GEMM stages the input once PER TAP — a 256 x 128 tile's K step moves
// 48 KB (32 KB of it gathered input) for 4.2 MFLOP, and that L2 -> LDS stream, not the MFMA, bounds it
// (~0.3 of the MFMA peak).  Here the output tile is a 16 x 16 pixel RECTANGLE of one
// image, and each 64-channel chunk of its 18 x 18 input halo is staged ONCE and read by all nine taps
// (shifted LDS windows); only the 16 KB weight slice of a tap is staged per K step.  Per 9 K steps:
// 41.5 KB of halo + 9 x 16 KB of weights = 186 KB instead of 432 KB (2.3x fewer staged bytes per FLOP).
// Everything else is conv_pipe's structure:
//  * 256 pixels x 128 (or 64) channels per tile on 8 waves of 64 x 64 (64 x 32);
//  * K step = one tap of one 64-channel chunk (two 32-deep halves); weights through a 3-slot LDS ring
//    with two slots in flight (LDS-DMA, counted vmcnt waits, raw s_barrier); the halo double-buffered,
//    the next chunk's halo issued at the first K step of the current chunk (9 steps of cover);
//  * the barrier in the middle of a K step: every LDS read has 16 MFMAs to hide behind;
//  * persistent workgroups (one per CU), tiles grouped per XCD, the channel tiles of one pixel tile on
//    one XCD; BatchNorm statistics in registers across a workgroup's tiles, one partial row each;
//  * register-transposed epilogue with 16-B row stores (round 4; the LDS transpose before it).
// Halo LDS rows are 128 B (64 channels); row r stores logical 16-B chunk c at slot c ^ (r & 7), which is
// conflict-free for ds_read_b128 at EVERY starting row (the tap shifts start fragments at arbitrary rows;
// conv_pipe's (r >> 1) & 7 swizzle conflicts 2-way there — checked with a bank model of the four
// ds_read_b128 lane groups).
#include <algorithm>

#include "common.h"
#include "conv_epi.h"
#include "conv_hpipe.h"
#include "conv_pipe.h"
#include "tile.h"

namespace ym {

Policy g_hpipe_force{-1};

namespace {

constexpr int HF = 0;   // forward: fp16 x fp16
constexpr int HD = 1;   // data gradient (of a stride-1 conv): bf16 x bf16, taps flipped

constexpr int TS = 16;                    // output tile side (pixels)
constexpr int HS = TS + 2;                // halo side
constexpr int HROWS = HS * HS;            // 324 halo pixels
constexpr int HPIECES = (HROWS + 7) / 8;  // 41 DMA pieces of 8 pixel rows (the last half out of range)
constexpr int HBUF = HPIECES * 1024;      // bytes per halo buffer
constexpr int RB = 128;                   // 64 channels x 2 B per LDS row

struct HArgs {
    const bf16_t* x; int64_t x_bs, x_ld;     // input view (forward: x; data gradient: dz)
    const bf16_t* w;                          // [Nout][3][3][Kin]
    void* y; int64_t y_bs, y_ld;              // output view
    float* st_sum; float* st_sq;              // [rows][Nout] or null
    int H, W, Kin, Nout, N;
    int out_f32, accumulate;
    int ntiles;                               // channel tiles
    int tpr, tpi;                             // tiles per tile-row (W / 16), per image
    int mt_total;                             // pixel tiles: N * tpi
};

__device__ __forceinline__ int fsw128(int r) { return (r >> 1) & 7; }   // weight rows (aligned reads)

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

// runtime (wave-uniform) vmcnt: the pending-DMA count after the stage a step needs depends on whether
// a halo was issued in between
__device__ __forceinline__ void vm_wait_n(int n) {
    switch (n) {
        case 0: vm_wait<0>(); break;
        case 1: vm_wait<1>(); break;
        case 2: vm_wait<2>(); break;
        case 3: vm_wait<3>(); break;
        case 4: vm_wait<4>(); break;
        case 5: vm_wait<5>(); break;
        case 6: vm_wait<6>(); break;
        case 7: vm_wait<7>(); break;
        case 8: vm_wait<8>(); break;
        case 9: vm_wait<9>(); break;
        case 10: vm_wait<10>(); break;
        case 11: vm_wait<11>(); break;
        default: vm_wait<12>(); break;
    }
}

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

// WRES (64 -> 64 channels, one 64-channel chunk): the layer's whole weight tensor (9 taps x 64 x 64, 72 KB)
// is staged into LDS once per workgroup and stays resident; the K loop then stages only the halo (41 pieces
// per 9 K steps) and waits only before a chunk's first step for its halo
// RO: K-step issue order as conv_pipe_kernel's (ym_conv_set_pipe_order): 1 pins every fragment read ahead of the half
// step of MFMAs it covers (the next step's first-half reads right after the barrier, before the DMAs)
template <int BN, int WM, int WN, int MODE, bool WRES = false, int RO = 0>
__global__ void __launch_bounds__(WM * WN * 64, 1) conv_hpipe_kernel(HArgs a) {
    constexpr int NS = WRES ? 9 : 4;          // weight ring: slot of step g computing, g+1..g+3 in flight (WRES:
                                              // the 9 taps, resident)
    constexpr int NW = WM * WN;
    static_assert(NW == 8, "8 waves");
    constexpr int AI = BN / 8 / NW;           // weight DMA pieces per wave per step
    constexpr int TM = BN / WM / 16;          // 16-channel subtiles per wave
    constexpr int TN = TS / WN;               // tile rows (16-pixel subtiles) per wave
    constexpr int WSLOT = BN * RB;
    constexpr int WCH = BN / WM;              // channels per wave
    constexpr int HI_MAX = (HPIECES + NW - 1) / NW;   // halo pieces of wave 0 (others one fewer or equal)
    static_assert(AI >= 1 && TM >= 1 && TN >= 1 && TN % 2 == 0, "tile");
    static_assert(2 * HBUF + NS * WSLOT <= 160 * 1024, "LDS budget");
    __shared__ __attribute__((aligned(16))) char smem[2 * HBUF + NS * WSLOT];
    char* const hbuf0 = smem;
    char* const wring = smem + 2 * HBUF;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave / WN, wc = wave % WN;
    const int fc = lane >> 4, fr = lane & 15;
    const int CC = a.Kin >> 6;                // 64-channel chunks
    const int hi_w = (HPIECES - wave + NW - 1) / NW;   // this wave's halo pieces (wave-uniform)

    // ---- this workgroup's tiles: channel tile fixed, pixel tiles of its XCD's range (as conv_pipe)
    const int G8 = int(gridDim.x) >> 3;
    const int xcd = int(blockIdx.x) & 7, q = int(blockIdx.x) >> 3;
    const int nt = q % a.ntiles, qq = q / a.ntiles, qstride = G8 / a.ntiles;
    const int per = (a.mt_total + 7) >> 3;
    const int mt_lo = xcd * per + qq, mt_hi = min(xcd * per + per, a.mt_total);
    const int ntile = mt_lo < mt_hi ? (mt_hi - mt_lo + qstride - 1) / qstride : 0;
    const int n0 = nt * BN;
    const int spt = 9 * CC;                   // K steps per tile
    const int total = ntile * spt;

    // weight DMA rows (fixed): row r of the A image = output channel n0 + r
    const uint32_t wrow_b = uint32_t(9 * a.Kin) * 2u;
    const __amdgpu_buffer_rsrc_t wres = make_rsrc(a.w, int64_t(a.Nout) * wrow_b);
    uint32_t a_off[AI];
#pragma unroll
    for (int j = 0; j < AI; ++j) {
        const int r = (wave * AI + j) * 8 + (lane >> 3);
        const int ch = n0 + r;
        a_off[j] = ch < a.Nout ? uint32_t(ch) * wrow_b + uint32_t((lane & 7) ^ fsw128(r)) * 16u : OOB;
    }
    const __amdgpu_buffer_rsrc_t xres = make_rsrc(a.x, int64_t(a.N) * a.x_bs * 2);

    // ---- issue side: weight stage s -> (chunk, tap); halo of global chunk h -> (tile, chunk)
    // weight stage s into its ring slot; past the stream's end (live false) the DMAs fetch nothing but still
    // count, so every step issues AI of them and the counted waits stay constant
    // issue position of the weight stream (stage s = g + NS): tap / chunk / ring slot advanced per stage — round 5: the
    // divisions by the steps per tile (s % spt, / 9, % NS) this replaced ran twice per step on each side of the loop
    int w_tap = 0, w_cc = 0, w_slot = 0;
    auto issue_w = [&](bool live) {
        if constexpr (WRES) return;
        const uint32_t soff = uint32_t(w_tap * a.Kin + w_cc * 64) * 2u;
        char* st = wring + w_slot * WSLOT;
#pragma unroll
        for (int j = 0; j < AI; ++j) dma16(wres, st + (wave * AI + j) * 1024, live ? a_off[j] : OOB, soff);
        if (++w_tap == 9) {
            w_tap = 0;
            if (++w_cc == CC) w_cc = 0;
        }
        w_slot = w_slot == NS - 1 ? 0 : w_slot + 1;
    };
    uint32_t hoff[HI_MAX];                    // per-lane halo offsets of the tile being staged
    int h_tile = -1;
    auto issue_h = [&](int h) {
        const int t = h / CC, cc = h - t * CC;
        if (t != h_tile) {
            h_tile = t;
            const int mt = mt_lo + t * qstride;
            const int n = mt / a.tpi, rem = mt - n * a.tpi;
            const int ty = rem / a.tpr, tx = rem - ty * a.tpr;
#pragma unroll
            for (int j = 0; j < HI_MAX; ++j) {
                const int hr = (wave + NW * j) * 8 + (lane >> 3);
                const int iy = ty * TS - 1 + hr / HS, ix = tx * TS - 1 + hr % HS;
                const bool ok = hr < HROWS && uint32_t(iy) < uint32_t(a.H) && uint32_t(ix) < uint32_t(a.W);
                hoff[j] = ok ? uint32_t((int64_t(n) * a.x_bs + (int64_t(iy) * a.W + ix) * a.x_ld) * 2) +
                                   uint32_t((lane & 7) ^ (hr & 7)) * 16u
                             : OOB;
            }
        }
        char* hb = hbuf0 + (h & 1) * HBUF;
#pragma unroll
        for (int j = 0; j < HI_MAX; ++j)
            if (j < hi_w) dma16(xres, hb + (wave + NW * j) * 1024, hoff[j], uint32_t(cc * 64) * 2u);
    };

    // per-lane fragment offsets: A as conv_pipe; B = halo rows of this wave's tile rows
    uint32_t offA[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
        const int ra = wr * (BN / WM) + fr;
        offA[kk] = uint32_t(ra * RB + (((kk * 4 + fc) ^ fsw128(ra)) << 4));
    }
    bf16x8 f0a[TM], f0b[TN], f1a[TM], f1b[TN];
    // compute-side position of a step: (kh, kw) of its tap, its weight ring slot, the halo buffer of its chunk
    struct Pos { int kh, kw, slot, hb; };
    auto next_pos = [&](Pos p) {
        if (++p.kw == 3) {
            p.kw = 0;
            if (++p.kh == 3) { p.kh = 0; p.hb ^= 1; }       // a chunk's 9 taps done: the next chunk's halo buffer
        }
        p.slot = p.slot == NS - 1 ? 0 : p.slot + 1;
        return p;
    };
    auto read_frags = [&](bf16x8* fa, bf16x8* fb, Pos p, int kk) {
        const int dh = MODE == HF ? p.kh : 2 - p.kh, dw = MODE == HF ? p.kw : 2 - p.kw;
        const char* As = wring + (WRES ? (p.kh * 3 + p.kw) : p.slot) * WSLOT + offA[kk];
        const char* Hs = hbuf0 + p.hb * HBUF;
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(As + i * 16 * RB);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int hr = (wc * TN + j + dh) * HS + fr + dw;
            fb[j] = *reinterpret_cast<const bf16x8*>(Hs + hr * RB + (((kk * 4 + fc) ^ (hr & 7)) << 4));
        }
    };
    f32x4 acc[TM][TN];
    auto mma = [&](const bf16x8* fa, const bf16x8* fb) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                if constexpr (MODE == HF)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, fa[i]),
                                                                        __builtin_bit_cast(f16x8, fb[j]), acc[i][j], 0,
                                                                        0, 0);
                else
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
            }
    };

    float ssum[TM][4], ssq[TM][4];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) ssum[i][r] = ssq[i][r] = 0.f;

    // ---- prologue: halo of chunk 0, weight stages 0..3; stage 0 and the halo landed everywhere
    const int nchunks = ntile * CC;
    if (total > 0) issue_h(0);
    if constexpr (WRES) {
        // every tap's weight slice, once (slot t = tap t; one 64-channel chunk)
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
            for (int j = 0; j < AI; ++j)
                dma16(wres, wring + t * WSLOT + (wave * AI + j) * 1024, total > 0 ? a_off[j] : OOB,
                      uint32_t(t * a.Kin) * 2u);
        vm_wait<0>();
    } else {
#pragma unroll
        for (int s = 0; s < NS; ++s)
            issue_w(s < total);
        vm_wait_n(AI * (NS - 1));
    }
    step_barrier();
    Pos pos{0, 0, 0, 0};
    if (total > 0) read_frags(f0a, f0b, pos, 0);

    int ct = 0, ck = 0;
    int c9 = 0, hc = 0;                       // g % 9 and g / 9 (the step's tap and global chunk), kept by counting
    for (int g = 0; g < total; ++g) {
        if (ck == 0) {
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        read_frags(f1a, f1b, pos, 1);
        mma(f0a, f0b);
        if constexpr (RO == 1) {
            __builtin_amdgcn_sched_group_barrier(0x100, TM + TN, 0);               // this step's second-half reads
            __builtin_amdgcn_sched_group_barrier(0x008, TM * TN, 0);               // first-half MFMAs
        }
        // stage g+1 must have landed (own DMAs); stages g+2 and g+3 may stay in flight, and so may halos
        // issued in steps g-2 and g-1 (after stage g+1, when those steps began a chunk with a successor)
        if (WRES) {
            // the only in-loop DMA is the next chunk's halo (issued 9 steps ahead): retire it before its first read
            if (g + 1 < total && c9 == 8) vm_wait<0>();
        } else if (g + 1 < total) {
            // a halo issued in step g-1 or g-2 (a chunk's first step, when a next chunk exists) is younger than stage
            // g+1 and may stay in flight
            vm_wait_n(2 * AI + ((c9 == 1 || c9 == 2) && hc + 1 < nchunks ? hi_w : 0));
        }
        step_barrier();
        // the halo buffer of chunk h-1 and the weight slot of step g are free (their reads returned before
        // the barrier): the next chunk's halo at its predecessor's first step, then weight stage g+4
        if (c9 == 0 && hc + 1 < nchunks) issue_h(hc + 1);
        // the weight DMAs one at a time between the second half's MFMAs (a burst held both waves of a SIMD
        // off the MFMA pipe), then the next step's first-half reads (harmless past the end)
        issue_w(g + NS < total);
        const Pos npos = next_pos(pos);
        read_frags(f0a, f0b, npos, 0);
        pos = npos;
        if (++c9 == 9) { c9 = 0; ++hc; }
        mma(f1a, f1b);
        if constexpr (RO == 1) {
            __builtin_amdgcn_sched_group_barrier(0x100, TM + TN, 0);               // next-step reads first
            if constexpr (!WRES) {
#pragma unroll
                for (int d = 0; d < AI; ++d) {
                    __builtin_amdgcn_sched_group_barrier(0x008, (TM * TN) / (AI + 1), 0);  // MFMAs
                    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                    // one weight DMA
                }
                __builtin_amdgcn_sched_group_barrier(0x008, TM * TN - AI * ((TM * TN) / (AI + 1)), 0);
            } else {
                __builtin_amdgcn_sched_group_barrier(0x008, TM * TN, 0);
            }
        } else if constexpr (!WRES) {
#pragma unroll
            for (int d = 0; d < AI; ++d) {
                __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                    // one weight DMA
                __builtin_amdgcn_sched_group_barrier(0x008, (TM * TN) / (AI + 1), 0);  // MFMAs
            }
            __builtin_amdgcn_sched_group_barrier(0x100, TM + TN, 0);                  // next-step reads
            __builtin_amdgcn_sched_group_barrier(0x008, TM * TN - AI * ((TM * TN) / (AI + 1)), 0);
        }
        if (++ck < spt) continue;
        ck = 0;

        // ---- epilogue of tile ct: register-transposed 16-B row stores (conv_epi.h epilogue_regs; round 4: no LDS
        // area, no waits on LDS round trips)
        const int mt = mt_lo + ct * qstride;
        ++ct;
        const int n = mt / a.tpi, rem = mt - n * a.tpi;
        const int ty = rem / a.tpr, tx = rem - ty * a.tpr;
        const int wch0 = n0 + wr * WCH;
        const int64_t ybytes = (int64_t(a.N - 1) * a.y_bs + int64_t(a.H) * a.W * a.y_ld) * 2;
        const __amdgpu_buffer_rsrc_t yres = make_rsrc(a.y, ybytes);
        // wave-local pixel q: tile row wc * TN + (q >> 4), column q & 15 (every pixel of a tile is in the map)
        auto pix_off = [&](int q) -> uint32_t {
            const int oy = ty * TS + wc * TN + (q >> 4), ox = tx * TS + (q & 15);
            return uint32_t((int64_t(n) * a.y_bs + (int64_t(oy) * a.W + ox) * a.y_ld + wch0) * 2);
        };
        auto pix_ok = [](int) -> bool { return true; };
        epilogue_regs<TM, TN>(acc, ssum, ssq, a.st_sum != nullptr, lane, wch0, a.Nout, yres, a.out_f32 == 2,
                              a.accumulate != 0, pix_off, pix_ok);
    }

    if (a.st_sum) {
        vm_wait<0>();
        __syncthreads();
        float (*red)[WN][BN] = reinterpret_cast<float (*)[WN][BN]>(smem);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float s = ssum[i][r], sq = ssq[i][r];
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) {
                    s += __shfl_xor(s, o, 64);
                    sq += __shfl_xor(sq, o, 64);
                }
                if (fr == 0) {
                    const int cl = wr * (BN / WM) + i * 16 + fc * 4 + r;
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
                a.st_sum[int64_t(row) * a.Nout + ch] = ps;
                a.st_sq[int64_t(row) * a.Nout + ch] = pq;
            }
        }
    }
}

}  // namespace

HPipePlan hpipe_plan(const ym_conv_desc* d, int dgrad) {
    HPipePlan p{};
    const int mode = g_hpipe_force >= 0 ? g_hpipe_force : 1;
    if (!d || mode == 0) return p;
    if (d->k != 3 || d->stride != 1 || d->pad != 1) return p;
    if (d->h != d->oh || d->w != d->ow || d->h % TS || d->w % TS) return p;
    const int kin = dgrad ? d->cout : d->cin, nout = dgrad ? d->cin : d->cout;
    // >= 128 output channels: the 64-channel tile (8 MFMAs per half step and wave) measured slower than
    // conv_halo.hip on the 64-channel 80x80 layers (0.080 vs 0.070 ms fwd, s@640 bs64)
    if (kin % 64 != 0 || nout % 8 != 0) return p;
    // 64 -> 64: the weight-resident 64-channel tile (cfg 2; same process, s@640 bs64 80x80: fwd 67 -> 57 us,
    // dgrad 57 -> 53 us against conv_halo); other < 128-channel layers stay on conv_halo
    const bool wres = kin == 64 && nout == 64;
    if (nout < 128 && !wres) return p;
    const int64_t in_ld = dgrad ? d->y_ld : d->x_ld, in_bs = dgrad ? d->y_bs : d->x_bs;
    const int64_t out_ld = dgrad ? d->x_ld : d->y_ld, out_bs = dgrad ? d->x_bs : d->y_bs;
    if (in_ld % 8 || in_bs % 8 || out_ld % 8 || out_bs % 8) return p;
    if (!dgrad && d->out_f32 == 1) return p;                     // Detect's fp32 bias convs: conv.hip
    if (int64_t(d->n) * in_bs * 2 >= (int64_t(1) << 31) || int64_t(d->n) * out_bs * 2 >= (int64_t(1) << 31)) return p;
    p.cfg = nout >= 128 ? 0 : (wres ? 2 : 1);
    const int bn = p.cfg == 0 ? 128 : 64;
    const int ntiles = (nout + bn - 1) / bn;
    const int64_t tiles = select_n(d) * (d->h / TS) * (d->w / TS);
    if (mode == 1 && tiles * ntiles < 512) return p;          // several tiles per CU (tail imbalance)
    // default: the weight-resident 64 -> 64 tile only — since round 4 the pipelined implicit GEMM (conv_pipe.hip)
    // runs the >= 128-output-channel 80x80 layers 9-12 % faster than the 128-channel halo tile (same-process
    // A/B, profiles/r04/hpipe_vs_pipe_ab.txt; round 3 measured the opposite before conv_pipe's 16-wave rework);
    // policy 2 still runs every eligible configuration (parity tests)
    if (mode == 1 && p.cfg != 2) return p;
    int grid = 256;
    const int unit = 8 * ntiles;
    grid = (grid / unit) * unit;
    if (grid < unit) return p;
    p.grid = grid;
    p.rows = grid / ntiles;
    p.ok = 1;
    return p;
}

int hpipe_launch(const HPipePlan& p, const ym_conv_desc* d, int dgrad, const uint16_t* x, const uint16_t* w, void* y,
                 float* st_sum, float* st_sq, hipStream_t st) {
    HArgs a{};
    a.x = x;
    a.w = w;
    a.y = y;
    a.N = d->n;
    a.H = d->h;
    a.W = d->w;
    if (!dgrad) {
        a.x_bs = d->x_bs; a.x_ld = d->x_ld; a.y_bs = d->y_bs; a.y_ld = d->y_ld;
        a.Kin = d->cin; a.Nout = d->cout;
        a.out_f32 = d->out_f32;
        a.st_sum = st_sum; a.st_sq = st_sq;
    } else {
        a.x_bs = d->y_bs; a.x_ld = d->y_ld; a.y_bs = d->x_bs; a.y_ld = d->x_ld;
        a.Kin = d->cout; a.Nout = d->cin;
        a.out_f32 = 0;
    }
    a.accumulate = d->accumulate;
    const int bn = p.cfg == 0 ? 128 : 64;
    a.ntiles = (a.Nout + bn - 1) / bn;
    a.tpr = a.W / TS;
    a.tpi = (a.H / TS) * a.tpr;
    a.mt_total = a.N * a.tpi;
    if (p.cfg == 2) {
#ifdef YM_EXPERIMENTS
        if (g_pipe_order) {
            if (!dgrad) conv_hpipe_kernel<64, 1, 8, HF, true, 1><<<dim3(p.grid), dim3(512), 0, st>>>(a);
            else conv_hpipe_kernel<64, 1, 8, HD, true, 1><<<dim3(p.grid), dim3(512), 0, st>>>(a);
            return 0;
        }
#endif
        if (!dgrad) conv_hpipe_kernel<64, 1, 8, HF, true><<<dim3(p.grid), dim3(512), 0, st>>>(a);
        else conv_hpipe_kernel<64, 1, 8, HD, true><<<dim3(p.grid), dim3(512), 0, st>>>(a);
        return 0;
    }
    if (!dgrad) {
        if (p.cfg == 0) conv_hpipe_kernel<128, 2, 4, HF><<<dim3(p.grid), dim3(512), 0, st>>>(a);
        else conv_hpipe_kernel<64, 1, 8, HF><<<dim3(p.grid), dim3(512), 0, st>>>(a);
    } else {
        if (p.cfg == 0) conv_hpipe_kernel<128, 2, 4, HD><<<dim3(p.grid), dim3(512), 0, st>>>(a);
        else conv_hpipe_kernel<64, 1, 8, HD><<<dim3(p.grid), dim3(512), 0, st>>>(a);
    }
    return 0;
}

}  // namespace ym
