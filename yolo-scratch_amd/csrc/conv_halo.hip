// 3x3 stride-1 convolutions with a halo-staged input operand (gfx950, MFMA 16x16x32).
//
// Same arithmetic as conv.hip's implicit GEMM (forward fp16 x fp16, data gradient bf16 x bf16,
// fp32 accumulate; reference nn.Conv2d in Conv / Bottleneck / Detect,
// /root/reference/yolo_scratch_cuda/models/yolo11_modules.py:21-47, 221-234), but the output tile
// is a spatial rectangle of one image (TH x TW pixels, <= TP) and the input operand is staged ONCE
// per 32-channel chunk as the tile's input halo ((TH+2) x (TW+2) pixels), not once per tap: the nine
// taps of the chunk read shifted windows of the same LDS image.  The implicit GEMM re-stages every
// input pixel for each of the 9 taps, and that L2 -> LDS stream is what bounds it (measured: the
// staging alone takes 87 % of its time on the 80x80 128->128 layer); the halo cuts the input
// stream ~6x, leaving the weight rows (one 32-channel x BN slice per tap) as the main stream.
//
// K loop: steps k = (32-channel chunk cc, kernel row kh), each step = the row's 3 taps.  LDS: two halo images (chunk cc and cc+1) and an
// NW-deep ring of weight slices, all filled by LDS-DMA (buffer_load ... lds) with source-side
// swizzle, counted vmcnt waits (the halo of the next chunk and NW-2 weight slices stay in flight)
// and raw barriers.  64-B LDS rows (32 channels): row r's 16-B chunk c lives in slot c ^ F(r) (fsw64 below).
// Pixels of a fragment map to halo rows through a per-lane base (row-major tile, any TW), so tile
// rectangles need not be powers of two (40x40 maps use 40 x 6 tiles); pixels past the map edge are
// computed on zero-padded halo rows and masked in the epilogue.
// Data gradient of a stride-1 3x3 conv = the same kernel with the [cin][kh][kw][cout] weight copy
// and flipped tap offsets.
#include <algorithm>

#include "common.h"
#include "conv_epi.h"
#include "conv_halo.h"
#include "bn_fold.h"
#include "tile.h"

namespace ym {
namespace {

constexpr int H_FWD = 0, H_DGRAD = 1;

struct HaloArgs {
    const bf16_t* x; int64_t x_bs, x_ld;     // input view (fwd: activations fp16; dgrad: dz bf16)
    const bf16_t* w;                          // [Nout][3][3][Kin]
    void* y; int64_t y_bs, y_ld;              // output view
    const float* bias;
    float* st_sum; float* st_sq;              // [gridDim.x][Nout] or null
    int GH, GW, Kin;                          // input map
    int OH, OW, Nout;                         // output map (== input map, stride 1)
    int N;
    int TH, TW, HWd, HP;                      // tile rows/cols, halo width, halo rows
    int RT, CT;                               // tiles per image: rows, cols
    int ntiles;
    int out_mode, accumulate;                 // out_mode: 0 bf16, 1 fp32, 2 fp16
    int ep_lds;                               // 16-bit output via the register-transposed epilogue (conv_epi.h)
    BnFoldArgs fold;                          // BatchNorm finalize as the tail (ym_conv_fwd_bn); gamma null = off
};

// 64-B LDS rows (32 channels): row r's 16-B chunk c lives in slot c ^ F(r), F(r) = 2 * ((r >> 2) & 1).
// A ds_read_b128 lane group reads 16 rows s + fr at chunks c (fr in {0-3, 12-15}) and c ^ 1
// (fr in {4-11}) (or the reverse); rows s+k, s+k+4, s+k+8, s+k+12 share bank quads and land on
// chunks {c, c^3, c^1, c^2} for EVERY start s — the halo fragments start at arbitrary rows (tap
// shifts, tile rows), where the earlier F = {0,3,2,1}[(r>>2)&3] conflicted 1.8-2.4x
// (bank-conflict model over the kernel's fragment rows: 7.3-9.4 LDS cycles per read -> 4.0-6.4).
__device__ __forceinline__ int fsw64(int r) { return ((r >> 2) & 1) << 1; }

// one 1-KiB LDS-DMA piece: lane l's 16 bytes from rsrc + voff + soff land at lds + 16 l.  (A function, not the builtin
// written inline in the kernel's lambdas: there hipcc's host pass silently dropped the kernels' launch stubs.)
__device__ __forceinline__ void dma16h(__amdgpu_buffer_rsrc_t r, char* lds, uint32_t voff, uint32_t soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
    asm volatile("" ::: "memory");
}
// wave-uniform count -> immediate: waits until at most n of this wave's vector-memory ops are pending
template <int MAXN>
__device__ __forceinline__ void wait_vm_dyn(int n) {
    if constexpr (MAXN == 0) {
        wait_vm<0>();
    } else {
        if (n >= MAXN) wait_vm<MAXN>();
        else wait_vm_dyn<MAXN - 1>(n);
    }
}

__device__ __forceinline__ void raw_barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// WPX x WCO waves; wave tile TPW x 16 pixels by TCW x 16 channels; HI halo DMA instructions per
// wave (halo capacity HI * waves * 16 rows); NW-deep weight ring.  EV: the eval-mode Conv block instance
// (ym_conv_fwd_eval: BatchNorm / SiLU / residual in the register epilogue; e is not read by the other instances)
template <int WPX, int WCO, int TPW, int TCW, int HI, int NW, int MODE, bool EV = false>
__global__ void __launch_bounds__(WPX * WCO * 64) __attribute__((amdgpu_waves_per_eu(1, 2)))
conv_halo_kernel(HaloArgs a, EvalArgs e) {
    constexpr int NWV = WPX * WCO, NT = NWV * 64;
    constexpr int BN = WCO * TCW * 16;            // output channels per tile
    static_assert(WPX * TPW * 16 <= 512, "pixel capacity per tile");
    // one K step = one 32-channel chunk x one kernel row (3 taps): the weight slot holds 3 x BN rows
    constexpr int WI = 3 * BN / 16 / NWV;         // weight DMA instructions per wave per step (16 rows each)
    constexpr int HPAD = HI * NWV * 16;           // halo rows per buffer
    constexpr int HBUF = HPAD * 64, WSLOT = 3 * BN * 64;
    static_assert(WI >= 1 && WI * 16 * NWV == 3 * BN && (BN & (BN - 1)) == 0, "weight staging map");
    static_assert(NW >= 3 && NW <= 8, "ring depth");
    __shared__ __attribute__((aligned(16))) char smem[2 * HBUF + NW * WSLOT];
    char* const hbuf = smem;
    char* const wring = smem + 2 * HBUF;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wp = wave / WCO, wc = wave % WCO;
    const int fc = lane >> 4, fr = lane & 15;
    const int n0 = blockIdx.y * BN;
    const int CC = (a.Kin + 31) >> 5;
    const int nk = CC * 3;
    const uint32_t wrow_b = uint32_t(9 * a.Kin) * 2u;
    const uint32_t xld_b = uint32_t(a.x_ld) * 2u;
    const int HWd = a.HWd;

    // weight DMA: instruction j of this wave fills slot rows (wave*WI + j)*16 + lane/4 (row = tap-in-row x BN + channel),
    // 16-B slot lane%4
    const __amdgpu_buffer_rsrc_t wres = make_rsrc(a.w, int64_t(a.Nout) * wrow_b);
    // per-lane weight offsets including the lane's swizzled 16-B chunk; the step's (kernel row, 32-channel chunk) goes
    // in the DMA's scalar soffset (Kin % 32 == 0, halo_plan): no vector instructions per DMA (round 5: the per-DMA
    // bounds selects of the generic form were ~5 VALU each, and the kernel ran 7.7 VALU per MFMA)
    // (Kin % 32 != 0: the last chunk's lanes past Kin go out of range in a separate, branched-to issue loop)
    uint32_t a_off[WI];
    int a_ch[WI];
#pragma unroll
    for (int j = 0; j < WI; ++j) {
        const int r = (wave * WI + j) * 16 + (lane >> 2);
        const int ti = r / BN, co = n0 + (r & (BN - 1));
        a_ch[j] = ((lane & 3) ^ fsw64(r)) * 8;
        a_off[j] = co < a.Nout ? uint32_t(co) * wrow_b + uint32_t(ti * a.Kin) * 2u + uint32_t(a_ch[j]) * 2u : OOB;
    }
    const int k_tail = (a.Kin & 31) ? (a.Kin >> 5) : -1;       // the partial last chunk, if any
    // tile-invariant geometry of this lane's halo DMA rows and fragment pixels (hoisted out of the tile loop)
    int h_r[HI], h_c[HI], h_ch[HI];
#pragma unroll
    for (int j = 0; j < HI; ++j) {
        const int r = (wave * HI + j) * 16 + (lane >> 2);
        h_r[j] = r < a.HP ? r / HWd : -(1 << 20);               // rows past the halo: never in the map
        h_c[j] = r - (r / HWd) * HWd;
        h_ch[j] = ((lane & 3) ^ fsw64(r)) * 8;
    }
    const int ntp0 = a.TH * a.TW;
    int f_ph[TPW], f_pw[TPW], hb[TPW];
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
        const int p = (wp * TPW + j) * 16 + fr;
        f_ph[j] = p < ntp0 ? p / a.TW : (1 << 20);              // pixels past the tile: never in the output
        f_pw[j] = p - (p / a.TW) * a.TW;
        hb[j] = p < ntp0 ? (p / a.TW) * HWd + f_pw[j] : 0;
    }
    float ssum[TCW][4], ssq[TCW][4];
#pragma unroll
    for (int i = 0; i < TCW; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) ssum[i][r] = ssq[i][r] = 0.f;

    const int ntp = a.TH * a.TW;
    const int xcd = blockIdx.x & 7, lstride = gridDim.x >> 3;
    const int per_xcd = (a.ntiles + 7) >> 3;
    const int t_end = min((xcd + 1) * per_xcd, a.ntiles);
    for (int tile = xcd * per_xcd + (blockIdx.x >> 3); tile < t_end; tile += lstride) {
        const int per_img = a.RT * a.CT;
        const int n = tile / per_img, rem = tile - n * per_img;
        const int oh0 = (rem / a.CT) * a.TH, ow0 = (rem % a.CT) * a.TW;
        const int ih0 = oh0 - 1, iw0 = ow0 - 1;
        const __amdgpu_buffer_rsrc_t xres = make_rsrc(a.x + int64_t(n) * a.x_bs, a.x_bs * 2);
        // halo DMA rows of this lane (chunk offsets in soffset); vmask bit j: fragment pixel j lies in the output (the
        // register epilogue's statistics mask)
        uint32_t h_off[HI];
#pragma unroll
        for (int j = 0; j < HI; ++j) {
            const int gh = ih0 + h_r[j], gw = iw0 + h_c[j];
            const bool ok = uint32_t(gh) < uint32_t(a.GH) && uint32_t(gw) < uint32_t(a.GW);
            h_off[j] = ok ? uint32_t(gh * a.GW + gw) * xld_b + uint32_t(h_ch[j]) * 2u : OOB;
        }
        uint32_t vmask = 0;
#pragma unroll
        for (int j = 0; j < TPW; ++j) vmask |= (oh0 + f_ph[j] < a.OH && ow0 + f_pw[j] < a.OW ? 1u : 0u) << j;

        auto issue_halo = [&](int cc) {
            char* dst = hbuf + (cc & 1) * HBUF;
            if (cc == k_tail) {
#pragma unroll
                for (int j = 0; j < HI; ++j)
                    dma16h(xres, dst + (wave * HI + j) * 1024, cc * 32 + h_ch[j] < a.Kin ? h_off[j] : OOB, uint32_t(cc) * 64u);
                return;
            }
#pragma unroll
            for (int j = 0; j < HI; ++j) dma16h(xres, dst + (wave * HI + j) * 1024, h_off[j], uint32_t(cc) * 64u);
        };
        // weight stream position (step k's chunk / kernel row / ring slot), advanced per issued step
        int w_cc = 0, w_kh = 0, w_slot = 0;
        auto issue_w = [&]() {
            char* dst = wring + w_slot * WSLOT;
            const uint32_t soff = uint32_t(w_kh * 3 * a.Kin + w_cc * 32) * 2u;
            if (w_cc == k_tail) {
#pragma unroll
                for (int j = 0; j < WI; ++j)
                    dma16h(wres, dst + (wave * WI + j) * 1024, w_cc * 32 + a_ch[j] < a.Kin ? a_off[j] : OOB, soff);
            } else {
#pragma unroll
                for (int j = 0; j < WI; ++j) dma16h(wres, dst + (wave * WI + j) * 1024, a_off[j], soff);
            }
            if (++w_kh == 3) { w_kh = 0; ++w_cc; }
            w_slot = w_slot == NW - 1 ? 0 : w_slot + 1;
        };

        f32x4 acc[TCW][TPW];
#pragma unroll
        for (int i = 0; i < TCW; ++i)
#pragma unroll
            for (int j = 0; j < TPW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

        raw_barrier();                    // every wave is done with the previous tile's buffers
        issue_halo(0);
#pragma unroll
        for (int s = 0; s < NW - 1; ++s)
            if (s < nk) issue_w();
        int cc = 0, kh = 0, slot = 0;
        for (int k = 0; k < nk; ++k) {
            // pending after the wait: the younger weight slots, and the next chunk's halo when it was
            // issued after this step's weights (at kernel row 0 of this chunk)
            const int yw = min(NW - 2, nk - 1 - k);
            const int pend = WI * yw + ((kh >= 1 && kh < NW - 1 && cc + 1 < CC) ? HI : 0);
            wait_vm_dyn<WI * (NW - 2) + HI>(pend);
            raw_barrier();
            if (kh == 0 && cc + 1 < CC) issue_halo(cc + 1);
            if (k + NW - 1 < nk) issue_w();

            const char* As = wring + slot * WSLOT;
            slot = slot == NW - 1 ? 0 : slot + 1;
            const char* Hs = hbuf + (cc & 1) * HBUF;
            // the three taps of kernel row kh: the fragment reads of tap ti+1 are issued ahead of the
            // MFMAs of tap ti (two register sets; the order is pinned with sched_group_barrier, the
            // compiler otherwise re-reads one A fragment at a time behind an lgkmcnt(0))
            // A rows r = ti*BN + wc*TCW*16 + i*16 + fr share F[(r>>2)&3] over i and ti: one base address
            const int ra = wc * (TCW * 16) + fr;
            const char* ap = As + ra * 64 + ((fc ^ fsw64(ra)) << 4);
            int hbt[TPW];
#pragma unroll
            for (int j = 0; j < TPW; ++j) hbt[j] = hb[j] + (MODE == H_FWD ? kh * HWd : (2 - kh) * HWd + 2);
            auto load_tap = [&](int ti, bf16x8* af, bf16x8* bfr) {
#pragma unroll
                for (int i = 0; i < TCW; ++i)
                    af[i] = *reinterpret_cast<const bf16x8*>(ap + ti * (BN * 64) + i * 1024);
#pragma unroll
                for (int j = 0; j < TPW; ++j) {
                    const int r = MODE == H_FWD ? hbt[j] + ti : hbt[j] - ti;
                    bfr[j] = *reinterpret_cast<const bf16x8*>(Hs + r * 64 + ((fc ^ fsw64(r)) << 4));
                }
            };
            auto mma_tap = [&](const bf16x8* af, const bf16x8* bfr) {
#pragma unroll
                for (int i = 0; i < TCW; ++i)
#pragma unroll
                    for (int j = 0; j < TPW; ++j) {
                        if constexpr (MODE == H_FWD)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, af[i]),
                                                                               __builtin_bit_cast(f16x8, bfr[j]),
                                                                               acc[i][j], 0, 0, 0);
                        else
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
                    }
            };
            bf16x8 fa0[TCW], fb0[TPW], fa1[TCW], fb1[TPW];
            load_tap(0, fa0, fb0);
            load_tap(1, fa1, fb1);
            mma_tap(fa0, fb0);
            __builtin_amdgcn_sched_group_barrier(0x100, TCW + TPW, 0);   // tap 0 reads
            __builtin_amdgcn_sched_group_barrier(0x100, TCW + TPW, 0);   // tap 1 reads
            __builtin_amdgcn_sched_group_barrier(0x008, TCW * TPW, 0);   // tap 0 MFMAs
            load_tap(2, fa0, fb0);
            mma_tap(fa1, fb1);
            __builtin_amdgcn_sched_group_barrier(0x100, TCW + TPW, 0);   // tap 2 reads
            __builtin_amdgcn_sched_group_barrier(0x008, TCW * TPW, 0);   // tap 1 MFMAs
            mma_tap(fa0, fb0);
            __builtin_amdgcn_sched_group_barrier(0x008, TCW * TPW, 0);   // tap 2 MFMAs
            if (++kh == 3) { kh = 0; ++cc; }
        }

        if (a.ep_lds) {
            // register-only transpose (conv_epi.h epilogue_regs: no LDS, no barrier; the statistics masked by the
            // tile's vmask) — round 4: -2..-6 % against the LDS transpose it replaced (halo_reg_epilogue_ab.txt)
            const __amdgpu_buffer_rsrc_t yres = make_rsrc(a.y, int64_t(a.N) * a.y_bs * 2);
            const int wch0 = n0 + wc * (TCW * 16);
            auto pix_off = [&](int q) -> uint32_t {
                const int p = wp * TPW * 16 + q;
                const int ph = p / a.TW, pw = p - ph * a.TW;
                const int oh = oh0 + ph, ow = ow0 + pw;
                if (p >= ntp || oh >= a.OH || ow >= a.OW) return OOB;
                return uint32_t((int64_t(n) * a.y_bs + int64_t(oh * a.OW + ow) * a.y_ld + wch0) * 2);
            };
            auto pix_ok = [&](int q) -> bool { return (vmask >> (q >> 4)) & 1u; };
            if constexpr (EV) {
                const EvalEpi ee{e.sc, e.sh, e.act, make_rsrc(e.res, e.res ? e.res_bytes : 0), e.res != nullptr};
                auto res_off = [&](int q) -> uint32_t {
                    const int p = wp * TPW * 16 + q;
                    const int ph = p / a.TW, pw = p - ph * a.TW;
                    const int oh = oh0 + ph, ow = ow0 + pw;
                    if (p >= ntp || oh >= a.OH || ow >= a.OW) return OOB;
                    return uint32_t((int64_t(n) * e.r_bs + int64_t(oh * a.OW + ow) * e.r_ld + wch0) * 2);
                };
                epilogue_regs_x<TCW, TPW>(acc, ssum, ssq, false, lane, wch0, a.Nout, yres, true, false, pix_off, pix_ok,
                                          &ee, res_off);
            } else {
                epilogue_regs<TCW, TPW>(acc, ssum, ssq, a.st_sum != nullptr, lane, wch0, a.Nout, yres, a.out_mode == 2,
                                        a.accumulate != 0 && a.out_mode == 0, pix_off, pix_ok);
            }
            continue;
        }
        // epilogue: lane holds channels cb..cb+3 of pixel p
#pragma unroll
        for (int j = 0; j < TPW; ++j) {
            const int p = (wp * TPW + j) * 16 + fr;
            const int ph = p / a.TW, pw = p - ph * a.TW;
            const int oh = oh0 + ph, ow = ow0 + pw;
            if (p >= ntp || oh >= a.OH || ow >= a.OW) continue;
            const int64_t obase = int64_t(n) * a.y_bs + int64_t(oh * a.OW + ow) * a.y_ld;
#pragma unroll
            for (int i = 0; i < TCW; ++i) {
                const int cb = n0 + wc * (TCW * 16) + i * 16 + fc * 4;
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
                if (a.out_mode == 2) {
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
                } else if (a.out_mode == 1) {
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
        float (*red)[WPX][BN] = reinterpret_cast<float (*)[WPX][BN]>(smem);   // [sum|sq][pixel wave][channel]
        wait_vm<0>();
        raw_barrier();                    // staging LDS is free again
#pragma unroll
        for (int i = 0; i < TCW; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float s = ssum[i][r], q = ssq[i][r];
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) {
                    s += __shfl_xor(s, o, 64);
                    q += __shfl_xor(q, o, 64);
                }
                if (fr == 0) {
                    const int cl = wc * (TCW * 16) + i * 16 + fc * 4 + r;
                    red[0][wp][cl] = s;
                    red[1][wp][cl] = q;
                }
            }
        __syncthreads();
        for (int c = tid; c < BN; c += NT) {
            const int ch = n0 + c;
            if (ch < a.Nout) {
                float ps = 0.f, pq = 0.f;
#pragma unroll
                for (int w = 0; w < WPX; ++w) { ps += red[0][w][c]; pq += red[1][w][c]; }
                stat_store(&a.st_sum[int64_t(blockIdx.x) * a.Nout + ch], ps, a.fold.gamma != nullptr);
                stat_store(&a.st_sq[int64_t(blockIdx.x) * a.Nout + ch], pq, a.fold.gamma != nullptr);
            }
        }
        if (a.fold.gamma) bn_fold_tail<BN, NT>(a.fold, a.st_sum, a.st_sq, a.Nout, int(blockIdx.y), int(gridDim.x), smem);
    }
}

// tile configurations: C8 = 8 waves, 256 pixels x 128 channels; C4 = 4 waves, 128 pixels x 64 channels
struct Cfg {
    int tp, bn, hpad;
};
constexpr Cfg C8{256, 128, 3 * 8 * 16};
constexpr Cfg C4{128, 64, 4 * 4 * 16};

// tile rectangle for a pixel capacity tp: 16-wide when the map allows, else whole map rows
static bool pick_rect(int OH, int OW, int tp, int hpad, int& TH, int& TW) {
    if (OW % 16 == 0 && OW >= 16) TW = 16;
    else if (OW <= tp / 2) TW = OW;
    else return false;
    TH = std::min(tp / TW, OH);
    if (TH < 1 || (TH + 2) * (TW + 2) > hpad) return false;
    const int RT = (OH + TH - 1) / TH;
    // used fraction of the computed pixels (tile capacity and the last row of tiles)
    const double util = double(OH) * OW / (double(RT) * TH * TW) * double(TH * TW) / tp;
    return util >= 0.74;
}

}  // namespace

Policy g_halo_force{-1};

HaloPlan halo_plan(const ym_conv_desc* d, int dgrad) {
    HaloPlan p{};
    // policy (ym_conv_set_halo): 0 never, 1 wherever it applies, 2 maps <= 24 wide (the 20x20 layers), 3 (the
    // default) maps <= 48 wide or <= 64 output channels — with the pipelined kernel taking the >= 128-channel
    // layers first, this rule measured 2953 vs 2940 img/s over rule 2 (s@640 bs64)
    const int force = g_halo_force >= 0 ? g_halo_force : 3;
    if (force == 0) return p;
    const int ow_ = dgrad ? d->w : d->ow, cout_ = dgrad ? d->cin : d->cout;
    if (force == 2 && ow_ > 24) return p;
    if (force == 3 && ow_ > 48 && cout_ > 64) return p;
    // 3x3, stride 1, pad 1, channels in whole 16-B chunks
    const int cin = dgrad ? d->cout : d->cin, cout = dgrad ? d->cin : d->cout;
    const int GH = dgrad ? d->oh : d->h, GW = dgrad ? d->ow : d->w;
    const int OH = dgrad ? d->h : d->oh, OW = dgrad ? d->w : d->ow;
    if (d->k != 3 || d->stride != 1 || d->pad != 1 || GH != OH || GW != OW) return p;
    if (cin % 8 != 0 || cout < 64) return p;
    const int64_t xbs = dgrad ? d->y_bs : d->x_bs;
    if (xbs * 2 >= (int64_t(1) << 31)) return p;
    // C8 when it still gives one workgroup per CU, else C4
    for (int c = 0; c < 2; ++c) {
        const Cfg cf = c == 0 ? C8 : C4;
        int TH, TW;
        if (!pick_rect(OH, OW, cf.tp, cf.hpad, TH, TW)) continue;
        const int RT = (OH + TH - 1) / TH, CT = (OW + TW - 1) / TW;
        const int64_t tiles = int64_t(d->n) * RT * CT;
        const int nco = (cout + cf.bn - 1) / cf.bn;
        const int64_t sel_tiles = select_n(d) * RT * CT;
        if (c == 0 && (sel_tiles * nco < 256 || cout <= 64)) continue;   // 128-channel tiles need >= 65 channels
        if (tiles >= (int64_t(1) << 30)) continue;
        p.ok = 1;
        p.cfg = c;
        p.TH = TH; p.TW = TW; p.RT = RT; p.CT = CT;
        p.ntiles = int(tiles);
        p.nco = nco;
        int gx = (p.ntiles + 7) & ~7;
        gx = std::min(gx, std::max(8, (2048 / nco) & ~7));   // bounded BN partial rows
        p.gx = gx;
        return p;
    }
    return p;
}

int halo_launch(const HaloPlan& p, const ym_conv_desc* d, int dgrad, const uint16_t* x, const uint16_t* w, void* y,
                const float* bias, float* st_sum, float* st_sq, hipStream_t st, const ym_bn_fold* fold,
                const EvalArgs* ev) {
    HaloArgs a{};
    a.x = x;
    a.w = w;
    a.y = y;
    a.bias = bias;
    a.st_sum = st_sum; a.st_sq = st_sq;
    a.N = d->n;
    if (!dgrad) {
        a.x_bs = d->x_bs; a.x_ld = d->x_ld; a.y_bs = d->y_bs; a.y_ld = d->y_ld;
        a.GH = d->h; a.GW = d->w; a.Kin = d->cin; a.OH = d->oh; a.OW = d->ow; a.Nout = d->cout;
        a.out_mode = d->out_f32;
    } else {
        a.x_bs = d->y_bs; a.x_ld = d->y_ld; a.y_bs = d->x_bs; a.y_ld = d->x_ld;
        a.GH = d->oh; a.GW = d->ow; a.Kin = d->cout; a.OH = d->h; a.OW = d->w; a.Nout = d->cin;
        a.out_mode = 0;
    }
    a.accumulate = d->accumulate;
    a.TH = p.TH; a.TW = p.TW; a.HWd = p.TW + 2; a.HP = (p.TH + 2) * (p.TW + 2);
    // 16-B epilogue stores of transposed pixel rows (round 2 through LDS: 64-ch 80x80 fwd 0.076 -> 0.070 ms, dgrad
    // 0.066 -> 0.058; round 4 in registers)
    a.ep_lds = !bias && a.out_mode != 1 && a.y_ld % 8 == 0 && a.y_bs % 8 == 0 &&
               int64_t(d->n) * a.y_bs * 2 < (int64_t(1) << 31) && reinterpret_cast<uintptr_t>(y) % 16 == 0;
    a.RT = p.RT; a.CT = p.CT; a.ntiles = p.ntiles;
    if (!dgrad && st_sum) a.fold = bn_fold_args(fold);
    const dim3 grid(p.gx, p.nco);
    const EvalArgs e = ev ? *ev : EvalArgs{};
    // the eval epilogue: the fp16 register epilogue of the C4 tile (C8's eval instance spills)
    if (ev && (dgrad || !a.ep_lds || st_sum || p.cfg == 0)) return -1;
    if (p.cfg == 0) {
        if (dgrad) hipLaunchKernelGGL((conv_halo_kernel<4, 2, 4, 4, 3, 3, H_DGRAD>), grid, dim3(512), 0, st, a, e);
        else hipLaunchKernelGGL((conv_halo_kernel<4, 2, 4, 4, 3, 3, H_FWD>), grid, dim3(512), 0, st, a, e);
    } else {
        // 4-deep weight ring (round 4, same-process A/B: -1..-5 % against 3 slots; 6 slots cost the second
        // workgroup per CU: +47..+61 %, profiles/r04/halo_ring_depth_ab.txt)
        if (dgrad) hipLaunchKernelGGL((conv_halo_kernel<2, 2, 4, 2, 4, 4, H_DGRAD>), grid, dim3(256), 0, st, a, e);
        else if (ev) hipLaunchKernelGGL((conv_halo_kernel<2, 2, 4, 2, 4, 4, H_FWD, true>), grid, dim3(256), 0, st, a, e);
        else hipLaunchKernelGGL((conv_halo_kernel<2, 2, 4, 2, 4, 4, H_FWD>), grid, dim3(256), 0, st, a, e);
    }
    return 0;
}

}  // namespace ym
