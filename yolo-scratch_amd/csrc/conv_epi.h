// Conv epilogue shared by the pipelined implicit GEMM (conv_pipe.hip) and the halo-staged 3x3
// kernel (conv_halo.hip): MFMA accumulators -> BatchNorm statistics -> 16-bit NHWC stores.
//
// A 16x16 MFMA accumulator gives each lane 4 consecutive channels of ONE pixel, so storing it
// straight out costs one 8-B store per (subtile, lane), 16 pixels x 32 B per instruction: scattered
// partial-line writes whose issue and drain held a 256 x 128 tile's epilogue at ~40 % of the tile's
// time (measured, tools/pipe_abl.sh ablation 5).  Here each 16-pixel slice of the wave's
// accumulators is transposed through a small per-wave LDS area (swizzled 16-B chunks: conflict-free
// writes and reads) and stored as 16-B pieces of each pixel's contiguous channel run (8 lanes = 128 B),
// with raw buffer stores whose out-of-tile pixels fall out of range (a fixed instruction count, no
// branches).
#pragma once
#include "common.h"
#include "tile.h"

namespace ym {

// acc[i][j][r]: channel wch0 + i*16 + fc*4 + r, wave-local pixel q = j*16 + fr (fc = lane>>4, fr = lane&15).
// WCH = 16 * TM channels of this wave; ep: this wave's LDS area (16 * WCH * 2 bytes).
// pix_off(q) -> byte offset of wave-local pixel q's channel wch0 in the output (OOB when the pixel
// is outside the map / tile).  half: fp16 (1) or bf16 (0) output; accumulate: add into the bf16 output.
template <int TM, int TN, class PixOff>
__device__ __forceinline__ void epilogue_store(f32x4 (&acc)[TM][TN], float (&ssum)[TM][4], float (&ssq)[TM][4],
                                               bool stats, char* ep, int lane, int wch0, int nout,
                                               __amdgpu_buffer_rsrc_t yres, bool half, bool accumulate,
                                               PixOff pix_off) {
    constexpr int WCH = 16 * TM;
    constexpr int CPR = WCH * 2 / 16;          // 16-B chunks per pixel row of this wave
    constexpr int RPS = 64 / CPR;              // pixel rows per store instruction
    static_assert(CPR >= 1 && CPR <= 8 && 16 % RPS == 0, "epilogue transpose geometry");
    const int fc = lane >> 4, fr = lane & 15;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const bool pvalid = pix_off(j * 16 + fr) != OOB;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int cb = wch0 + i * 16 + fc * 4;
            if (stats && pvalid) {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (cb + r < nout) {
                        const float v = acc[i][j][r];
                        ssum[i][r] += v;
                        ssq[i][r] += v * v;
                    }
            }
            uint2 o;
            if (half) {
                o.x = pk2h(acc[i][j][0], acc[i][j][1]);
                o.y = pk2h(acc[i][j][2], acc[i][j][3]);
            } else {
                o.x = pk2bf(acc[i][j][0], acc[i][j][1]);
                o.y = pk2bf(acc[i][j][2], acc[i][j][3]);
            }
            const int byte = (i * 16 + fc * 4) * 2;                    // within the pixel row
            const int chunk = (byte >> 4) ^ (fr & (CPR - 1));          // swizzled 16-B chunk
            *reinterpret_cast<uint2*>(ep + fr * (WCH * 2) + chunk * 16 + (byte & 15)) = o;
        }
#pragma unroll
        for (int h = 0; h < 16 / RPS; ++h) {
            const int p = h * RPS + lane / CPR, c = lane % CPR;
            uint4 v = *reinterpret_cast<const uint4*>(ep + p * (WCH * 2) + ((c ^ (p & (CPR - 1))) * 16));
            uint32_t off = pix_off(j * 16 + p);
            if (off != OOB) {
                if (wch0 + c * 8 < nout) off += uint32_t(c) * 16u;
                else off = OOB;
            }
            if (accumulate) {                                          // gradient fan-in (bf16)
                const uint4 old = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(yres, off, 0, 0));
                uint32_t ww[4] = {v.x, v.y, v.z, v.w}, oo[4] = {old.x, old.y, old.z, old.w};
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    ww[e] = pk2bf(bf2f(bf16_t(ww[e] & 0xffff)) + bf2f(bf16_t(oo[e] & 0xffff)),
                                  bf2f(bf16_t(ww[e] >> 16)) + bf2f(bf16_t(oo[e] >> 16)));
                v = make_uint4(ww[0], ww[1], ww[2], ww[3]);
            }
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v),
                                                   yres, off, 0, 0);
        }
    }
}

// Eval-mode Conv block epilogue (ym_conv_fwd_eval): the running-statistics BatchNorm (scale / shift per output
// channel), SiLU when act, then + the fp16 residual (res_off(q): byte offset of wave-local pixel q's channel wch0 in the
// residual view) — ym_bn_apply's arithmetic (fp32, one fp16 rounding), applied to the accumulators before the pack
// instead of to a stored fp16 z.
struct EvalEpi {
    const float* sc; const float* sh;
    int act;
    __amdgpu_buffer_rsrc_t rres;
    int res;
};

// Register-only form (round 3; the pipelined kernel's data gradient): each pair of 16-pixel subtiles (ja, jb) is exchanged
// between lane rows with v_permlane16_swap (rows 1 / 3 of ja's packed values <-> rows 0 / 2 of jb's), after which
// lane (fc, fr) holds 8 consecutive channels (i*16 + (fc >> 1)*8 ..) of ONE pixel (subtile fc odd ? jb : ja, row
// fr): one 16-B store per lane and channel subtile, 32 pixels x 32 B per instruction, TM * TN / 2 stores per lane.
// No LDS: an LDS transpose makes hipcc drain every in-flight LDS-DMA stage (vmcnt(0)) in front of it.
// pix_off(q) as above (byte offset of wave-local pixel q's channel wch0, OOB outside); nout % 8 == 0.
// pix_ok(q): pixel q of the wave lies inside the output (the statistics' mask; a compare, where pix_off also
// decomposes the pixel).
// ea: the eval-mode BatchNorm / SiLU / residual (a null constant for every other caller: no code, no registers),
// res_off its residual offsets (see EvalEpi).
template <int TM, int TN, class PixOff, class PixOk, class ResOff>
__device__ __forceinline__ void epilogue_regs_x(f32x4 (&acc)[TM][TN], float (&ssum)[TM][4], float (&ssq)[TM][4],
                                                bool stats, int lane, int wch0, int nout,
                                                __amdgpu_buffer_rsrc_t yres, bool half, bool accumulate,
                                                PixOff pix_off, PixOk pix_ok, const EvalEpi* ea, ResOff res_off) {
    static_assert(TN % 2 == 0, "subtile pairs");
    const int fc = lane >> 4, fr = lane & 15;
    if (ea) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int cb = wch0 + i * 16 + fc * 4;
            if (cb >= nout) continue;                                  // nout % 8 == 0: all four or none
            const float4 s4 = *reinterpret_cast<const float4*>(ea->sc + cb);
            const float4 h4 = *reinterpret_cast<const float4*>(ea->sh + cb);
            const float sv[4] = {s4.x, s4.y, s4.z, s4.w}, hv[4] = {h4.x, h4.y, h4.z, h4.w};
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float t = fmaf(acc[i][j][r], sv[r], hv[r]);
                    acc[i][j][r] = ea->act ? silu_f(t) : t;
                }
        }
        if (ea->res) {                                                 // + residual in fp32, one rounding (as ym_bn_apply)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const uint32_t b = res_off(j * 16 + fr);
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const int co = i * 16 + fc * 4;
                    const uint32_t off = b != OOB && wch0 + co < nout ? b + uint32_t(co) * 2u : OOB;
                    const uint2 rv = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(ea->rres, off, 0, 0));
                    acc[i][j][0] += h2f(uint16_t(rv.x & 0xffff));
                    acc[i][j][1] += h2f(uint16_t(rv.x >> 16));
                    acc[i][j][2] += h2f(uint16_t(rv.y & 0xffff));
                    acc[i][j][3] += h2f(uint16_t(rv.y >> 16));
                }
            }
        }
    }
    if (stats) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            if (!pix_ok(j * 16 + fr)) continue;
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int cb = wch0 + i * 16 + fc * 4;
                if (cb < nout) {                                       // nout % 8 == 0: all four or none
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float v = acc[i][j][r];
                        ssum[i][r] += v;
                        ssq[i][r] = fmaf(v, v, ssq[i][r]);
                    }
                }
            }
        }
    }
    auto pack = [&](float lo, float hi) -> uint32_t {
        return half ? pk2h(lo, hi) : pk2bf(lo, hi);
    };
#pragma unroll
    for (int jp = 0; jp < TN / 2; ++jp) {
        const int ja = 2 * jp, jb = ja + 1;
        const uint32_t base = pix_off((fc & 1 ? jb : ja) * 16 + fr);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const uint32_t x0 = pack(acc[i][ja][0], acc[i][ja][1]), x1 = pack(acc[i][ja][2], acc[i][ja][3]);
            const uint32_t y0 = pack(acc[i][jb][0], acc[i][jb][1]), y1 = pack(acc[i][jb][2], acc[i][jb][3]);
            const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
            const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
            uint4 v = make_uint4(s0[0], s1[0], s0[1], s1[1]);
            const int co = i * 16 + (fc >> 1) * 8;                     // channel offset within the wave
            const uint32_t off = base != OOB && wch0 + co < nout ? base + uint32_t(co) * 2u : OOB;
            if (accumulate) {                                          // gradient fan-in (bf16)
                const uint4 old = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(yres, off, 0, 0));
                uint32_t ww[4] = {v.x, v.y, v.z, v.w}, oo[4] = {old.x, old.y, old.z, old.w};
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    ww[e] = pk2bf(bf2f(bf16_t(ww[e] & 0xffff)) + bf2f(bf16_t(oo[e] & 0xffff)),
                                  bf2f(bf16_t(ww[e] >> 16)) + bf2f(bf16_t(oo[e] >> 16)));
                v = make_uint4(ww[0], ww[1], ww[2], ww[3]);
            }

            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v),
                                                   yres, off, 0, 0);
        }
    }
}

// The same epilogue for 32x32 MFMA accumulators (v_mfma_f32_32x32x16): acc[i][j][r] is channel
// wch0 + i*32 + 8*(r>>2) + 4*h + (r&3) of wave-local pixel q = j*32 + p (h = lane>>5, p = lane&31): each register group
// g = r>>2 holds 4 consecutive channels of one pixel, the other 4 of that 8-channel run in the partner lane l ^ 32.
// Groups (2k, 2k+1) are exchanged between the lane halves with v_permlane32_swap (the upper half of 2k's packed values
// <-> the lower half of 2k+1's), after which lane l holds channels i*32 + 8*(2k + h) .. +7 of pixel j*32 + p: one 16-B
// store per lane and group pair, 32 pixels x 2 runs per instruction, TM * TN * 2 stores per lane.  Statistics: ssum /
// ssq[i][r] for the 16 channels the lane's registers hold (summed over the lane's pixels; the caller reduces over p).
template <int TM, int TN, class PixOff, class PixOk, class ResOff>
__device__ __forceinline__ void epilogue_regs32_x(f32x16 (&acc)[TM][TN], float (&ssum)[TM][16], float (&ssq)[TM][16],
                                                  bool stats, int lane, int wch0, int nout,
                                                  __amdgpu_buffer_rsrc_t yres, bool half, bool accumulate,
                                                  PixOff pix_off, PixOk pix_ok, const EvalEpi* ea, ResOff res_off) {
    const int h = lane >> 5, p = lane & 31;
    if (ea) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int cb = wch0 + i * 32 + 8 * g + 4 * h;
                if (cb >= nout) continue;                              // nout % 8 == 0: all four or none
                const float4 s4 = *reinterpret_cast<const float4*>(ea->sc + cb);
                const float4 h4 = *reinterpret_cast<const float4*>(ea->sh + cb);
                const float sv[4] = {s4.x, s4.y, s4.z, s4.w}, hv[4] = {h4.x, h4.y, h4.z, h4.w};
#pragma unroll
                for (int j = 0; j < TN; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float t = fmaf(acc[i][j][4 * g + r], sv[r], hv[r]);
                        acc[i][j][4 * g + r] = ea->act ? silu_f(t) : t;
                    }
            }
        if (ea->res) {                                                 // + residual in fp32, one rounding (as ym_bn_apply)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const uint32_t b = res_off(j * 32 + p);
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const int co = i * 32 + 8 * g + 4 * h;
                        const uint32_t off = b != OOB && wch0 + co < nout ? b + uint32_t(co) * 2u : OOB;
                        const uint2 rv =
                            __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(ea->rres, off, 0, 0));
                        acc[i][j][4 * g + 0] += h2f(uint16_t(rv.x & 0xffff));
                        acc[i][j][4 * g + 1] += h2f(uint16_t(rv.x >> 16));
                        acc[i][j][4 * g + 2] += h2f(uint16_t(rv.y & 0xffff));
                        acc[i][j][4 * g + 3] += h2f(uint16_t(rv.y >> 16));
                    }
            }
        }
    }
    if (stats) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            if (!pix_ok(j * 32 + p)) continue;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    if (wch0 + i * 32 + 8 * g + 4 * h >= nout) continue;   // nout % 8 == 0: all four or none
#pragma unroll
                    for (int r = 4 * g; r < 4 * g + 4; ++r) {
                        const float v = acc[i][j][r];
                        ssum[i][r] += v;
                        ssq[i][r] = fmaf(v, v, ssq[i][r]);
                    }
                }
        }
    }
    auto pack = [&](float lo, float hi) -> uint32_t {
        return half ? pk2h(lo, hi) : pk2bf(lo, hi);
    };
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const uint32_t base = pix_off(j * 32 + p);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int ga = 8 * k, gb = 8 * k + 4;                  // registers of groups 2k and 2k + 1
                const uint32_t x0 = pack(acc[i][j][ga], acc[i][j][ga + 1]), x1 = pack(acc[i][j][ga + 2], acc[i][j][ga + 3]);
                const uint32_t y0 = pack(acc[i][j][gb], acc[i][j][gb + 1]), y1 = pack(acc[i][j][gb + 2], acc[i][j][gb + 3]);
                const auto s0 = __builtin_amdgcn_permlane32_swap(x0, y0, false, false);
                const auto s1 = __builtin_amdgcn_permlane32_swap(x1, y1, false, false);
                uint4 v = make_uint4(s0[0], s1[0], s0[1], s1[1]);
                const int co = i * 32 + 8 * (2 * k + h);               // channel offset within the wave
                const uint32_t off = base != OOB && wch0 + co < nout ? base + uint32_t(co) * 2u : OOB;
                if (accumulate) {                                      // gradient fan-in (bf16)
                    const uint4 old = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(yres, off, 0, 0));
                    uint32_t ww[4] = {v.x, v.y, v.z, v.w}, oo[4] = {old.x, old.y, old.z, old.w};
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        ww[e] = pk2bf(bf2f(bf16_t(ww[e] & 0xffff)) + bf2f(bf16_t(oo[e] & 0xffff)),
                                      bf2f(bf16_t(ww[e] >> 16)) + bf2f(bf16_t(oo[e] >> 16)));
                    v = make_uint4(ww[0], ww[1], ww[2], ww[3]);
                }
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v),
                                                       yres, off, 0, 0);
            }
    }
}

template <int TM, int TN, class PixOff, class PixOk>
__device__ __forceinline__ void epilogue_regs(f32x4 (&acc)[TM][TN], float (&ssum)[TM][4], float (&ssq)[TM][4],
                                              bool stats, int lane, int wch0, int nout,
                                              __amdgpu_buffer_rsrc_t yres, bool half, bool accumulate,
                                              PixOff pix_off, PixOk pix_ok) {
    epilogue_regs_x<TM, TN>(acc, ssum, ssq, stats, lane, wch0, nout, yres, half, accumulate, pix_off, pix_ok, nullptr,
                            pix_off);
}

}  // namespace ym
