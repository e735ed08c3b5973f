// Halo-staged 3x3 stride-1 convolution (conv_halo.hip): applicability plan + launch, used by
// ym_conv_fwd / ym_conv_dgrad in conv.hip before they fall back to the implicit GEMM.
#pragma once
#include "common.h"

namespace ym {


struct HaloPlan {
    int ok;              // the halo kernel handles this conv
    int cfg;             // 0: 8 waves, 256 px x 128 ch tiles; 1: 4 waves, 128 px x 64 ch
    int TH, TW, RT, CT;  // tile rectangle, tiles per image (rows, cols)
    int ntiles, nco;     // pixel tiles, channel tiles
    int gx;              // grid x (= rows of the BN statistics partials)
};

// -1: default policy (3); 0 never; 1 wherever it applies; 2 maps <= 24 wide; 3 maps <= 48
// wide or <= 64 output channels (ym_conv_set_halo)
extern Policy g_halo_force;

// dgrad = 0: forward conv described by d; 1: its data gradient
HaloPlan halo_plan(const ym_conv_desc* d, int dgrad);
// fold: the BatchNorm finalize as the launch's tail (ym_conv_fwd_bn; forward with statistics only) or null
// ev: the eval-mode Conv block epilogue (ym_conv_fwd_eval: forward, fp16 output view, no statistics) or null
int halo_launch(const HaloPlan& p, const ym_conv_desc* d, int dgrad, const uint16_t* x, const uint16_t* w, void* y,
                const float* bias, float* st_sum, float* st_sq, hipStream_t st, const ym_bn_fold* fold = nullptr,
                const EvalArgs* ev = nullptr);

}  // namespace ym
