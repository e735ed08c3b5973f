// Halo-staged persistent pipelined 3x3 stride-1 convolution (conv_hpipe.hip): applicability plan +
// launch, used by ym_conv_fwd / ym_conv_dgrad in conv.hip ahead of the other conv kernels.
#pragma once
#include "common.h"

namespace ym {

struct HPipePlan {
    int ok;          // the halo-pipelined kernel handles this conv
    int cfg;         // 0: 128-channel tiles, 1: 64-channel tiles, 2: 64 -> 64 with the weights resident in LDS
    int grid;        // workgroups (persistent; a multiple of 8 * channel tiles)
    int rows;        // rows of the BN statistics partials (= grid / channel tiles)
};

// selection policy (ym_conv_set_hpipe): -1 default (1); 0 never; 1 the weight-resident 64 -> 64 layers with >= 512 tiles;
// 2 every eligible layer
extern Policy g_hpipe_force;

HPipePlan hpipe_plan(const ym_conv_desc* d, int dgrad);
int hpipe_launch(const HPipePlan& p, const ym_conv_desc* d, int dgrad, const uint16_t* x, const uint16_t* w, void* y,
                 float* st_sum, float* st_sq, hipStream_t st);

}  // namespace ym
