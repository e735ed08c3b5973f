// Direct MFMA convolution with register-resident weights (conv_direct.hip): applicability plan +
// launch, tried by ym_conv_fwd / ym_conv_dgrad in conv.hip before the other conv kernels.
#pragma once
#include "common.h"

namespace ym {

struct DirectPlan {
    int ok;          // the direct kernel handles this conv
    int variant;     // template instance (conv_direct.hip: kVariants)
    int grid;        // workgroups (= rows of the BN statistics partials)
};

// -1: default policy; 0 never; 1 maps of >= 1 M output pixels; 2 any size
extern Policy g_direct_force;

// inference: a forward without BatchNorm statistics (the eval path) — under the default policy it takes the kernel from
// 200 k output pixels (the 160x160 stage from 8 images up) instead of 1 M
DirectPlan direct_plan(const ym_conv_desc* d, int dgrad, bool inference = false);
int direct_launch(const DirectPlan& p, const ym_conv_desc* d, int dgrad, const uint16_t* x, const uint16_t* w,
                  void* y, float* st_sum, float* st_sq, hipStream_t st);

}  // namespace ym
