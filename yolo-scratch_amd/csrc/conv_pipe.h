// Persistent, software-pipelined implicit-GEMM convolution (conv_pipe.hip): applicability plan +
// launch, used by ym_conv_fwd / ym_conv_dgrad in conv.hip ahead of the halo kernel and the
// 2-stage implicit GEMM.
#pragma once
#include "common.h"

namespace ym {


struct PipePlan {
    int ok;          // the pipelined kernel handles this conv
    int cfg;         // tile configuration (conv_pipe.hip: kCfg)
    int grid;        // workgroups (persistent; a multiple of 8 * channel tiles)
    int rows;        // rows of the BN statistics partials (= grid / channel tiles)
};

// -1: default policy (3); 0 never; 1 layers of >= 1024 tiles, >= 128 channels; 2 >= 256
// tiles; 3 the wider rule of pipe_plan (ym_conv_set_pipe)
extern Policy g_pipe_force;
#ifdef YM_EXPERIMENTS
extern Policy g_pipe_order;     // K-step issue order of the pipelined kernels (conv_pipe / conv_hpipe RO; measurement only)
#endif

// dgrad = 0: forward conv described by d; 1: its data gradient
PipePlan pipe_plan(const ym_conv_desc* d, int dgrad);
// fold: the BatchNorm finalize as the launch's tail (ym_conv_fwd_bn; forward with statistics only) or null
int pipe_launch(const PipePlan& p, const ym_conv_desc* d, int dgrad, const uint16_t* x, const uint16_t* w, void* y,
                const float* bias, float* st_sum, float* st_sq, hipStream_t st, const ym_bn_fold* fold = nullptr);
// the eval-mode Conv block instance (ym_conv_fwd_eval): d's forward with the running-statistics BatchNorm / SiLU /
// residual e in the epilogue, into the fp16 y view (pipe_eval_ok: the plan's single-class forward); 0 on success
bool pipe_eval_ok(const PipePlan& p, const ym_conv_desc* d);
int pipe_launch_eval(const PipePlan& p, const ym_conv_desc* d, const uint16_t* x, const uint16_t* w, uint16_t* y,
                     const EvalArgs& e, hipStream_t st);

}  // namespace ym
