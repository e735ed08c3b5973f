/*
 * libyolomi — kernel-selection policy overrides (tests, tuning and A/B measurement; not needed to train or infer).
 *
 * The shipping library decides every kernel, tile and split from the call's arguments alone.  These setters override
 * those decisions process-wide: the parity tests force every kernel instance onto shapes the defaults would route
 * elsewhere (tests/test_gpu_conv.py), and the A/B tools (tools/, bench.py YM_LIB_SET) compare policies in one process.
 * No setting changes a result beyond fp32 summation order.
 *
 * Threading contract (the entry points of yolomi.h are reentrant and thread-safe):
 *  - each policy is an atomic int: a setter racing a launch on another thread is not a data race — that launch
 *    runs entirely under the old or entirely under the new setting;
 *  - a setting applies to calls that START after the setter returns; nothing already enqueued changes;
 *  - answers derived from the policies (ym_conv_algo, ym_conv_kernel, ym_conv_fwd_eval_ok, every *_workspace_size)
 *    hold for the setting they were computed under.  ym_policy_generation() increases on every setter call: a
 *    caller that caches such an answer keys the cache on it (yolomi/graph.py does).  A workspace sized under one
 *    setting and passed to a call made under another is checked by that call: too small, and the call runs the
 *    form that needs none (ym_conv_fwd_eval: unsplit; ym_conv_wgrad: YM_ERR_ARG, no launch).
 * Every setter returns the previous value; out-of-range values restore the default.
 */
#ifndef YOLOMI_EXPERIMENTAL_H
#define YOLOMI_EXPERIMENTAL_H

#ifdef __cplusplus
extern "C" {
#endif

/* Number of setter calls so far (any setter of this header): a cache key for policy-dependent answers. */
unsigned ym_policy_generation(void);

/* Kernel selection as if the batch held n images (0: the real batch, the default): every size rule
 * and tile choice below evaluates at n, the launch geometry at the real batch — a small-batch parity
 * test runs the kernel instances of a large-batch step.  Returns the previous setting.  Process-wide;
 * not for use while other threads plan or launch convolutions. */
int ym_conv_set_select_batch(int n);
/* Selection policy of the halo-staged kernel for later calls: -1 default, 0 never, 1 wherever it
 * applies, 2 maps <= 24 wide, 3 (default) maps <= 48 wide or <= 64 output channels.  Returns the
 * previous setting.  Process-wide; not for use while other threads launch convolutions. */
int ym_conv_set_halo(int mode);
/* Selection policy of the persistent pipelined implicit GEMM (conv_pipe.hip) for later calls: -1
 * default, 0 never, 1 layers of >= 1024 256-pixel tiles with >= 128 output channels, 2 every eligible
 * layer of >= 256 tiles, 3 (default) every 1x1 and the 3x3 with >= 128 output channels (forward: or
 * inputs) at >= 256 tiles, never a stride-2 data gradient.  Returns the previous setting.
 * Process-wide, like ym_conv_set_halo. */
int ym_conv_set_pipe(int mode);
/* Selection policy of the direct register-weight kernel (conv_direct.hip: 32-128-channel 1x1 / 3x3
 * layers) for later calls: -1 default, 0 never, 1 maps of >= 1 M output pixels (default), 2 any size, 3 >= 200 k
 * output pixels.
 * Returns the previous setting.  Process-wide, like ym_conv_set_halo. */
int ym_conv_set_direct(int mode);
/* Selection policy of the halo-staged pipelined 3x3 stride-1 kernel (conv_hpipe.hip: 16x16-pixel tiles,
 * each 64-channel chunk of the 18x18 input halo staged once for all nine taps): -1 default, 0 never,
 * 1 the weight-resident 64 -> 64 layers with >= 512 tiles (default), 2 every eligible layer; returns the previous setting. */
int ym_conv_set_hpipe(int mode);
/* Workgroups per weight-gradient launch the split-K plan aims for (default 256, tuned in the training step where
 * the weight gradients share the GPU with the data gradients; <= 0 restores it).  Returns the previous setting.
 * Process-wide, like ym_conv_set_halo; a workspace size queried under one setting serves only that setting. */
int ym_wgrad_set_target(int wgs);
/* Fold policy of ym_conv_fwd_bn for later calls: -1 default (on), 0 never (conv, then ym_bn_finalize), 1 on.
 * Returns the previous setting.  Process-wide, like ym_conv_set_halo. */
int ym_conv_set_fold(int mode);
/* Stage / ring configuration of ym_conv_fwd_eval's implicit GEMM (0: 32-deep K stages x 3, 1: 64 x 3 (default),
 * 2: 64 x 4); <0 restores the default.  Returns the previous setting.  Process-wide, like ym_conv_set_halo. */
int ym_conv_set_eval_cfg(int cfg);
/* Eval GEMM outputs of <= 32 channels on a 128 x 32 tile (1, default; <0 restores it) or the 128 x 64 one (0).
 * Returns the previous setting. */
int ym_conv_set_eval_narrow(int on);
/* The small-grid K-split's tile threshold (yolomi.h ym_conv_fwd_eval_workspace_size): split layers of <= max_tiles
 * 128x64 tiles and >= 12 K stages (default 64; 0 never; <0 restores the default); returns the previous setting. */
int ym_conv_set_eval_split(int max_tiles);
/* The K-split's K-stage threshold (split layers of >= min_stages 64-deep stages; default 12; <0 restores it) and the
 * tile count at or below which an eval conv the halo kernel would take runs the 2-stage GEMM instead (default 0). */
int ym_conv_set_eval_split_nk(int min_stages);
/* Layers the pipelined implicit GEMM takes (>= 256 tiles: large maps / batches) run its eval instance (1, default;
 * <0 restores it) or, with 0, are not eval-epilogue cases (ym_conv_fwd + ym_bn_apply). */
int ym_conv_set_eval_pipe(int on);
/* Layers whose training kernel has no eval instance, run through one anyway (bit mask; default 0; <0 restores it):
 * bit 0 the halo kernel's 8-wave tile -> the 2-stage GEMM's eval instance, bit 1 the halo-pipelined 3x3 kernel ->
 * the halo C4 / 2-stage GEMM eval instances.  Returns the previous setting. */
int ym_conv_set_eval_route(int mask);
int ym_conv_set_eval_gemm_tiles(int max_tiles);
/* Policy of the fused backward statistics + finalize for later calls: -1 default (= 2), 0 never, 1 on maps up
 * to 25600 pixels (20x20 x 64 images), 2 up to 102400 (40x40 x 64).  Returns the previous setting.  Process-wide,
 * like ym_conv_set_halo. */
int ym_bn_set_bwd_fold(int mode);

#ifdef YM_EXPERIMENTS
/* Measurement library only (make -C yolo-scratch_amd/csrc exp -> libyolomi_exp.so; NOT exported by libyolomi.so):
 * conv_pipe experiment instances — 1 the 8-wave 256x128 tile, 10-13 ablations that skip DMAs or MFMAs (WRONG results
 * by design, for timing only), 20 the generic control path.  0 restores the shipped kernels. */
int ym_pipe_set_exp(int v);
/* MFMA shape of the persistent pipelined implicit GEMM (round 6, measured slower: profiles/r06/pipe_mfma_order_ab.txt):
 * 0 (default) v_mfma_f32_16x16x32 on the shipped tiles, 1 v_mfma_f32_32x32x16 on the same tiles, 2 v_mfma_f32_32x32x16 with the 256 x 128 tile on 8 waves of 64 x 64 instead
 * of 16 of 32 x 64.  Returns the previous setting. */
int ym_conv_set_pipe_mfma(int mode);
/* K-step issue order of the pipelined kernels (round 6, measured slower: profiles/r06/pipe_mfma_order_ab.txt):
 * 0 (default) stage DMAs first after the barrier, the next stage's fragment reads late; 1 every fragment read pinned ahead of the half step of MFMAs it covers.  Returns the
 * previous setting. */
int ym_conv_set_pipe_order(int mode);
/* Loop form of the pipelined kernel's single-class training instances (round 6): 0 one flat loop over the workgroup's K
 * steps, 1 nested tiles x K steps with each tile's first step peeled, 2 (default, shipped) as 1 with the LDS ring slot
 * carried as a byte offset.  Out of range restores 2.  Returns the previous setting. */
int ym_conv_set_pipe_loop(int mode);
/* Tap lookahead of the 3x3 weight-gradient kernel (round 6): 0 each tap's input fragments read right before its MFMAs,
 * 1 one tap ahead.  Out of range restores the shipped setting.  Returns the previous setting. */
int ym_wgrad_set_lookahead(int la);
/* K order of the pipelined kernel's single-class forward (round 6): 0 channel chunk innermost everywhere, 1 tap
 * innermost everywhere (the taps that re-read the same input pixels back to back), anything else (default) the shipped
 * rule — tap innermost on the stride-2 3x3 forwards reading maps >= 128 wide.  Returns the previous setting. */
int ym_conv_set_pipe_taporder(int mode);
/* Loop form of the pipelined kernel's eval instance (round 6): 2 the nested form the training instances ship, anything
 * else (default) the flat loop.  Returns the previous setting. */
int ym_conv_set_pipe_eval_loop(int mode);
#endif

#ifdef __cplusplus
}
#endif
#endif
