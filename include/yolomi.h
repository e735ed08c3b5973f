/*
 * libyolomi — MI355X (gfx950) C-ABI for the YOLOv11 training/eval hot path.
 *
 * The reference (Pratye/yolo-scratch) has no native code: its hot path is
 * PyTorch ATen called from Python.  Every entry point below replaces one
 * implicit ATen call site of the reference (cited per function, paths
 * relative to /root/reference/yolo_scratch_cuda/).  The Python drop-in
 * modules (yolo-scratch_amd/{models,losses,train_yolo11_cuda.py}) bind these
 * with ctypes.
 *
 * Conventions
 *  - All pointers are DEVICE pointers unless stated; buffers are allocated by
 *    the caller (PyTorch caching allocator); the library never allocates or
 *    frees caller memory and keeps no TENSOR state between calls.  The only
 *    process-wide state is configuration: the kernel selection policies, whose
 *    override setters live in yolomi_experimental.h (tests / tuning only, atomic, see the contract
 *    there); a policy never changes a result beyond fp32 summation order.  The library reads no
 *    environment variables.
 *  - `stream` is a hipStream_t (0 = legacy default stream); every call is
 *    asynchronous on it and performs no device-wide synchronisation.
 *  - Activations are NHWC.  An "activation view" is (base pointer, batch
 *    stride, pixel stride `ld`), all in elements; channel c of pixel p of
 *    image n lives at base[n*bstride + p*ld + c].  Channel slices (concat /
 *    split) are expressed by offsetting `base` and keeping `ld`.
 *  - 16-bit tensors are raw uint16 bit patterns.  Activations are fp16,
 *    gradients bf16, pre-BatchNorm conv outputs fp16, master weights fp32
 *    (converted per step to an fp16 forward copy and a bf16 dgrad copy).
 *  - Return value: YM_OK (0) or a negative YM_ERR_*; ym_last_error() gives a
 *    thread-local message.  Nothing throws across the ABI.
 */
#ifndef YOLOMI_H
#define YOLOMI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define YM_OK 0
#define YM_ERR_ARG -1
#define YM_ERR_HIP -2
#define YM_ERR_UNSUPPORTED -3

const char* ym_last_error(void);
int ym_version(void);

/* ------------------------------------------------------------------ postprocess
 * Replaces decode_predictions_for_metrics / nms_simple /
 * calculate_iou_batch_simple (train_yolo11_cuda.py:265-437).
 */

/* IoU of one box against m boxes, fp32, reference op order
 * (calculate_iou_batch_simple, train_yolo11_cuda.py:402-437). */
int ym_iou_row(const float* box1, const float* boxes2, int64_t m, float* out, void* stream);

/* Workspace bytes for ym_decode_nms / ym_nms_batched with B images of N rows. */
size_t ym_nms_workspace_size(int64_t B, int64_t N);

/* decode_predictions_for_metrics (train_yolo11_cuda.py:265-358) for a batch.
 * pred: (B, N, 4+C) fp32 rows [x, y, w, h, score_0..score_{C-1}] with row
 * stride `row_stride` (>= 4+C) and image stride `img_stride` (elements).
 * Per image b: rows with max score > conf are kept in row order, converted
 * xywh->xyxy, greedy class-agnostic NMS (suppress IoU > iou_thr), then
 * boxes / img_size clamped to [0,1].  Outputs (capacity N per image, image b
 * at offset b*N): out_count[b], out_boxes[(b*N+k)*4..], out_scores, out_labels
 * (argmax class, int64), out_index (row index of the kept box within the
 * filtered set, i.e. nms_simple's keep list), in descending-score order. */
int ym_decode_nms(const float* pred, int64_t B, int64_t N, int64_t C, int64_t row_stride, int64_t img_stride,
                  float conf, float iou_thr, float img_size, void* workspace, size_t workspace_bytes,
                  int32_t* out_count, float* out_boxes, float* out_scores, int64_t* out_labels,
                  int64_t* out_index, void* stream);
/* The same with a row's elements `col_stride` apart (1: ym_decode_nms): the anchor-major view pred.transpose(1, 2)
 * of the (B, 4+C, A) eval output is read in place (row_stride 1, col_stride A), no contiguous copy. */
int ym_decode_nms_strided(const float* pred, int64_t B, int64_t N, int64_t C, int64_t row_stride,
                          int64_t img_stride, int64_t col_stride, float conf, float iou_thr, float img_size,
                          void* workspace, size_t workspace_bytes, int32_t* out_count, float* out_boxes,
                          float* out_scores, int64_t* out_labels, int64_t* out_index, void* stream);

/* nms_simple (train_yolo11_cuda.py:361-399) on one set of n xyxy boxes:
 * keep[0..*count) are indices into boxes in kept (score-descending) order. */
int ym_nms(const float* boxes, const float* scores, int64_t n, float iou_thr, void* workspace,
           size_t workspace_bytes, int64_t* keep, int32_t* count, void* stream);


/* ------------------------------------------------------------------ detection metrics
 * Replaces evaluate_detections / calculate_iou_batch / calculate_ap
 * (utils/metrics.py:49-81, :84-274, :277-323).
 */

/* Workspace bytes for ym_eval_detections. */
size_t ym_eval_workspace_size(int64_t n_img, int64_t n_pred, int n_thr);

/* evaluate_detections over n_img images, all on the device, no host sync.
 * Predictions of image b are rows pred_off[b]..pred_off[b+1) of pred_boxes (xyxy fp32,
 * n_pred x 4) / pred_scores; its GT boxes rows gt_off[b]..gt_off[b+1) of gt_boxes
 * (n_gt x 4).  pred_off / gt_off are device int64 arrays of n_img+1 prefix offsets.
 * thresholds (host, n_thr <= 15 doubles) are the IoU thresholds matched at once;
 * the first n_ap give mAP50-95 (their mean) and mAP50 (the first); pr_index selects
 * the threshold precision / recall are counted at (the reference uses 0.5).
 * max_gt_per_img <= 4096.  out (device, n_thr + 7 doubles): AP per threshold, then
 * precision, recall, mAP50, mAP50-95, TP, FP, predictions kept by conf. */
int ym_eval_detections(const float* pred_boxes, const float* pred_scores, const int64_t* pred_off,
                       const float* gt_boxes, const int64_t* gt_off, int64_t n_img, int64_t n_pred, int64_t n_gt,
                       int64_t max_gt_per_img, const double* thresholds, int n_thr, int n_ap, int pr_index,
                       float conf, void* workspace, size_t workspace_bytes, double* out, void* stream);

/* calculate_ap (utils/metrics.py:277-323) on one flat detection list: scores[n] and
 * is_tp[n] (0/1); workspace ym_eval_workspace_size(1, n, 1).  out (device, 8 doubles):
 * out[0] = AP (0 when n_gt == 0 or n == 0), the rest as ym_eval_detections. */
int ym_eval_ap(const float* scores, const uint8_t* is_tp, int64_t n, int64_t n_gt, void* workspace,
               size_t workspace_bytes, double* out, void* stream);

/* calculate_iou_batch (utils/metrics.py:49-81): out[i*m+j] = IoU(boxes1[i], boxes2[j]),
 * xyxy fp32 in the reference's op order. */
int ym_iou_matrix(const float* boxes1, const float* boxes2, int64_t n, int64_t m, float* out, void* stream);

/* ------------------------------------------------------------------ convolution
 * Replaces nn.Conv2d forward/backward inside Conv (models/yolo11_modules.py:21-33)
 * and the Detect head's bias convs (:221-234).  NHWC; fp16 forward / bf16 backward MFMA, fp32 accumulate.
 */
typedef struct {
    int32_t n, h, w, cin;      /* input  (n, h, w, cin)  */
    int32_t oh, ow, cout;      /* output (n, oh, ow, cout) */
    int32_t k, stride, pad;    /* square kernel */
    int64_t x_bs, x_ld;        /* input view: image stride, pixel stride (elements) */
    int64_t y_bs, y_ld;        /* output view */
    int32_t out_f32;           /* fwd output: 0 bf16, 1 fp32, 2 fp16 (pre-BatchNorm z) */
    int32_t accumulate;        /* add into the destination instead of overwriting */
} ym_conv_desc;

typedef struct {
    const float* src;          /* fp32 OIHW master weight */
    uint16_t* dst_fwd;         /* fp16 [cout][kh][kw][cin] (forward) or NULL */
    uint16_t* dst_t;           /* bf16 [cin][kh][kw][cout] (dgrad) or NULL */
    int64_t elem_offset;       /* running element offset of this entry */
    int32_t cout, cin, kh, kw;
    int32_t cout_t;            /* row length of dst_t (>= cout; zero padding is the caller's) */
} ym_wprep_entry;

/* Rows of the BN statistics partials of the 2-stage implicit GEMM's forward alone, for m output pixels
 * (kept for callers that size by shape only; NOT the row count of other conv kernels — use
 * ym_conv_fwd_stat_rows). */
int ym_conv_stat_blocks(int64_t m, int cout);
/* Rows of the BN statistics partials ym_conv_fwd writes for this bias-free conv: the kernels use
 * different grids (the direct kernel: CUs x occupancy; the pipelined kernels: 256 / channel tiles;
 * the halo kernel: its tile grid; the implicit GEMM: ym_conv_stat_blocks).  stat_sum / stat_sq MUST
 * hold ym_conv_fwd_stat_rows(d) x cout floats each, with the selection policies below unchanged
 * between this call and the forward. */
int ym_conv_fwd_stat_rows(const ym_conv_desc* d);
/* Which kernel ym_conv_fwd (dgrad = 0, bias-free) / ym_conv_dgrad (dgrad = 1) runs for d: 4 = the
 * halo-staged pipelined 3x3 kernel, 3 = the direct register-weight kernel, 2 = the persistent
 * pipelined implicit GEMM, 1 = the halo-staged 3x3 stride-1 kernel, 0 = the 2-stage implicit GEMM. */
int ym_conv_algo(const ym_conv_desc* d, int dgrad);
/* The kernel INSTANCE a bias-free forward (dir 0), data gradient (1) or weight gradient (2) of d runs:
 * returns an id (algo x 1000 + template instance; weight gradients >= 10000; -1 for a bad argument) and,
 * if name != NULL, writes its name (e.g. "direct v3", "pipe 256x128", "wgrad3 s2 64x64 8x8 deep"). */
int ym_conv_kernel(const ym_conv_desc* d, int dir, char* name, int name_len);
/* y = conv(x, w) (+bias), x fp16 NHWC view, w fp16 [cout][kh][kw][cin], k in 1..3; optional per-block
 * channel sum / sum-of-squares partials [ym_conv_fwd_stat_rows(d)][cout] for training BatchNorm
 * (BatchNorm2d batch stats; not together with a bias).  accumulate is not supported for fp16 output
 * (out_f32 = 2). */
int ym_conv_fwd(const ym_conv_desc* d, const uint16_t* x, const uint16_t* w, void* y, const float* bias,
                float* stat_sum, float* stat_sq, void* stream);
/* dx (+)= conv_transpose(dz, w) using the [cin][kh][kw][cout] weight copy. */
int ym_conv_dgrad(const ym_conv_desc* d, const uint16_t* dz, const uint16_t* wt, uint16_t* dx, void* stream);
/* Weight gradient dW (fp32 OIHW) = sum over output pixels of dz (x) x, overwriting dw_oihw or adding
 * into it (accumulate = 1).  The K (pixel) axis is split over workgroups; the fp32 partials go to
 * `workspace` (ym_conv_wgrad_workspace_size bytes) and are reduced by the library: no atomics
 * into, and no zero-fill of, dw_oihw.  dz bf16 with the y_* view, x fp16 with the x_* view. */
size_t ym_conv_wgrad_workspace_size(const ym_conv_desc* d);
int ym_conv_wgrad(const ym_conv_desc* d, const uint16_t* dz, const uint16_t* x, void* workspace,
                  size_t workspace_bytes, float* dw_oihw, int accumulate, void* stream);
/* Stem conv (3x3) on the fp32 NCHW image of ch = 1..4 planes (model.0, yaml row 0: Conv(ch, c, 3, 2); the reference's
 * build_yolo11(ch=...), models/yolo11_model.py:23, 258); y = NULL: statistics only. */
int ym_conv_first_fwd(const float* img, const float* w_oihw, uint16_t* y, float* stat_sum, float* stat_sq, int n,
                      int h, int w, int oh, int ow, int cout, int stride, int pad, int ch, int blocks, void* stream);
/* Eval-mode stem Conv block in one launch (inference): the stem conv, BatchNorm with the running-statistics scale /
 * shift, SiLU if act, written into the fp16 activation view y (strides y_bs / y_ld, multiples of 8, y 16-B aligned)
 * — what ym_conv_first_fwd + ym_bn_apply compute, without the statistics, the fp16 z and the apply launch. */
int ym_conv_first_fwd_eval(const float* img, const float* w_oihw, const float* scale, const float* shift, int act,
                           uint16_t* y, int64_t y_bs, int64_t y_ld, int n, int h, int w, int oh, int ow, int cout,
                           int stride, int pad, int ch, void* stream);
/* dW (+)= stem weight gradient (ch image planes); per-workgroup partials in `workspace`
 * (ym_conv_first_wgrad_workspace_size bytes), summed in a fixed order (bit-reproducible). */
size_t ym_conv_first_wgrad_workspace_size(int cout, int ch);
int ym_conv_first_wgrad(const uint16_t* dz, const float* img, float* dw_oihw, int n, int h, int w, int oh, int ow,
                        int cout, int stride, int pad, int ch, float* workspace, size_t workspace_bytes, void* stream);
size_t ym_stem_bwd_wgrad_workspace_size(int cout);
/* Stored-z stem backward: dz = BatchNorm-backward apply of dy on the STORED fp16 z (dense
 * [m][cout]) straight into the weight-gradient partials (dz never written) — replaces
 * ym_bn_bwd_apply + ym_conv_first_wgrad; cout 16 / 32 / 64; workspace ym_stem_bwd_wgrad_workspace_size(cout). */
int ym_stem_bwd_wgrad_stored(const uint16_t* dy, int64_t d_bs, int64_t d_ld, const uint16_t* z, const float* img,
                             const float* bnv, const float* coef, float* dw_oihw, float* workspace,
                             size_t workspace_bytes, int n, int h, int w, int oh, int ow, int cout, int stride, int pad,
                             void* stream);
/* Depthwise 3x3 s1 p1 (Attention.pe, yolo11_modules.py:122); input channel c reads source
 * channel (c / gsz) * gstride + goff + c % gsz of the x view. */
int ym_dw3x3_fwd(const uint16_t* x, int64_t x_bs, int64_t x_ld, int gsz, int gstride, int goff, const float* w,
                 uint16_t* y, float* stat_sum, float* stat_sq, int n, int h, int wd, int c, int blocks, void* stream);
/* Eval-mode form in one launch: + BatchNorm with the running-statistics scale / shift, SiLU if act, + the fp16
 * residual view res (NULL: none; strides multiples of 4) into the fp16 y view (strides multiples of 8, 16-B aligned) —
 * ym_dw3x3_fwd + ym_bn_apply without the statistics, the z round trip and the apply launch. */
int ym_dw3x3_fwd_eval(const uint16_t* x, int64_t x_bs, int64_t x_ld, int gsz, int gstride, int goff, const float* w,
                      const float* scale, const float* shift, int act, const uint16_t* res, int64_t r_bs, int64_t r_ld,
                      uint16_t* y, int64_t y_bs, int64_t y_ld, int n, int h, int wd, int c, void* stream);
size_t ym_dw3x3_bwd_workspace_size(int c);
int ym_dw3x3_bwd(const uint16_t* x, int64_t x_bs, int64_t x_ld, int gsz, int gstride, int goff, const float* w,
                 const uint16_t* dz, uint16_t* dx, int64_t dx_bs, int64_t dx_ld, float* dw, int n, int h, int wd,
                 int c, int accumulate, float* workspace, size_t workspace_bytes, void* stream);
/* All conv weights fp32 OIHW -> fp16 forward / bf16 dgrad layouts in one launch (table in device memory).
 * ym_prep_weights_fwd: the fp16 forward copies only (dst_t ignored) — for tables without data-gradient copies
 * (an eval plan's): one grid row of workgroups, no LDS tile. */
int ym_prep_weights(const ym_wprep_entry* table_dev, int n_entries, int64_t total_elems, void* stream);
int ym_prep_weights_fwd(const ym_wprep_entry* table_dev, int n_entries, int64_t total_elems, void* stream);

/* ------------------------------------------------------------------ BatchNorm2d (train) + SiLU
 * Replaces BatchNorm2d + the shared in-place SiLU of Conv (models/yolo11_modules.py:24-33;
 * eps 1e-3 / momentum 0.03 from yolo11_model.py:183-185).  z is the dense (m, c) conv output in
 * fp16 (written by ym_conv_fwd with out_f32 = 2); dz (bf16) may overwrite it in place.
 */
/* scratch for the two-level partial reductions of ym_bn_finalize / ym_bn_bwd_finalize: fp64 rows
 * plus ticket counters.  Zero it once before first use (the library leaves the counters at zero
 * after every call); calls sharing one workspace must be ordered (same stream). */
size_t ym_bn_workspace_size(int c);
/* BatchNorm parameters for ym_conv_fwd_bn: the arguments of ym_bn_finalize after the statistics rows. */
typedef struct {
    const float* gamma;
    const float* beta;
    float* running_mean;       /* running statistics (momentum update) or NULL */
    float* running_var;
    int64_t* num_batches_tracked;
    float* scale;              /* outputs, [c] each: gamma * rstd, beta - mean * scale, mean, rstd */
    float* shift;
    float* mean;
    float* rstd;
    void* workspace;           /* ym_bn_workspace_size(c) bytes, zeroed once (shared with ym_bn_finalize) */
    double count;              /* elements per channel (n * oh * ow) */
    float momentum;
    float eps;
} ym_bn_fold;
/* Conv forward + BatchNorm statistics AND their finalize: ym_conv_fwd (stat_sum / stat_sq as there, bias-free,
 * fp16 z) followed by ym_bn_finalize over its rows, with the same outputs.  Where ym_conv_fwd_bn_fused(d) is 1
 * the finalize runs as the conv launch's tail (the last workgroup of each channel tile folds the tile's rows in
 * fp64, fixed order) instead of a second launch; elsewhere the two launches run in order. */
int ym_conv_fwd_bn_fused(const ym_conv_desc* d);
int ym_conv_fwd_bn(const ym_conv_desc* d, const uint16_t* x, const uint16_t* w, void* y, float* stat_sum,
                   float* stat_sq, const ym_bn_fold* bn, void* stream);
int ym_bn_finalize(const float* part_sum, const float* part_sq, int parts, int c, double count, const float* gamma,
                   const float* beta, float* running_mean, float* running_var, int64_t* num_batches_tracked,
                   float momentum, float eps, float* scale, float* shift, float* mean, float* rstd, void* workspace,
                   void* stream);
/* Eval-mode Conv block in ONE launch (inference): conv -> BatchNorm with the running-statistics scale / shift
 * (ym_bn_eval_coeff[_batch]) -> SiLU if act -> + residual, written into the fp16 activation view y — what
 * ym_conv_fwd (fp16 z) + ym_bn_apply compute, without the z round trip and the apply launch (Conv.forward of
 * yolo11_modules.py:21-47 in eval mode).  d describes the conv with d->y_bs / d->y_ld the OUTPUT VIEW's strides
 * (out_f32 = 2, accumulate 0); the residual (or NULL) is an fp16 view with strides r_bs / r_ld (elements, multiples
 * of 4).  ym_conv_fwd_eval_ok(d) is 1 where the kernel this conv selects has the eval epilogue (the halo-staged 3x3
 * kernel's 4-wave tile, the 2-stage implicit GEMM); elsewhere run ym_conv_fwd + ym_bn_apply.  Bias-free convs only. */
int ym_conv_fwd_eval_ok(const ym_conv_desc* d);
/* Small grids (a bs-1 forward's late layers: a few dozen tiles, each walking a long K serially) run as a K-split: the
 * GEMM launch writes ks fp32 partial slices into the caller's workspace and a second launch applies BatchNorm / SiLU /
 * residual to their sum.  ym_conv_fwd_eval_workspace_size(d) is the workspace that takes (0: one launch); with a
 * NULL or smaller workspace the call runs unsplit.  By default layers of <= 64 128x64 tiles and >= 12 K stages split
 * (yolomi_experimental.h ym_conv_set_eval_split); a workspace size holds for the policy it was queried under. */
size_t ym_conv_fwd_eval_workspace_size(const ym_conv_desc* d);
int ym_conv_fwd_eval(const ym_conv_desc* d, const uint16_t* x, const uint16_t* w, const float* scale,
                     const float* shift, int act, const uint16_t* res, int64_t r_bs, int64_t r_ld, uint16_t* y,
                     void* workspace, size_t workspace_bytes, void* stream);
/* Eval-mode coefficients of many BatchNorm layers in ONE launch (the eval forward's per-layer
 * ym_bn_eval_coeff calls were 77 launches per YOLOv11-s forward); table in device memory. */
typedef struct ym_bn_eval_entry {
    const float* gamma; const float* beta; const float* running_mean; const float* running_var;
    float* scale; float* shift;
    int32_t c; float eps;
} ym_bn_eval_entry;
int ym_bn_eval_coeff_batch(const ym_bn_eval_entry* table_dev, int n_entries, void* stream);
int ym_bn_eval_coeff(int c, const float* gamma, const float* beta, const float* running_mean,
                     const float* running_var, float eps, float* scale, float* shift, void* stream);
/* out_view = act(z*scale+shift) (+ res_view); act: 0 identity, 1 SiLU; hw = pixels per image */
int ym_bn_apply(const uint16_t* z, int64_t m, int c, int hw, const float* scale, const float* shift, int act,
                const uint16_t* res, int64_t r_bs, int64_t r_ld, uint16_t* out, int64_t o_bs, int64_t o_ld,
                float* out32, void* stream);   /* out32: optional fp32 dense copy (SPPF pool chain) */
int ym_bn_bwd_blocks(int64_t m, int c);
int ym_bn_bwd_reduce(const uint16_t* dy, int64_t d_bs, int64_t d_ld, const uint16_t* z, int64_t m, int c, int hw,
                     const float* scale, const float* shift, const float* mean, const float* rstd, int act,
                     float* part_sum, float* part_dot, void* stream);
int ym_bn_bwd_finalize(const float* part_sum, const float* part_dot, int parts, int c, double count,
                       const float* gamma, const float* rstd, float* dgamma, float* dbeta, int accumulate,
                       float* coef, void* workspace, void* stream);
/* Backward statistics AND finalize in one launch on the small maps (m <= 102400 pixels = 40x40 x 64
 * images, c % 64 == 0):
 * ym_bn_bwd_reduce followed by ym_bn_bwd_finalize over its rows, with the same outputs (dgamma / dbeta /
 * coef; part_sum / part_dot as scratch rows, ym_bn_bwd_blocks(m, c) x c floats each).  Where
 * ym_bn_bwd_fold_ok(m, c) is 0 it runs those two launches. */
int ym_bn_bwd_fold_ok(int64_t m, int c);
int ym_bn_bwd_reduce_fold(const uint16_t* dy, int64_t d_bs, int64_t d_ld, const uint16_t* z, int64_t m, int c, int hw,
                          const float* scale, const float* shift, const float* mean, const float* rstd, int act,
                          float* part_sum, float* part_dot, const float* gamma, float* dgamma, float* dbeta,
                          int accumulate, float* coef, void* workspace, void* stream);
int ym_bn_bwd_apply(const uint16_t* dy, int64_t d_bs, int64_t d_ld, const uint16_t* z, int64_t m, int c, int hw,
                    const float* scale, const float* shift, const float* mean, const float* rstd, int act,
                    const float* coef, uint16_t* dz, void* stream);
/* ym_bn_bwd_apply that also writes the residual branch's gradient from the same dy read:
 * dres (+)= dy into the bf16 view (r_bs, r_ld) — the shortcut of Bottleneck (yolo11_modules.py:47)
 * and Attention.pe (:134); replaces a separate ym_view_axpy pass. */
int ym_bn_bwd_apply_res(const uint16_t* dy, int64_t d_bs, int64_t d_ld, const uint16_t* z, int64_t m, int c, int hw,
                        const float* scale, const float* shift, const float* mean, const float* rstd, int act,
                        const float* coef, uint16_t* dz, uint16_t* dres, int64_t r_bs, int64_t r_ld,
                        int r_accumulate, void* stream);

/* ------------------------------------------------------------------ graph ops
 * SPPF max-pool (yolo11_modules.py:92-105), nearest 2x upsample (yaml head rows 11, 14),
 * C2PSA attention core (yolo11_modules.py:124-136), view conversions, Detect grad split.
 */
/* SPPF's chained 5x5 / stride 1 / pad 2 pools on fp32 values (first-max tie semantics of the fp32
 * reference).  Forward: y (dense fp32), code (dense uint8 window argmax kh*5+kw) and an fp16 copy
 * into the view yv.  Backward (gather over the argmax codes, no atomics):
 * out = init_view (bf16, optional) + sum of dy over the windows whose argmax is the pixel, written
 * to dx (dense fp32, optional) and/or the bf16 view dxv (added to it when accumulate). */
/* SPPF's three chained 5x5 pools in one launch per direction (models/yolo11_modules.py:100-104),
 * the chain kept in LDS (maps with h*w*cg*13 <= 96 KiB, cg = 8 or 4 channels per block; see
 * ym_sppf_supported).  fwd: x = fp32 cv1 output (m, c); code = 3 argmax planes (m, c) each;
 * y1..y3 = the fp16 concat slices (common bs / ld); p_out (optional) = the fp32 pool outputs as 3
 * planes.  bwd: g1..g3 = the bf16 gradients of the slices (common bs / ld); the routed gradient of
 * slice 0 written (or accumulated) into dxv, optionally also as fp32 into dx32.  Bit-identical to
 * three chained ym_maxpool5_f32_fwd / _bwd calls. */
int ym_sppf_supported(int h, int w, int c);
int ym_sppf_fwd(const float* x, uint8_t* code, uint16_t* y1, uint16_t* y2, uint16_t* y3, int64_t y_bs, int64_t y_ld,
                float* p_out, int n, int h, int w, int c, void* stream);
int ym_sppf_bwd(const uint8_t* code, const uint16_t* g1, const uint16_t* g2, const uint16_t* g3, int64_t g_bs,
                int64_t g_ld, uint16_t* dxv, int64_t v_bs, int64_t v_ld, int accumulate, float* dx32, int n, int h,
                int w, int c, void* stream);
int ym_maxpool5_f32_fwd(const float* x, float* y, uint8_t* code, uint16_t* yv, int64_t y_bs, int64_t y_ld, int n,
                        int h, int w, int c, void* stream);
int ym_maxpool5_f32_bwd(const uint8_t* code, const float* dy, const uint16_t* init, int64_t i_bs, int64_t i_ld,
                        float* dx, uint16_t* dxv, int64_t v_bs, int64_t v_ld, int accumulate, int n, int h, int w,
                        int c, void* stream);
int ym_upsample2_fwd(const uint16_t* x, int64_t x_bs, int64_t x_ld, uint16_t* y, int64_t y_bs, int64_t y_ld, int n,
                     int h, int w, int c, void* stream);
int ym_upsample2_bwd(const uint16_t* dy, int64_t d_bs, int64_t d_ld, uint16_t* dx, int64_t x_bs, int64_t x_ld, int n,
                     int h, int w, int c, int accumulate, void* stream);
int ym_view_to_f32(const uint16_t* x, int64_t bs, int64_t ld, float* y, int64_t m, int c, int hw, void* stream);
int ym_f32_to_view(const float* x, uint16_t* y, int64_t bs, int64_t ld, int64_t m, int c, int hw, int accumulate,
                   void* stream);
/* dhead (B, A, 64+nc) fp32 rows of one pyramid level -> bf16 dz for the box / cls 1x1 convs
 * (cls zero-padded to a multiple of 8 channels, dz_cls rows of round_up(nc, 8)) and bias grads (+=); nc 1..1024. */
size_t ym_head_grad_workspace_size(void);
int ym_head_grad(const float* dhead, int64_t a_total, int64_t a_off, int hw, int64_t m, int nc, uint16_t* dz_box,
                 uint16_t* dz_cls, float* dbias_box, float* dbias_cls, float* workspace, size_t workspace_bytes,
                 void* stream);
int ym_attn_fwd(const uint16_t* qkv, int64_t q_bs, int64_t q_ld, int b, int heads, int n, int key_dim, int head_dim,
                float scale, uint16_t* out, int64_t o_bs, int64_t o_ld, float* lse, void* stream);
size_t ym_attn_workspace_size(int b, int heads, int n);
int ym_attn_bwd(const uint16_t* qkv, int64_t q_bs, int64_t q_ld, const uint16_t* out, int64_t o_bs, int64_t o_ld,
                const uint16_t* dout, int64_t d_bs, int64_t d_ld, const float* lse, int b, int heads, int n,
                float scale, float* workspace, uint16_t* dqkv, int64_t g_bs, int64_t g_ld, int acc_q, int acc_k,
                int acc_v, void* stream);
/* Concat.forward (models/yolo11_modules.py:284-285) of contiguous tensors along one dimension, and
 * its backward: `rows` runs of `width_bytes`, source pitch `src_pitch`, destination pitch `dst_pitch`
 * (bytes).  A device-to-device strided copy on the stream. */
int ym_copy2d(void* dst, int64_t dst_pitch, const void* src, int64_t src_pitch, int64_t width_bytes, int64_t rows,
              void* stream);
/* dst_view = src_view (+ dst_view when accumulate); src NULL zero-fills dst */
int ym_view_axpy(const uint16_t* x, int64_t x_bs, int64_t x_ld, uint16_t* y, int64_t y_bs, int64_t y_ld, int64_t m,
                 int c, int hw, int accumulate, int half, void* stream);   /* half: 1 fp16 data, 0 bf16 */

/* ------------------------------------------------------------------ detection loss + decode
 * Replaces v8DetectionLoss.__call__ and its TaskAlignedAssigner / BboxLoss
 * (losses/yolo_v8_loss.py:64-538) and Detect.inference (models/yolo11_modules.py:248-266).
 * head: (B, A, 64+nc) fp32 rows, levels concatenated (level l: h[l] x w[l] anchors, stride[l]).
 * Host arrays: level_h, level_w, strides.  Targets: the collate batch dict on the device
 * (batch_idx int64 (N,), cls int64 (N,1), bboxes fp32 (N,4) normalised xyxy); M = max boxes
 * per image.  gt_box (B,M,4) / gt_lab (B,M) / gt_valid (B,M) are caller-allocated outputs.
 * out[0] = loss (sum(items) * B), out[1..3] = items (box, cls, dfl with gains), out[4] = tss,
 * out[5] = number of foreground anchors.
 */
size_t ym_loss_workspace_size(int64_t B, int64_t A, int M);
int ym_loss_fwd(const float* head, int64_t B, int64_t A, int nc, int nl, const int* level_h, const int* level_w,
                const float* strides, const int64_t* batch_idx, const int64_t* cls, const float* bboxes,
                int64_t n_targets, int M, float imgsz_h, float imgsz_w, void* workspace, size_t workspace_bytes,
                float* gt_box, float* gt_lab, int* gt_valid, float* out, void* stream);
/* dhead = d(out[0] * grad_out[0]) / d head, using the assignment left in the workspace by ym_loss_fwd. */
int ym_loss_bwd(const float* head, int64_t B, int64_t A, int nc, int nl, const int* level_h, const int* level_w,
                const float* strides, int M, void* workspace, size_t workspace_bytes, const float* gt_box,
                const float* gt_lab, const float* out, const float* grad_out, float* dhead, void* stream);
/* Device pointers to the assignment (target_gt_idx, fg_mask, target-score magnitude) in the workspace. */
int ym_loss_assignment(void* workspace, int64_t B, int64_t A, int M, const int** tgi, const int** fg,
                       const float** norm);
/* TaskAlignedAssigner.forward (losses/yolo_v8_loss.py:78-180) on explicit tensors, for M >= 1 (the
 * M = 0 early return :100-108 is the caller's): pd_scores (B,A,nc) probabilities, pd_bboxes (B,A,4)
 * pixel xyxy, anc_points (A,2) pixels, gt_labels (B,M) float, gt_bboxes (B,M,4) (16-B aligned),
 * mask_gt (B,M) float.  Outputs: target_labels (B,A) float, target_bboxes (B,A,4), target_scores
 * (B,A,nc), fg_mask (B,A) uint8, target_gt_idx (B,A) int64 — the reference's 5-tuple.  Same kernels
 * (and quirks Q1-Q3) as ym_loss_fwd's fused assignment; alpha / beta / eps are the class's (align =
 * score^alpha * IoU^beta, norm eps; the fused loss uses 0.5 / 4 / 1e-9). */
size_t ym_tal_assign_workspace_size(int64_t B, int64_t A, int M);
int ym_tal_assign(const float* pd_scores, const float* pd_bboxes, const float* anc_points, const float* gt_labels,
                  const float* gt_bboxes, const float* mask_gt, int64_t B, int64_t A, int nc, int M, float alpha,
                  float beta, float eps, void* workspace, size_t workspace_bytes, float* target_labels, float* target_bboxes, float* target_scores,
                  uint8_t* fg_mask, int64_t* target_gt_idx, void* stream);
/* BboxLoss.forward (losses/yolo_v8_loss.py:280-324): pred_dist (B,A,64), pred_bboxes / target_bboxes
 * (B,A,4) grid units, anchor_points (A,2), target_scores (B,A,nc), tss device scalar (target_scores_sum),
 * fg_mask (B,A) uint8.  out[0] = loss_iou, out[1] = loss_dfl.  The backward writes
 * d(grad_out[0] * loss_iou + grad_out[1] * loss_dfl) / d pred_dist, d pred_bboxes (zero off foreground). */
size_t ym_bbox_loss_workspace_size(int64_t B, int64_t A);
int ym_bbox_loss_fwd(const float* pred_dist, const float* pred_bboxes, const float* anchor_points,
                     const float* target_bboxes, const float* target_scores, const float* tss, const uint8_t* fg_mask,
                     int64_t B, int64_t A, int nc, void* workspace, size_t workspace_bytes, float* out, void* stream);
int ym_bbox_loss_bwd(const float* pred_dist, const float* pred_bboxes, const float* anchor_points,
                     const float* target_bboxes, const float* target_scores, const float* tss, const uint8_t* fg_mask,
                     int64_t B, int64_t A, int nc, const float* grad_out, float* dpred_dist, float* dpred_bboxes,
                     void* stream);
/* y (B, 4+nc, A): xywh * stride from the DFL projection with weights dfl_w[16], sigmoid(cls). */
int ym_detect_decode(const float* head, int64_t B, int64_t A, int nc, int nl, const int* level_h,
                     const int* level_w, const float* strides, const float* dfl_w, float* y, void* stream);
/* DFL.forward (models/yolo11_modules.py:189-192) called standalone: x (B, 4*c1, A) fp32 -> softmax over the
 * c1 bins of each side -> 1x1 conv with w[c1] -> y (B, 4, A).  ym_dfl_bwd writes dx = d(sum y*dy)/dx. */
int ym_dfl_fwd(const float* x, int64_t B, int64_t A, int c1, const float* w, float* y, void* stream);
int ym_dfl_bwd(const float* x, int64_t B, int64_t A, int c1, const float* w, const float* dy, float* dx,
               void* stream);

/* ------------------------------------------------------------------ data path
 * Stretch-resize of a batch of grayscale uint8 images (packed back to back in `src`; meta[3b..3b+2]
 * = {byte offset, h0, w0}) to size x size with OpenCV's fixed-point INTER_LINEAR, /255 -> fp32
 * (batch, 1, size, size).  Replaces cv2.resize + astype(float32)/255 of the reference loader
 * (datasets/crater_dataset_cuda.py:182-184, 253). */
int ym_resize_linear_u8(const uint8_t* src, const int64_t* meta, int batch, int size, float* out, void* stream);

/* ------------------------------------------------------------------ optimizer tail
 * clip_grad_norm_(params, max_norm) + AdamW.step() over every parameter (train_yolo11_cuda.py:58-62,
 * 440-451).  The parameters form one flat index space: entry e covers elements [offset, offset + n)
 * of its own fp32 param / grad / exp_avg / exp_avg_sq tensors (offsets ascending from 0). */
typedef struct {
    float* p;
    const float* g;
    float* m;                  /* exp_avg */
    float* v;                  /* exp_avg_sq */
    int64_t offset, n;
} ym_adamw_entry;
/* Blocks (= fp32 partials) of ym_grad_norm over `total` elements. */
int ym_grad_norm_blocks(int64_t total);
/* norm[0] = ||all grads||_2 (deterministic two-level sum; partials: ym_grad_norm_blocks floats). */
int ym_grad_norm(const ym_adamw_entry* table_dev, int n_entries, int64_t total, float* partials, float* norm,
                 void* stream);
/* torch.optim.AdamW update (amsgrad=False, maximize=False) at step `step` (>= 1, already incremented)
 * on g * min(1, max_norm / (norm[0] + 1e-6)); max_norm <= 0: no clipping (norm may be NULL). */
int ym_adamw(const ym_adamw_entry* table_dev, int n_entries, int64_t total, double lr, double beta1, double beta2,
             double eps, double weight_decay, int64_t step, float max_norm, const float* norm, void* stream);

#ifdef __cplusplus
}
#endif
#endif
