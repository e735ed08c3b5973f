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
 *    frees caller memory and keeps no state between calls.
 *  - `stream` is a hipStream_t (0 = legacy default stream); every call is
 *    asynchronous on it and performs no device-wide synchronisation.
 *  - Activations are NHWC.  An "activation view" is (base pointer, batch
 *    stride, pixel stride `ld`), all in elements; channel c of pixel p of
 *    image n lives at base[n*bstride + p*ld + c].  Channel slices (concat /
 *    split) are expressed by offsetting `base` and keeping `ld`.
 *  - bf16 tensors are raw uint16 bit patterns.
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

/* nms_simple (train_yolo11_cuda.py:361-399) on one set of n xyxy boxes:
 * keep[0..*count) are indices into boxes in kept (score-descending) order. */
int ym_nms(const float* boxes, const float* scores, int64_t n, float iou_thr, void* workspace,
           size_t workspace_bytes, int64_t* keep, int32_t* count, void* stream);

#ifdef __cplusplus
}
#endif
#endif
