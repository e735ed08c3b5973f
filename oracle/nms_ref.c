/* C restatement of the reference's NMS postprocess — TEST ORACLE ONLY.
 *
 * nms_simple (/root/reference/yolo_scratch_cuda/train_yolo11_cuda.py:361-399)
 * with calculate_iou_batch_simple (:402-437): class-agnostic greedy NMS, boxes
 * sorted by score descending, a box is dropped when IoU(kept, box) > thr.
 * IoU is evaluated in the reference's fp32 op order
 *     inter = clamp(min(x2)-max(x1),0) * clamp(min(y2)-max(y1),0)
 *     union = area1 + area2 - inter;   iou = inter / (union + 1e-6f)
 * Build with -ffp-contract=off so no FMA changes a rounding.  The reference's
 * argsort is unstable; ties are broken here by ascending index (golden inputs
 * are tie-free).
 */
#include <stdint.h>
#include <stdlib.h>

static const float *g_scores;

static int cmp_desc(const void *a, const void *b) {
    int32_t i = *(const int32_t *)a, j = *(const int32_t *)b;
    float si = g_scores[i], sj = g_scores[j];
    if (si > sj) return -1;
    if (si < sj) return 1;
    return (i > j) - (i < j);
}

float oracle_iou(const float *a, const float *b) {
    float x1 = a[0] > b[0] ? a[0] : b[0];
    float y1 = a[1] > b[1] ? a[1] : b[1];
    float x2 = a[2] < b[2] ? a[2] : b[2];
    float y2 = a[3] < b[3] ? a[3] : b[3];
    float iw = x2 - x1, ih = y2 - y1;
    iw = iw < 0.0f ? 0.0f : iw;
    ih = ih < 0.0f ? 0.0f : ih;
    float inter = iw * ih;
    float a1 = (a[2] - a[0]) * (a[3] - a[1]);
    float a2 = (b[2] - b[0]) * (b[3] - b[1]);
    float uni = a1 + a2;
    uni = uni - inter;
    return inter / (uni + 1e-6f);
}

void oracle_iou_row(const float *b1, const float *b2, int64_t m, float *out) {
    for (int64_t j = 0; j < m; ++j) out[j] = oracle_iou(b1, b2 + 4 * j);
}

/* returns the number of kept boxes; keep[] receives indices into boxes[] */
int64_t oracle_nms(const float *boxes, const float *scores, int64_t n, float thr, int64_t *keep) {
    if (n <= 0) return 0;
    int32_t *ord = (int32_t *)malloc(sizeof(int32_t) * n);
    uint8_t *dead = (uint8_t *)calloc(n, 1);
    for (int64_t i = 0; i < n; ++i) ord[i] = (int32_t)i;
    g_scores = scores;
    qsort(ord, n, sizeof(int32_t), cmp_desc);
    int64_t nk = 0;
    for (int64_t p = 0; p < n; ++p) {
        if (dead[p]) continue;
        int32_t i = ord[p];
        keep[nk++] = i;
        for (int64_t q = p + 1; q < n; ++q)
            if (!dead[q] && oracle_iou(boxes + 4 * i, boxes + 4 * ord[q]) > thr) dead[q] = 1;
    }
    free(ord);
    free(dead);
    return nk;
}
