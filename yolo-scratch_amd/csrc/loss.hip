// v8 detection loss on gfx950: target preprocess, task-aligned assignment with the
// reference's forced-assignment quirks, CIoU + DFL + BCE forward, analytic backward,
// and the eval-mode Detect.inference decode.
//
// Follows /root/reference/yolo_scratch_cuda/losses/yolo_v8_loss.py:
//   preprocess :501-527, bbox_decode :529-538, TaskAlignedAssigner :64-270
//   (Q1: no top-k — positives are in-box anchors; Q2: loop 1 :117-139 and the
//   sequential loop 2 :146-162; select_highest_overlaps :226-244; Q3 GT-axis
//   normalisation :172-178), BboxLoss :280-324, v8DetectionLoss :372-499
//   (gains 7.5/0.5/1.5, tss = max(sum, 1), loss.sum()*B).
// Compiled with -ffp-contract=off: assignment decisions (in-box tests, argmax
// over IoU) use the reference's fp32 op order.
//
// Data layout: head (B, A, 64+nc) fp32 rows (one row per anchor, the three
// pyramid levels concatenated like the reference's torch.cat over levels).
//
// Kernels (per call of ym_loss_fwd): gt_prep (B threads) -> assign_scan (grid
// over anchors: decode, IoU vs every GT, in-box counts, per-GT argmax via
// packed 64-bit atomicMax) -> assign_resolve (one workgroup per image: loop 1,
// select_highest_overlaps, the sequential loop 2 on compact per-GT state, final
// select, target-score norm) -> loss_partial (per anchor BCE / CIoU / DFL) ->
// loss_final.  ym_loss_bwd recomputes per anchor and writes d loss / d head.
#include <algorithm>

#include "common.h"

namespace ym {
namespace {

constexpr int REG = 16;
constexpr int MAXLV = 4;
constexpr float EPS_IOU = 1e-7f;
constexpr float EPS_TAL = 1e-9f;

struct Levels {
    int n;
    int64_t off[MAXLV + 1];   // anchor offsets (cumulative)
    int w[MAXLV];
    float stride[MAXLV];
};

__device__ __forceinline__ void anchor_of(const Levels& L, int64_t a, float& ax, float& ay, float& s) {
    int l = 0;
    while (l + 1 < L.n && a >= L.off[l + 1]) ++l;
    int64_t p = a - L.off[l];
    int row = int(p / L.w[l]), col = int(p - int64_t(row) * L.w[l]);
    ax = float(col) + 0.5f;
    ay = float(row) + 0.5f;
    s = L.stride[l];
}

// softmax-expectation of 16 bins (bbox_decode :534-536); returns dist and fills p
__device__ __forceinline__ float dfl_expect(const float* x, float* p) {
    float m = x[0];
#pragma unroll
    for (int k = 1; k < REG; ++k) m = fmaxf(m, x[k]);
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < REG; ++k) { p[k] = expf(x[k] - m); s += p[k]; }
    float inv = 1.0f / s, d = 0.f;
#pragma unroll
    for (int k = 0; k < REG; ++k) { p[k] *= inv; d += p[k] * float(k); }
    return d;
}

// bbox_iou(xyxy, CIoU=False) with the reference's eps placement (:33-44)
__device__ __forceinline__ float iou_xyxy(float a0, float a1, float a2, float a3, float b0, float b1, float b2, float b3) {
    float w1 = a2 - a0, h1 = a3 - a1 + EPS_IOU;
    float w2 = b2 - b0, h2 = b3 - b1 + EPS_IOU;
    float iw = fminf(a2, b2) - fmaxf(a0, b0);
    float ih = fminf(a3, b3) - fmaxf(a1, b1);
    iw = iw < 0.f ? 0.f : iw;
    ih = ih < 0.f ? 0.f : ih;
    float inter = iw * ih;
    float uni = w1 * h1 + w2 * h2 - inter + EPS_IOU;
    return inter / uni;
}

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

// ---------------------------------------------------------------- preprocess (:501-527)
// gt_box[b][j] pixel xyxy (bbox * [ih, iw, ih, iw] as imgsz.repeat(2)), gt_lab, valid; stable per-image order
// one wave per image: the targets are scanned 64 at a time, each image's rows keep the batch order
// (ballot + prefix popcount), the first M of them are kept
__global__ void __launch_bounds__(64) gt_prep_kernel(const int64_t* __restrict__ bidx, const int64_t* __restrict__ cls,
                                                     const float* __restrict__ boxes, int64_t N, int B, int M, float ih,
                                                     float iw, float4* __restrict__ gt_box, float* __restrict__ gt_lab,
                                                     int* __restrict__ gt_valid) {
    const int b = blockIdx.x, lane = threadIdx.x;
    const unsigned long long below = (1ull << lane) - 1ull;
    int j = 0;
    for (int64_t t0 = 0; t0 < N && j < M; t0 += 64) {
        const int64_t t = t0 + lane;
        const bool mine = t < N && bidx[t] == b;
        const unsigned long long mask = __ballot(mine);
        const int slot = j + int(__popcll(mask & below));
        if (mine && slot < M) {
            const float* r = boxes + 4 * t;
            gt_box[b * M + slot] = make_float4(r[0] * ih, r[1] * iw, r[2] * ih, r[3] * iw);
            gt_lab[b * M + slot] = float(cls[t]);
            gt_valid[b * M + slot] = 1;
        }
        j += int(__popcll(mask));
    }
    for (int s = min(j, M) + lane; s < M; s += 64) {
        gt_box[b * M + s] = make_float4(0.f, 0.f, 0.f, 0.f);
        gt_lab[b * M + s] = 0.f;
        gt_valid[b * M + s] = 0;
    }
}

struct AssignWs {
    float4* pbox;        // [B][A] predicted xyxy in grid units
    int* cnt0;           // [B][A] in-box & valid count
    int* g0;             // [B][A] first in-box & valid gt
    int* gmax;           // [B][A] argmax_g IoU (first)
    int* fcnt;           // [B][A] loop-1 forced count   (zeroed)
    int* fgg;            // [B][A] loop-1 forced gt
    int* r1;             // [B][A] row after the first select
    int* tgi;            // [B][A] final target gt index
    float* norm;         // [B][A] target-score magnitude (0 when background)
    int* fg;             // [B][A] foreground flag
    unsigned long long* amax;   // [B][M] packed (iou bits << 32 | ~a)   (zeroed)
    int* gcnt;           // [B][M] in-box positives per gt           (zeroed)
    double* part;        // [nblk][5] loss partials (cls, box, dfl, tss, num_fg)
    float* out;          // [8] loss, items[3], tss, num_fg ...
};

// ---------------------------------------------------------------- assignment inputs
// The assigner reads its predictions through one of two sources: the fused loss's (B, A, 64+nc) head rows
// (boxes decoded here, v8DetectionLoss.__call__ :408-422), or the explicit tensors a direct
// TaskAlignedAssigner.forward call passes (pd_scores already sigmoided, pd_bboxes / anc_points in pixels).
struct HeadSrc {
    const float* head;
    int64_t A;
    int no;
    Levels L;
    // pixel-space predicted box + anchor centre; stores the grid-unit box the loss re-reads
    __device__ void box(int b, int64_t a, AssignWs& w, float& px1, float& py1, float& px2, float& py2, float& cx,
                        float& cy) const {
        const float* x = head + (int64_t(b) * A + a) * no;
        float ax, ay, s;
        anchor_of(L, a, ax, ay, s);
        float p[REG], d[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) d[k] = dfl_expect(x + k * REG, p);
        float x1 = ax - d[0], y1 = ay - d[1], x2 = ax + d[2], y2 = ay + d[3];
        w.pbox[int64_t(b) * A + a] = make_float4(x1, y1, x2, y2);
        px1 = x1 * s; py1 = y1 * s; px2 = x2 * s; py2 = y2 * s;
        cx = ax * s; cy = ay * s;                        // anchor_points * stride_tensor
    }
    __device__ float4 pixbox(int b, int64_t a, const AssignWs& w) const {
        float ax, ay, s;
        anchor_of(L, a, ax, ay, s);
        float4 pb = w.pbox[int64_t(b) * A + a];
        return make_float4(pb.x * s, pb.y * s, pb.z * s, pb.w * s);
    }
    __device__ float score(int b, int64_t a, int lab) const { return sigm(head[(int64_t(b) * A + a) * no + 64 + lab]); }
};

struct PlainSrc {
    const float* scores;    // (B, A, nc) probabilities
    const float* boxes;     // (B, A, 4) xyxy pixels
    const float* anc;       // (A, 2) pixels
    int64_t A;
    int nc;
    __device__ void box(int b, int64_t a, AssignWs&, float& px1, float& py1, float& px2, float& py2, float& cx,
                        float& cy) const {
        const float* r = boxes + (int64_t(b) * A + a) * 4;
        px1 = r[0]; py1 = r[1]; px2 = r[2]; py2 = r[3];
        cx = anc[2 * a]; cy = anc[2 * a + 1];
    }
    __device__ float4 pixbox(int b, int64_t a, const AssignWs&) const {
        const float* r = boxes + (int64_t(b) * A + a) * 4;
        return make_float4(r[0], r[1], r[2], r[3]);
    }
    __device__ float score(int b, int64_t a, int lab) const { return scores[(int64_t(b) * A + a) * nc + lab]; }
};

// ---------------------------------------------------------------- assignment, pass 1
template <class Src>
__global__ void __launch_bounds__(256) assign_scan_kernel(Src src, int64_t A, const float4* __restrict__ gt_box,
                                                          const int* __restrict__ gt_valid, int M, AssignWs w) {
    extern __shared__ unsigned long long s_amax[];    // [M]
    int* s_cnt = reinterpret_cast<int*>(s_amax + M);   // [M]
    const int b = blockIdx.y;
    for (int g = threadIdx.x; g < M; g += blockDim.x) { s_amax[g] = 0ull; s_cnt[g] = 0; }
    __syncthreads();
    const int64_t a = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const bool live = a < A;
    // every lane runs the gt loop (dead lanes with zero keys) so the per-gt argmax and in-box counts
    // reduce over the wave first (shuffles / ballot) and take one LDS atomic per wave, not per lane
    float px1 = 0.f, py1 = 0.f, px2 = 0.f, py2 = 0.f, cx = 0.f, cy = 0.f;
    if (live) src.box(b, a, w, px1, py1, px2, py2, cx, cy);
    int cnt = 0, first = -1, gm = 0;
    float best = -1.f;
    const int lane = threadIdx.x & 63;
    for (int g = 0; g < M; ++g) {
        const float4 gb = gt_box[b * M + g];
        float iou = iou_xyxy(px1, py1, px2, py2, gb.x, gb.y, gb.z, gb.w);
        iou = iou < 0.f ? 0.f : iou;                     // .clamp_(0) (:199)
        if (iou > best) { best = iou; gm = g; }
        // select_candidates_in_gts (:210-224): min(l, t, r, b) > eps
        const float l = cx - gb.x, t = cy - gb.y, r = gb.z - cx, bo = gb.w - cy;
        const float mn = fminf(fminf(l, t), fminf(r, bo));
        const bool inb = live && mn > EPS_TAL && gt_valid[b * M + g];
        if (inb) {
            ++cnt;
            if (first < 0) first = g;
        }
        const unsigned long long pos = __ballot(inb);
        if (lane == 0 && pos) atomicAdd(&s_cnt[g], int(__popcll(pos)));
        // wave max of the packed (iou, ~a) key: the first anchor of the best IoU
        uint32_t hi = live ? __float_as_uint(iou) : 0u, lo = live ? 0xffffffffu - uint32_t(a) : 0u;
        // most (wave, gt) pairs overlap nowhere: every key's iou bits are then 0 and the wave max is lane 0's
        // (the lowest anchor; lane 0 is live whenever any lane is), so the 12 shuffles are skipped
        if (!__ballot(hi != 0u)) {
            if (lane == 0 && live) atomicMax(&s_amax[g], uint64_t(lo));
            continue;
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const uint32_t h2 = __shfl_xor(hi, o, 64), l2 = __shfl_xor(lo, o, 64);
            if (h2 > hi || (h2 == hi && l2 > lo)) { hi = h2; lo = l2; }
        }
        if (lane == 0) atomicMax(&s_amax[g], (uint64_t(hi) << 32) | uint64_t(lo));
    }
    if (live) {
        w.cnt0[int64_t(b) * A + a] = cnt;
        w.g0[int64_t(b) * A + a] = first;
        w.gmax[int64_t(b) * A + a] = gm;
    }
    __syncthreads();
    for (int g = threadIdx.x; g < M; g += blockDim.x) {
        atomicMax(&w.amax[int64_t(b) * M + g], s_amax[g]);
        if (s_cnt[g]) atomicAdd(&w.gcnt[int64_t(b) * M + g], s_cnt[g]);
    }
}

// ---------------------------------------------------------------- assignment, pass 2 (one workgroup per image)
constexpr int RES_THREADS = 1024;

__global__ void __launch_bounds__(RES_THREADS) assign_resolve_kernel(const float* __restrict__ head, int64_t A, int no,
                                                                    int nc, const float4* __restrict__ gt_box,
                                                                    const float* __restrict__ gt_lab,
                                                                    const int* __restrict__ gt_valid, int M,
                                                                    AssignWs w) {
    extern __shared__ int sm[];
    int* cnt2 = sm;                 // [M]
    int* f2a = sm + M;              // [M] loop-2 forced anchors
    int* f2g = sm + 2 * M;          // [M] loop-2 forced gts
    int* modA = sm + 3 * M;         // [M] modified anchors (current tgi/fg)
    int* modT = sm + 4 * M;         // [M]
    __shared__ int nf2, nmod;
    const int b = blockIdx.x;
    const int64_t base = int64_t(b) * A;
    for (int g = threadIdx.x; g < M; g += blockDim.x) cnt2[g] = 0;
    if (threadIdx.x == 0) { nf2 = 0; nmod = 0; }
    // loop 1: a valid gt with no in-box anchor takes its best-IoU anchor (the in-box branch cannot fire)
    for (int g = threadIdx.x; g < M; g += blockDim.x) {
        if (gt_valid[b * M + g] && w.gcnt[int64_t(b) * M + g] == 0) {
            int64_t a = int64_t(0xffffffffu - uint32_t(w.amax[int64_t(b) * M + g] & 0xffffffffull));
            atomicAdd(&w.fcnt[base + a], 1);
            w.fgg[base + a] = g;
        }
    }
    __threadfence_block();
    __syncthreads();
    // select_highest_overlaps #1: every row ends with at most one gt
    for (int64_t a = threadIdx.x; a < A; a += blockDim.x) {
        int c0 = w.cnt0[base + a], fc = w.fcnt[base + a];
        int tot = c0 + fc, r;
        if (tot == 0) r = -1;
        else if (tot == 1) r = c0 ? w.g0[base + a] : w.fgg[base + a];
        else r = w.gmax[base + a];
        w.r1[base + a] = r;
        if (r >= 0) atomicAdd(&cnt2[r], 1);
    }
    __threadfence_block();
    __syncthreads();
    // loop 2 (sequential in gt order; tgi/fg edits feed later checks)
    if (threadIdx.x == 0) {
        for (int g = 0; g < M; ++g) {
            if (!gt_valid[b * M + g] || cnt2[g] > 0) continue;
            int a = int(0xffffffffu - uint32_t(w.amax[int64_t(b) * M + g] & 0xffffffffull));
            int cur = -2;
            for (int k = 0; k < nmod; ++k)
                if (modA[k] == a) cur = modT[k];
            if (cur == -2) cur = w.r1[base + a];
            if (cur >= 0) cnt2[cur]--;
            bool found = false;
            for (int k = 0; k < nmod; ++k)
                if (modA[k] == a) { modT[k] = g; found = true; }
            if (!found) { modA[nmod] = a; modT[nmod] = g; nmod++; }
            cnt2[g]++;
            f2a[nf2] = a;
            f2g[nf2] = g;
            nf2++;
        }
    }
    __syncthreads();
    // final select + target scores (get_targets :246-270, normalisation :172-178)
    for (int64_t a = threadIdx.x; a < A; a += blockDim.x) {
        int r = w.r1[base + a];
        int add = 0, last = -1;
        for (int k = 0; k < nf2; ++k)
            if (f2a[k] == a) { ++add; last = f2g[k]; }
        int el = (r >= 0 ? 1 : 0) + add;
        int t = 0, f = 0;
        if (el == 1) { t = r >= 0 ? r : last; f = 1; }
        else if (el >= 2) { t = w.gmax[base + a]; f = 1; }
        w.tgi[base + a] = t;
        w.fg[base + a] = f;
    }
}

// target-score magnitude: align = sigmoid(cls[label])^alpha * IoU^beta (:206), norm = align*IoU/(align+eps)
// (v8DetectionLoss: alpha 0.5, beta 4, eps 1e-9; the class defaults alpha 1, beta 6 for a standalone assigner)
template <class Src>
__global__ void assign_norm_kernel(Src src, int64_t A, const float4* __restrict__ gt_box,
                                   const float* __restrict__ gt_lab, int M, AssignWs w, float alpha, float beta,
                                   float eps) {
    const int b = blockIdx.y;
    const int64_t a = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (a >= A) return;
    const int64_t i = int64_t(b) * A + a;
    if (!w.fg[i]) { w.norm[i] = 0.f; return; }
    float4 pb = src.pixbox(b, a, w);
    int t = w.tgi[i];
    float4 gb = gt_box[b * M + t];
    float iou = iou_xyxy(pb.x, pb.y, pb.z, pb.w, gb.x, gb.y, gb.z, gb.w);
    iou = iou < 0.f ? 0.f : iou;
    int lab = int(gt_lab[b * M + t]);
    float sc = src.score(b, a, lab);
    float align = (alpha == 0.5f ? sqrtf(sc) : powf(sc, alpha)) * powf(iou, beta);
    w.norm[i] = align * iou / (align + eps);
}

// ---------------------------------------------------------------- loss terms
struct CiouOut { float ciou, g[4]; };

// CIoU of pred (x1,y1,x2,y2) vs target (bbox_iou(..., CIoU=True), :25-56) and d ciou / d pred
__device__ CiouOut ciou_grad(float x1, float y1, float x2, float y2, float X1, float Y1, float X2, float Y2, bool want) {
    const float eps = EPS_IOU;
    float w1 = x2 - x1, h1 = y2 - y1 + eps;
    float w2 = X2 - X1, h2 = Y2 - Y1 + eps;
    float mnx = fminf(x2, X2), mxx = fmaxf(x1, X1);
    float mny = fminf(y2, Y2), mxy = fmaxf(y1, Y1);
    float iw = mnx - mxx, ih = mny - mxy;
    float iwc = iw < 0.f ? 0.f : iw, ihc = ih < 0.f ? 0.f : ih;
    float inter = iwc * ihc;
    float uni = w1 * h1 + w2 * h2 - inter + eps;
    float iou = inter / uni;
    float cw = fmaxf(x2, X2) - fminf(x1, X1);
    float ch = fmaxf(y2, Y2) - fminf(y1, Y1);
    float c2 = cw * cw + ch * ch + eps;
    float sx = X1 + X2 - x1 - x2, sy = Y1 + Y2 - y1 - y2;
    float rho2 = (sx * sx + sy * sy) / 4.0f;
    const float k4 = 4.0f / (3.14159265358979323846f * 3.14159265358979323846f);
    float dat = atanf(w2 / h2) - atanf(w1 / h1);
    float v = k4 * dat * dat;
    float alpha = v / (v - iou + (1.0f + eps));
    CiouOut o;
    o.ciou = iou - (rho2 / c2 + v * alpha);
    if (!want) return o;
    // torch.minimum/maximum backward split the gradient on ties; clamp passes where input >= 0
    auto lt_w = [](float a, float b) { return a < b ? 1.0f : (a == b ? 0.5f : 0.0f); };
    float d_iw_dx2 = lt_w(x2, X2), d_iw_dx1 = -lt_w(X1, x1);     // min(x2,X2) - max(x1,X1)
    float d_ih_dy2 = lt_w(y2, Y2), d_ih_dy1 = -lt_w(Y1, y1);
    float miw = iw >= 0.f ? 1.f : 0.f, mih = ih >= 0.f ? 1.f : 0.f;
    // d inter
    float dI[4] = {ihc * miw * d_iw_dx1, iwc * mih * d_ih_dy1, ihc * miw * d_iw_dx2, iwc * mih * d_ih_dy2};
    // d (w1*h1): w1 = x2 - x1, h1 = y2 - y1 + eps
    float dWH[4] = {-h1, -w1, h1, w1};
    float dcw_dx2 = lt_w(X2, x2), dcw_dx1 = -lt_w(x1, X1);      // max(x2,X2) - min(x1,X1)
    float dch_dy2 = lt_w(Y2, y2), dch_dy1 = -lt_w(y1, Y1);
    float dC2[4] = {2.f * cw * dcw_dx1, 2.f * ch * dch_dy1, 2.f * cw * dcw_dx2, 2.f * ch * dch_dy2};
    float dR[4] = {-sx / 2.0f, -sy / 2.0f, -sx / 2.0f, -sy / 2.0f};
    // v = k4 * (atan(w2/h2) - atan(w1/h1))^2 ; r = w1/h1
    float r = w1 / h1;
    float datan = 1.0f / (1.0f + r * r);
    float dv_dr = k4 * 2.0f * dat * (-datan);
    float dr[4] = {-1.0f / h1, w1 / (h1 * h1), 1.0f / h1, -w1 / (h1 * h1)};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        float dunion = dWH[k] - dI[k];
        float diou = (dI[k] - iou * dunion) / uni;
        float dpen = dR[k] / c2 - rho2 * dC2[k] / (c2 * c2) + alpha * dv_dr * dr[k];
        o.g[k] = diou - dpen;
    }
    return o;
}

__device__ __forceinline__ float bce(float x, float t) {
    float mv = fmaxf(-x, 0.f);
    return (1.0f - t) * x + mv + logf(expf(-mv) + expf(-x - mv));
}

// one thread per anchor; block partials (double) of cls, box, dfl, tss.  The workgroup's class logits (a contiguous run
// of 256 head rows) are staged through LDS by coalesced loads first (round 5: each lane read its own 20 B at a 276-B
// row stride); every thread's arithmetic and summation order is unchanged.
constexpr int LOSS_NC_LDS = 16;                 // class counts staged through LDS (larger ones read the rows directly)
__global__ void __launch_bounds__(256) loss_partial_kernel(const float* __restrict__ head, int64_t A, int no, int nc,
                                                           Levels L, const float4* __restrict__ gt_box,
                                                           const float* __restrict__ gt_lab, int M, AssignWs w) {
    __shared__ double red[5][256];
    __shared__ float s_cls[256 * LOSS_NC_LDS];
    const int b = blockIdx.y;
    const int64_t a0 = int64_t(blockIdx.x) * blockDim.x;
    const int64_t a = a0 + threadIdx.x;
    const bool staged = nc <= LOSS_NC_LDS;
    if (staged) {
        const int na = int(min(int64_t(blockDim.x), A - a0));
        const float* xr = head + (int64_t(b) * A + a0) * no;
        // element e of the run's class block = (row aa, class c); (aa, c) stepped without a division per element
        const int q = int(blockDim.x) / nc, r = int(blockDim.x) - q * nc;
        int aa = threadIdx.x / nc, c = threadIdx.x - aa * nc;
        for (int e = threadIdx.x; e < na * nc; e += blockDim.x) {
            s_cls[e] = xr[int64_t(aa) * no + 64 + c];
            c += r;
            aa += q;
            if (c >= nc) { c -= nc; ++aa; }
        }
        __syncthreads();
    }
    double lc = 0, lb = 0, ld = 0, ts = 0, nf = 0;
    if (a < A) {
        const int64_t i = int64_t(b) * A + a;
        const float* x = head + i * no;
        const int f = w.fg[i];
        const float nm = w.norm[i];
        int lab = 0;
        if (f) lab = int(gt_lab[b * M + w.tgi[i]]);
        const float* xc = staged ? s_cls + threadIdx.x * nc : x + 64;
        for (int c = 0; c < nc; ++c) {
            float t = (f && c == lab) ? nm : 0.f;
            lc += bce(xc[c], t);
        }
        if (f) {
            ts = nm;
            nf = 1;
            float ax, ay, s;
            anchor_of(L, a, ax, ay, s);
            float4 pb = w.pbox[i];
            float4 gb = gt_box[b * M + w.tgi[i]];
            float X1 = gb.x / s, Y1 = gb.y / s, X2 = gb.z / s, Y2 = gb.w / s;   // target_bboxes /= stride
            CiouOut ci = ciou_grad(pb.x, pb.y, pb.z, pb.w, X1, Y1, X2, Y2, false);
            lb = double((1.0f - ci.ciou) * nm);
            // DFL (bbox2dist :327-330 then _df_loss :312-324)
            float tgt[4] = {ax - X1, ay - Y1, X2 - ax, Y2 - ay};
            float acc = 0.f;
            for (int k = 0; k < 4; ++k) {
                float t = fminf(fmaxf(tgt[k], 0.f), REG - 1 - 0.01f);
                t = fminf(fmaxf(t, 0.f), REG - 1 - 0.01f);
                int tl = int(t);
                float wl = float(tl + 1) - t, wr = 1.0f - wl;
                const float* xs = x + k * REG;
                float m = xs[0];
                for (int j = 1; j < REG; ++j) m = fmaxf(m, xs[j]);
                float se = 0.f;
                for (int j = 0; j < REG; ++j) se += expf(xs[j] - m);
                float lse = m + logf(se);
                acc += (lse - xs[tl]) * wl + (lse - xs[tl + 1]) * wr;
            }
            ld = double(acc / 4.0f * nm);
        }
    }
    red[0][threadIdx.x] = lc;
    red[1][threadIdx.x] = lb;
    red[2][threadIdx.x] = ld;
    red[3][threadIdx.x] = ts;
    red[4][threadIdx.x] = nf;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o)
            for (int k = 0; k < 5; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x < 5) w.part[(int64_t(blockIdx.y) * gridDim.x + blockIdx.x) * 5 + threadIdx.x] = red[threadIdx.x][0];
}

// out: [0] loss, [1..3] items (box, cls, dfl with gains), [4] tss, [5] num_fg
__global__ void loss_final_kernel(int nparts, int B, AssignWs w) {
    __shared__ double red[5][256];
    double s[5] = {0, 0, 0, 0, 0};
    for (int p = threadIdx.x; p < nparts; p += blockDim.x)
        for (int k = 0; k < 5; ++k) s[k] += w.part[int64_t(p) * 5 + k];
    for (int k = 0; k < 5; ++k) red[k][threadIdx.x] = s[k];
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o)
            for (int k = 0; k < 5; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        float tss = fmaxf(float(red[3][0]), 1.0f);
        float lcls = float(red[0][0]) / tss, lbox = float(red[1][0]) / tss, ldfl = float(red[2][0]) / tss;
        float ib = lbox * 7.5f, ic = lcls * 0.5f, id = ldfl * 1.5f;
        w.out[1] = ib;
        w.out[2] = ic;
        w.out[3] = id;
        w.out[0] = (ib + ic + id) * float(B);
        w.out[4] = tss;
        w.out[5] = float(red[4][0]);
    }
}

// d loss / d head rows; gscale = d(total)/d(loss) (autograd's incoming grad, device scalar).
// A workgroup's 256 anchors are one contiguous run of 256 x no floats of head / dhead: the background rows' zero DFL
// gradients are stored a row (256 B) per wave instruction and the class-logit gradients element by element over the
// run (round 5 — the thread-per-row form stored 4 B per lane at a 276-B row stride), then each foreground anchor's
// thread writes its 64 DFL / box gradients (2-3 % of the rows).  Same arithmetic per element.
__global__ void __launch_bounds__(256) loss_bwd_kernel(const float* __restrict__ head, int64_t A, int no, int nc, int B,
                                                       Levels L, const float4* __restrict__ gt_box,
                                                       const float* __restrict__ gt_lab, int M, AssignWs w,
                                                       const float* __restrict__ gout, float* __restrict__ dhead) {
    __shared__ int s_f[256], s_lab[256];
    __shared__ float s_nm[256];
    const int b = blockIdx.y;
    const int64_t a0 = int64_t(blockIdx.x) * blockDim.x;
    const int na = int(min(int64_t(blockDim.x), A - a0));
    const int tid = threadIdx.x;
    const float k = gout[0] * float(B) / w.out[4];
    if (tid < na) {
        const int64_t i = int64_t(b) * A + a0 + tid;
        const int f = w.fg[i];
        s_f[tid] = f;
        s_nm[tid] = w.norm[i];
        s_lab[tid] = f ? int(gt_lab[b * M + w.tgi[i]]) : 0;
    }
    __syncthreads();
    {
        const int64_t r0 = (int64_t(b) * A + a0) * no;
        const float* xr = head + r0;
        float* dr = dhead + r0;
        // background rows' 64 zero DFL gradients: wave wv stores rows wv*64 .. wv*64+63, one row per store
        // instruction, skipping foreground rows by a wave-uniform bit of a ballot (no memory read in the loop)
        const int wv = tid >> 6, lane = tid & 63, rb = wv * 64;
        const unsigned long long bg = __ballot(rb + lane < na && !s_f[rb + lane]);
        for (int r = 0; r < 64; ++r)
            if ((bg >> r) & 1ull) dr[int64_t(rb + r) * no + lane] = 0.f;
        // class-logit gradients, element e = (row aa, class c) of the run's class block, stepped without divisions
        const int q = int(blockDim.x) / nc, rr = int(blockDim.x) - q * nc;
        int aa = tid / nc, c = tid - aa * nc;
        for (int e = tid; e < na * nc; e += blockDim.x, c += rr, aa += q) {
            if (c >= nc) { c -= nc; ++aa; }
            const int64_t o = int64_t(aa) * no + 64 + c;
            const float t = (s_f[aa] && c == s_lab[aa]) ? s_nm[aa] : 0.f;
            dr[o] = 0.5f * k * (sigm(xr[o]) - t);
        }
    }
    if (tid >= na || !s_f[tid]) return;
    const int64_t a = a0 + tid;
    const int64_t i = int64_t(b) * A + a;
    const float* x = head + i * no;
    float* dx = dhead + i * no;
    const float nm = s_nm[tid];
    float ax, ay, s;
    anchor_of(L, a, ax, ay, s);
    float4 gb = gt_box[b * M + w.tgi[i]];
    float X1 = gb.x / s, Y1 = gb.y / s, X2 = gb.z / s, Y2 = gb.w / s;
    float p[4][REG], d[4];
    for (int q = 0; q < 4; ++q) d[q] = dfl_expect(x + q * REG, p[q]);
    float x1 = ax - d[0], y1 = ay - d[1], x2 = ax + d[2], y2 = ay + d[3];
    CiouOut ci = ciou_grad(x1, y1, x2, y2, X1, Y1, X2, Y2, true);
    // L_box = (1 - ciou) * nm ; d dist: x1 = ax - d0, y1 = ay - d1, x2 = ax + d2, y2 = ay + d3
    float gd[4] = {ci.g[0], ci.g[1], -ci.g[2], -ci.g[3]};       // d(1-ciou)/d dist = -dciou/dxy * dxy/ddist
    float tgt[4] = {ax - X1, ay - Y1, X2 - ax, Y2 - ay};
    for (int q = 0; q < 4; ++q) {
        float gbox = 7.5f * k * nm * gd[q];
        float t = fminf(fmaxf(tgt[q], 0.f), REG - 1 - 0.01f);
        int tl = int(t);
        float wl = float(tl + 1) - t, wr = 1.0f - wl;
        float gdfl = 1.5f * k * nm / 4.0f;
        for (int j = 0; j < REG; ++j) {
            float pj = p[q][j];
            float g = gbox * pj * (float(j) - d[q]);
            g += gdfl * ((wl + wr) * pj - (j == tl ? wl : 0.f) - (j == tl + 1 ? wr : 0.f));
            dx[q * REG + j] = g;
        }
    }
}

// Detect.inference (yolo11_modules.py:248-266): y (B, 4+nc, A) = [xywh * stride, sigmoid(cls)]
__global__ void detect_decode_kernel(const float* __restrict__ head, int64_t A, int no, int nc, Levels L,
                                     const float* __restrict__ dflw, float* __restrict__ y) {
    const int b = blockIdx.y;
    const int64_t a = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (a >= A) return;
    const float* x = head + (int64_t(b) * A + a) * no;
    float ax, ay, s;
    anchor_of(L, a, ax, ay, s);
    float d[4], p[REG];
    for (int q = 0; q < 4; ++q) {
        dfl_expect(x + q * REG, p);
        float acc = 0.f;
        for (int j = 0; j < REG; ++j) acc += p[j] * dflw[j];
        d[q] = acc;
    }
    float x1 = ax - d[0], y1 = ay - d[1], x2 = ax + d[2], y2 = ay + d[3];
    float* yb = y + int64_t(b) * (4 + nc) * A;
    yb[0 * A + a] = (x1 + x2) / 2 * s;
    yb[1 * A + a] = (y1 + y2) / 2 * s;
    yb[2 * A + a] = (x2 - x1) * s;
    yb[3 * A + a] = (y2 - y1) * s;
    for (int c = 0; c < nc; ++c) yb[(4 + c) * A + a] = sigm(x[64 + c]);
}

// ---------------------------------------------------------------- TaskAlignedAssigner.forward on explicit tensors
// mask_gt (float, the reference's `if mask_gt[b, g]` truthiness) -> int valid flags
__global__ void mask_valid_kernel(const float* __restrict__ mask_gt, int64_t n, int* __restrict__ valid) {
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n) valid[i] = mask_gt[i] != 0.f;
}

// get_targets (:246-270) + target_scores normalisation (:172-178) on the final assignment:
// labels = gt_labels[b, tgi] clamped to [0, nc] (float, like gt_labels), boxes = gt_bboxes[b, tgi],
// scores = one-hot(label) * norm on foreground rows, fg (bool) and tgi (int64)
__global__ void assign_targets_kernel(int64_t A, int nc, const float4* __restrict__ gt_box,
                                      const float* __restrict__ gt_lab, int M, AssignWs w, float* __restrict__ t_lab,
                                      float4* __restrict__ t_box, float* __restrict__ t_sc, uint8_t* __restrict__ fg_out,
                                      int64_t* __restrict__ tgi_out) {
    const int b = blockIdx.y;
    const int64_t a = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (a >= A) return;
    const int64_t i = int64_t(b) * A + a;
    const int t = w.tgi[i], f = w.fg[i];
    float lab = gt_lab[b * M + t];
    lab = fminf(fmaxf(lab, 0.f), float(nc));
    t_lab[i] = lab;
    t_box[i] = gt_box[b * M + t];
    const int li = int(lab);
    const float nm = w.norm[i];
    for (int c = 0; c < nc; ++c) t_sc[i * nc + c] = (f && c == li) ? nm : 0.f;
    fg_out[i] = uint8_t(f);
    tgi_out[i] = int64_t(t);
}

// ---------------------------------------------------------------- BboxLoss.forward on explicit tensors (:280-324)
// one thread per anchor; partials (double) of the CIoU and DFL sums over foreground anchors
struct BoxIn {
    const float* pdist;     // (B, A, 64)
    const float* pbox;      // (B, A, 4) grid units
    const float* anc;       // (A, 2) grid units
    const float* tbox;      // (B, A, 4) grid units
    const float* tsc;       // (B, A, nc)
    const uint8_t* fg;      // (B, A)
    int64_t A;
    int nc;
};

__device__ __forceinline__ float box_weight(const BoxIn& in, int64_t i) {
    float wsum = 0.f;                                    // target_scores.sum(-1) (:298)
    for (int c = 0; c < in.nc; ++c) wsum += in.tsc[i * in.nc + c];
    return wsum;
}

__global__ void __launch_bounds__(256) bbox_loss_partial_kernel(BoxIn in, double* __restrict__ part) {
    __shared__ double red[2][256];
    const int b = blockIdx.y;
    const int64_t a = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    double li = 0, ld = 0;
    if (a < in.A) {
        const int64_t i = int64_t(b) * in.A + a;
        if (in.fg[i]) {
            const float wt = box_weight(in, i);
            const float* pb = in.pbox + i * 4;
            const float* tb = in.tbox + i * 4;
            CiouOut ci = ciou_grad(pb[0], pb[1], pb[2], pb[3], tb[0], tb[1], tb[2], tb[3], false);
            li = double((1.0f - ci.ciou) * wt);
            const float ax = in.anc[2 * a], ay = in.anc[2 * a + 1];
            float tgt[4] = {ax - tb[0], ay - tb[1], tb[2] - ax, tb[3] - ay};
            float acc = 0.f;
            for (int k = 0; k < 4; ++k) {
                float t = fminf(fmaxf(tgt[k], 0.f), REG - 1 - 0.01f);
                int tl = int(t);
                float wl = float(tl + 1) - t, wr = 1.0f - wl;
                const float* xs = in.pdist + i * 64 + k * REG;
                float m = xs[0];
                for (int j = 1; j < REG; ++j) m = fmaxf(m, xs[j]);
                float se = 0.f;
                for (int j = 0; j < REG; ++j) se += expf(xs[j] - m);
                float lse = m + logf(se);
                acc += (lse - xs[tl]) * wl + (lse - xs[tl + 1]) * wr;
            }
            ld = double(acc / 4.0f * wt);
        }
    }
    red[0][threadIdx.x] = li;
    red[1][threadIdx.x] = ld;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) {
            red[0][threadIdx.x] += red[0][threadIdx.x + o];
            red[1][threadIdx.x] += red[1][threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x < 2) part[(int64_t(blockIdx.y) * gridDim.x + blockIdx.x) * 2 + threadIdx.x] = red[threadIdx.x][0];
}

// out[0] = loss_iou, out[1] = loss_dfl (each sum / target_scores_sum)
__global__ void bbox_loss_final_kernel(const double* __restrict__ part, int nparts, const float* __restrict__ tss,
                                       float* __restrict__ out) {
    __shared__ double red[2][256];
    double s0 = 0, s1 = 0;
    for (int p = threadIdx.x; p < nparts; p += blockDim.x) { s0 += part[2 * p]; s1 += part[2 * p + 1]; }
    red[0][threadIdx.x] = s0;
    red[1][threadIdx.x] = s1;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) {
            red[0][threadIdx.x] += red[0][threadIdx.x + o];
            red[1][threadIdx.x] += red[1][threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out[0] = float(red[0][0]) / tss[0];
        out[1] = float(red[1][0]) / tss[0];
    }
}

// d(g0 * loss_iou + g1 * loss_dfl) / d pred_bboxes and / d pred_dist (zero on background rows)
__global__ void __launch_bounds__(256) bbox_loss_bwd_kernel(BoxIn in, const float* __restrict__ tss,
                                                            const float* __restrict__ gout, float* __restrict__ dpdist,
                                                            float* __restrict__ dpbox) {
    const int b = blockIdx.y;
    const int64_t a = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (a >= in.A) return;
    const int64_t i = int64_t(b) * in.A + a;
    float* gd = dpdist + i * 64;
    float* gb = dpbox + i * 4;
    if (!in.fg[i]) {
        for (int j = 0; j < 64; ++j) gd[j] = 0.f;
        for (int j = 0; j < 4; ++j) gb[j] = 0.f;
        return;
    }
    const float wt = box_weight(in, i);
    const float* pb = in.pbox + i * 4;
    const float* tb = in.tbox + i * 4;
    CiouOut ci = ciou_grad(pb[0], pb[1], pb[2], pb[3], tb[0], tb[1], tb[2], tb[3], true);
    const float kiou = -gout[0] * wt / tss[0];
    for (int j = 0; j < 4; ++j) gb[j] = kiou * ci.g[j];
    const float ax = in.anc[2 * a], ay = in.anc[2 * a + 1];
    float tgt[4] = {ax - tb[0], ay - tb[1], tb[2] - ax, tb[3] - ay};
    const float kdfl = gout[1] * wt / (4.0f * tss[0]);
    for (int k = 0; k < 4; ++k) {
        float t = fminf(fmaxf(tgt[k], 0.f), REG - 1 - 0.01f);
        int tl = int(t);
        float wl = float(tl + 1) - t, wr = 1.0f - wl;
        const float* xs = in.pdist + i * 64 + k * REG;
        float p[REG];
        dfl_expect(xs, p);
        for (int j = 0; j < REG; ++j)
            gd[k * REG + j] = kdfl * ((wl + wr) * p[j] - (j == tl ? wl : 0.f) - (j == tl + 1 ? wr : 0.f));
    }
}

inline size_t al(size_t x) { return (x + 255) & ~size_t(255); }

struct Carve {
    AssignWs w;
    size_t bytes;
};

Carve carve(void* base, int64_t B, int64_t A, int M, int64_t nparts) {
    char* p = static_cast<char*>(base);
    size_t off = 0;
    auto take = [&](size_t n) { char* r = p ? p + off : nullptr; off += al(n); return r; };
    Carve c;
    size_t BA = size_t(B) * A, BM = size_t(B) * std::max(M, 1);
    // zeroed region first (one memset)
    c.w.amax = reinterpret_cast<unsigned long long*>(take(BM * 8));
    c.w.gcnt = reinterpret_cast<int*>(take(BM * 4));
    c.w.fcnt = reinterpret_cast<int*>(take(BA * 4));
    c.w.pbox = reinterpret_cast<float4*>(take(BA * 16));
    c.w.cnt0 = reinterpret_cast<int*>(take(BA * 4));
    c.w.g0 = reinterpret_cast<int*>(take(BA * 4));
    c.w.gmax = reinterpret_cast<int*>(take(BA * 4));
    c.w.fgg = reinterpret_cast<int*>(take(BA * 4));
    c.w.r1 = reinterpret_cast<int*>(take(BA * 4));
    c.w.tgi = reinterpret_cast<int*>(take(BA * 4));
    c.w.norm = reinterpret_cast<float*>(take(BA * 4));
    c.w.fg = reinterpret_cast<int*>(take(BA * 4));
    c.w.part = reinterpret_cast<double*>(take(size_t(nparts) * 5 * 8));
    c.bytes = off;
    return c;
}

size_t zero_bytes(int64_t B, int64_t A, int M) {
    size_t BA = size_t(B) * A, BM = size_t(B) * std::max(M, 1);
    return al(BM * 8) + al(BM * 4) + al(BA * 4);
}

}  // namespace
}  // namespace ym

using namespace ym;

static Levels make_levels(int nl, const int* lh, const int* lw, const float* strides) {
    Levels L{};
    L.n = nl;
    L.off[0] = 0;
    for (int l = 0; l < nl; ++l) {
        L.off[l + 1] = L.off[l] + int64_t(lh[l]) * lw[l];
        L.w[l] = lw[l];
        L.stride[l] = strides[l];
    }
    return L;
}

extern "C" size_t ym_loss_workspace_size(int64_t B, int64_t A, int M) {
    int64_t nparts = B * ((A + 255) / 256);
    return carve(nullptr, B, A, M, nparts).bytes + 256;
}

extern "C" int ym_loss_fwd(const float* head, int64_t B, int64_t A, int nc, int nl, const int* level_h,
                           const int* level_w, const float* strides, const int64_t* batch_idx, const int64_t* cls,
                           const float* bboxes, int64_t n_targets, int M, float imgsz_h, float imgsz_w,
                           void* workspace, size_t workspace_bytes, float* gt_box, float* gt_lab, int* gt_valid,
                           float* out, void* stream) {
    YM_CHECK_ARG(nl >= 1 && nl <= MAXLV, "ym_loss_fwd: 1..4 levels");
    YM_CHECK_ARG(nc >= 1 && nc <= 1024, "ym_loss_fwd: nc=%d out of range (1..1024)", nc);
    YM_CHECK_ARG(M >= 0 && M <= 4096, "ym_loss_fwd: M=%d out of range", M);
    hipStream_t st = as_stream(stream);
    Levels L = make_levels(nl, level_h, level_w, strides);
    YM_CHECK_ARG(L.off[nl] == A, "ym_loss_fwd: level sizes do not sum to A");
    const int no = 64 + nc;
    const int64_t nparts = B * ((A + 255) / 256);
    Carve c = carve(workspace, B, A, M, nparts);
    YM_CHECK_ARG(workspace_bytes >= c.bytes, "ym_loss_fwd: workspace too small");
    AssignWs w = c.w;
    w.out = out;
    if (hipMemsetAsync(workspace, 0, zero_bytes(B, A, M), st) != hipSuccess) return YM_ERR_HIP;
    dim3 ga(unsigned((A + 255) / 256), unsigned(B));
    if (M > 0) {
        hipLaunchKernelGGL(gt_prep_kernel, dim3(unsigned(B)), dim3(64), 0, st, batch_idx, cls, bboxes,
                           n_targets, int(B), M, imgsz_h, imgsz_w, reinterpret_cast<float4*>(gt_box), gt_lab, gt_valid);
        HeadSrc src{head, A, no, L};
        hipLaunchKernelGGL(assign_scan_kernel<HeadSrc>, ga, dim3(256), size_t(M) * 12, st, src, A,
                           reinterpret_cast<const float4*>(gt_box), gt_valid, M, w);
        hipLaunchKernelGGL(assign_resolve_kernel, dim3(unsigned(B)), dim3(RES_THREADS), size_t(M) * 5 * sizeof(int),
                           st, head, A, no, nc, reinterpret_cast<const float4*>(gt_box), gt_lab, gt_valid, M, w);
        hipLaunchKernelGGL(assign_norm_kernel<HeadSrc>, ga, dim3(256), 0, st, src, A,
                           reinterpret_cast<const float4*>(gt_box), gt_lab, M, w, 0.5f, 4.0f, EPS_TAL);
    } else {
        // no targets in the batch (:100-108 early return): all background
        if (hipMemsetAsync(w.fg, 0, size_t(B) * A * 4, st) != hipSuccess) return YM_ERR_HIP;
        if (hipMemsetAsync(w.tgi, 0, size_t(B) * A * 4, st) != hipSuccess) return YM_ERR_HIP;
        if (hipMemsetAsync(w.norm, 0, size_t(B) * A * 4, st) != hipSuccess) return YM_ERR_HIP;
    }
    hipLaunchKernelGGL(loss_partial_kernel, ga, dim3(256), 0, st, head, A, no, nc, L,
                       reinterpret_cast<const float4*>(gt_box), gt_lab, M, w);
    hipLaunchKernelGGL(loss_final_kernel, dim3(1), dim3(256), 0, st, int(nparts), int(B), w);
    YM_LAUNCH_CHECK("ym_loss_fwd");
    return YM_OK;
}

extern "C" int ym_loss_bwd(const float* head, int64_t B, int64_t A, int nc, int nl, const int* level_h,
                           const int* level_w, const float* strides, int M, void* workspace, size_t workspace_bytes,
                           const float* gt_box, const float* gt_lab, const float* out, const float* grad_out,
                           float* dhead, void* stream) {
    hipStream_t st = as_stream(stream);
    Levels L = make_levels(nl, level_h, level_w, strides);
    const int64_t nparts = B * ((A + 255) / 256);
    Carve c = carve(workspace, B, A, M, nparts);
    YM_CHECK_ARG(workspace_bytes >= c.bytes, "ym_loss_bwd: workspace too small");
    AssignWs w = c.w;
    w.out = const_cast<float*>(out);
    dim3 ga(unsigned((A + 255) / 256), unsigned(B));
    hipLaunchKernelGGL(loss_bwd_kernel, ga, dim3(256), 0, st, head, A, 64 + nc, nc, int(B), L,
                       reinterpret_cast<const float4*>(gt_box), gt_lab, M, w, grad_out, dhead);
    YM_LAUNCH_CHECK("ym_loss_bwd");
    return YM_OK;
}

extern "C" int ym_loss_assignment(void* workspace, int64_t B, int64_t A, int M, const int** tgi, const int** fg,
                                  const float** norm) {
    const int64_t nparts = B * ((A + 255) / 256);
    Carve c = carve(workspace, B, A, M, nparts);
    *tgi = c.w.tgi;
    *fg = c.w.fg;
    *norm = c.w.norm;
    return YM_OK;
}

extern "C" int ym_detect_decode(const float* head, int64_t B, int64_t A, int nc, int nl, const int* level_h,
                                const int* level_w, const float* strides, const float* dfl_w, float* y, void* stream) {
    Levels L = make_levels(nl, level_h, level_w, strides);
    YM_CHECK_ARG(L.off[nl] == A, "ym_detect_decode: level sizes do not sum to A");
    dim3 ga(unsigned((A + 255) / 256), unsigned(B));
    hipLaunchKernelGGL(detect_decode_kernel, ga, dim3(256), 0, as_stream(stream), head, A, 64 + nc, nc, L, dfl_w, y);
    YM_LAUNCH_CHECK("ym_detect_decode");
    return YM_OK;
}

// DFL.forward (yolo11_modules.py:189-192) on its own: x (B, 4*c1, A) -> softmax over the c1 bins of each
// side -> 1x1 conv with the module's c1 weights -> y (B, 4, A).  One thread per (anchor, side, image); the
// bins of a side are c1 rows A apart, so a wave's loads of one bin are one contiguous 256-B segment.
constexpr int DFL_MAX = 64;

__global__ void dfl_fwd_kernel(const float* __restrict__ x, int64_t A, int c1, const float* __restrict__ w,
                               float* __restrict__ y) {
    const int64_t a = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const int q = blockIdx.y, b = blockIdx.z;
    if (a >= A) return;
    const float* xs = x + (int64_t(b) * 4 + q) * c1 * A + a;
    float v[DFL_MAX];
    float m = -INFINITY;
    for (int j = 0; j < c1; ++j) { v[j] = xs[int64_t(j) * A]; m = fmaxf(m, v[j]); }
    float s = 0.f;
    for (int j = 0; j < c1; ++j) { v[j] = expf(v[j] - m); s += v[j]; }
    float acc = 0.f;
    for (int j = 0; j < c1; ++j) acc += (v[j] / s) * w[j];
    y[(int64_t(b) * 4 + q) * A + a] = acc;
}

// softmax backward in autograd's order: dp_j = w_j * dy, dx_j = p_j * (dp_j - sum_k p_k dp_k)
__global__ void dfl_bwd_kernel(const float* __restrict__ x, int64_t A, int c1, const float* __restrict__ w,
                               const float* __restrict__ dy, float* __restrict__ dx) {
    const int64_t a = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const int q = blockIdx.y, b = blockIdx.z;
    if (a >= A) return;
    const int64_t base = (int64_t(b) * 4 + q) * c1 * A + a;
    float v[DFL_MAX];
    float m = -INFINITY;
    for (int j = 0; j < c1; ++j) { v[j] = x[base + int64_t(j) * A]; m = fmaxf(m, v[j]); }
    float s = 0.f;
    for (int j = 0; j < c1; ++j) { v[j] = expf(v[j] - m); s += v[j]; }
    const float g = dy[(int64_t(b) * 4 + q) * A + a];
    float e = 0.f;
    for (int j = 0; j < c1; ++j) { v[j] = v[j] / s; e += v[j] * (w[j] * g); }
    for (int j = 0; j < c1; ++j) dx[base + int64_t(j) * A] = v[j] * (w[j] * g - e);
}

extern "C" int ym_dfl_fwd(const float* x, int64_t B, int64_t A, int c1, const float* w, float* y, void* stream) {
    YM_CHECK_ARG(c1 >= 1 && c1 <= DFL_MAX, "ym_dfl_fwd: c1=%d out of range (1..%d)", c1, DFL_MAX);
    YM_CHECK_ARG(B >= 0 && A >= 0 && B <= 65535, "ym_dfl_fwd: B=%lld A=%lld", (long long)B, (long long)A);
    if (B == 0 || A == 0) return YM_OK;
    dim3 g(unsigned((A + 255) / 256), 4, unsigned(B));
    hipLaunchKernelGGL(dfl_fwd_kernel, g, dim3(256), 0, as_stream(stream), x, A, c1, w, y);
    YM_LAUNCH_CHECK("ym_dfl_fwd");
    return YM_OK;
}

extern "C" int ym_dfl_bwd(const float* x, int64_t B, int64_t A, int c1, const float* w, const float* dy, float* dx,
                          void* stream) {
    YM_CHECK_ARG(c1 >= 1 && c1 <= DFL_MAX, "ym_dfl_bwd: c1=%d out of range (1..%d)", c1, DFL_MAX);
    YM_CHECK_ARG(B >= 0 && A >= 0 && B <= 65535, "ym_dfl_bwd: B=%lld A=%lld", (long long)B, (long long)A);
    if (B == 0 || A == 0) return YM_OK;
    dim3 g(unsigned((A + 255) / 256), 4, unsigned(B));
    hipLaunchKernelGGL(dfl_bwd_kernel, g, dim3(256), 0, as_stream(stream), x, A, c1, w, dy, dx);
    YM_LAUNCH_CHECK("ym_dfl_bwd");
    return YM_OK;
}

// TaskAlignedAssigner.forward (yolo_v8_loss.py:78-180) on explicit tensors; M >= 1 (the M = 0 early return
// :100-108 is the caller's).  Outputs: target_labels (B,A) f32, target_bboxes (B,A,4), target_scores
// (B,A,nc), fg_mask (B,A) u8, target_gt_idx (B,A) i64.
extern "C" size_t ym_tal_assign_workspace_size(int64_t B, int64_t A, int M) {
    return ym_loss_workspace_size(B, A, M) + 256 + size_t(B) * std::max(M, 1) * 4;
}

extern "C" int ym_tal_assign(const float* pd_scores, const float* pd_bboxes, const float* anc_points,
                             const float* gt_labels, const float* gt_bboxes, const float* mask_gt, int64_t B,
                             int64_t A, int nc, int M, float alpha, float beta, float eps, void* workspace,
                             size_t workspace_bytes, float* target_labels,
                             float* target_bboxes, float* target_scores, uint8_t* fg_mask, int64_t* target_gt_idx,
                             void* stream) {
    YM_CHECK_ARG(M >= 1 && M <= 4096, "ym_tal_assign: M=%d out of range (1..4096)", M);
    YM_CHECK_ARG(nc >= 1 && nc <= 1024, "ym_tal_assign: nc=%d out of range (1..1024)", nc);
    YM_CHECK_ARG((reinterpret_cast<uintptr_t>(gt_bboxes) & 15) == 0, "ym_tal_assign: gt_bboxes not 16-B aligned");
    YM_CHECK_ARG((reinterpret_cast<uintptr_t>(target_bboxes) & 15) == 0, "ym_tal_assign: target_bboxes not 16-B aligned");
    hipStream_t st = as_stream(stream);
    const int64_t nparts = B * ((A + 255) / 256);
    Carve c = carve(workspace, B, A, M, nparts);
    const size_t vbytes = size_t(B) * M * 4;
    YM_CHECK_ARG(workspace_bytes >= c.bytes + vbytes, "ym_tal_assign: workspace too small");
    int* valid = reinterpret_cast<int*>(static_cast<char*>(workspace) + c.bytes);
    AssignWs w = c.w;
    if (hipMemsetAsync(workspace, 0, zero_bytes(B, A, M), st) != hipSuccess) return YM_ERR_HIP;
    hipLaunchKernelGGL(mask_valid_kernel, dim3(unsigned((B * M + 255) / 256)), dim3(256), 0, st, mask_gt, B * M, valid);
    dim3 ga(unsigned((A + 255) / 256), unsigned(B));
    PlainSrc src{pd_scores, pd_bboxes, anc_points, A, nc};
    const float4* gb = reinterpret_cast<const float4*>(gt_bboxes);
    hipLaunchKernelGGL(assign_scan_kernel<PlainSrc>, ga, dim3(256), size_t(M) * 12, st, src, A, gb, valid, M, w);
    hipLaunchKernelGGL(assign_resolve_kernel, dim3(unsigned(B)), dim3(RES_THREADS), size_t(M) * 5 * sizeof(int), st,
                       nullptr, A, 0, nc, gb, gt_labels, valid, M, w);
    hipLaunchKernelGGL(assign_norm_kernel<PlainSrc>, ga, dim3(256), 0, st, src, A, gb, gt_labels, M, w, alpha, beta,
                       eps);
    hipLaunchKernelGGL(assign_targets_kernel, ga, dim3(256), 0, st, A, nc, gb, gt_labels, M, w, target_labels,
                       reinterpret_cast<float4*>(target_bboxes), target_scores, fg_mask, target_gt_idx);
    YM_LAUNCH_CHECK("ym_tal_assign");
    return YM_OK;
}

// BboxLoss.forward (yolo_v8_loss.py:280-324): out[0] = loss_iou, out[1] = loss_dfl; tss is a device scalar
extern "C" size_t ym_bbox_loss_workspace_size(int64_t B, int64_t A) { return size_t(B) * ((A + 255) / 256) * 16; }

extern "C" int ym_bbox_loss_fwd(const float* pred_dist, const float* pred_bboxes, const float* anchor_points,
                                const float* target_bboxes, const float* target_scores, const float* tss,
                                const uint8_t* fg_mask, int64_t B, int64_t A, int nc, void* workspace,
                                size_t workspace_bytes, float* out, void* stream) {
    YM_CHECK_ARG(nc >= 1 && nc <= 1024, "ym_bbox_loss_fwd: nc=%d out of range (1..1024)", nc);
    YM_CHECK_ARG(workspace_bytes >= ym_bbox_loss_workspace_size(B, A), "ym_bbox_loss_fwd: workspace too small");
    hipStream_t st = as_stream(stream);
    BoxIn in{pred_dist, pred_bboxes, anchor_points, target_bboxes, target_scores, fg_mask, A, nc};
    dim3 ga(unsigned((A + 255) / 256), unsigned(B));
    double* part = static_cast<double*>(workspace);
    hipLaunchKernelGGL(bbox_loss_partial_kernel, ga, dim3(256), 0, st, in, part);
    hipLaunchKernelGGL(bbox_loss_final_kernel, dim3(1), dim3(256), 0, st, part, int(ga.x * ga.y), tss, out);
    YM_LAUNCH_CHECK("ym_bbox_loss_fwd");
    return YM_OK;
}

extern "C" int ym_bbox_loss_bwd(const float* pred_dist, const float* pred_bboxes, const float* anchor_points,
                                const float* target_bboxes, const float* target_scores, const float* tss,
                                const uint8_t* fg_mask, int64_t B, int64_t A, int nc, const float* grad_out,
                                float* dpred_dist, float* dpred_bboxes, void* stream) {
    BoxIn in{pred_dist, pred_bboxes, anchor_points, target_bboxes, target_scores, fg_mask, A, nc};
    dim3 ga(unsigned((A + 255) / 256), unsigned(B));
    hipLaunchKernelGGL(bbox_loss_bwd_kernel, ga, dim3(256), 0, as_stream(stream), in, tss, grad_out, dpred_dist,
                       dpred_bboxes);
    YM_LAUNCH_CHECK("ym_bbox_loss_bwd");
    return YM_OK;
}
