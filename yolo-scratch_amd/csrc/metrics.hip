// Detection metrics on the GPU: P / R / mAP50 / mAP50-95 (gfx950).
//
// Replaces evaluate_detections / calculate_iou_batch / calculate_ap
// (/root/reference/yolo_scratch_cuda/utils/metrics.py:49-81, :84-274, :277-323).
// Class-agnostic greedy matching, exactly the reference's decisions:
//   * per image, predictions with score >= conf (fp32 compare, :117) in score-descending
//     order (stable: equal scores keep their input order, :161);
//   * each prediction takes the best *unmatched* GT (max IoU, first index on ties,
//     :184-190) and is a TP iff (double)IoU >= threshold (:194), which marks that GT;
//     no unmatched GT left -> FP (:175-179); an image without GT -> all FP (:156-160);
//   * IoU in the reference's fp32 op order (:67-79), this file is built -ffp-contract=off;
//   * AP (:277-323): detections of all images sorted by score descending with the TPs
//     ahead of the FPs on equal scores (Python's stable sort of tp_list + fp_list),
//     precision = tpc / (tpc + fpc + 1e-6), all-point envelope, sum of
//     delta-recall x envelope over the recall steps.  Computed in fp64.
//
// Pipeline (one stream, no host sync):
//   1. key1        per image block: key (image, score>=conf ? 0 : 1, ~score) + input index
//   2. radix sort  hipCUB, stable: per-image score order, filtered predictions last
//   3. match       one block per image, one wave per IoU threshold (all thresholds at
//                  once); GT boxes staged in LDS, each lane owns GTs lane+64k and keeps
//                  their "matched" bits in a 64-bit register mask (<= 4096 GT / image);
//                  prediction chunks staged in LDS; the wave's argmax is a shuffle
//                  reduction.  Emits one AP sort key per (threshold, prediction):
//                  (threshold, ~score, FP bit) -- filtered predictions get ~0 (sorted last)
//   4. radix sort  hipCUB over the 37-bit keys: per threshold, score descending, TP first
//   5. AP          chunked (2048 detections / block): TP counts -> exclusive scan ->
//                  per-chunk precision max -> reverse scan (envelope carry) -> per-chunk
//                  term sums -> fixed-order final sum (deterministic).
#include "common.h"

#include <hipcub/hipcub.hpp>

namespace ym {
namespace {

constexpr int MAX_THR = 15;          // thresholds per call (AP sort key field is 4 bits, 15 = filtered)
constexpr int GT_LDS = 2048;         // GT boxes staged in LDS per image (more: read through L2)
constexpr int GT_MAX = 4096;         // 64 lanes x 64-bit matched mask
constexpr int PCH = 512;             // predictions staged per LDS chunk
constexpr int AP_T = 256;            // threads of the AP kernels
constexpr int AP_ITEMS = 8;
constexpr int AP_CH = AP_T * AP_ITEMS;

struct Thr {
    double t[MAX_THR];
};

__host__ __device__ inline size_t al256(size_t x) { return (x + 255) & ~size_t(255); }

__device__ __forceinline__ float iou_ref(float4 a, float4 b) {
    float x1 = fmaxf(a.x, b.x), y1 = fmaxf(a.y, b.y);
    float x2 = fminf(a.z, b.z), y2 = fminf(a.w, b.w);
    float iw = x2 - x1, ih = y2 - y1;
    iw = iw < 0.0f ? 0.0f : iw;
    ih = ih < 0.0f ? 0.0f : ih;
    float inter = iw * ih;
    float a1 = (a.z - a.x) * (a.w - a.y);
    float a2 = (b.z - b.x) * (b.w - b.y);
    float uni = a1 + a2;
    uni = uni - inter;
    return inter / (uni + 1e-6f);
}

// 32-bit key that sorts ascending in descending-score order
__device__ __forceinline__ uint32_t desc_key(float s) {
    uint32_t u = __float_as_uint(s);
    uint32_t ord = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    return ~ord;
}

struct Ws {
    uint64_t* k1in;   // [n_pred]
    uint64_t* k1out;
    int32_t* v1in;    // [n_pred] input index
    int32_t* v1out;
    uint64_t* k2in;   // [n_thr][n_pred]
    uint64_t* k2out;
    int32_t* tcnt;    // [n_thr][cps] TP per chunk
    int32_t* tbase;   // [n_thr][cps] exclusive prefix
    int32_t* ttot;    // [n_thr]
    double* cmax;     // [n_thr][cps] chunk max precision
    double* carry;    // [n_thr][cps] max precision of later chunks
    double* psum;     // [n_thr][cps] chunk term sums
    int32_t* nvalid;  // [1] filtered-in predictions (all images)
    int32_t* bad;     // [1] an image exceeded GT_MAX
    void* cub;
    size_t cub_bytes;
};

inline int key1_bits(int64_t n_img) {
    int nb = 0;
    while ((int64_t(1) << nb) < n_img) ++nb;
    return 33 + nb;
}

size_t cub_bytes_for(int64_t n_img, int64_t n_pred, int n_thr) {
    size_t a = 0, b = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, a, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                       (const int32_t*)nullptr, (int32_t*)nullptr, int(n_pred), 0, key1_bits(n_img));
    (void)hipcub::DeviceRadixSort::SortKeys(nullptr, b, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                      int(n_pred * n_thr), 0, 37);
    return a > b ? a : b;
}

size_t layout(char* base, int64_t n_img, int64_t n_pred, int n_thr, Ws* w) {
    size_t n = size_t(n_pred), cps = size_t((n_pred + AP_CH - 1) / AP_CH), nt = size_t(n_thr);
    size_t off = 0;
    auto take = [&](size_t bytes) { char* p = base ? base + off : nullptr; off += al256(bytes); return p; };
    Ws v;
    v.k1in = (uint64_t*)take(n * 8);
    v.k1out = (uint64_t*)take(n * 8);
    v.v1in = (int32_t*)take(n * 4);
    v.v1out = (int32_t*)take(n * 4);
    v.k2in = (uint64_t*)take(n * nt * 8);
    v.k2out = (uint64_t*)take(n * nt * 8);
    v.tcnt = (int32_t*)take(nt * cps * 4);
    v.tbase = (int32_t*)take(nt * cps * 4);
    v.ttot = (int32_t*)take(nt * 4);
    v.cmax = (double*)take(nt * cps * 8);
    v.carry = (double*)take(nt * cps * 8);
    v.psum = (double*)take(nt * cps * 8);
    v.nvalid = (int32_t*)take(8);
    v.bad = v.nvalid + 1;
    v.cub_bytes = cub_bytes_for(n_img, n_pred, n_thr);
    v.cub = take(v.cub_bytes);
    if (w) *w = v;
    return off;
}

// ---------------------------------------------------------------- 1. per-image sort keys
__global__ __launch_bounds__(256) void key1_kernel(const float* __restrict__ score, const int64_t* __restrict__ poff,
                                                   float conf, Ws w) {
    const int64_t b = blockIdx.x;
    const int64_t p0 = poff[b], p1 = poff[b + 1];
    for (int64_t i = p0 + threadIdx.x; i < p1; i += blockDim.x) {
        float s = score[i];
        uint64_t excl = s >= conf ? 0u : 1u;
        w.k1in[i] = (uint64_t(b) << 33) | (excl << 32) | uint64_t(desc_key(s));
        w.v1in[i] = int32_t(i);
    }
}

// ---------------------------------------------------------------- 3. greedy matching
// blockDim = 64 * n_thr; wave t matches at threshold t.
__global__ __launch_bounds__(64 * MAX_THR) void match_kernel(
    const float4* __restrict__ pbox, const float* __restrict__ pscore, const int64_t* __restrict__ poff,
    const float4* __restrict__ gbox, const int64_t* __restrict__ goff, float conf, Thr thr, int64_t n_pred, Ws w) {
    __shared__ float4 sg[GT_LDS];
    __shared__ float4 sp[PCH];
    __shared__ uint32_t sd[PCH];
    __shared__ uint8_t sv[PCH];
    const int b = blockIdx.x;
    const int tid = threadIdx.x, nthr = blockDim.x;
    const int t = tid >> 6, lane = tid & 63;
    const int64_t p0 = poff[b], p1 = poff[b + 1];
    const int64_t g0 = goff[b];
    int G = int(goff[b + 1] - g0);
    if (G > GT_MAX) {                       // host checks too; never match partially
        if (tid == 0) atomicOr(w.bad, 1);
        G = 0;
    }
    const float4* gb = gbox + g0;
    if (G <= GT_LDS) {
        for (int j = tid; j < G; j += nthr) sg[j] = gb[j];
        gb = sg;
    }
    const double th = thr.t[t];
    const uint64_t tkey = uint64_t(t) << 33;
    uint64_t* keys = w.k2in + int64_t(t) * n_pred;
    uint64_t used = 0;                      // bit k: GT lane + 64k matched
    int nvalid = 0;
    for (int64_t c0 = p0; c0 < p1; c0 += PCH) {
        const int n = int(p1 - c0 < PCH ? p1 - c0 : PCH);
        __syncthreads();
        for (int i = tid; i < n; i += nthr) {
            int o = w.v1out[c0 + i];
            float s = pscore[o];
            sp[i] = pbox[o];
            sd[i] = desc_key(s);
            sv[i] = s >= conf;
        }
        __syncthreads();
        for (int i = 0; i < n; ++i) {
            const int64_t p = c0 + i;
            if (!sv[i]) {                   // filtered out: sorted last in its image
                if (lane == 0) keys[p] = ~uint64_t(0);
                continue;
            }
            ++nvalid;
            uint64_t fp = 1;
            if (G > 0) {
                const float4 a = sp[i];
                float best = -INFINITY;
                int bj = INT32_MAX;
                for (int k = 0; k * 64 < G; ++k) {
                    int j = lane + 64 * k;
                    if (j < G && !((used >> k) & 1)) {
                        float v = iou_ref(a, gb[j]);
                        if (v > best || bj == INT32_MAX) {
                            best = v;
                            bj = j;
                        }
                    }
                }
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) {
                    float ob = __shfl_xor(best, o, 64);
                    int oj = __shfl_xor(bj, o, 64);
                    if (oj != INT32_MAX && (bj == INT32_MAX || ob > best || (ob == best && oj < bj))) {
                        best = ob;
                        bj = oj;
                    }
                }
                if (bj != INT32_MAX && double(best) >= th) {
                    fp = 0;
                    if (lane == (bj & 63)) used |= uint64_t(1) << (bj >> 6);
                }
            }
            if (lane == 0) keys[p] = tkey | (uint64_t(sd[i]) << 1) | fp;
        }
    }
    if (tid == 0) atomicAdd(w.nvalid, nvalid);
}

// ---------------------------------------------------------------- block scans (256 threads)
template <typename T, typename Op>
__device__ T block_scan_incl(T v, Op op, T* sm, bool reverse) {
    const int tid = threadIdx.x;
    const int pos = reverse ? AP_T - 1 - tid : tid;
    sm[pos] = v;
    __syncthreads();
    for (int o = 1; o < AP_T; o <<= 1) {
        T x = pos >= o ? op(sm[pos - o], sm[pos]) : sm[pos];
        __syncthreads();
        sm[pos] = x;
        __syncthreads();
    }
    T r = sm[pos];
    __syncthreads();
    return r;
}

struct AddI {
    __device__ int operator()(int a, int b) const { return a + b; }
};
struct MaxD {
    __device__ double operator()(double a, double b) const { return a > b ? a : b; }
};
struct AddD {
    __device__ double operator()(double a, double b) const { return a + b; }
};

// ---------------------------------------------------------------- 5. AP over the sorted keys
// grid (cps, n_thr); segment t = sorted keys [t*NV, (t+1)*NV)
__global__ __launch_bounds__(AP_T) void ap_count_kernel(Ws w, int cps) {
    __shared__ int sm[AP_T];
    const int c = blockIdx.x, t = blockIdx.y;
    const int64_t NV = *w.nvalid;
    const uint64_t* key = w.k2out + t * NV;
    int cnt = 0;
    for (int e = 0; e < AP_ITEMS; ++e) {
        int64_t j = int64_t(c) * AP_CH + threadIdx.x * AP_ITEMS + e;
        if (j < NV) cnt += !(key[j] & 1);
    }
    cnt = block_scan_incl(cnt, AddI(), sm, false);
    if (threadIdx.x == AP_T - 1) w.tcnt[t * cps + c] = cnt;
}

// one block per threshold.  mode 0: exclusive scan of the chunk TP counts (+ segment total);
// mode 1: carry[c] = max(cmax[c+1..cps)), 0 past the end (the reference's trailing 0 sentinel)
__global__ __launch_bounds__(AP_T) void ap_scan_kernel(Ws w, int cps, int mode) {
    __shared__ int si[AP_T];
    __shared__ double sd[AP_T];
    __shared__ int itot;
    __shared__ double nxt[AP_T + 1];
    const int t = blockIdx.x;
    if (mode == 0) {
        int run = 0;
        for (int c0 = 0; c0 < cps; c0 += AP_T) {
            int c = c0 + threadIdx.x;
            int v = c < cps ? w.tcnt[t * cps + c] : 0;
            int inc = block_scan_incl(v, AddI(), si, false);
            if (c < cps) w.tbase[t * cps + c] = run + inc - v;
            if (threadIdx.x == AP_T - 1) itot = inc;
            __syncthreads();
            run += itot;
            __syncthreads();
        }
        if (threadIdx.x == 0) w.ttot[t] = run;
        return;
    }
    double run = 0.0;
    for (int r = (cps + AP_T - 1) / AP_T - 1; r >= 0; --r) {
        int c = r * AP_T + threadIdx.x;
        double v = c < cps ? w.cmax[t * cps + c] : 0.0;
        double inc = block_scan_incl(v, MaxD(), sd, true);   // this chunk and later ones of the round
        nxt[threadIdx.x] = inc;
        if (threadIdx.x == 0) nxt[AP_T] = run;
        __syncthreads();
        double later = nxt[AP_T];
        if (threadIdx.x + 1 < AP_T) later = nxt[threadIdx.x + 1] > later ? nxt[threadIdx.x + 1] : later;
        if (c < cps) w.carry[t * cps + c] = later;
        double first = nxt[0];
        __syncthreads();
        run = first > run ? first : run;
    }
}

// mode 0: chunk max of precision -> cmax;  mode 1: envelope terms -> psum
__global__ __launch_bounds__(AP_T) void ap_chunk_kernel(Ws w, int cps, double n_gt, int mode) {
    __shared__ int si[AP_T];
    __shared__ double sd[AP_T];
    const int c = blockIdx.x, t = blockIdx.y;
    const int64_t NV = *w.nvalid;
    const uint64_t* key = w.k2out + t * NV;
    const int64_t j0 = int64_t(c) * AP_CH + threadIdx.x * AP_ITEMS;
    int flags = 0, cnt = 0;
    for (int e = 0; e < AP_ITEMS; ++e) {
        int64_t j = j0 + e;
        int tp = j < NV ? !(key[j] & 1) : 0;
        flags |= tp << e;
        cnt += tp;
    }
    const int inc = block_scan_incl(cnt, AddI(), si, false);
    int tpc = w.tbase[t * cps + c] + inc - cnt;     // TPs before this thread's first element
    int tpcs[AP_ITEMS];
    double prec[AP_ITEMS];
    double tmax = 0.0;
    for (int e = 0; e < AP_ITEMS; ++e) {
        int64_t j = j0 + e;
        tpc += (flags >> e) & 1;
        tpcs[e] = tpc;
        prec[e] = j < NV ? double(tpc) / (double(j + 1) + 1e-6) : 0.0;
        tmax = prec[e] > tmax ? prec[e] : tmax;
    }
    if (mode == 0) {
        double m = block_scan_incl(tmax, MaxD(), sd, false);
        if (threadIdx.x == AP_T - 1) w.cmax[t * cps + c] = m;
        return;
    }
    // envelope: max over this and every later detection of the segment
    double after = block_scan_incl(tmax, MaxD(), sd, true);      // this thread and later threads
    __shared__ double nxt[AP_T + 1];
    nxt[threadIdx.x] = after;
    if (threadIdx.x == 0) nxt[AP_T] = w.carry[t * cps + c];
    __syncthreads();
    double env = nxt[AP_T];
    if (threadIdx.x + 1 < AP_T) env = nxt[threadIdx.x + 1] > env ? nxt[threadIdx.x + 1] : env;
    // walk backwards so env is the suffix max at each element; terms summed front to back
    double term[AP_ITEMS];
    for (int e = AP_ITEMS - 1; e >= 0; --e) {
        env = prec[e] > env ? prec[e] : env;
        term[e] = ((flags >> e) & 1) ? (double(tpcs[e]) / n_gt - double(tpcs[e] - 1) / n_gt) * env : 0.0;
    }
    double sum = 0.0;
    for (int e = 0; e < AP_ITEMS; ++e) sum += term[e];
    sum = block_scan_incl(sum, AddD(), sd, false);
    if (threadIdx.x == AP_T - 1) w.psum[t * cps + c] = sum;
}

// numpy.add.reduce's pairwise order for n <= 128 (8 accumulators), used for np.mean of the APs
__device__ double np_sum_small(const double* a, int n) {
    if (n < 8) {
        double r = -0.0;
        for (int i = 0; i < n; ++i) r += a[i];
        return r;
    }
    double r[8];
    for (int k = 0; k < 8; ++k) r[k] = a[k];
    int i = 8;
    for (; i < n - (n % 8); i += 8)
        for (int k = 0; k < 8; ++k) r[k] += a[i + k];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
}

// out: [n_thr] AP, then precision, recall, mAP50, mAP50-95, tp, fp, n_valid
__global__ void ap_final_kernel(Ws w, int cps, int n_thr, int n_ap, int pr_index, double n_gt, double* out) {
    if (threadIdx.x != 0) return;
    double ap[MAX_THR];
    const int64_t NV = *w.nvalid;
    const bool bad = *w.bad != 0;
    for (int t = 0; t < n_thr; ++t) {
        double s = 0.0;
        for (int c = 0; c < cps; ++c) s += w.psum[t * cps + c];
        ap[t] = (n_gt == 0.0 || NV == 0) ? 0.0 : s;
        out[t] = bad ? NAN : ap[t];
    }
    const double tp = w.ttot[pr_index], fp = double(NV) - tp;
    double* o = out + n_thr;
    o[0] = (tp + fp) > 0 ? tp / (tp + fp) : 0.0;
    o[1] = n_gt > 0 ? tp / n_gt : 0.0;
    o[2] = n_ap > 0 ? ap[0] : 0.0;
    o[3] = n_ap > 0 ? np_sum_small(ap, n_ap) / double(n_ap) : 0.0;
    o[4] = tp;
    o[5] = fp;
    o[6] = double(NV);
    if (bad)
        for (int k = 0; k < 4; ++k) o[k] = NAN;
}

// calculate_ap on a flat list: one AP key per detection (score, TP flag)
__global__ __launch_bounds__(256) void ap_list_keys_kernel(const float* __restrict__ score,
                                                           const uint8_t* __restrict__ is_tp, int64_t n, Ws w) {
    int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i == 0) {
        *w.nvalid = int32_t(n);
        *w.bad = 0;
    }
    if (i < n) w.k2in[i] = (uint64_t(desc_key(score[i])) << 1) | uint64_t(is_tp[i] ? 0 : 1);
}

// calculate_iou_batch: (n, m) IoU matrix, reference fp32 op order
__global__ __launch_bounds__(256) void iou_matrix_kernel(const float4* __restrict__ a, const float4* __restrict__ b,
                                                         int64_t n, int64_t m, float* __restrict__ out) {
    int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (idx < n * m) out[idx] = iou_ref(a[idx / m], b[idx % m]);
}

int launch_ap(const Ws& w, int cps, int n_thr, double n_gt, hipStream_t st) {
    hipLaunchKernelGGL(ap_count_kernel, dim3(cps, n_thr), dim3(AP_T), 0, st, w, cps);
    YM_LAUNCH_CHECK("eval ap_count");
    hipLaunchKernelGGL(ap_scan_kernel, dim3(n_thr), dim3(AP_T), 0, st, w, cps, 0);
    YM_LAUNCH_CHECK("eval ap_scan");
    hipLaunchKernelGGL(ap_chunk_kernel, dim3(cps, n_thr), dim3(AP_T), 0, st, w, cps, n_gt, 0);
    YM_LAUNCH_CHECK("eval ap_max");
    hipLaunchKernelGGL(ap_scan_kernel, dim3(n_thr), dim3(AP_T), 0, st, w, cps, 1);
    YM_LAUNCH_CHECK("eval ap_carry");
    hipLaunchKernelGGL(ap_chunk_kernel, dim3(cps, n_thr), dim3(AP_T), 0, st, w, cps, n_gt, 1);
    YM_LAUNCH_CHECK("eval ap_terms");
    return YM_OK;
}

}  // namespace
}  // namespace ym

using namespace ym;

extern "C" size_t ym_eval_workspace_size(int64_t n_img, int64_t n_pred, int n_thr) {
    if (n_pred < 1) n_pred = 1;
    return layout(nullptr, n_img, n_pred, n_thr, nullptr);
}

extern "C" int ym_eval_detections(const float* pred_boxes, const float* pred_scores, const int64_t* pred_off,
                                  const float* gt_boxes, const int64_t* gt_off, int64_t n_img, int64_t n_pred,
                                  int64_t n_gt, int64_t max_gt_per_img, const double* thresholds, int n_thr, int n_ap,
                                  int pr_index, float conf, void* workspace, size_t workspace_bytes, double* out,
                                  void* stream) {
    YM_CHECK_ARG(n_img >= 0 && n_pred >= 0 && n_gt >= 0, "ym_eval_detections: negative size");
    YM_CHECK_ARG(n_thr >= 1 && n_thr <= MAX_THR, "ym_eval_detections: n_thr=%d outside 1..%d", n_thr, MAX_THR);
    YM_CHECK_ARG(n_ap >= 0 && n_ap <= n_thr && pr_index >= 0 && pr_index < n_thr,
                 "ym_eval_detections: bad n_ap / pr_index");
    YM_CHECK_ARG(max_gt_per_img <= GT_MAX, "ym_eval_detections: %lld GT boxes in one image (max %d)",
                 (long long)max_gt_per_img, GT_MAX);
    YM_CHECK_ARG(n_pred < (int64_t(1) << 31) / MAX_THR, "ym_eval_detections: too many predictions");
    YM_CHECK_ARG(n_img < (int64_t(1) << 30), "ym_eval_detections: too many images");
    hipStream_t st = as_stream(stream);
    const int64_t np1 = n_pred < 1 ? 1 : n_pred;
    YM_CHECK_ARG(workspace_bytes >= layout(nullptr, n_img, np1, n_thr, nullptr),
                 "ym_eval_detections: workspace too small (%zu)", workspace_bytes);
    Ws w;
    layout(static_cast<char*>(workspace), n_img, np1, n_thr, &w);
    Thr thr{};
    for (int t = 0; t < n_thr; ++t) thr.t[t] = thresholds[t];
    const int cps = int((np1 + AP_CH - 1) / AP_CH);
    if (hipMemsetAsync(w.nvalid, 0, 8, st) != hipSuccess) return YM_ERR_HIP;
    if (hipMemsetAsync(w.ttot, 0, n_thr * sizeof(int32_t), st) != hipSuccess) return YM_ERR_HIP;
    if (hipMemsetAsync(w.psum, 0, size_t(n_thr) * cps * sizeof(double), st) != hipSuccess) return YM_ERR_HIP;
    if (n_img > 0 && n_pred > 0) {
        hipLaunchKernelGGL(key1_kernel, dim3(unsigned(n_img)), dim3(256), 0, st, pred_scores, pred_off, conf, w);
        YM_LAUNCH_CHECK("eval key1");
        size_t cb = w.cub_bytes;
        if (hipcub::DeviceRadixSort::SortPairs(w.cub, cb, w.k1in, w.k1out, w.v1in, w.v1out, int(n_pred), 0, key1_bits(n_img),
                                               st) != hipSuccess) {
            set_error("ym_eval_detections: per-image sort failed");
            return YM_ERR_HIP;
        }
        hipLaunchKernelGGL(match_kernel, dim3(unsigned(n_img)), dim3(64 * n_thr), 0, st,
                           reinterpret_cast<const float4*>(pred_boxes), pred_scores, pred_off,
                           reinterpret_cast<const float4*>(gt_boxes), gt_off, conf, thr, n_pred, w);
        YM_LAUNCH_CHECK("eval match");
        cb = w.cub_bytes;
        if (hipcub::DeviceRadixSort::SortKeys(w.cub, cb, w.k2in, w.k2out, int(n_pred * n_thr), 0, 37, st) !=
            hipSuccess) {
            set_error("ym_eval_detections: AP sort failed");
            return YM_ERR_HIP;
        }
        int rc = launch_ap(w, cps, n_thr, double(n_gt), st);
        if (rc != YM_OK) return rc;
    }
    hipLaunchKernelGGL(ap_final_kernel, dim3(1), dim3(64), 0, st, w, cps, n_thr, n_ap, pr_index, double(n_gt), out);
    YM_LAUNCH_CHECK("eval ap_final");
    return YM_OK;
}

extern "C" int ym_eval_ap(const float* scores, const uint8_t* is_tp, int64_t n, int64_t n_gt, void* workspace,
                          size_t workspace_bytes, double* out, void* stream) {
    YM_CHECK_ARG(n >= 0 && n_gt >= 0, "ym_eval_ap: negative size");
    YM_CHECK_ARG(n < (int64_t(1) << 31) / MAX_THR, "ym_eval_ap: too many detections");
    hipStream_t st = as_stream(stream);
    const int64_t np1 = n < 1 ? 1 : n;
    YM_CHECK_ARG(workspace_bytes >= layout(nullptr, 1, np1, 1, nullptr), "ym_eval_ap: workspace too small (%zu)",
                 workspace_bytes);
    Ws w;
    layout(static_cast<char*>(workspace), 1, np1, 1, &w);
    const int cps = int((np1 + AP_CH - 1) / AP_CH);
    if (hipMemsetAsync(w.nvalid, 0, 8, st) != hipSuccess) return YM_ERR_HIP;
    if (hipMemsetAsync(w.ttot, 0, sizeof(int32_t), st) != hipSuccess) return YM_ERR_HIP;
    if (hipMemsetAsync(w.psum, 0, size_t(cps) * sizeof(double), st) != hipSuccess) return YM_ERR_HIP;
    if (n > 0) {
        hipLaunchKernelGGL(ap_list_keys_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, st, scores, is_tp, n,
                           w);
        YM_LAUNCH_CHECK("eval ap keys");
        size_t cb = w.cub_bytes;
        if (hipcub::DeviceRadixSort::SortKeys(w.cub, cb, w.k2in, w.k2out, int(n), 0, 33, st) != hipSuccess) {
            set_error("ym_eval_ap: sort failed");
            return YM_ERR_HIP;
        }
        int rc = launch_ap(w, cps, 1, double(n_gt), st);
        if (rc != YM_OK) return rc;
    }
    hipLaunchKernelGGL(ap_final_kernel, dim3(1), dim3(64), 0, st, w, cps, 1, 1, 0, double(n_gt), out);
    YM_LAUNCH_CHECK("eval ap_final");
    return YM_OK;
}

extern "C" int ym_iou_matrix(const float* boxes1, const float* boxes2, int64_t n, int64_t m, float* out,
                             void* stream) {
    YM_CHECK_ARG(n >= 0 && m >= 0, "ym_iou_matrix: negative size");
    if (n == 0 || m == 0) return YM_OK;
    hipLaunchKernelGGL(iou_matrix_kernel, dim3(unsigned((n * m + 255) / 256)), dim3(256), 0, as_stream(stream),
                       reinterpret_cast<const float4*>(boxes1), reinterpret_cast<const float4*>(boxes2), n, m, out);
    YM_LAUNCH_CHECK("ym_iou_matrix");
    return YM_OK;
}
