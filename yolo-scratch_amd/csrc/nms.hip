// Decode + class-agnostic greedy NMS, one workgroup per image (gfx950).
//
// Replaces decode_predictions_for_metrics / nms_simple / calculate_iou_batch_simple
// (/root/reference/yolo_scratch_cuda/train_yolo11_cuda.py:265-437).  Bit-exact
// with the reference on tie-free scores: the IoU is evaluated in the same fp32
// op order and this file is compiled with -ffp-contract=off.
//
// Pipeline per call
//   1. rowmax kernel      grid over rows: max/argmax over the C class scores,
//                         `> conf` flag, xywh -> xyxy            (:296-329)
//   2. nms_image kernel   one 1024-thread workgroup per image:
//        a. order-preserving compaction of flagged rows (block scan)
//        b. bitonic sort of 64-bit keys (~score, filtered index): score
//           descending, index ascending (the reference's argsort is unstable;
//           golden inputs are tie-free)                          (:377)
//        c. greedy loop: the head box is broadcast through LDS, every thread
//           tests the boxes it holds in registers, drops IoU > thr, and a
//           block min-reduction finds the next alive head        (:380-397)
//        d. write kept boxes / img_size clamped to [0,1]          (:342-350)
#include <cstdlib>

#include "common.h"
#include "tile.h"

namespace ym {
namespace {

constexpr int NMS_THREADS = 1024;
constexpr int NMS_WAVES = NMS_THREADS / 64;
constexpr int SORT_LDS_KEYS = 16384;   // 128 KiB of keys in LDS
constexpr int REG_ITEMS = 8;           // boxes held in registers per thread (K <= 8192)

struct Ws {
    float4* box;      // [B][N] xyxy of every row
    float* score;     // [B][N]
    int32_t* label;   // [B][N]
    int32_t* flag;    // [B][N]
    int32_t* frow;    // [B][N] filtered index -> row
    uint64_t* keys;   // [B][KP] (global sort path; sorted keys of the bitmask path)
    float4* sbox;     // [B][N] boxes in sorted order      (bitmask path)
    uint64_t* mask;   // [B][N][Wn] suppression bitmask    (bitmask path)
    int32_t* kcount;  // [B] candidates after the filter   (bitmask path)
};

// Bitmask path (small batches: one image is too little work for one workgroup's greedy loop):
// sort per image, then the upper-triangular IoU > thr bitmask of the sorted candidates over the
// whole GPU, then a chunked greedy scan per image.  Needs the [64][Wn] chunk double buffer in LDS.
constexpr int64_t BM_MAX_B = 8;
constexpr int64_t BM_MAX_WN = 150;            // N <= 9600 (640x640: 8400 anchors)
inline bool bitmask_path(int64_t B, int64_t N) { return B <= BM_MAX_B && (N + 63) / 64 <= BM_MAX_WN && N >= 128; }

__host__ __device__ inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

inline int64_t pow2_at_least(int64_t x) {
    int64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

inline size_t bitmask_bytes(int64_t B, int64_t N) {
    if (!bitmask_path(B, N)) return 0;
    const size_t n = size_t(B) * size_t(N), wn = size_t((N + 63) / 64);
    return align256(n * 16) + align256(n * wn * 8) + align256(size_t(B) * 4);
}

inline Ws carve(void* base, int64_t B, int64_t N) {
    char* p = static_cast<char*>(base);
    size_t n = size_t(B) * size_t(N);
    Ws w;
    w.box = reinterpret_cast<float4*>(p);   p += align256(n * sizeof(float4));
    w.score = reinterpret_cast<float*>(p);  p += align256(n * sizeof(float));
    w.label = reinterpret_cast<int32_t*>(p); p += align256(n * sizeof(int32_t));
    w.flag = reinterpret_cast<int32_t*>(p); p += align256(n * sizeof(int32_t));
    w.frow = reinterpret_cast<int32_t*>(p); p += align256(n * sizeof(int32_t));
    w.keys = reinterpret_cast<uint64_t*>(p); p += align256(size_t(B) * pow2_at_least(N) * 8);
    w.sbox = nullptr; w.mask = nullptr; w.kcount = nullptr;
    if (bitmask_path(B, N)) {
        const size_t wn = size_t((N + 63) / 64);
        w.sbox = reinterpret_cast<float4*>(p);   p += align256(n * 16);
        w.mask = reinterpret_cast<uint64_t*>(p); p += align256(n * wn * 8);
        w.kcount = reinterpret_cast<int32_t*>(p);
    }
    return w;
}

inline size_t ws_bytes(int64_t B, int64_t N) {
    size_t n = size_t(B) * size_t(N);
    return align256(n * 16) + 4 * align256(n * 4) + align256(size_t(B) * pow2_at_least(N) * 8) + bitmask_bytes(B, N) +
           256;
}

// IoU in the reference's op order (train_yolo11_cuda.py:418-435).
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

__device__ __forceinline__ uint32_t desc_bits(float s) {
    uint32_t u = __float_as_uint(s);
    uint32_t ord = (u & 0x80000000u) ? ~u : (u | 0x80000000u);   // ascending-order bits
    return ~ord;                                                  // descending
}

// ---------------------------------------------------------------- stage 1
// thread per row (C small) — max/argmax with the first maximal index winning; cs: the stride between a row's
// elements (1: row-major rows; A: the anchor-major view of the (B, 4+nc, A) eval output, read coalesced across rows)
__global__ void rowmax_thread_kernel(const float* __restrict__ pred, int64_t B, int64_t N, int64_t C,
                                     int64_t rs, int64_t is, int64_t cs, float conf, Ws w) {
    int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= B * N) return;
    int64_t b = i / N, n = i - b * N;
    const float* r = pred + b * is + n * rs;
    float mx = r[4 * cs];
    int lab = 0;
    for (int64_t c = 1; c < C; ++c) {
        float v = r[(4 + c) * cs];
        if (v > mx) { mx = v; lab = int(c); }
    }
    float x = r[0], y = r[cs], hw = r[2 * cs] / 2.0f, hh = r[3 * cs] / 2.0f;
    w.box[i] = make_float4(x - hw, y - hh, x + hw, y + hh);
    w.score[i] = mx;
    w.label[i] = lab;
    w.flag[i] = (mx > conf) ? 1 : 0;
}

// wave per row (C large, e.g. the literal (B, 4+nc, A) eval layout)
__global__ void rowmax_wave_kernel(const float* __restrict__ pred, int64_t B, int64_t N, int64_t C,
                                   int64_t rs, int64_t is, int64_t cs, float conf, Ws w) {
    int64_t i = int64_t(blockIdx.x) * (blockDim.x / 64) + threadIdx.x / 64;
    int lane = threadIdx.x & 63;
    if (i >= B * N) return;
    int64_t b = i / N, n = i - b * N;
    const float* r = pred + b * is + n * rs;
    float mx = -INFINITY;
    int64_t lab = INT64_MAX;
    for (int64_t c = lane; c < C; c += 64) {
        float v = r[(4 + c) * cs];
        if (v > mx || (v == mx && c < lab)) { mx = v; lab = c; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        float om = __shfl_xor(mx, o, 64);
        int64_t ol = __shfl_xor(lab, o, 64);
        if (om > mx || (om == mx && ol < lab)) { mx = om; lab = ol; }
    }
    if (lane == 0) {
        float x = r[0], y = r[cs], hw = r[2 * cs] / 2.0f, hh = r[3 * cs] / 2.0f;
        w.box[i] = make_float4(x - hw, y - hh, x + hw, y + hh);
        w.score[i] = mx;
        w.label[i] = int32_t(lab);
        w.flag[i] = (mx > conf) ? 1 : 0;
    }
}

// direct candidates (nms_simple): every box is a candidate
__global__ void direct_kernel(const float4* __restrict__ boxes, const float* __restrict__ scores, int64_t n, Ws w) {
    int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    w.box[i] = boxes[i];
    w.score[i] = scores[i];
    w.label[i] = 0;
    w.flag[i] = 1;
}

// ---------------------------------------------------------------- stage 2 helpers
__device__ int block_excl_scan(int v, int* sh, int& total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) sh[wv] = x;
    __syncthreads();
    if (wv == 0) {
        int s = lane < NMS_WAVES ? sh[lane] : 0;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            int y = __shfl_up(s, o, 64);
            if (lane >= o) s += y;
        }
        if (lane < NMS_WAVES) sh[lane] = s;
    }
    __syncthreads();
    int before = (wv > 0 ? sh[wv - 1] : 0) + x - v;
    total = sh[NMS_WAVES - 1];
    __syncthreads();
    return before;
}

__device__ int block_min(int v, int* sh) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    if (lane == 0) sh[wv] = v;
    __syncthreads();
    int r = sh[0];
#pragma unroll
    for (int k = 1; k < NMS_WAVES; ++k) r = min(r, sh[k]);
    __syncthreads();
    return r;
}

template <bool IN_LDS>
__device__ void bitonic(uint64_t* keys, int P) {
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < P; i += NMS_THREADS) {
                int l = i ^ j;
                if (l > i) {
                    uint64_t a = keys[i], c = keys[l];
                    bool up = (i & k) == 0;
                    if ((a > c) == up) { keys[i] = c; keys[l] = a; }
                }
            }
            if (IN_LDS) __syncthreads();
            else { __threadfence_block(); __syncthreads(); }
        }
    }
}

// ---------------------------------------------------------------- stage 2
template <bool SORT_ONLY>
__global__ void __launch_bounds__(NMS_THREADS)
nms_image_kernel(int64_t N, int64_t KP, float iou_thr, float img_size, int clamp_norm, Ws w,
                 int32_t* __restrict__ out_count, float* __restrict__ out_boxes, float* __restrict__ out_scores,
                 int64_t* __restrict__ out_labels, int64_t* __restrict__ out_index) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    uint64_t* skeys = reinterpret_cast<uint64_t*>(smem);            // SORT_LDS_KEYS
    __shared__ int sh[NMS_WAVES + 1];
    __shared__ float4 head_box;
    __shared__ int kept_pos_count;

    const int64_t b = blockIdx.x;
    const int tid = threadIdx.x;
    const int64_t base = b * N;

    // a. order-preserving compaction (chunk per thread)
    const int cpt = int((N + NMS_THREADS - 1) / NMS_THREADS);
    const int64_t r0 = int64_t(tid) * cpt;
    int cnt = 0;
    for (int k = 0; k < cpt; ++k) {
        int64_t r = r0 + k;
        if (r < N) cnt += w.flag[base + r];
    }
    int K;
    int off = block_excl_scan(cnt, sh, K);
    for (int k = 0; k < cpt; ++k) {
        int64_t r = r0 + k;
        if (r < N && w.flag[base + r]) w.frow[base + off++] = int32_t(r);
    }
    __syncthreads();
    if (K == 0) {
        if (tid == 0) {
            out_count[b] = 0;
            if (SORT_ONLY) w.kcount[b] = 0;
        }
        return;
    }
    if constexpr (SORT_ONLY) {        // bitmask path: the sort runs over the whole GPU (nms_rank_kernel)
        for (int64_t r = tid; r < N; r += NMS_THREADS) w.flag[base + r] = 0;   // rank counters
        if (tid == 0) w.kcount[b] = K;
        return;
    }

    // b. sort (score desc, filtered index asc)
    int P = 1;
    while (P < K) P <<= 1;
    const bool lds_sort = P <= SORT_LDS_KEYS;
    uint64_t* keys = lds_sort ? skeys : (w.keys + b * KP);   // KP >= P
    for (int i = tid; i < P; i += NMS_THREADS) {
        uint64_t key = ~0ull;
        if (i < K) key = (uint64_t(desc_bits(w.score[base + w.frow[base + i]])) << 32) | uint32_t(i);
        keys[i] = key;
    }
    __syncthreads();
    // the LDS image is sorted through the __shared__ pointer itself (ds_ instructions); the generic
    // `keys` pointer would compile to flat loads/stores, ~10x slower for the 91 bitonic stages
    if (lds_sort) bitonic<true>(skeys, P);
    else bitonic<false>(w.keys + b * KP, P);

    // c. greedy loop; sorted position s -> filtered index f = keys[s] low bits
    float4 mybox[REG_ITEMS];
    bool alive[REG_ITEMS];
    const bool in_regs = K <= REG_ITEMS * NMS_THREADS;
    if (in_regs) {
#pragma unroll
        for (int it = 0; it < REG_ITEMS; ++it) {
            int s = tid + it * NMS_THREADS;
            alive[it] = s < K;
            if (s < K) {
                int f = int(uint32_t(keys[s]));
                mybox[it] = w.box[base + w.frow[base + f]];
            }
        }
    }
    // alive flags for the large-K path live in out_index scratch as bytes: reuse w.flag (now free)
    int32_t* galive = w.flag + base;
    if (!in_regs) {
        for (int s = tid; s < K; s += NMS_THREADS) galive[s] = 1;
    }
    if (tid == 0) kept_pos_count = 0;
    __syncthreads();

    int head = 0;
    while (head < K) {
        // record + broadcast the head box: from the registers of the thread that holds sorted
        // position `head` (no dependent global loads on the serial path), or from HBM for K > 8192
        if (in_regs) {
            if (tid == (head & (NMS_THREADS - 1))) {
                const int hit = head / NMS_THREADS;
#pragma unroll
                for (int it = 0; it < REG_ITEMS; ++it)
                    if (it == hit) head_box = mybox[it];
            }
        } else if (tid == 0) {
            int f = int(uint32_t(keys[head]));
            head_box = w.box[base + w.frow[base + f]];
        }
        if (tid == 0) {
            out_index[base + kept_pos_count] = head;   // sorted position for now
            kept_pos_count++;
        }
        __syncthreads();
        const float4 hb = head_box;
        int next = INT32_MAX;
        if (in_regs) {
#pragma unroll
            for (int it = 0; it < REG_ITEMS; ++it) {
                int s = tid + it * NMS_THREADS;
                if (alive[it] && s > head) {
                    float v = iou_ref(hb, mybox[it]);
                    if (!(v <= iou_thr)) alive[it] = false;     // reference keeps IoU <= thr (:396)
                    else next = min(next, s);
                } else if (s <= head) {
                    alive[it] = false;
                }
            }
        } else {
            for (int s = tid; s < K; s += NMS_THREADS) {
                if (s > head && galive[s]) {
                    int f = int(uint32_t(keys[s]));
                    float v = iou_ref(hb, w.box[base + w.frow[base + f]]);
                    if (!(v <= iou_thr)) galive[s] = 0;
                    else next = min(next, s);
                }
            }
        }
        head = block_min(next, sh);
    }
    __syncthreads();

    // d. outputs
    const int nk = kept_pos_count;
    for (int k = tid; k < nk; k += NMS_THREADS) {
        int s = int(out_index[base + k]);
        int f = int(uint32_t(keys[s]));
        int64_t row = base + w.frow[base + f];
        float4 bx = w.box[row];
        if (clamp_norm) {
            bx.x = fminf(fmaxf(bx.x / img_size, 0.0f), 1.0f);
            bx.y = fminf(fmaxf(bx.y / img_size, 0.0f), 1.0f);
            bx.z = fminf(fmaxf(bx.z / img_size, 0.0f), 1.0f);
            bx.w = fminf(fmaxf(bx.w / img_size, 0.0f), 1.0f);
        }
        int64_t o = base + k;
        reinterpret_cast<float4*>(out_boxes)[o] = bx;
        out_scores[o] = w.score[row];
        out_labels[o] = w.label[row];
        out_index[o] = f;
    }
    if (tid == 0) out_count[b] = nk;
}

// Sort of the filtered candidates (bitmask path) by rank: the keys (score descending, filtered
// index ascending) are unique, so key i goes to position #{j : key_j < key_i}.  K^2 comparisons
// over a (key tile i, key tile j) grid; the per-tile counts are integer atomics into rank[] (w.flag,
// zeroed by the compaction kernel) — order-independent, so the result is exact.
__device__ __forceinline__ uint64_t cand_key(const Ws& w, int64_t base, int f) {
    return (uint64_t(desc_bits(w.score[base + w.frow[base + f]])) << 32) | uint32_t(f);
}

__global__ void __launch_bounds__(256) nms_rank_kernel(int64_t N, Ws w) {
    __shared__ uint64_t tile[256];
    const int64_t b = blockIdx.z;
    const int K = w.kcount[b];
    const int i0 = blockIdx.x * 256, j0 = blockIdx.y * 256;
    if (i0 >= K || j0 >= K) return;
    const int64_t base = b * N;
    const int i = i0 + threadIdx.x;
    tile[threadIdx.x] = j0 + int(threadIdx.x) < K ? cand_key(w, base, j0 + threadIdx.x) : ~0ull;
    __syncthreads();
    if (i >= K) return;
    const uint64_t ki = cand_key(w, base, i);
    const int jn = min(256, K - j0);
    int cnt = 0;
    for (int jj = 0; jj < jn; ++jj) cnt += tile[jj] < ki;
    if (cnt) atomicAdd(&w.flag[base + i], cnt);
}

__global__ void nms_rank_scatter_kernel(int64_t N, int64_t KP, Ws w) {
    const int64_t b = blockIdx.y;
    const int K = w.kcount[b];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= K) return;
    const int64_t base = b * N;
    const int r = w.flag[base + i];
    w.keys[b * KP + r] = cand_key(w, base, i);
    w.sbox[base + r] = w.box[base + w.frow[base + i]];
}

// maskT[b][cb][i] bit j-64cb = (j > i) && !(IoU(i, j) <= thr) for sorted positions i, j < K; only
// cb >= i/64 is written (the scan reads the upper triangle).  Block = 64 rows of one row block.
// Grid: x = the upper triangle's Wn (Wn + 1) / 2 (row block, column block) pairs, t = cb (cb + 1) / 2 + rb
// (half the blocks of a square grid, whose lower half only returned), z = image.
__global__ void __launch_bounds__(64) nms_mask_kernel(int64_t N, int Wn, float iou_thr, Ws w) {
    __shared__ float4 cols[64];
    const int tri = blockIdx.x;
    int cb = int((sqrtf(8.0f * float(tri) + 1.0f) - 1.0f) * 0.5f);
    while (cb * (cb + 1) / 2 > tri) --cb;
    while ((cb + 1) * (cb + 2) / 2 <= tri) ++cb;
    const int rb = tri - cb * (cb + 1) / 2;
    const int64_t b = blockIdx.z;
    const int K = w.kcount[b];
    if (rb * 64 >= K || cb * 64 >= K) return;
    const int t = threadIdx.x;
    const int64_t base = b * N;
    const int j0 = cb * 64;
    if (j0 + t < K) cols[t] = w.sbox[base + j0 + t];
    __syncthreads();
    const int i = rb * 64 + t;
    if (i >= K) return;
    const float4 bi = w.sbox[base + i];
    uint64_t word = 0;
    const int jn = min(64, K - j0);
    for (int jj = 0; jj < jn; ++jj) {
        const int j = j0 + jj;
        if (j > i && !(iou_ref(bi, cols[jj]) <= iou_thr)) word |= uint64_t(1) << jj;
    }
    w.mask[(b * Wn + cb) * N + i] = word;          // column-major: column cb, row i
}

// Greedy scan, ONE wave per image, visiting only what the kept rows need (round 1's workgroup scan read the
// whole upper triangle: every earlier row of every column, ~K^2/128 words per image).  A chunk c's
// removed bits come from two places:
//  * NEAR rows (the previous group of 4 chunks and the earlier chunks of this group): the words
//    D(c', c) = column c, rows 64c'..64c'+63 are loaded one group AHEAD (they do not depend on any
//    decision; coalesced 512-B wave loads) and read under the kept bits of chunk c';
//  * FAR rows (two or more groups back): each lane accumulates, for the column blocks it owns
//    (cb = lane + 64k), the words of every kept row; a group's kept rows are gathered at the start
//    of the next group and joined at the start of the one after (the loads fly during a group).
// The per-chunk work is then one wave OR, the fixpoint of the chunk's 64x64 diagonal block and the
// keep update: no workgroup barrier, and ~(kept x Wn + 26 x 64 x groups) words read instead of the
// triangle.  Same decisions as nms_scan_kernel (a box is kept iff no earlier kept box has
// IoU > thr with it): the removed bits of chunk c are the OR over ALL kept rows j < 64c of
// mask[j][c], split into near and far.
constexpr int SCAN_WL = (BM_MAX_WN + 63) / 64;      // column-block words per lane (far bits)

// OR over the 64 lanes by DPP (row prefix-ORs, then row broadcasts 15 / 31; the total lands in lane
// 63): a dozen VALU steps instead of a chain of 12 cross-lane permutes
__device__ __forceinline__ uint32_t wave_or32_dpp(uint32_t v) {
    v |= uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x111, 0xf, 0xf, false));   // row_shr:1
    v |= uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x112, 0xf, 0xf, false));   // row_shr:2
    v |= uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x114, 0xf, 0xf, false));   // row_shr:4
    v |= uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x118, 0xf, 0xf, false));   // row_shr:8
    v |= uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x142, 0xa, 0xf, false));   // row_bcast:15
    v |= uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x143, 0xc, 0xf, false));   // row_bcast:31
    return uint32_t(__builtin_amdgcn_readlane(int(v), 63));
}
__device__ __forceinline__ uint64_t wave_or64_dpp(uint64_t v) {
    return (uint64_t(wave_or32_dpp(uint32_t(v >> 32))) << 32) | wave_or32_dpp(uint32_t(v));
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    return (uint64_t(uint32_t(__builtin_amdgcn_readlane(int(uint32_t(v >> 32)), l))) << 32) |
           uint32_t(__builtin_amdgcn_readlane(int(uint32_t(v)), l));
}
constexpr int SCAN_RB = 8;                          // kept rows per group gathered asynchronously

__global__ void __launch_bounds__(64) nms_scan_wave_kernel(int64_t N, int64_t KP, int Wn, float img_size, Ws w,
                                                           int32_t* __restrict__ out_count,
                                                           float* __restrict__ out_boxes,
                                                           float* __restrict__ out_scores,
                                                           int64_t* __restrict__ out_labels,
                                                           int64_t* __restrict__ out_index) {
    __shared__ int rows_sh[256];
    const int64_t b = blockIdx.x;
    const int lane = threadIdx.x;
    const int K = w.kcount[b];
    const int64_t base = b * N;
    if (K == 0) {
        if (lane == 0) out_count[b] = 0;
        return;
    }
    const int nch = (K + 63) / 64;
    const int ngr = (nch + 3) / 4;
    const uint64_t* mcol = w.mask + int64_t(b) * Wn * N;     // column cb: mcol + cb * N, row-indexed
    // raw buffer loads over this image's mask: 32-bit byte offsets, and every guarded-off load reads 0
    // through an out-of-range offset instead of a branch (one wave runs alone per image: its
    // instruction count is the kernel's time)
    const __amdgpu_buffer_rsrc_t mres = make_rsrc(mcol, int64_t(Wn) * N * 8);
    auto ld8 = [&](uint32_t off) -> uint64_t {
        const uint2 v = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(mres, off, 0, 0));
        return (uint64_t(v.y) << 32) | v.x;
    };

    uint64_t far[SCAN_WL];
#pragma unroll
    for (int k = 0; k < SCAN_WL; ++k) far[k] = 0;
    // D(c', c) for the 4 chunks q of a group: slot s <-> c' = 4g - 4 + s (s <= 4 + q)
    uint64_t dcur[4][8], dnx[4][8];
    auto load_group = [&](int g, uint64_t (&d)[4][8]) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int c = 4 * g + q;
            const uint32_t col = c < nch ? uint32_t(c * int(N) + lane) * 8u : OOB;
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                if (s > 4 + q) {
                    d[q][s] = 0;
                    continue;
                }
                const int cp = 4 * g - 4 + s;
                d[q][s] = ld8(col == OOB || cp < 0 ? OOB : col + uint32_t(cp) * 512u);
            }
        }
    };
    uint64_t kprev[4] = {0, 0, 0, 0};                 // kept bits of the previous group's chunks
    uint64_t pend[SCAN_RB][SCAN_WL];                   // far words of the gathered rows, in flight
#pragma unroll
    for (int r = 0; r < SCAN_RB; ++r)
#pragma unroll
        for (int k = 0; k < SCAN_WL; ++k) pend[r][k] = 0;
    int nkept = 0;
    load_group(0, dcur);
    for (int g = 0; g < ngr; ++g) {
        // Everything loaded at the previous group's start (this group's D blocks, the far words of
        // group g-2's kept rows) has had a whole group of decisions to arrive: wait for it HERE, once,
        // explicitly.  (Left to the compiler, the loop-carried loads got conservative vmcnt waits
        // inside the chunk loop that also waited for the loads issued at THIS group's start.)
        __builtin_amdgcn_s_waitcnt(0x0F70);            // vmcnt(0), expcnt / lgkmcnt untouched
#pragma unroll
        for (int r = 0; r < SCAN_RB; ++r)
#pragma unroll
            for (int k = 0; k < SCAN_WL; ++k) far[k] |= pend[r][k];
        if (g >= 1)
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int s = 0; s < 8; ++s) dcur[q][s] = dnx[q][s];
        // next group's D blocks, and the far words (columns cb >= 4(g+1), beyond group g's near window)
        // of group g-1's kept rows: in flight during this group, used from the next group on
        if (g + 1 < ngr) load_group(g + 1, dnx);
        int nr = 0;
        if (g >= 1) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint64_t kb = kprev[q];
                if ((kb >> lane) & 1)
                    rows_sh[nr + __popcll(kb & ((uint64_t(1) << lane) - 1))] = 64 * (4 * (g - 1) + q) + lane;
                nr += __popcll(kb);
            }
            __builtin_amdgcn_wave_barrier();
        }
        const int cb_lo = 4 * (g + 1);
        auto row_words = [&](int j, uint64_t* dst) {
#pragma unroll
            for (int k = 0; k < SCAN_WL; ++k) {
                const int cb = lane + 64 * k;
                dst[k] = ld8(j >= 0 && cb >= cb_lo && cb < Wn ? uint32_t(cb * int(N) + j) * 8u : OOB);
            }
        };
        const int npend = min(nr, SCAN_RB);
#pragma unroll
        for (int r = 0; r < SCAN_RB; ++r) row_words(r < npend ? rows_sh[r] : -1, pend[r]);
        for (int r = SCAN_RB; r < nr; ++r) {   // > SCAN_RB kept rows: synchronously
            uint64_t t[SCAN_WL];
            row_words(rows_sh[r], t);
#pragma unroll
            for (int k = 0; k < SCAN_WL; ++k) far[k] |= t[k];
        }
        uint64_t kcur[4] = {0, 0, 0, 0};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int c = 4 * g + q;
            if (c >= nch) break;
            // near rows: previous group (slots 0..3) and this group's earlier chunks (slots 4..4+q-1):
            // each lane ORs the words of its kept rows, then one DPP OR over the wave
            uint64_t nl = 0;
#pragma unroll
            for (int s = 0; s < 4 + q; ++s)
                if ((((s < 4 ? kprev[s] : kcur[s - 4]) >> lane) & 1)) nl |= dcur[q][s];
            const uint64_t near = wave_or64_dpp(nl);
            // far rows: column c's word lives in lane c & 63, slot c >> 6
            const int kw = c >> 6;
            uint64_t fw = far[0];
#pragma unroll
            for (int k = 1; k < SCAN_WL; ++k)
                if (kw == k) fw = far[k];
            const uint64_t rem = near | readlane64(fw, c & 63);
            const int rows = min(64, K - 64 * c);
            const uint64_t diag = dcur[q][4 + q];
            // the diagonal block greedily, one iteration per KEPT row (~1-2 per chunk): the lowest
            // undecided bit s survives, and its row (lane s's word, bits > s only) removes later bits
            uint64_t und = ~rem & (rows == 64 ? ~uint64_t(0) : ((uint64_t(1) << rows) - 1));
            uint64_t alive = 0;
            while (und) {
                const int sl = __builtin_ctzll(und);
                alive |= uint64_t(1) << sl;
                und &= ~readlane64(diag, sl) & ~(uint64_t(1) << sl);
            }
            if ((alive >> lane) & 1) out_index[base + nkept + __popcll(alive & ((uint64_t(1) << lane) - 1))] = 64 * c + lane;
            nkept += __popcll(alive);
            kcur[q] = alive;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) kprev[q] = kcur[q];
    }
    __syncthreads();                                 // this wave's out_index stores are visible to its loads
    // outputs in kept order (sorted position -> filtered index -> row)
    for (int k = lane; k < nkept; k += 64) {
        const int spos = int(out_index[base + k]);
        const int f = int(uint32_t(w.keys[b * KP + spos]));
        const int64_t row = base + w.frow[base + f];
        float4 bx = w.box[row];
        bx.x = fminf(fmaxf(bx.x / img_size, 0.0f), 1.0f);
        bx.y = fminf(fmaxf(bx.y / img_size, 0.0f), 1.0f);
        bx.z = fminf(fmaxf(bx.z / img_size, 0.0f), 1.0f);
        bx.w = fminf(fmaxf(bx.w / img_size, 0.0f), 1.0f);
        reinterpret_cast<float4*>(out_boxes)[base + k] = bx;
        out_scores[base + k] = w.score[row];
        out_labels[base + k] = w.label[row];
        out_index[base + k] = f;
    }
    if (lane == 0) out_count[b] = nkept;
}

int launch_nms(int64_t B, int64_t Nalloc, float iou_thr, float img_size, int clamp_norm, Ws w,
               int32_t* out_count, float* out_boxes, float* out_scores, int64_t* out_labels, int64_t* out_index,
               hipStream_t st) {
    size_t lds = size_t(SORT_LDS_KEYS) * sizeof(uint64_t);
    if (w.mask && clamp_norm) {
        const int Wn = int((Nalloc + 63) / 64);
        const int64_t KP = pow2_at_least(Nalloc);
        hipLaunchKernelGGL(nms_image_kernel<true>, dim3(unsigned(B)), dim3(NMS_THREADS), lds, st, Nalloc, KP, iou_thr,
                           img_size, clamp_norm, w, out_count, out_boxes, out_scores, out_labels, out_index);
        const unsigned nt = unsigned((Nalloc + 255) / 256);
        hipLaunchKernelGGL(nms_rank_kernel, dim3(nt, nt, unsigned(B)), dim3(256), 0, st, Nalloc, w);
        hipLaunchKernelGGL(nms_rank_scatter_kernel, dim3(nt, unsigned(B)), dim3(256), 0, st, Nalloc, KP, w);
        hipLaunchKernelGGL(nms_mask_kernel, dim3(unsigned(Wn * (Wn + 1) / 2), 1, unsigned(B)), dim3(64), 0, st, Nalloc,
                           Wn, iou_thr, w);
        hipLaunchKernelGGL(nms_scan_wave_kernel, dim3(unsigned(B)), dim3(64), 0, st, Nalloc, KP, Wn, img_size, w,
                           out_count, out_boxes, out_scores, out_labels, out_index);
        YM_LAUNCH_CHECK("nms bitmask path");
        return YM_OK;
    }
    hipLaunchKernelGGL(nms_image_kernel<false>, dim3(unsigned(B)), dim3(NMS_THREADS), lds, st, Nalloc,
                       pow2_at_least(Nalloc), iou_thr, img_size,
                       clamp_norm, w, out_count, out_boxes, out_scores, out_labels, out_index);
    YM_LAUNCH_CHECK("nms_image_kernel");
    return YM_OK;
}

}  // namespace
}  // namespace ym

using namespace ym;

extern "C" size_t ym_nms_workspace_size(int64_t B, int64_t N) { return 2 * ws_bytes(B, N); }

__global__ void ym_iou_row_kernel(const float4* __restrict__ b1, const float4* __restrict__ b2, int64_t m,
                                  float* __restrict__ out) {
    int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < m) out[i] = iou_ref(*b1, b2[i]);
}

extern "C" int ym_iou_row(const float* box1, const float* boxes2, int64_t m, float* out, void* stream) {
    YM_CHECK_ARG(m >= 0, "ym_iou_row: m < 0");
    if (m == 0) return YM_OK;
    hipLaunchKernelGGL(ym_iou_row_kernel, dim3(unsigned((m + 255) / 256)), dim3(256), 0, as_stream(stream),
                       reinterpret_cast<const float4*>(box1), reinterpret_cast<const float4*>(boxes2), m, out);
    YM_LAUNCH_CHECK("ym_iou_row");
    return YM_OK;
}

extern "C" int ym_decode_nms_strided(const float* pred, int64_t B, int64_t N, int64_t C, int64_t row_stride,
                                     int64_t img_stride, int64_t col_stride, float conf, float iou_thr, float img_size,
                                     void* workspace, size_t workspace_bytes, int32_t* out_count, float* out_boxes,
                                     float* out_scores, int64_t* out_labels, int64_t* out_index, void* stream) {
    YM_CHECK_ARG(B >= 0 && N >= 0 && C >= 1, "ym_decode_nms: bad shape B=%lld N=%lld C=%lld", (long long)B,
                 (long long)N, (long long)C);
    YM_CHECK_ARG(col_stride >= 1 && (col_stride > 1 || row_stride >= 4 + C), "ym_decode_nms: row_stride < 4+C");
    YM_CHECK_ARG(N < (int64_t(1) << 30), "ym_decode_nms: N too large");
    if (B == 0) return YM_OK;
    hipStream_t st = as_stream(stream);
    if (N == 0) return hipMemsetAsync(out_count, 0, B * sizeof(int32_t), st) == hipSuccess ? YM_OK : YM_ERR_HIP;
    YM_CHECK_ARG(workspace_bytes >= ws_bytes(B, N), "ym_decode_nms: workspace too small (%zu < %zu)",
                 workspace_bytes, ws_bytes(B, N));
    Ws w = carve(workspace, B, N);
    if (C <= 64)
        hipLaunchKernelGGL(rowmax_thread_kernel, dim3(unsigned((B * N + 255) / 256)), dim3(256), 0, st, pred, B, N,
                           C, row_stride, img_stride, col_stride, conf, w);
    else
        hipLaunchKernelGGL(rowmax_wave_kernel, dim3(unsigned((B * N + 3) / 4)), dim3(256), 0, st, pred, B, N, C,
                           row_stride, img_stride, col_stride, conf, w);
    YM_LAUNCH_CHECK("rowmax");
    return launch_nms(B, N, iou_thr, img_size, 1, w, out_count, out_boxes, out_scores, out_labels, out_index, st);
}

extern "C" int ym_decode_nms(const float* pred, int64_t B, int64_t N, int64_t C, int64_t row_stride,
                             int64_t img_stride, float conf, float iou_thr, float img_size, void* workspace,
                             size_t workspace_bytes, int32_t* out_count, float* out_boxes, float* out_scores,
                             int64_t* out_labels, int64_t* out_index, void* stream) {
    return ym_decode_nms_strided(pred, B, N, C, row_stride, img_stride, 1, conf, iou_thr, img_size, workspace,
                                 workspace_bytes, out_count, out_boxes, out_scores, out_labels, out_index, stream);
}

extern "C" int ym_nms(const float* boxes, const float* scores, int64_t n, float iou_thr, void* workspace,
                      size_t workspace_bytes, int64_t* keep, int32_t* count, void* stream) {
    YM_CHECK_ARG(n >= 0, "ym_nms: n < 0");
    hipStream_t st = as_stream(stream);
    if (n == 0) return hipMemsetAsync(count, 0, sizeof(int32_t), st) == hipSuccess ? YM_OK : YM_ERR_HIP;
    YM_CHECK_ARG(workspace_bytes >= ws_bytes(1, n) + ws_bytes(1, n), "ym_nms: workspace too small");
    Ws w = carve(workspace, 1, n);
    // scratch outputs (boxes/scores/labels) after the candidate arrays
    char* extra = static_cast<char*>(workspace) + ws_bytes(1, n);
    float* ob = reinterpret_cast<float*>(extra);
    float* os = reinterpret_cast<float*>(extra + align256(n * 16));
    int64_t* ol = reinterpret_cast<int64_t*>(extra + align256(n * 16) + align256(n * 4));
    hipLaunchKernelGGL(direct_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, st,
                       reinterpret_cast<const float4*>(boxes), scores, n, w);
    YM_LAUNCH_CHECK("nms direct");
    return launch_nms(1, n, iou_thr, 1.0f, 0, w, count, ob, os, ol, keep, st);
}
