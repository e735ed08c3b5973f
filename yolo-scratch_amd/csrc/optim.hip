// AdamW step and gradient-norm clipping over every parameter of a model in three launches (gfx950).
//
// Replaces the optimizer tail of the reference's training step,
// torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=10.0) + optim.AdamW(...).step()
// (/root/reference/yolo_scratch_cuda/train_yolo11_cuda.py:58-62, 440-451).  PyTorch's fused
// multi-tensor AdamW and foreach norm spend ~0.5 ms per s@640 step on 45 MB of parameters (244
// tensors, 7 + 6 launches, 0.9 TB/s); here the parameters are one flat index space described by a
// table of (param, grad, exp_avg, exp_avg_sq) pointers, so the whole update is a single
// HBM-streaming pass (28 B per parameter) and the clip coefficient never leaves the device.
//
// grad_sqnorm_kernel:      block b sums g^2 over elements [b*4096, (b+1)*4096) (per thread in index
//   order, then an xor tree, then the waves in order): deterministic.
// grad_norm_finish_kernel: one block folds the partials in order (fp64) -> total norm (fp32).
// adamw_kernel:            per element, torch.optim.AdamW's update (decoupled weight decay,
//   bias corrections; amsgrad / maximize not supported) on g * clip, clip = min(1, max_norm /
//   (norm + 1e-6)) as clip_grad_norm_ computes it (no clipping when max_norm <= 0).
#include <cmath>

#include "common.h"

namespace ym {
namespace {

constexpr int OPT_THREADS = 256, OPT_PER_THREAD = 16, OPT_CHUNK = OPT_THREADS * OPT_PER_THREAD;

// entry holding flat element i (offsets ascending, entry e covers [offset, offset + n))
__device__ __forceinline__ int find_entry(const ym_adamw_entry* __restrict__ tab, int n_entries, int64_t i) {
    int lo = 0, hi = n_entries - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (tab[mid].offset <= i) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

__global__ void __launch_bounds__(OPT_THREADS) grad_sqnorm_kernel(const ym_adamw_entry* __restrict__ tab, int n_entries,
                                                                  int64_t total, float* __restrict__ partials) {
    __shared__ float red[OPT_THREADS / 64];
    const int64_t i0 = int64_t(blockIdx.x) * OPT_CHUNK + threadIdx.x;
    float s = 0.f;
    if (i0 < total) {
        int e = find_entry(tab, n_entries, i0);
        for (int k = 0; k < OPT_PER_THREAD; ++k) {
            const int64_t i = i0 + int64_t(k) * OPT_THREADS;
            if (i >= total) break;
            while (i >= tab[e].offset + tab[e].n) ++e;
            const float g = tab[e].g[i - tab[e].offset];
            s += g * g;
        }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) partials[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ void __launch_bounds__(256) grad_norm_finish_kernel(const float* __restrict__ partials, int n,
                                                               float* __restrict__ norm) {
    __shared__ double red[4];
    double s = 0.0;
    for (int i = threadIdx.x; i < n; i += 256) s += double(partials[i]);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) norm[0] = float(sqrt((red[0] + red[1]) + (red[2] + red[3])));
}

// scalars as torch forms them: Python-double expressions rounded once to fp32 (decay = 1 - lr*wd,
// omb1 = 1 - beta1, omb2 = 1 - beta2, step_size = lr / bc1, bc2_sqrt = sqrt(bc2))
__global__ void __launch_bounds__(OPT_THREADS) adamw_kernel(const ym_adamw_entry* __restrict__ tab, int n_entries,
                                                            int64_t total, float decay, float omb1, float beta2,
                                                            float omb2, float eps, float step_size, float bc2_sqrt,
                                                            float max_norm, const float* __restrict__ norm) {
    const int64_t i0 = int64_t(blockIdx.x) * OPT_CHUNK + threadIdx.x;
    if (i0 >= total) return;
    float clip = 1.f;
    if (max_norm > 0.f && norm) clip = fminf(max_norm / (norm[0] + 1e-6f), 1.f);
    int e = find_entry(tab, n_entries, i0);
    for (int k = 0; k < OPT_PER_THREAD; ++k) {
        const int64_t i = i0 + int64_t(k) * OPT_THREADS;
        if (i >= total) break;
        while (i >= tab[e].offset + tab[e].n) ++e;
        const ym_adamw_entry& t = tab[e];
        const int64_t j = i - t.offset;
        const float g = t.g[j] * clip;
        float m = t.m[j], v = t.v[j];
        m = m + omb1 * (g - m);                          // exp_avg.lerp_(grad, 1 - beta1)
        v = v * beta2 + omb2 * g * g;                    // exp_avg_sq.mul_(beta2).addcmul_(g, g, 1 - beta2)
        const float denom = sqrtf(v) / bc2_sqrt + eps;
        t.p[j] = t.p[j] * decay - step_size * (m / denom);
        t.m[j] = m;
        t.v[j] = v;
    }
}

}  // namespace
}  // namespace ym

using namespace ym;

extern "C" int ym_grad_norm_blocks(int64_t total) { return int((total + OPT_CHUNK - 1) / OPT_CHUNK); }

extern "C" int ym_grad_norm(const ym_adamw_entry* table_dev, int n_entries, int64_t total, float* partials,
                            float* norm, void* stream) {
    YM_CHECK_ARG(table_dev && partials && norm && n_entries > 0, "ym_grad_norm: null argument");
    const int nb = ym_grad_norm_blocks(total);
    hipStream_t st = as_stream(stream);
    if (nb > 0)
        hipLaunchKernelGGL(grad_sqnorm_kernel, dim3(unsigned(nb)), dim3(OPT_THREADS), 0, st, table_dev, n_entries, total,
                           partials);
    hipLaunchKernelGGL(grad_norm_finish_kernel, dim3(1), dim3(256), 0, st, partials, nb, norm);
    YM_LAUNCH_CHECK("ym_grad_norm");
    return YM_OK;
}

extern "C" int ym_adamw(const ym_adamw_entry* table_dev, int n_entries, int64_t total, double lr, double beta1,
                        double beta2, double eps, double weight_decay, int64_t step, float max_norm, const float* norm,
                        void* stream) {
    YM_CHECK_ARG(table_dev && n_entries > 0 && step >= 1, "ym_adamw: bad arguments");
    YM_CHECK_ARG(max_norm <= 0.f || norm, "ym_adamw: clipping needs the norm from ym_grad_norm");
    if (total == 0) return YM_OK;
    // bias corrections in double on the host, as torch computes them from the Python step count
    const double bc1 = 1.0 - std::pow(beta1, double(step));
    const double bc2 = 1.0 - std::pow(beta2, double(step));
    hipLaunchKernelGGL(adamw_kernel, dim3(unsigned(ym_grad_norm_blocks(total))), dim3(OPT_THREADS), 0, as_stream(stream),
                       table_dev, n_entries, total, float(1.0 - lr * weight_decay), float(1.0 - beta1), float(beta2),
                       float(1.0 - beta2), float(eps), float(lr / bc1), float(std::sqrt(bc2)), max_norm, norm);
    YM_LAUNCH_CHECK("ym_adamw");
    return YM_OK;
}
