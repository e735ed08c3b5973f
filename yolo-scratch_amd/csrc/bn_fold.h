// BatchNorm finalize as the tail of a conv forward launch (ym_conv_fwd_bn), shared by the pipelined and the
// halo-staged kernels.  Every workgroup of channel tile nt has published its statistics row write-through
// (agent-scope stores); after its stores drained (vmcnt(0)) and a workgroup barrier, one lane takes an
// agent-scope ticket; the workgroup that takes the last one (rows - 1) folds the tile's rows in fp64 in a
// fixed order (THREADS / BN row subsets with 8 rows' loads in flight, then in subset order) and writes what
// ym_bn_finalize writes for those channels, then re-arms the ticket (the pattern of bn.hip's finalize: the
// launch's tail pays ~5 us instead of a second launch).
#pragma once
#include "common.h"

namespace ym {

struct BnFoldArgs {
    const float* gamma; const float* beta;    // null gamma: no fold
    float* rm; float* rv; int64_t* nbt;       // running statistics (or null), num_batches_tracked
    float* scale; float* shift; float* mean; float* rstd;
    unsigned* cnt;                            // one ticket per channel tile (the BN workspace's counters)
    double count;
    float mom, eps;
};

static inline BnFoldArgs bn_fold_args(const ym_bn_fold* f) {
    BnFoldArgs a{};
    if (!f) return a;
    a.gamma = f->gamma; a.beta = f->beta;
    a.rm = f->running_mean; a.rv = f->running_var; a.nbt = f->num_batches_tracked;
    a.scale = f->scale; a.shift = f->shift; a.mean = f->mean; a.rstd = f->rstd;
    a.cnt = static_cast<unsigned*>(f->workspace);
    a.count = f->count; a.mom = f->momentum; a.eps = f->eps;
    return a;
}

// the row store of a kernel's statistics epilogue: write-through when a fold follows
__device__ __forceinline__ void stat_store(float* p, float v, bool fold) {
    if (fold) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}

template <int BN, int THREADS>
__device__ __forceinline__ void bn_fold_tail(const BnFoldArgs& f, const float* st_sum, const float* st_sq, int Nout,
                                             int nt, int rows, char* smem) {
    constexpr int K = THREADS / BN;
    static_assert(K >= 1 && THREADS % BN == 0, "fold geometry");
    // the flag lives in the kernel's (now free) staging LDS past the fold's partials: a __shared__ variable of its
    // own would add 4 B to kernels sized to exactly two workgroups per CU (conv_halo C4: 2 x 80 KB)
    int& last_sh = *reinterpret_cast<int*>(smem + THREADS * 16);
    const int tid = threadIdx.x;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        const unsigned t = __hip_atomic_fetch_add(&f.cnt[nt], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last_sh = t == unsigned(rows - 1);
    }
    __syncthreads();
    if (!last_sh) return;
    double (*part)[2][BN] = reinterpret_cast<double (*)[2][BN]>(smem);      // [K][sum|sq][channel]
    const int cl = tid % BN, k = tid / BN, ch = nt * BN + cl;
    auto ld = [&](const float* p, int r) {
        return __hip_atomic_load(const_cast<float*>(p) + int64_t(r) * Nout + ch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    double s = 0.0, q = 0.0;
    if (ch < Nout) {
        int r = k;
        for (; r + 7 * K < rows; r += 8 * K) {
            float vs[8], vq[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                vs[u] = ld(st_sum, r + u * K);
                vq[u] = ld(st_sq, r + u * K);
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                s += double(vs[u]);
                q += double(vq[u]);
            }
        }
        for (; r < rows; r += K) {
            s += double(ld(st_sum, r));
            q += double(ld(st_sq, r));
        }
    }
    part[k][0][cl] = s;
    part[k][1][cl] = q;
    __syncthreads();
    if (tid == 0) f.cnt[nt] = 0u;                 // re-armed for the next launch (same stream)
    if (k != 0 || ch >= Nout) return;
    s = 0.0;
    q = 0.0;
    for (int j = 0; j < K; ++j) {
        s += part[j][0][cl];
        q += part[j][1][cl];
    }
    if (f.nbt && nt == 0 && cl == 0) *f.nbt += 1;
    const double mu = s / f.count;
    double var = q / f.count - mu * mu;
    if (var < 0) var = 0;
    const double rstd = 1.0 / sqrt(var + double(f.eps));
    const float sc = float(double(f.gamma[ch]) * rstd);
    f.scale[ch] = sc;
    f.shift[ch] = float(double(f.beta[ch]) - mu * double(sc));
    f.mean[ch] = float(mu);
    f.rstd[ch] = float(rstd);
    if (f.rm) {
        const double unb = f.count > 1 ? var * f.count / (f.count - 1) : var;
        f.rm[ch] = float((1.0 - f.mom) * f.rm[ch] + f.mom * mu);
        f.rv[ch] = float((1.0 - f.mom) * f.rv[ch] + f.mom * unb);
    }
}

}  // namespace ym
