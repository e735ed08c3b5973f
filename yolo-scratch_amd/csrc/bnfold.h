// BatchNorm statistics finalized by the kernel that produces them (conv forward epilogues, the
// backward statistics pass): no separate finalize launch on the critical path.
//
// Every workgroup writes its slice of one partial row ([rows][C] fp32 sum / square-sum, or sum(g) /
// sum(g*xhat) in the backward), then takes a ticket on its row GROUP's counter (groups of `gs`
// consecutive rows, at most 32 groups).  The workgroup drawing a group's last ticket folds the
// group's rows (fp64, in row order) into one level-2 row, then takes a ticket on the top counter;
// the one drawing the last top ticket folds the level-2 rows (in group order) and runs the
// finalize, and every folder re-arms the counter it consumed.  The result does not depend on
// which workgroups finish first: bit-reproducible.  Visibility hand-off per MI355X_MICROARCH.md
// (inter-workgroup visibility, "valid forms"): the partial rows are stored write-through (relaxed
// agent-scope atomic stores = `sc1` vector stores) -> every wave vmcnt(0) -> barrier -> one lane's
// relaxed agent fetch_add; the last arriver: barrier -> `sc1` loads (relaxed agent atomic loads),
// no fence on either side.  No release fence: an agent release writes back the XCD's whole dirty L2 (the
// conv's freshly written z), which measured +35 us per conv launch when every workgroup paid it.
// Vector memory operations only; nothing spins.
#pragma once
#include "common.h"

namespace ym {

struct BnFold {
    unsigned* cnt;            // [ngroups + 1] tickets, zero between launches (null: no fused finalize)
    double* p2;               // [ngroups][2][C] level-2 rows
    int rows, gs, ngroups;    // partial rows, rows per group, groups
    int per_row;              // workgroups writing slices of each row (channel tiles)
    int bwd;                  // 0: forward statistics, 1: backward (dgamma / dbeta / apply coefficients)
    double count;             // pixels per channel
    const float* gamma; const float* beta;
    float* running_mean; float* running_var; int64_t* nbt;
    float momentum, eps;
    float* scale; float* shift; float* mean; float* rstd;   // forward outputs
    const float* rstd_in;     // backward: the forward's rstd
    float* dgamma; float* dbeta; int accumulate; float* coef;   // backward outputs
};

// host: fill the grouping fields for `rows` partial rows written by `per_row` workgroups each
inline void bn_fold_groups(BnFold& f, int rows, int per_row) {
    f.rows = rows;
    f.per_row = per_row;
    f.gs = (rows + 31) / 32;
    f.ngroups = (rows + f.gs - 1) / f.gs;
}

// host: the forward fold of a ym_bn_train over `count` pixels (grouping filled in by the launcher);
// the workspace is ym_bn_workspace_size(c): 256 B of counters, then the level-2 rows
inline BnFold bn_fold_fwd(const ym_bn_train* t, double count) {
    BnFold f{};
    f.cnt = static_cast<unsigned*>(t->workspace);
    f.p2 = reinterpret_cast<double*>(static_cast<char*>(t->workspace) + 256);
    f.bwd = 0;
    f.count = count;
    f.gamma = t->gamma; f.beta = t->beta;
    f.running_mean = t->running_mean; f.running_var = t->running_var; f.nbt = t->num_batches_tracked;
    f.momentum = t->momentum; f.eps = t->eps;
    f.scale = t->scale; f.shift = t->shift; f.mean = t->mean; f.rstd = t->rstd;
    return f;
}

// write-through store / L1-bypassing load of hand-off data (sc1 vector memory operations)
__device__ __forceinline__ void st_wt(float* p, float v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt(double* p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// a partial-row store: write-through when a fused fold will read it (wt), plain otherwise
__device__ __forceinline__ void st_row(float* p, float v, bool wt) {
    if (wt) st_wt(p, v);
    else *p = v;
}
__device__ __forceinline__ float ld_wt(const float* p) {
    return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_wt(const double* p) {
    return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void bn_fold_finish(const BnFold& f, int C, int c, double s, double q) {
    if (!f.bwd) {
        if (f.nbt && c == 0) *f.nbt += 1;
        const double mu = s / f.count;
        double var = q / f.count - mu * mu;
        if (var < 0) var = 0;
        const double rstd = 1.0 / sqrt(var + double(f.eps));
        const float sc = float(double(f.gamma[c]) * rstd);
        f.scale[c] = sc;
        f.shift[c] = float(double(f.beta[c]) - mu * double(sc));
        f.mean[c] = float(mu);
        f.rstd[c] = float(rstd);
        if (f.running_mean) {
            const double unb = f.count > 1 ? var * f.count / (f.count - 1) : var;
            f.running_mean[c] = float((1.0 - f.momentum) * f.running_mean[c] + f.momentum * mu);
            f.running_var[c] = float((1.0 - f.momentum) * f.running_var[c] + f.momentum * unb);
        }
    } else {
        if (f.dgamma) f.dgamma[c] = float(f.accumulate ? f.dgamma[c] + q : q);
        if (f.dbeta) f.dbeta[c] = float(f.accumulate ? f.dbeta[c] + s : s);
        f.coef[c] = f.gamma[c] * f.rstd_in[c];
        f.coef[C + c] = float(s / f.count);
        f.coef[2 * C + c] = float(q / f.count);
    }
}

// one lane takes the ticket; returns (to every thread) whether this workgroup drew the last one.
// flag: one int of the caller's LDS, free once every thread has passed the entry barrier
__device__ __forceinline__ bool bn_ticket(unsigned* counter, unsigned expected, int* flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = t + 1 == expected;
    }
    __syncthreads();
    const bool r = *flag != 0;
    __syncthreads();              // the flag's LDS word is the caller's again
    return r;
}

// Called by EVERY thread of a workgroup after its slice of partial row `row` is stored with st_wt; `lds` is any
// 4 bytes of the kernel's LDS that no thread reads after this call starts.
__device__ __forceinline__ void bn_fold_tail(const BnFold& f, const float* ps, const float* pq, int C, int row,
                                             void* lds) {
    int* flag = static_cast<int*>(lds);
    const int nt = blockDim.x * blockDim.y * blockDim.z;
    const int tid = threadIdx.x + blockDim.x * (threadIdx.y + blockDim.y * threadIdx.z);
    const int g = row / f.gs;
    const int r0 = g * f.gs, r1 = min(f.rows, r0 + f.gs);
    if (!bn_ticket(&f.cnt[g], unsigned((r1 - r0) * f.per_row), flag)) return;
    for (int c = tid; c < C; c += nt) {
        double s = 0.0, q = 0.0;
        for (int r = r0; r < r1; ++r) {
            s += double(ld_wt(&ps[int64_t(r) * C + c]));
            q += double(ld_wt(&pq[int64_t(r) * C + c]));
        }
        st_wt(&f.p2[(int64_t(g) * 2 + 0) * C + c], s);
        st_wt(&f.p2[(int64_t(g) * 2 + 1) * C + c], q);
    }
    if (tid == 0) f.cnt[g] = 0u;                       // re-armed: every ticket of this group is in
    if (!bn_ticket(&f.cnt[f.ngroups], unsigned(f.ngroups), flag)) return;
    for (int c = tid; c < C; c += nt) {
        double s = 0.0, q = 0.0;
        for (int k = 0; k < f.ngroups; ++k) {
            s += ld_wt(&f.p2[(int64_t(k) * 2 + 0) * C + c]);
            q += ld_wt(&f.p2[(int64_t(k) * 2 + 1) * C + c]);
        }
        bn_fold_finish(f, C, c, s, q);
    }
    if (tid == 0) f.cnt[f.ngroups] = 0u;
}

}  // namespace ym
