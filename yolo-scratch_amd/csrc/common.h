// Shared device/host helpers for libyolomi (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <stdint.h>
#include <stdio.h>

#include <atomic>

#include "../../include/yolomi.h"
#include "../../include/yolomi_experimental.h"

namespace ym {

// thread-local last-error string behind ym_last_error()
void set_error(const char* fmt, ...);

#define YM_CHECK_ARG(cond, ...)                    \
    do {                                           \
        if (!(cond)) {                             \
            ::ym::set_error(__VA_ARGS__);          \
            return YM_ERR_ARG;                     \
        }                                          \
    } while (0)

#define YM_LAUNCH_CHECK(what)                                                        \
    do {                                                                             \
        hipError_t e_ = hipGetLastError();                                           \
        if (e_ != hipSuccess) {                                                      \
            ::ym::set_error("%s: launch failed: %s", what, hipGetErrorString(e_));   \
            return YM_ERR_HIP;                                                       \
        }                                                                            \
    } while (0)

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// A process-wide selection policy behind a yolomi_experimental.h setter: an atomic int (a setter racing a launch
// is a data race no more — the launch sees the old or the new value, whole); every store bumps g_policy_gen, so a
// caller that caches a policy-dependent answer (ym_conv_fwd_eval_ok, a workspace size) can tell it went stale
// (ym_policy_generation).  Reads are relaxed: a policy orders nothing but itself.
extern std::atomic<unsigned> g_policy_gen;
struct Policy {
    std::atomic<int> v;
    explicit constexpr Policy(int x) : v(x) {}
    operator int() const { return v.load(std::memory_order_relaxed); }
    int set(int x) {
        const int prev = v.exchange(x, std::memory_order_relaxed);
        g_policy_gen.fetch_add(1, std::memory_order_relaxed);
        return prev;
    }
};

// Conv kernel selection batch (ym_conv_set_select_batch): when > 0 the selection rules of every conv
// kernel (size thresholds, tile shapes) evaluate as if the batch held this many images, while the
// launch geometry still follows the real batch — so a small-batch parity test runs exactly the kernel
// instances a large-batch training step selects.  0 (the default): the real batch.
extern Policy g_select_n;
static inline int64_t select_n(const ym_conv_desc* d) { return g_select_n > 0 ? int64_t(g_select_n) : int64_t(d->n); }

// the weight-gradient kernel instance ym_conv_wgrad runs for d (wgrad.hip; ym_conv_kernel dir 2)
int wgrad_kernel(const ym_conv_desc* d, char* name, size_t len);

// eval-mode Conv block epilogue arguments (ym_conv_fwd_eval; conv_epi.h EvalEpi is built from them in the kernel):
// BatchNorm scale / shift from the running statistics, SiLU when act, and an fp16 residual view (res null: none;
// r_bs / r_ld its image / pixel strides in elements; res_bytes its extent from res for the buffer resource).
// ks > 1: the K-split form (the 2-stage GEMM only): blockIdx.z walks K slice z of ks and stores its fp32 partial sums to
// part[z][M][Nout]; eval_fold_kernel applies the epilogue to their sum
struct EvalArgs {
    const float* sc; const float* sh;
    int act;
    const uint16_t* res; int64_t res_bytes;
    int64_t r_bs, r_ld;
    int ks; float* part;
};

typedef uint16_t bf16_t;   // raw bf16 bits in memory

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
// round-to-nearest-even f32 -> bf16 (v_cvt_pk_bf16_f32; NaN stays a quiet NaN)
__device__ __forceinline__ bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }
// two floats -> packed bf16 pair (lo in bits 0..15): one v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t pk2bf(float lo, float hi) {
    typedef float f2_t __attribute__((ext_vector_type(2)));
    typedef __bf16 b2_t __attribute__((ext_vector_type(2)));
    f2_t v = {lo, hi};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, b2_t));
}

// fp16 bits <-> f32 (pre-BatchNorm conv outputs are kept in fp16: 3 more mantissa bits than
// bf16 where normalisation amplifies rounding; |z| is clamped below the fp16 range)
__device__ __forceinline__ float h2f(uint16_t v) { return __half2float(__ushort_as_half(v)); }
// the clamp is one v_med3_f32 (IEEE minNum semantics: a NaN input comes out as -65504, as the fminf / fmaxf pair gave)
__device__ __forceinline__ uint16_t f2h(float f) {
    f = __builtin_amdgcn_fmed3f(f, -65504.f, 65504.f);
    return __half_as_ushort(__float2half(f));
}
// two floats -> packed fp16 pair (lo in bits 0..15), clamped: two v_med3_f32 + one v_cvt_pk_f16_f32 (round 5: the
// per-value fminf / fmaxf / cvt / shift / or sequence it replaces was 7 VALU per pair, a third of the 1x1 conv
// epilogues' vector instructions)
__device__ __forceinline__ uint32_t pk2h(float lo, float hi) {
    typedef float f2_t __attribute__((ext_vector_type(2)));
    typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
    f2_t v = {__builtin_amdgcn_fmed3f(lo, -65504.f, 65504.f), __builtin_amdgcn_fmed3f(hi, -65504.f, 65504.f)};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, h2_t));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// SiLU with the hardware reciprocal (v_rcp_f32, ~1 ulp; results are stored in 16 bits)
__device__ __forceinline__ float silu_f(float u) { return u * __builtin_amdgcn_rcpf(1.0f + __expf(-u)); }

}  // namespace ym
