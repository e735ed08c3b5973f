// MFMA fragment types and raw-buffer helpers shared by the conv / wgrad kernels (gfx950).
#pragma once
#include "common.h"

namespace ym {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t OOB = 0x80000000u;          // buffer offset past num_records: loads return 0
constexpr int RSRC_FLAGS = 0x00020000;         // raw buffer, 32-bit data format (gfx9 dword3)

// buffer resource over [base, base + bytes); bytes clamped below 2^31 so OOB is always out of range
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0,
                                             int(bytes < 0x7fffffff ? (bytes > 0 ? bytes : 0) : 0x7fffffff),
                                             RSRC_FLAGS);
}

__device__ __forceinline__ uint4 buf_load16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// 8 fp16 -> 8 bf16 (v_cvt_f32_f16 + v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint4 h8_to_bf8(uint4 h) {
    uint32_t w[4] = {h.x, h.y, h.z, h.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) w[e] = pk2bf(h2f(uint16_t(w[e] & 0xffff)), h2f(uint16_t(w[e] >> 16)));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// q = x / d, r = x % d for x < 2^24 (exact as a float), d >= 1, inv_d = 1.0f / d: the float estimate is within one of
// the quotient, one compare-and-correct each way (~8 VALU against ~25 for a 32-bit integer division)
__device__ __forceinline__ void fdivmod(uint32_t x, uint32_t d, float inv_d, uint32_t& q, uint32_t& r) {
    uint32_t e = uint32_t(float(x) * inv_d);
    int rem = int(x) - int(e * d);
    e = rem < 0 ? e - 1 : (rem >= int(d) ? e + 1 : e);
    q = e;
    r = x - e * d;
}

}  // namespace ym
