// Ping-pong structure microbenchmark (gfx950): one 512-thread workgroup per CU, 8 waves in two groups of
// four; per iteration every wave reads 8 fragments (ds_read_b128) and issues NDMA LDS-DMA pieces (L2-resident
// source), barrier, runs 16 v_mfma_f32_16x16x32_f16, barrier.  PP: group 1 one barrier behind (ping-pong);
// otherwise all waves load, then all compute.  Reports shader cycles per interval (s_memtime of block 0) —
// the floor of the conv kernels' K-loop structure, without any conv bookkeeping.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/pp_micro.hip -o tools/pp_micro
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int N>
__device__ __forceinline__ void vmw() {
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}
__device__ __forceinline__ void bar_wait_first() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ void bar_then_wait() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_sched_barrier(0);
}

// MODE 0: ping-pong, lgkmcnt before the barrier; 1: ping-pong, lgkmcnt after; 2: lockstep (no stagger);
// 3: MFMAs only (no reads, no barriers); 4: ping-pong with no MFMAs (load structure alone)
template <int MODE, int NDMA>
__global__ void __launch_bounds__(512, 1) pp_kernel(const char* src, float* out, long long* clk, int iters) {
    __shared__ __attribute__((aligned(16))) char lds[96 * 1024];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wave >> 2;
    const int fc = lane >> 4, fr = lane & 15;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(src) + size_t(blockIdx.x) * 65536,
                                                                       (short)0, 65536, 0x00020000);
    const int ra = (grp * 64 + fr) * 128 + ((fc ^ ((fr >> 1) & 7)) << 4);
    const int rb = 16384 + ((wave & 3) * 64 + fr) * 128 + ((fc ^ ((fr >> 1) & 7)) << 4);
    f16x8 fa[4], fb[4];
    f32x4 acc[4][4];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < 1024; ++i) lds[(tid * 1024 + i) % (96 * 1024)] = char(i * 7 + tid);   // any bytes
    __syncthreads();
    long long t0 = __builtin_amdgcn_s_memtime();
    long long r0 = __builtin_amdgcn_s_memrealtime();
    if ((MODE == 0 || MODE == 1 || MODE == 4) && grp == 1) bar_wait_first();
    for (int it = 0; it < iters; ++it) {
        if constexpr (MODE != 3) {
#pragma unroll
            for (int i = 0; i < 4; ++i) fa[i] = *reinterpret_cast<const f16x8*>(lds + ra + i * 2048);
#pragma unroll
            for (int j = 0; j < 4; ++j) fb[j] = *reinterpret_cast<const f16x8*>(lds + rb + j * 2048);
#pragma unroll
            for (int d = 0; d < NDMA; ++d)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(lds + 65536 + (wave * 4 + d) * 1024),
                                                         16, uint32_t(lane * 16), uint32_t(((it * 8 + wave * 4 + d) & 63) * 1024), 0, 0);
            if constexpr (NDMA > 0) vmw<NDMA * 2>();
            if constexpr (MODE == 1) bar_then_wait();
            else bar_wait_first();
        }
        if constexpr (MODE != 4) {
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[i], fb[j], acc[i][j], 0, 0, 0);
            __builtin_amdgcn_s_setprio(0);
        }
        if constexpr (MODE != 3) bar_wait_first();
    }
    if ((MODE == 0 || MODE == 1 || MODE == 4) && grp == 0) bar_wait_first();
    vmw<0>();
    long long t1 = __builtin_amdgcn_s_memtime();
    long long r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.f;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (MODE == 4) s += float(fa[0][0]) + float(fb[0][1]);
    out[blockIdx.x * 512 + tid] = s;
    if (blockIdx.x == 0 && tid == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}

template <int MODE, int NDMA>
void run(const char* name, const char* src, float* out, long long* clk) {
    const int iters = 2000;
    pp_kernel<MODE, NDMA><<<256, 512>>>(src, out, clk, iters);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    pp_kernel<MODE, NDMA><<<256, 512>>>(src, out, clk, iters);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    long long c[2];
    CK(hipMemcpy(c, clk, sizeof(c), hipMemcpyDeviceToHost));
    const double ghz = double(c[0]) / (double(c[1]) / 100e6) / 1e9;
    // per iteration a wave runs one load and one compute interval; MFMA-bound = 2 x 16 x 16 = 512 cycles
    const double tf = 256.0 * 8 * 16 * 16384.0 * iters / (ms * 1e-3) / 1e12;
    printf("%-34s NDMA %d: %7.1f cycles/iter (MFMA floor 512) clock %.2f GHz  %6.0f TF/s  %.3f ms\n", name, NDMA,
           double(c[0]) / iters, ghz, tf, ms);
}

int main() {
    char* src;
    float* out;
    long long* clk;
    CK(hipMalloc(&src, 256 * 65536));
    CK(hipMalloc(&out, 256 * 512 * 4));
    CK(hipMalloc(&clk, 64));
    CK(hipMemset(src, 0x3c, 256 * 65536));
    run<3, 0>("mfma only (no reads, no barrier)", src, out, clk);
    run<2, 0>("lockstep reads+mfma", src, out, clk);
    run<0, 0>("ping-pong, wait then barrier", src, out, clk);
    run<1, 0>("ping-pong, barrier then wait", src, out, clk);
    run<4, 0>("ping-pong loads only", src, out, clk);
    run<0, 1>("ping-pong, wait then barrier", src, out, clk);
    run<0, 2>("ping-pong, wait then barrier", src, out, clk);
    run<0, 3>("ping-pong, wait then barrier", src, out, clk);
    run<1, 3>("ping-pong, barrier then wait", src, out, clk);
    run<2, 3>("lockstep reads+mfma", src, out, clk);
    run<4, 3>("ping-pong loads only", src, out, clk);
    return 0;
}
