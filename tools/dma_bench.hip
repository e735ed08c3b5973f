// Staging-rate microbenchmark (gfx950): how fast can one workgroup per CU move bytes from L2 / MALL
// into LDS by LDS-DMA (buffer_load_dwordx4 ... lds), or into registers by buffer_load_dwordx4, as a
// function of the waves per CU and the pieces each wave keeps in flight?  No compute: this is the
// ceiling the implicit-GEMM conv kernels' operand staging runs under.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/dma_bench.hip -o tools/dma_bench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, bytes, 0x00020000);
}

template <int N>
__device__ __forceinline__ void vmw() {
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// every wave streams `iters` pieces of 1 KiB (64 lanes x 16 B) from its workgroup's region into a private
// LDS ring of RING pieces, keeping DEPTH pieces in flight (counted vmcnt)
template <int DEPTH, int RING, int MAXW = 16>
__global__ void dma_kernel(const char* src, int region, int iters, int* sink) {
    __shared__ __attribute__((aligned(16))) char lds[MAXW * RING * 1024];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const char* base = src + size_t(blockIdx.x) * region;
    const __amdgpu_buffer_rsrc_t r = rsrc(base, region);
    const int npieces = region / 1024;
    int p = wave;
    for (int i = 0; i < iters; ++i) {
        char* dst = lds + (wave * RING + (i % RING)) * 1024;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)dst, 16,
                                                 uint32_t(p) * 1024u + lane * 16u, 0, 0, 0);
        p += nw;
        if (p >= npieces) p -= npieces;
        vmw<DEPTH>();
    }
    vmw<0>();
    __syncthreads();
    if (threadIdx.x == 0) sink[blockIdx.x] = lds[blockIdx.x & 1023];
}

template <int DEPTH>
__global__ void reg_kernel(const char* src, int region, int iters, int* sink) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const char* base = src + size_t(blockIdx.x) * region;
    const __amdgpu_buffer_rsrc_t r = rsrc(base, region);
    const int npieces = region / 1024;
    uint32_t acc = 0;
    int p = wave;
    for (int i = 0; i < iters; i += DEPTH) {
        uint4 v[DEPTH];
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            v[d] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, uint32_t(p) * 1024u + lane * 16u, 0, 0));
            p += nw;
            if (p >= npieces) p -= npieces;
        }
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) acc ^= v[d].x ^ v[d].y ^ v[d].z ^ v[d].w;
    }
    if (acc == 0x12345678u) sink[blockIdx.x] = acc;
}

int main(int argc, char** argv) {
    const int ncu = 256;
    const size_t maxb = size_t(ncu) * (4 << 20);
    char* src;
    int* sink;
    CK(hipMalloc(&src, maxb));
    CK(hipMalloc(&sink, 4096 * 4));
    CK(hipMemset(src, 1, maxb));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int iters = 4096;
    printf("kind   waves depth region_KB  GB/s/CU  TB/s_chip\n");
    for (int region_kb : {64, 1024, 4096}) {
        for (int kind = 0; kind < 2; ++kind) {
            for (int waves : {4, 8, 16}) {
                for (int depth : {2, 4, 8, 16}) {
                    auto launch = [&]() {
                        dim3 g(ncu), b(64 * waves);
                        const int reg = region_kb * 1024;
                        if (kind == 0) {
                            if (depth == 2) dma_kernel<2, 4><<<g, b>>>(src, reg, iters, sink);
                            if (depth == 4) dma_kernel<4, 6><<<g, b>>>(src, reg, iters, sink);
                            if (depth == 8) dma_kernel<8, 9><<<g, b>>>(src, reg, iters, sink);
                            if (depth == 16) {
                                if (waves > 8) return false;
                                dma_kernel<16, 17, 8><<<g, b>>>(src, reg, iters, sink);
                            }
                        } else {
                            if (depth == 2) reg_kernel<2><<<g, b>>>(src, reg, iters, sink);
                            if (depth == 4) reg_kernel<4><<<g, b>>>(src, reg, iters, sink);
                            if (depth == 8) reg_kernel<8><<<g, b>>>(src, reg, iters, sink);
                            if (depth == 16) reg_kernel<16><<<g, b>>>(src, reg, iters, sink);
                        }
                        return true;
                    };
                    if (!launch()) continue;
                    CK(hipDeviceSynchronize());
                    CK(hipEventRecord(e0));
                    const int reps = 5;
                    for (int r = 0; r < reps; ++r) launch();
                    CK(hipEventRecord(e1));
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    const double bytes = double(ncu) * waves * iters * 1024.0 * reps;
                    const double gbs = bytes / (ms * 1e-3) / 1e9;
                    printf("%s %5d %5d %9d %8.1f %9.2f\n", kind ? "reg " : "dma ", waves, depth, region_kb, gbs / ncu,
                           gbs / 1e3);
                    fflush(stdout);
                }
            }
        }
    }
    return 0;
}
