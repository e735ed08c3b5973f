// Image preprocessing for the crater data path (gfx950): stretch-resize of grayscale uint8
// images to S x S with OpenCV's fixed-point INTER_LINEAR arithmetic, then /255 to fp32 NCHW.
//
// Replaces cv2.resize(im, (S, S), interpolation=cv2.INTER_LINEAR) + astype(float32) / 255 in the
// reference loader (/root/reference/yolo_scratch_cuda/datasets/crater_dataset_cuda.py:182-184,
// 253).  The reference does it per image on the CPU in DataLoader workers; here the workers only
// decode, the raw uint8 bytes cross PCIe (1/4 of the fp32 tensor) and one launch resizes the batch.
//
// Arithmetic (OpenCV resizeGeneric_, fixed-point 8U path, INTER_RESIZE_COEF_BITS = 11):
//   fx = float((dx + 0.5) * (W0 / S) - 0.5) in double, sx = floor(fx), fx -= sx;
//   sx < 0 -> (sx, fx) = (0, 0);  sx >= W0 - 1 -> (sx, fx) = (W0 - 1, 0);
//   a0 = rint((1 - fx) * 2048), a1 = rint(fx * 2048)  (saturate_cast<short>: round half to even)
//   h(r) = src[r][sx] * a0 + src[r][min(sx + 1, W0 - 1)] * a1            (the same for rows)
//   out = ((b0 * (h(sy) >> 4)) >> 16) + ((b1 * (h(sy1) >> 4)) >> 16) + 2) >> 2, clamped to 0..255
//        (the vertical rounding of OpenCV's SIMD path, which covers every column when S % 16 == 0)
// Images already S x S are copied unchanged (the reference skips the resize there, :183).
#include <algorithm>

#include "common.h"

namespace ym {
namespace {

__device__ __forceinline__ void lin_coeff(int d, double scale, int n, int& s, int& a0, int& a1) {
    float f = float((d + 0.5) * scale - 0.5);
    int si = int(floorf(f));
    f -= float(si);
    if (si < 0) { f = 0.f; si = 0; }
    if (si >= n - 1) { f = 0.f; si = n - 1; }
    s = si;
    a0 = __float2int_rn((1.f - f) * 2048.f);
    a1 = __float2int_rn(f * 2048.f);
}

// meta[b] = {byte offset of image b in src, h0, w0}; out (B, 1, S, S) fp32
__global__ void resize_linear_u8_kernel(const uint8_t* __restrict__ src, const int64_t* __restrict__ meta, int S,
                                        int64_t total, float* __restrict__ out) {
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
         i += int64_t(gridDim.x) * blockDim.x) {
        const int64_t b = i / (int64_t(S) * S);
        const int p = int(i - b * int64_t(S) * S);
        const int dy = p / S, dx = p - dy * S;
        const uint8_t* im = src + meta[3 * b];
        const int h0 = int(meta[3 * b + 1]), w0 = int(meta[3 * b + 2]);
        int v;
        if (h0 == S && w0 == S) {
            v = im[p];
        } else {
            int sx, a0, a1, sy, b0, b1;
            lin_coeff(dx, double(w0) / S, w0, sx, a0, a1);
            lin_coeff(dy, double(h0) / S, h0, sy, b0, b1);
            const int sx1 = min(sx + 1, w0 - 1), sy1 = min(sy + 1, h0 - 1);
            const uint8_t* r0 = im + int64_t(sy) * w0;
            const uint8_t* r1 = im + int64_t(sy1) * w0;
            const int h0v = int(r0[sx]) * a0 + int(r0[sx1]) * a1;
            const int h1v = int(r1[sx]) * a0 + int(r1[sx1]) * a1;
            v = (((b0 * (h0v >> 4)) >> 16) + ((b1 * (h1v >> 4)) >> 16) + 2) >> 2;
            v = min(max(v, 0), 255);
        }
        out[i] = float(v) / 255.0f;
    }
}

}  // namespace
}  // namespace ym

using namespace ym;

extern "C" int ym_resize_linear_u8(const uint8_t* src, const int64_t* meta, int batch, int size, float* out,
                                   void* stream) {
    YM_CHECK_ARG(src && meta && out && batch >= 0 && size > 0, "ym_resize_linear_u8: bad arguments");
    const int64_t total = int64_t(batch) * size * size;
    if (total == 0) return YM_OK;
    const int64_t blocks = std::min<int64_t>((total + 255) / 256, 16384);
    hipLaunchKernelGGL(resize_linear_u8_kernel, dim3(unsigned(blocks)), dim3(256), 0, as_stream(stream), src, meta, size,
                       total, out);
    YM_LAUNCH_CHECK("ym_resize_linear_u8");
    return YM_OK;
}
