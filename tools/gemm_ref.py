"""Reference timings (NOT the product path): hipBLASLt via torch.matmul on the GEMM each conv layer is
equivalent to — a 1x1 conv is exactly Y[M, N] = X[M, K] W[N, K]^T over NHWC pixels; a 3x3 conv is priced as
its im2col GEMM (K = 9 Cin, the operand materialised, so it is an upper bound on what a GEMM engine does with
the same FLOPs).  Tells whether a gap to the MFMA peak is the kernel structure or the shape.
usage: python tools/gemm_ref.py
"""
import torch

SHAPES = [  # (label, M, K, N)   s@640 bs64 layers
    ("1x1 512->512 20x20", 64 * 400, 512, 512),
    ("1x1 768->512 20x20", 64 * 400, 768, 512),
    ("1x1 1024->512 20x20", 64 * 400, 1024, 512),
    ("1x1 384->256 40x40", 64 * 1600, 384, 256),
    ("1x1 768->256 40x40", 64 * 1600, 768, 256),
    ("1x1 192->256 80x80", 64 * 6400, 192, 256),
    ("1x1 512->128 80x80", 64 * 6400, 512, 128),
    ("1x1 96->128 160x160", 64 * 25600, 96, 128),
    ("3x3 128->128 80x80 (im2col)", 64 * 6400, 1152, 128),
    ("3x3 128->128 40x40 (im2col)", 64 * 1600, 1152, 128),
    ("3x3 256->256 s2 40x40 (im2col)", 64 * 1600, 2304, 256),
    ("3x3 128->128 20x20 (im2col)", 64 * 400, 1152, 128),
]


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    print(f"{'layer':34s} {'GFLOP':>7s} {'ms':>8s} {'TF/s':>7s} {'frac':>6s}")
    for label, M, K, N in SHAPES:
        a = torch.rand(M, K, device=dev, dtype=torch.float16, generator=g) * 2 - 1
        b = torch.rand(N, K, device=dev, dtype=torch.float16, generator=g) * 2 - 1
        for _ in range(3):
            torch.matmul(a, b.t())
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record()
        for _ in range(reps):
            torch.matmul(a, b.t())
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        fl = 2 * M * K * N
        print(f"{label:34s} {fl / 1e9:7.1f} {ms:8.3f} {fl / ms / 1e9:7.0f} {fl / ms / 1e9 / 2500:6.3f}")


if __name__ == "__main__":
    main()
