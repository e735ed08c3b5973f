"""wgrad3 tap lookahead (ym_wgrad_set_lookahead, measurement library): the weight gradient of every 3x3 shape of
tests/test_gpu_conv.py SHAPES plus s@640 bs64-sized layers, LA 1 against LA 0 — bit-identical expected (the same MFMAs
into the same accumulators in the same order; only the fragment reads move)."""
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
for p in (str(ROOT), str(ROOT / "yolo-scratch_amd"), str(ROOT / "tests")):
    sys.path.insert(0, p)


def main():
    import torch
    import test_gpu_conv as T
    from yolomi._lib import call, lib
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream().cuda_stream
    shapes = [s for s in T.SHAPES if s[5] == 3] + [
        (64, 80, 80, 128, 128, 3, 1, 1), (64, 160, 160, 64, 64, 3, 2, 1), (64, 40, 40, 256, 128, 3, 1, 1),
        (64, 20, 20, 128, 128, 3, 1, 1), (64, 40, 40, 256, 256, 3, 2, 1), (64, 160, 160, 32, 32, 3, 1, 1),
        (64, 80, 80, 64, 64, 3, 1, 1), (64, 20, 20, 256, 256, 3, 1, 1)]
    for shape in shapes:
        n, h, w, cin, cout, k, s, p = shape
        d, oh, ow = T._desc(*shape)
        g = torch.Generator().manual_seed(hash(shape) & 0xFFFF)
        x = torch.randn(n, h, w, cin, generator=g).half().to(dev)
        dz = torch.randn(n, oh, ow, cout, generator=g).bfloat16().to(dev)
        ws = torch.empty(max(lib().ym_conv_wgrad_workspace_size(ctypes.byref(d)) // 4, 1), dtype=torch.float32,
                         device=dev)
        outs = []
        for la in (0, 1):
            lib().ym_wgrad_set_lookahead(la)
            dw = torch.full((cout, cin, k, k), float("nan"), dtype=torch.float32, device=dev)
            call("ym_conv_wgrad", ctypes.byref(d), dz.data_ptr(), x.data_ptr(), ws.data_ptr(), ws.numel() * 4,
                 dw.data_ptr(), 0, st)
            outs.append(dw)
        torch.cuda.synchronize()
        assert torch.isfinite(outs[0]).all() and torch.equal(outs[0], outs[1]), shape
        print("bit-identical", shape, flush=True)
    lib().ym_wgrad_set_lookahead(-1)
    print("all shapes ok")


if __name__ == "__main__":
    main()
