"""ym_upsample2_fwd / ym_upsample2_bwd (misc.hip) — nn.Upsample(scale_factor=2, mode='nearest') of the
YOLOv11 head (yaml rows 11 and 14) and its gradient, on channel-slice views of wider buffers as the plan
uses them (the upsampled map is a slice of the following Concat).  Forward bit-exact against
F.interpolate; backward bit-exact against the fp32 sum of each 2x2 block in (row, column) order, plus
the existing gradient when accumulating, rounded once to bf16."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CASES = [  # (n, h, w, c, x channels, x offset, y channels, y offset)
    (4, 20, 20, 512, 512, 0, 768, 0),      # model.11 at s@640 (concat with a 256-channel skip)
    (4, 40, 40, 256, 256, 0, 384, 0),      # model.14
    (3, 7, 5, 24, 40, 8, 56, 16),          # ragged map, offset slices on both sides
    (1, 1, 1, 8, 8, 0, 8, 0),
    (2, 3, 9, 2048, 2048, 0, 2048, 0),     # rows wider than one workgroup
]


@pytest.mark.parametrize("n,h,w,c,xc,xo,yc,yo", CASES)
@pytest.mark.parametrize("accumulate", [0, 1])
def test_upsample2_fwd_bwd_bit_exact(n, h, w, c, xc, xo, yc, yo, accumulate):
    from yolomi._lib import call
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(n * 1000 + h * 10 + w + c + accumulate)
    xb = torch.randn(n, h, w, xc, generator=g, device=dev).to(torch.bfloat16)
    yb = torch.full((n, 2 * h, 2 * w, yc), 7.0, device=dev, dtype=torch.bfloat16)
    e = xb.element_size()
    call("ym_upsample2_fwd", xb.data_ptr() + e * xo, h * w * xc, xc, yb.data_ptr() + e * yo, 4 * h * w * yc, yc,
         n, h, w, c, None)
    torch.cuda.synchronize()
    x = xb[..., xo:xo + c].permute(0, 3, 1, 2).float()
    want = F.interpolate(x, scale_factor=2, mode="nearest").permute(0, 2, 3, 1).to(torch.bfloat16)
    assert torch.equal(yb[..., yo:yo + c].view(torch.int16), want.view(torch.int16))
    # the rest of the wider output buffer is untouched
    rest = torch.cat([yb[..., :yo], yb[..., yo + c:]], dim=-1)
    assert bool((rest == 7.0).all())

    dy = torch.randn(n, 2 * h, 2 * w, yc, generator=g, device=dev).to(torch.bfloat16)
    dx = torch.randn(n, h, w, xc, generator=g, device=dev).to(torch.bfloat16)
    dx0 = dx.clone()
    call("ym_upsample2_bwd", dy.data_ptr() + e * yo, 4 * h * w * yc, yc, dx.data_ptr() + e * xo, h * w * xc, xc,
         n, h, w, c, accumulate, None)
    torch.cuda.synchronize()
    d = dy[..., yo:yo + c].float()
    s = torch.zeros(n, h, w, c, device=dev)
    for a in range(2):
        for b in range(2):
            s = s + d[:, a::2, b::2, :]
    if accumulate:
        s = s + dx0[..., xo:xo + c].float()
    assert torch.equal(dx[..., xo:xo + c].view(torch.int16), s.to(torch.bfloat16).view(torch.int16))
    rest = torch.cat([dx[..., :xo], dx[..., xo + c:]], dim=-1)
    rest0 = torch.cat([dx0[..., :xo], dx0[..., xo + c:]], dim=-1)
    assert torch.equal(rest, rest0)


def test_upsample2_empty_map():
    from yolomi._lib import call
    call("ym_upsample2_fwd", None, 0, 8, None, 0, 8, 0, 4, 4, 8, None)
    call("ym_upsample2_bwd", None, 0, 8, None, 0, 8, 0, 4, 4, 8, 0, None)
    torch.cuda.synchronize()
