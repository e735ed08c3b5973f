"""ym_prep_weights (conv.hip): fp32 OIHW master weights -> fp16 [Cout][KH][KW][Cin] and bf16
[Cin][KH][KW][Cout_t], one launch over a table of entries — bit-exact against torch's own roundings.
The entry mix covers chunks inside one entry, chunks crossing several small entries, entries without a
transposed copy, padded transposed rows (cout_t > cout), long rows and a ragged total; the forward-only launch
(eval plans) on the same table.  More than 64 entries: both levels of the chunk -> entry search."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [  # (cout, cin, k, need_t, cout_t)
    (16, 3, 3, False, None),          # stem: no data gradient
    (32, 16, 3, True, None),
    (64, 64, 1, True, 80),            # padded transposed rows
    (3, 8, 1, True, None),            # tiny entries: chunks cross several of them
    (5, 8, 1, False, None),
    (7, 16, 3, True, 8),
    (512, 256, 3, True, None),        # ~290 chunks inside one entry
    (96, 192, 1, True, None),
    (255, 64, 1, True, 256),          # Detect-like odd cout
    (13, 24, 3, True, None),          # ragged tail
    (64, 512, 3, False, None),        # long rows (4608): chunks spanning 2 rows
] + [(8, 8, 1, i % 2 == 0, None) for i in range(70)] + [(24, 40, 3, True, None)]   # > 64 entries


def test_prep_weights_bit_exact():
    from yolomi._lib import WPrepEntry, call
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(7)
    ws, fwds, ts = [], [], []
    arr = (WPrepEntry * len(SHAPES))()
    off = 0
    for e, (co, ci, k, need_t, cout_t) in zip(arr, SHAPES):
        cout_t = cout_t or co
        w = (torch.randn(co, ci, k, k, generator=g) * 3).to(dev)
        fwd = torch.full((co, k, k, ci), 12345, dtype=torch.int16, device=dev).view(torch.float16)
        t = torch.zeros(ci, k, k, cout_t, dtype=torch.bfloat16, device=dev) if need_t else None
        ws.append(w), fwds.append(fwd), ts.append(t)
        e.src, e.dst_fwd, e.dst_t = w.data_ptr(), fwd.data_ptr(), (t.data_ptr() if t is not None else None)
        e.elem_offset, e.cout, e.cin, e.kh, e.kw, e.cout_t = off, co, ci, k, k, cout_t
        off += w.numel()
    table = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(dev)
    call("ym_prep_weights", table.data_ptr(), len(SHAPES), off, None)
    torch.cuda.synchronize()
    _check(ws, fwds, ts)


def test_prep_weights_fwd_only_bit_exact():
    """ym_prep_weights_fwd: the forward copies of the same table, bit-exact; the transposed destinations untouched."""
    from yolomi._lib import WPrepEntry, call
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(9)
    ws, fwds, ts = [], [], []
    arr = (WPrepEntry * len(SHAPES))()
    off = 0
    for e, (co, ci, k, need_t, cout_t) in zip(arr, SHAPES):
        cout_t = cout_t or co
        w = (torch.randn(co, ci, k, k, generator=g) * 3).to(dev)
        fwd = torch.full((co, k, k, ci), 12345, dtype=torch.int16, device=dev).view(torch.float16)
        t = torch.full((ci, k, k, cout_t), 777, dtype=torch.int16, device=dev).view(torch.bfloat16) if need_t else None
        ws.append(w), fwds.append(fwd), ts.append(t)
        e.src, e.dst_fwd, e.dst_t = w.data_ptr(), fwd.data_ptr(), (t.data_ptr() if t is not None else None)
        e.elem_offset, e.cout, e.cin, e.kh, e.kw, e.cout_t = off, co, ci, k, k, cout_t
        off += w.numel()
    table = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(dev)
    call("ym_prep_weights_fwd", table.data_ptr(), len(SHAPES), off, None)
    torch.cuda.synchronize()
    for (co, ci, k, need_t, cout_t), w, fwd, t in zip(SHAPES, ws, fwds, ts):
        assert torch.equal(fwd.view(torch.int16), w.permute(0, 2, 3, 1).half().view(torch.int16)), (co, ci, k)
        if t is not None:
            assert torch.all(t.view(torch.int16) == 777), (co, ci, k)


def _check(ws, fwds, ts):
    for (co, ci, k, need_t, cout_t), w, fwd, t in zip(SHAPES, ws, fwds, ts):
        cout_t = cout_t or co
        ref = w.permute(0, 2, 3, 1).half()
        assert torch.equal(fwd.view(torch.int16), ref.view(torch.int16)), (co, ci, k)
        if need_t:
            reft = torch.zeros_like(t)
            reft[..., :co] = w.permute(1, 2, 3, 0).bfloat16()
            assert torch.equal(t.view(torch.int16), reft.view(torch.int16)), (co, ci, k)
