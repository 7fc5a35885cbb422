"""GPU: the forward's one-launch head against the launches it replaces.

rgbac_forward_prologue (AutoEncoderRGB_Journal.py:209-217) = rgbac_mask_pyramid(round255) +
rgbac_nchw_to_nhwc + a zero fill, bit for bit.  The whole bf16 forward with it is bit-identical
in x_hat to the separate launches, and its scalars agree (the bits partials are the same
values: only who zeroes them changed)."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


def _alpha(B, H, W, seed):
    g = torch.Generator().manual_seed(seed)
    a = torch.rand((B, 1, H, W), generator=g)
    a[:, :, : H // 3] = 0.0                       # a transparent band, exact zeros
    a[:, :, -3:, :] = 1.0
    return a.cuda()


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("B,C,H,W,levels", [(2, 3, 256, 192, 4), (1, 3, 64, 64, 4),
                                            (3, 1, 96, 160, 3), (1, 3, 40, 72, 1)])
def test_prologue_equals_separate_launches(device, dt, B, C, H, W, levels):
    from rgbac import _lib
    from rgbac import runtime as rt
    from rgbac.layers.SupplyMask import mask_pyramid
    g = torch.Generator().manual_seed(7)
    x = torch.rand((B, C, H, W), generator=g).cuda()
    a = _alpha(B, H, W, 8)
    want_r, want_md = mask_pyramid(a, levels, round255=True)
    want_xf = rt.to_nhwc(x, dt)
    xf = torch.full_like(want_xf.t, float("nan"))
    md, h, w = [], H, W
    for _ in range(levels):
        h, w = (h - 1) // 2 + 1, (w - 1) // 2 + 1
        md.append(torch.full((B, 1, h, w), float("nan"), device=x.device))
    rounded = torch.full_like(a, float("nan"))
    zero = torch.full((1237,), float("nan"), dtype=torch.float64, device=x.device)
    ptrs = (ctypes.c_void_p * levels)(*[o.data_ptr() for o in md])
    _lib.call("rgbac_forward_prologue", _lib.dtype_code(dt), B, C, H, W, x.data_ptr(),
              xf.data_ptr(), want_xf.ldc, a.data_ptr(), 1, rounded.data_ptr(), levels, ptrs,
              zero.data_ptr(), zero.numel(), _lib.stream_ptr(x.device))
    torch.cuda.synchronize()
    assert torch.equal(xf.view(torch.int16 if dt == torch.bfloat16 else torch.int32),
                       want_xf.t.view(torch.int16 if dt == torch.bfloat16 else torch.int32))
    assert torch.equal(rounded, want_r)
    for got, want in zip(md, want_md):
        assert torch.equal(got, want)
    assert torch.equal(zero, torch.zeros_like(zero))


def test_prologue_rejects_unchunked_rows(device):
    from rgbac import _lib
    x = torch.rand((1, 3, 64, 64), device="cuda")
    a = torch.rand((1, 1, 64, 64), device="cuda")
    xf = torch.empty((1, 64, 64, 6), dtype=torch.bfloat16, device="cuda")
    md = [torch.empty(1, device="cuda")]
    ptrs = (ctypes.c_void_p * 1)(md[0].data_ptr())
    with pytest.raises(RuntimeError, match="16-byte NHWC row chunks"):
        _lib.call("rgbac_forward_prologue", _lib.BF16, 1, 3, 64, 64, x.data_ptr(), xf.data_ptr(),
                  6, a.data_ptr(), 0, None, 1, ptrs, None, 0, _lib.stream_ptr(x.device))


def test_rgb_forward_fused_head_bit_identical(device):
    """bf16 forward at the bench's config-2 shape with the one-launch prologue vs the separate
    launches: x_hat and the four scalars identical.  (The first forward of a shape tunes its
    tiles live: the GAUSS launches' candidates write bits partials at their own granularity, so
    the tuner re-zeroes them -- rgbac/runtime.py launch -- or the first bpp over-counts.)"""
    from bench import rgb_net, synth_inputs
    from rgbac.layers.SupplyMask import mask_pyramid
    from rgbac.models import AutoEncoderRGB_Journal as M
    net = rgb_net().cuda().eval().set_compute_dtype(torch.bfloat16)
    x, a = (t.cuda() for t in synth_inputs(8, 256, 256))
    _, me = mask_pyramid(a, 4)
    args = [x, a, a, *me]
    outs = {}
    old = M.FUSED_PROLOGUE
    try:
        for fused in (False, True):
            M.FUSED_PROLOGUE = fused
            with torch.no_grad():
                outs[fused] = [t.clone() for t in net(*args)]
            torch.cuda.synchronize()
    finally:
        M.FUSED_PROLOGUE = old
    a, b = outs[False], outs[True]
    assert torch.equal(a[0], b[0])
    for i in (1, 2, 3, 4):
        assert a[i].item() == b[i].item(), (i, a[i], b[i])
