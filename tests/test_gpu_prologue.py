"""GPU: the forward's one-launch head and tail against the launches they replace.

rgbac_forward_prologue (AutoEncoderRGB_Journal.py:209-217) = rgbac_mask_pyramid(round255) +
rgbac_nchw_to_nhwc + a zero fill, bit for bit.  rgbac_finalize_fused (:280-295) =
rgbac_finalize_ex in one launch through a last-arriving-block ticket: same per-image MSE
partials, the scalars equal up to fp64 summation order (4 combining waves instead of 16),
x_hat's NCHW copy bit-identical, and the ticket is back at zero after every launch (graph
replays reuse it).  The whole bf16 forward with both is bit-identical in x_hat to the separate
launches."""
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


@pytest.mark.parametrize("mode,B,H,W", [(0, 8, 256, 256), (0, 1, 64, 64), (1, 3, 128, 96),
                                        (0, 2, 1024, 512)])
def test_finalize_fused_equals_two_launches(device, mode, B, H, W):
    from rgbac import _lib
    from rgbac import runtime as rt
    g = torch.Generator().manual_seed(11)
    cx = 3 if mode == 0 else 1
    x = torch.rand((B, cx, H, W), generator=g).cuda()
    xh = rt.to_nhwc((x + 0.05 * torch.randn((B, cx, H, W), generator=g).cuda()).clamp(0, 1),
                    torch.bfloat16)
    mask = _alpha(B, H, W, 12)[:, 0].contiguous() if mode == 0 else None
    yb = torch.rand(10 * 77, generator=g, dtype=torch.float64).cuda() * 100
    zb = torch.rand(5, generator=g, dtype=torch.float64).cuda() * 10
    nd = _lib.finalize_scratch_doubles(B, H, W)

    def run(fused, ticket=None):
        scratch = torch.empty(nd, dtype=torch.float64, device="cuda")
        out = torch.empty(4, dtype=torch.float32, device="cuda")
        xo = torch.full((B, cx, H, W), float("nan"), device="cuda")
        head = (_lib.BF16, mode, B, cx, H, W, x.data_ptr(), xh.ptr(), xh.ldc, _lib.ptr(mask),
                yb.data_ptr(), yb.numel(), zb.data_ptr(), zb.numel(), scratch.data_ptr())
        if fused:
            _lib.call("rgbac_finalize_fused", *head, ticket.data_ptr(), out.data_ptr(),
                      xo.data_ptr(), _lib.stream_ptr(x.device))
        else:
            _lib.call("rgbac_finalize_ex", *head, out.data_ptr(), xo.data_ptr(),
                      _lib.stream_ptr(x.device))
        torch.cuda.synchronize()
        return out.cpu(), xo

    want, want_xo = run(False)
    ticket = torch.zeros(1, dtype=torch.int32, device="cuda")
    for _ in range(3):                             # the last arriver resets the ticket
        got, got_xo = run(True, ticket)
        assert ticket.item() == 0
        # same partials; the 4-wave combine adds them in another fixed fp64 order
        torch.testing.assert_close(got, want, rtol=2e-7, atol=0.0)
        assert torch.equal(got_xo, want_xo)


def test_rgb_forward_fused_head_and_tail_bit_identical(device):
    """bf16 forward at the bench's config-2 shape with the one-launch prologue / finalize vs
    the separate launches: x_hat identical, the scalars equal to fp64-order rounding."""
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
        assert abs(a[i].item() - b[i].item()) <= 1e-6 * abs(a[i].item()), (i, a[i], b[i])
