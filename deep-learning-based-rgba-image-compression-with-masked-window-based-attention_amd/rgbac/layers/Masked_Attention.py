"""Win_noShift_Attention block (reference: layers/Masked_Attention.py:143-189).

out = conv_a(x) * sigmoid(conv_b(attn(x, mask))) + x, with every conv on the
MFMA engine and the elementwise tails fused into conv epilogues:
  ResidualUnit:  1x1+GELU -> 3x3+GELU -> 1x1 (+identity, GELU in the epilogue)
  gate:          conv_b[3] epilogue computes a * sigmoid(v) + x directly.
(The name is the reference's: the shift IS applied, shift_size = ws/2.)"""
import ctypes
import os

import torch
import torch.nn as nn

from .. import _lib
from .. import runtime as rt
from ._blocks import conv1x1, conv3x3
from .masked_win_attention import WinBasedAttention, needs_grad


class ResidualUnit(nn.Module):
    """Masked_Attention.py:150-169 (nested class there; same state_dict keys)."""

    def __init__(self, N):
        super().__init__()
        self.conv = nn.Sequential(conv1x1(N, N // 2), nn.GELU(), conv3x3(N // 2, N // 2),
                                  nn.GELU(), conv1x1(N // 2, N))
        self.relu = nn.GELU()

    def nhwc(self, x):
        return run_residual_units([(self, x)])[0]

    def forward(self, x):
        rt.check_gpu(x)
        if needs_grad(self, x):
            from ..train_forward import layer_t, residual_unit_t
            return layer_t(lambda f: residual_unit_t(self, f), x)
        with torch.no_grad():
            return rt.to_nchw(self.nhwc(rt.to_nhwc(x, torch.float32)))


FUSED = os.environ.get("RGBAC_FUSED_RU", "1") != "0"


def _fused_ok(pairs):
    x = pairs[0][1]
    return (FUSED and x.t.dtype == torch.bfloat16 and x.C == 192 and x.H % 8 == 0 and
            x.W % 8 == 0 and len(pairs) <= 4)


def run_residual_units_fused(pairs):
    """The same units as ONE rgbac_residual_unit launch (csrc/fused.hip): both
    intermediates stay in LDS, one read of x and one write of y per pixel."""
    x0 = pairs[0][1]
    arr = (_lib.RuArgs * len(pairs))()
    outs, keep = [], []
    for i, (u, x) in enumerate(pairs):
        segs = [(x.C, x.ldc)]
        p1 = rt.packed(u.conv[0], x.t.dtype, segs)
        p2 = rt.packed(u.conv[2], x.t.dtype, [(p1.cout, rt.round_up(p1.cout, 8))])
        p3 = rt.packed(u.conv[4], x.t.dtype, [(p2.cout, rt.round_up(p2.cout, 8))])
        o = rt.new_feat(x.B, x.H, x.W, x.C, x.t.dtype, x.t.device)
        a = arr[i]
        a.dtype, a.channels, a.batch, a.h, a.w = _lib.BF16, x.C, x.B, x.H, x.W
        a.x, a.x_ldc = x.ptr(), x.ldc
        a.w1, a.w2, a.w3 = p1.w.data_ptr(), p2.w.data_ptr(), p3.w.data_ptr()
        a.w1_kpad, a.w2_kpad, a.w3_kpad = p1.k_pad, p2.k_pad, p3.k_pad
        a.b1, a.b2, a.b3 = p1.bias.data_ptr(), p2.bias.data_ptr(), p3.bias.data_ptr()
        a.out, a.out_ldc = o.ptr(), o.ldc
        outs.append(o)
        keep.append((p1, p2, p3))
    npix = x0.B * x0.H * x0.W
    C = x0.C
    flops = 2.0 * npix * len(pairs) * (C * C // 2 * 2 + 9 * (C // 2) ** 2)
    rt.timed(f"ru_fused_kernel<{C}, {C // 2}>", flops, 2 * npix * len(pairs) * 2 * C,
             lambda: _lib.call("rgbac_residual_unit", ctypes.addressof(arr), len(pairs),
                               _lib.stream_ptr(x0.t.device)),
             f"ru_fused_kernel g{len(pairs)} C{C} {x0.H}x{x0.W} B{x0.B}")
    return outs


def run_residual_units(pairs):
    """Independent ResidualUnits [(unit, x), ...] of equal shape as grouped launches:
    1x1+GELU, 3x3+GELU, 1x1 (+identity, GELU) -- three launches for all units
    (or one fused launch for bf16 C = 192)."""
    if _fused_ok(pairs):
        return run_residual_units_fused(pairs)
    return run_residual_units_unfused(pairs)


def run_residual_units_unfused(pairs):
    from .TransformRGB import prep_conv
    ts = rt.launch([prep_conv(u.conv[0], [x.src()], act="gelu") for u, x in pairs])
    ts = rt.launch([prep_conv(u.conv[2], [t.src()], act="gelu") for (u, _), t in zip(pairs, ts)])
    return rt.launch([prep_conv(u.conv[4], [t.src()], act="gelu", res0=x)
                      for (u, x), t in zip(pairs, ts)])


class Win_noShift_Attention(nn.Module):
    """Window-based self-attention module."""

    def __init__(self, dim, num_heads=8, window_size=8, shift_size=0):
        super().__init__()
        N = dim
        self.conv_a = nn.Sequential(ResidualUnit(N), ResidualUnit(N), ResidualUnit(N))
        self.attn = WinBasedAttention(dim=dim, num_heads=num_heads, window_size=window_size,
                                      shift_size=shift_size)
        self.conv_b = nn.Sequential(ResidualUnit(N), ResidualUnit(N), ResidualUnit(N),
                                    conv1x1(N, N))

    def nhwc(self, x, mask):
        # the trunk (conv_a) and the attention branch (attn -> conv_b) are independent
        # until the gate: their residual units run pairwise as 2-group launches
        b = self.attn.nhwc(x, mask)
        a = x
        for k in range(3):
            a, b = run_residual_units([(self.conv_a[k], a), (self.conv_b[k], b)])
        pk = rt.packed(self.conv_b[3], x.t.dtype, rt.segs_of(b.src()))
        return rt.conv(pk, [b.src()], act="gate", res1=a, res2=x)

    def forward(self, x, mask):
        rt.check_gpu(x, mask)
        if needs_grad(self, x):
            from ..train_forward import attention_block_t, layer_t
            return layer_t(lambda f: attention_block_t(self, f, mask), x)
        with torch.no_grad():
            return rt.to_nchw(self.nhwc(rt.to_nhwc(x, torch.float32), mask))
