"""Win_noShift_Attention block (reference: layers/Masked_Attention.py:143-189).

out = conv_a(x) * sigmoid(conv_b(attn(x, mask))) + x, with every conv on the
MFMA engine and the elementwise tails fused into conv epilogues:
  ResidualUnit:  1x1+GELU -> 3x3+GELU -> 1x1 (+identity, GELU in the epilogue)
  gate:          conv_b[3] epilogue computes a * sigmoid(v) + x directly.
(The name is the reference's: the shift IS applied, shift_size = ws/2.)"""
import torch
import torch.nn as nn

from .. import runtime as rt
from ._blocks import conv1x1, conv3x3
from .masked_win_attention import WinBasedAttention


class ResidualUnit(nn.Module):
    """Masked_Attention.py:150-169 (nested class there; same state_dict keys)."""

    def __init__(self, N):
        super().__init__()
        self.conv = nn.Sequential(conv1x1(N, N // 2), nn.GELU(), conv3x3(N // 2, N // 2),
                                  nn.GELU(), conv1x1(N // 2, N))
        self.relu = nn.GELU()

    def nhwc(self, x):
        dt = x.t.dtype
        c0, c2, c4 = self.conv[0], self.conv[2], self.conv[4]
        t = rt.conv(rt.packed(c0, dt, rt.segs_of(x.src())), [x.src()], act="gelu")
        t = rt.conv(rt.packed(c2, dt, rt.segs_of(t.src())), [t.src()], act="gelu")
        return rt.conv(rt.packed(c4, dt, rt.segs_of(t.src())), [t.src()], act="gelu", res0=x)

    def forward(self, x):
        rt.check_gpu(x)
        with torch.no_grad():
            return rt.to_nchw(self.nhwc(rt.to_nhwc(x, torch.float32)))


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
        a = x
        for ru in self.conv_a:
            a = ru.nhwc(a)
        b = self.attn.nhwc(x, mask)
        for ru in list(self.conv_b)[:3]:
            b = ru.nhwc(b)
        pk = rt.packed(self.conv_b[3], x.t.dtype, rt.segs_of(b.src()))
        return rt.conv(pk, [b.src()], act="gate", res1=a, res2=x)

    def forward(self, x, mask):
        rt.check_gpu(x, mask)
        with torch.no_grad():
            return rt.to_nchw(self.nhwc(rt.to_nhwc(x, torch.float32), mask))
