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
        return run_residual_units([(self, x)])[0]

    def forward(self, x):
        rt.check_gpu(x)
        with torch.no_grad():
            return rt.to_nchw(self.nhwc(rt.to_nhwc(x, torch.float32)))


def run_residual_units(pairs):
    """Independent ResidualUnits [(unit, x), ...] of equal shape as grouped launches:
    1x1+GELU, 3x3+GELU, 1x1 (+identity, GELU) -- three launches for all units."""
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
        with torch.no_grad():
            return rt.to_nchw(self.nhwc(rt.to_nhwc(x, torch.float32), mask))
