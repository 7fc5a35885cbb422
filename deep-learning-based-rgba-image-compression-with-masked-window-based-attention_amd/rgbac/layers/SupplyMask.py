"""SupplyMaskToTransform (reference: layers/SupplyMask.py:7-18) as one HIP
launch chain: six AvgPool2d(3, stride 2, padding 1, count_include_pad)."""
import ctypes

import torch
import torch.nn as nn

from .. import _lib
from .. import runtime as rt


def mask_pyramid(alpha, levels=6, round255=False):
    """alpha: fp32 (B,1,H,W) on the GPU -> (rounded or None, [level1..levelN])."""
    rt.check_gpu(alpha)
    a = alpha.contiguous().float()
    B, C, H, W = a.shape
    assert C == 1, "alpha must have one channel"
    outs, h, w = [], H, W
    for _ in range(levels):
        h, w = (h - 1) // 2 + 1, (w - 1) // 2 + 1
        outs.append(torch.empty((B, 1, h, w), dtype=torch.float32, device=a.device))
    rounded = torch.empty_like(a) if round255 else None
    ptrs = (ctypes.c_void_p * max(levels, 1))(*[o.data_ptr() for o in outs])
    _lib.call("rgbac_mask_pyramid", B, H, W, a.data_ptr(), 1 if round255 else 0,
              _lib.ptr(rounded), levels, ptrs, _lib.stream_ptr(a.device))
    return rounded, outs


class SupplyMaskToTransform(nn.Module):
    def __init__(self, kernel=3):
        super().__init__()
        assert kernel == 3, "the reference only uses kernel=3"
        self.pool = nn.AvgPool2d(kernel, stride=2, padding=1)

    def forward(self, inputs):
        return tuple(mask_pyramid(inputs, 6)[1])
