"""Unmasked shifted-window attention (reference: layers/win_attention.py).

Same kernels as masked_win_attention with ``masked=0``: every window is
attended and the shift mask is shared by all images (:161, :104)."""
import torch

from .. import runtime as rt
from .masked_win_attention import (WindowAttention, needs_grad, window_partition,  # noqa: F401
                                   window_reverse)
from .masked_win_attention import WinBasedAttention as _MaskedWinBasedAttention


class WinBasedAttention(_MaskedWinBasedAttention):
    masked = False

    def nhwc(self, x, img_alpha=None):
        return self.attn.run_nhwc(x, None, self.shift_size, False)

    def forward(self, x):
        rt.check_gpu(x)
        if needs_grad(self, x):
            from ..train_forward import layer_t, win_attention_t
            return layer_t(lambda f: win_attention_t(self, f, None), x)
        with torch.no_grad():
            return rt.to_nchw(self.nhwc(rt.to_nhwc(x, torch.float32)))
