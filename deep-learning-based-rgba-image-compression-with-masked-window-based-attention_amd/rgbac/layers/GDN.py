"""GDN / IGDN (reference: layers/GDN.py:9-94) on the MFMA conv engine.

The norm pool ``conv2d(x**2, gamma', beta')`` is a 1x1 GEMM over channels; it
runs through rgbac_conv2d with ``square_input`` (x**2 formed while staging the
B tile) and the GDN/IGDN epilogue ``x / sqrt(norm)`` / ``x * sqrt(norm)``
reading x at the same pixel, so a GDN costs one read of x, one write of y.
"""
import torch
import torch.nn as nn
from torch.autograd import Function

from .. import runtime as rt


class LowerBound(Function):
    """GDN.py:9-23: max(x, bound) with gradient passed where x >= bound or grad < 0."""

    @staticmethod
    def forward(ctx, inputs, bound):
        b = torch.ones_like(inputs) * bound
        ctx.save_for_backward(inputs, b)
        return torch.max(inputs, b)

    @staticmethod
    def backward(ctx, grad_output):
        inputs, b = ctx.saved_tensors
        pass_through = (inputs >= b) | (grad_output < 0)
        return pass_through.type(grad_output.dtype) * grad_output, None


class GDN(nn.Module):
    """y[i] = x[i] / sqrt(beta[i] + sum_j gamma[i, j] * x[j]^2)   (inverse: * sqrt)."""

    def __init__(self, ch, inverse=False, beta_min=1e-6, gamma_init=0.1,
                 reparam_offset=2 ** -18):
        super().__init__()
        self.inverse = inverse
        self.beta_min = beta_min
        self.gamma_init = gamma_init
        self.reparam_offset = reparam_offset
        self.build(ch)

    def build(self, ch):
        self.pedestal = self.reparam_offset ** 2
        self.beta_bound = (self.beta_min + self.reparam_offset ** 2) ** 0.5
        self.gamma_bound = self.reparam_offset
        self.beta = nn.Parameter(torch.sqrt(torch.ones(ch) + self.pedestal))
        g = self.gamma_init * torch.eye(ch) + self.pedestal
        self.gamma = nn.Parameter(torch.sqrt(g))

    def effective_params(self):
        """Reparametrised (beta', gamma') exactly as GDN.py:71-78 computes them (fp32): on the
        GPU one HIP launch each way (rgbac.autograd.GdnReparamFn, bit-identical to the torch
        graph below, which CPU tensors keep)."""
        if self.beta.is_cuda and self.gamma.is_cuda:
            from ..autograd import GdnReparamFn
            return GdnReparamFn.apply(self.beta, self.gamma, self.beta_bound, self.gamma_bound,
                                      self.pedestal)
        beta = LowerBound.apply(self.beta, self.beta_bound) ** 2 - self.pedestal
        gamma = LowerBound.apply(self.gamma, self.gamma_bound) ** 2 - self.pedestal
        return beta, gamma

    def _pack(self, dtype, C):
        key = (dtype, rt.PARAM_GEN, self.beta._version, self.gamma._version, self.beta.data_ptr(),
               self.gamma.data_ptr())
        ent = self.__dict__.get("_rgbac_gdn")
        if ent is None or ent[0] != key:
            with torch.no_grad():
                beta, gamma = self.effective_params()
            pk = rt.PackedConv(gamma.reshape(C, C, 1, 1), beta, rt.CONV, [(C, rt.round_up(C, 8))],
                               dtype)
            self.__dict__["_rgbac_gdn"] = (key, pk)
            ent = self.__dict__["_rgbac_gdn"]
        return ent[1]

    def nhwc(self, x, out=None):
        pk = self._pack(x.t.dtype, x.C)
        return rt.conv(pk, [x.src()], out=out, square=True,
                       act="igdn" if self.inverse else "gdn", res1=x)

    def forward(self, inputs):
        rt.check_gpu(inputs)
        shape = inputs.shape
        if inputs.dim() == 5:
            bs, ch, d, w, h = shape
            inputs = inputs.reshape(bs, ch, d * w, h)
        from .masked_win_attention import needs_grad
        if needs_grad(self, inputs):
            # differentiable like GDN.py:64-94 (LowerBound rule on beta/gamma included)
            from ..train_forward import gdn_t, layer_t
            return layer_t(lambda f: gdn_t(self, f), inputs).reshape(shape)
        with torch.no_grad():
            y = rt.to_nchw(self.nhwc(rt.to_nhwc(inputs, torch.float32)))
        return y.reshape(shape)
