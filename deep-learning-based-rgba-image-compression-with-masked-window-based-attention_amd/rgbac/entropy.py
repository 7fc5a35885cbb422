"""compressai-compatible entropy models, forward on the HIP path.

The reference takes ``EntropyBottleneck``, ``GaussianConditional`` and
``CompressionModel`` from compressai (imports at
models/AutoEncoderRGB_Journal.py:4-6; version unpinned, the no-arg
``CompressionModel()`` implies >= 1.2).  compressai is not vendored and not
installed, so these classes re-create its parameter/buffer layout (so
checkpoints load unchanged) and its forward semantics, which run in
rgbac_eb_forward / rgbac_gaussian_slice.  The rANS bitstream path
(compress/decompress) is out of scope for this round.
"""
import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from . import runtime as rt


class LowerBound(nn.Module):
    """compressai.ops.LowerBound: a buffer ``bound`` (state_dict key ``*.bound``)."""

    def __init__(self, bound):
        super().__init__()
        self.register_buffer("bound", torch.Tensor([float(bound)]))

    def forward(self, x):
        return torch.max(x, self.bound)


class _EntropyModel(nn.Module):
    def __init__(self, likelihood_bound=1e-9):
        super().__init__()
        self.use_likelihood_bound = likelihood_bound > 0
        if self.use_likelihood_bound:
            self.likelihood_lower_bound = LowerBound(likelihood_bound)
        self.register_buffer("_offset", torch.IntTensor())
        self.register_buffer("_quantized_cdf", torch.IntTensor())
        self.register_buffer("_cdf_length", torch.IntTensor())


class EntropyBottleneck(_EntropyModel):
    """Factorized prior (Ballé 2018), filters (3,3,3,3), compressai layout."""

    def __init__(self, channels, tail_mass=1e-9, init_scale=10, filters=(3, 3, 3, 3)):
        super().__init__()
        self.channels = int(channels)
        self.filters = tuple(int(f) for f in filters)
        self.init_scale = float(init_scale)
        self.tail_mass = float(tail_mass)
        f = (1,) + self.filters + (1,)
        scale = self.init_scale ** (1 / (len(self.filters) + 1))
        for i in range(len(self.filters) + 1):
            init = np.log(np.expm1(1 / scale / f[i + 1]))
            m = torch.Tensor(channels, f[i + 1], f[i]).fill_(init)
            self.register_parameter(f"_matrix{i:d}", nn.Parameter(m))
            b = torch.Tensor(channels, f[i + 1], 1)
            nn.init.uniform_(b, -0.5, 0.5)
            self.register_parameter(f"_bias{i:d}", nn.Parameter(b))
            if i < len(self.filters):
                fac = torch.zeros(channels, f[i + 1], 1)
                self.register_parameter(f"_factor{i:d}", nn.Parameter(fac))
        self.quantiles = nn.Parameter(
            torch.Tensor([-self.init_scale, 0, self.init_scale]).repeat(channels, 1, 1))
        target = np.log(2 / self.tail_mass - 1)
        self.register_buffer("target", torch.Tensor([-target, 0, target]))

    def _get_medians(self):
        return self.quantiles[:, :, 1:2]

    def packed_params(self):
        """[C][64] fp32 block consumed by rgbac_eb_forward (see csrc/entropy.hip)."""
        C = self.channels
        parts = [F.softplus(getattr(self, f"_matrix{i}").detach().float()).reshape(C, -1)
                 for i in range(5)]
        parts += [getattr(self, f"_bias{i}").detach().float().reshape(C, -1) for i in range(5)]
        parts += [torch.tanh(getattr(self, f"_factor{i}").detach().float()).reshape(C, -1)
                  for i in range(4)]
        parts.append(self._get_medians().detach().float().reshape(C, 1))
        p = torch.cat(parts, dim=1)
        assert p.shape[1] == 59
        return F.pad(p, (0, 64 - 59)).contiguous()

    def packed_params_cached(self):
        ps = [getattr(self, n) for n in sorted(self._parameters)]
        key = (rt.PARAM_GEN,) + tuple((q._version, q.data_ptr()) for q in ps)
        ent = self.__dict__.get("_rgbac_eb")
        if ent is None or ent[0] != key:
            with torch.no_grad():
                self.__dict__["_rgbac_eb"] = (key, self.packed_params())
            ent = self.__dict__["_rgbac_eb"]
        return ent[1]

    def _logits_cumulative(self, inputs, stop_gradient):
        logits = inputs
        for i in range(len(self.filters) + 1):
            m = getattr(self, f"_matrix{i}")
            b = getattr(self, f"_bias{i}")
            if stop_gradient:
                m, b = m.detach(), b.detach()
            logits = torch.matmul(F.softplus(m), logits) + b
            if i < len(self.filters):
                fac = getattr(self, f"_factor{i}")
                if stop_gradient:
                    fac = fac.detach()
                logits = logits + torch.tanh(fac) * torch.tanh(logits)
        return logits

    def loss(self):
        """Auxiliary quantile loss (compressai EntropyBottleneck.loss); tiny, host-side torch."""
        logits = self._logits_cumulative(self.quantiles, stop_gradient=True)
        return torch.abs(logits - self.target).sum()


class GaussianConditional(_EntropyModel):
    """compressai GaussianConditional(scale_table=None, scale_bound=0.11) layout."""

    def __init__(self, scale_table, scale_bound=0.11, tail_mass=1e-9):
        super().__init__()
        if scale_table is not None and not isinstance(scale_table, (list, tuple)):
            raise ValueError(f'Invalid type for scale_table "{type(scale_table)}"')
        self.tail_mass = float(tail_mass)
        if scale_bound is None and scale_table:
            scale_bound = scale_table[0]
        if scale_bound <= 0:
            raise ValueError("Invalid parameters")
        self.lower_bound_scale = LowerBound(scale_bound)
        self.register_buffer("scale_table",
                             torch.Tensor(tuple(float(s) for s in scale_table))
                             if scale_table else torch.Tensor())
        self.register_buffer("scale_bound", torch.Tensor([float(scale_bound)]))

    def update_scale_table(self, scale_table, force=False):
        if self._offset.numel() > 0 and not force:
            return False
        self.scale_table = torch.as_tensor(scale_table, dtype=torch.float32,
                                           device=self.scale_bound.device)
        return True


# ---------------------------------------------------------------- HIP calls
def eb_forward_hip(eb, z, z_hat, params, noise, partial, lik=None):
    """z, z_hat: Feat; params: packed_params(); partial: fp64 scratch."""
    npix = z.B * z.H * z.W
    rt.timed("eb_forward_kernel", 0.0, 2.0 * npix * z.C * z.t.element_size(),
              lambda: _lib.call("rgbac_eb_forward", _lib.dtype_code(z.t.dtype), npix, z.C,
                                z.ptr(), z.ldc, params.data_ptr(), _lib.ptr(noise), z_hat.ptr(),
                                z_hat.ldc, _lib.ptr(lik), partial.data_ptr(),
                                _lib.stream_ptr(z.t.device)))


def gaussian_slice_hip(y, ycoff, nch, mu, sc, hat, noise, partial, lik=None):
    """One slice of GaussianConditional.forward + ste_round, all Feats (NHWC)."""
    npix = y.B * y.H * y.W
    rt.timed("gaussian_slice_kernel", 0.0, 4.0 * npix * nch * y.t.element_size(),
              lambda: _lib.call("rgbac_gaussian_slice", _lib.dtype_code(y.t.dtype), npix, nch,
                                y.ptr(ycoff), y.ldc, mu.ptr(), mu.ldc, sc.ptr(), sc.ldc,
                                _lib.ptr(noise), hat.ptr(), hat.ldc, _lib.ptr(lik),
                                partial.data_ptr(), _lib.stream_ptr(y.t.device)))


def reduce_blocks(n):
    return _lib.load().rgbac_reduce_blocks(int(n))
