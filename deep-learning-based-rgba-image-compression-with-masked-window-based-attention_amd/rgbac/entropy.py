"""compressai-compatible entropy models, forward on the HIP path.

The reference takes ``EntropyBottleneck``, ``GaussianConditional`` and
``CompressionModel`` from compressai (imports at
models/AutoEncoderRGB_Journal.py:4-6; version unpinned, the no-arg
``CompressionModel()`` implies >= 1.2).  compressai is not vendored and not
installed, so these classes re-create its parameter/buffer layout (so
checkpoints load unchanged) and its forward semantics, which run in
rgbac_eb_forward / rgbac_gaussian_slice.  The bitstream side (``update`` -> CDF tables,
``build_indexes`` / ``quantize`` / ``dequantize``, ``compress`` / ``decompress``) follows
compressai's EntropyModel API; the tables are built by rgbac.ans.pmf_to_quantized_cdf and
the strings by the host rANS coder (csrc/rans.cpp), byte-compatible with compressai.ans.
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
        self.entropy_coder_precision = 16

    # compressai EntropyModel properties
    @property
    def offset(self):
        return self._offset

    @property
    def quantized_cdf(self):
        return self._quantized_cdf

    @property
    def cdf_length(self):
        return self._cdf_length

    def _check_cdf(self):
        if self._offset.numel() == 0 or self._quantized_cdf.numel() == 0:
            raise ValueError("Uninitialized CDFs. Run update() first")

    def _pmf_to_cdf(self, pmf, tail_mass, pmf_length, max_length):
        """EntropyModel._pmf_to_cdf: per row, quantise [pmf[:len], tail] to a 16-bit CDF."""
        from .ans import pmf_to_quantized_cdf
        cdf = torch.zeros((len(pmf_length), max_length + 2), dtype=torch.int32)
        pmf, tail_mass, lens = pmf.detach().cpu(), tail_mass.detach().cpu(), pmf_length.tolist()
        for i, p in enumerate(pmf):
            prob = torch.cat((p[:lens[i]], tail_mass[i]), dim=0)
            c = pmf_to_quantized_cdf(prob, self.entropy_coder_precision)
            cdf[i, :len(c)] = torch.tensor(c, dtype=torch.int32)
        return cdf.to(pmf_length.device)

    def tables(self):
        """(cdfs, cdf_lengths, offsets) packed for the host coder (cached per update)."""
        from .ans import CdfTables
        self._check_cdf()
        bufs = (self._quantized_cdf, self._cdf_length, self._offset)
        vers = tuple(b._version for b in bufs)
        ent = self.__dict__.get("_rgbac_tables")      # holds the buffers: identity is safe
        if ent is None or any(a is not b for a, b in zip(ent[0], bufs)) or ent[1] != vers:
            ent = (bufs, vers, CdfTables(*bufs))
            self.__dict__["_rgbac_tables"] = ent
        return ent[2]

    def quantize(self, inputs, mode, means=None):
        """EntropyModel.quantize for mode "symbols" / "dequantize" (inference)."""
        if mode not in ("symbols", "dequantize"):
            raise ValueError(f'Invalid quantization mode: "{mode}"')
        outputs = inputs.clone() if means is None else inputs - means
        outputs = torch.round(outputs)
        if mode == "dequantize":
            return outputs if means is None else outputs + means
        return outputs.int()

    @staticmethod
    def dequantize(inputs, means=None, dtype=torch.float):
        outputs = inputs.type(dtype)
        return outputs if means is None else outputs + means

    def compress(self, inputs, indexes, means=None):
        """EntropyModel.compress: one string per batch element."""
        from .ans import RansEncoder
        symbols = self.quantize(inputs, "symbols", means)
        tab = self.tables()
        sym, idx = symbols.cpu(), indexes.int().cpu()
        return [RansEncoder().encode_with_indexes(sym[i].reshape(-1), idx[i].reshape(-1), tab)
                for i in range(symbols.size(0))]

    def decompress(self, strings, indexes, dtype=torch.float, means=None):
        from .ans import RansDecoder
        tab = self.tables()
        outputs = torch.empty(indexes.size(), dtype=torch.int32)
        idx = indexes.int().cpu()
        for i, s in enumerate(strings):
            dec = RansDecoder()
            dec.set_stream(s)
            outputs[i] = torch.from_numpy(dec.decode_stream_np(idx[i].reshape(-1), tab)).reshape(
                outputs[i].size())
        return self.dequantize(outputs.to(indexes.device), means, dtype)


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

    def update(self, force=False, update_quantiles=False):
        """EntropyBottleneck.update: per-channel 16-bit CDFs of the factorized density over
        [median - minima, median + maxima] (+ tail bin)."""
        if self._offset.numel() > 0 and not force:
            return False
        with torch.no_grad():
            q = self.quantiles.detach()
            medians = q[:, 0, 1]
            minima = torch.clamp(torch.ceil(medians - q[:, 0, 0]).int(), min=0)
            maxima = torch.clamp(torch.ceil(q[:, 0, 2] - medians).int(), min=0)
            self._offset = -minima
            pmf_start = medians - minima
            pmf_length = maxima + minima + 1
            max_length = int(pmf_length.max().item())
            samples = torch.arange(max_length, device=q.device)[None, :] + pmf_start[:, None, None]
            lower = self._logits_cumulative(samples - 0.5, stop_gradient=True)
            upper = self._logits_cumulative(samples + 0.5, stop_gradient=True)
            pmf = (torch.sigmoid(upper) - torch.sigmoid(lower))[:, 0, :]
            tail_mass = torch.sigmoid(lower[:, 0, :1]) + torch.sigmoid(-upper[:, 0, -1:])
            self._quantized_cdf = self._pmf_to_cdf(pmf, tail_mass, pmf_length, max_length)
            self._cdf_length = pmf_length + 2
        return True

    def _build_indexes(self, size):
        N, C = size[0], size[1]
        view = (1, -1) + (1,) * (len(size) - 2)
        return torch.arange(C, dtype=torch.int32).view(*view).expand(N, *size[1:]).int()

    def compress(self, x):
        """EntropyBottleneck.compress(x) -> one string per image (indexes = channel)."""
        self._check_cdf()
        med = self._get_medians().detach().reshape(1, -1, *([1] * (x.dim() - 2)))
        return super().compress(x, self._build_indexes(x.size()), med)

    def decompress(self, strings, size):
        self._check_cdf()
        out_size = (len(strings), self._quantized_cdf.size(0), *size)
        med = self._get_medians().detach().reshape(1, -1, *([1] * len(size)))
        idx = self._build_indexes(out_size).to(self._quantized_cdf.device)
        return super().decompress(strings, idx, med.dtype, med)

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
        self.scale_table = torch.Tensor(tuple(float(s) for s in scale_table)).to(
            self.scale_bound.device)
        self.update()
        return True

    def update(self):
        """GaussianConditional.update: one 16-bit CDF per scale_table entry, centred
        Gaussian pmf over +-ceil(scale * multiplier) (+ tail bin)."""
        from scipy.stats import norm
        multiplier = -float(norm.ppf(self.tail_mass / 2))      # _standardized_quantile
        with torch.no_grad():
            st = self.scale_table
            pmf_center = torch.ceil(st * multiplier).int()
            pmf_length = 2 * pmf_center + 1
            max_length = int(torch.max(pmf_length).item())
            samples = torch.abs(torch.arange(max_length, device=st.device).int() -
                                pmf_center[:, None]).float()
            samples_scale = st.unsqueeze(1).float()
            upper = _std_cumulative((0.5 - samples) / samples_scale)
            lower = _std_cumulative((-0.5 - samples) / samples_scale)
            pmf = upper - lower
            tail_mass = 2 * lower[:, :1]
            self._quantized_cdf = self._pmf_to_cdf(pmf, tail_mass, pmf_length, max_length)
            self._offset = -pmf_center
            self._cdf_length = pmf_length + 2

    def build_indexes(self, scales):
        """GaussianConditional.build_indexes (API surface; the model path runs it in
        rgbac_gauss_code)."""
        scales = torch.max(scales, self.lower_bound_scale.bound.to(scales.device))
        indexes = scales.new_full(scales.size(), len(self.scale_table) - 1).int()
        for s in self.scale_table[:-1]:
            indexes -= (scales <= s).int()
        return indexes


def _std_cumulative(t):
    # GaussianConditional._standardized_cumulative
    return 0.5 * torch.erfc(float(-(2 ** -0.5)) * t)


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
