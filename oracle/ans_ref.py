"""Bitstream oracle (compress / decompress) -- TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this module, as the checker of the bitstream path
(rgbac.ans / csrc/rans.cpp / csrc/code.hip).  Pure Python for the integer coder
(small cases only) and PyTorch-CPU fp32 for the model arithmetic.

Restates, from compressai's published algorithm (the reference imports it at
models/AutoEncoderRGB_Journal.py:4-5; compressai is neither vendored nor installed,
version unpinned, >= 1.2 implied by the no-arg CompressionModel()):
  * ``pmf_to_quantized_cdf``           compressai/cpp_exts/ops/ops.cpp
  * ``BufferedRansEncoder`` / ``RansDecoder``   compressai/cpp_exts/rans/rans_interface.cpp
    over ryg_rans rans64.h (64-bit state, 32-bit words, 16-bit precision, 4-bit bypass)
  * ``gc_update`` / ``eb_update``      GaussianConditional.update / EntropyBottleneck.update
  * ``gc_build_indexes``               GaussianConditional.build_indexes
  * ``rgb_compress`` / ``rgb_decompress``  models/AutoEncoderRGB_Journal.py:312-416

PARITY STATUS: parity unpinned (no compressai here, no reference fixtures; see
DESIGN.md §2).  Pinned by hand-derived known answers (tests/test_ans.py: the one-symbol
stream of a two-symbol uniform table, pmf tables whose quantisation is exact, the
zero-frequency steal rule) and by encode -> decode identity.
"""
import math

import torch

from . import ref_model as ref

PRECISION = 16
BYPASS_PRECISION = 4
MAX_BYPASS_VAL = (1 << BYPASS_PRECISION) - 1
RANS_L = 1 << 31
MASK32 = (1 << 32) - 1


def pmf_to_quantized_cdf(pmf, precision=PRECISION):
    """ops.cpp pmf_to_quantized_cdf (float32 products, std::round = half away from zero)."""
    one = 1 << precision
    f32 = torch.tensor(list(pmf), dtype=torch.float32)
    scaled = (f32 * float(one)).tolist()        # float32 products, exact as in C++
    cdf = [0] + [int(math.floor(abs(v) + 0.5)) * (1 if v >= 0 else -1) for v in scaled]
    total = sum(cdf)
    if total == 0:
        raise ValueError("pmf has no mass")
    cdf = [(one * v) // total for v in cdf]
    for i in range(1, len(cdf)):
        cdf[i] += cdf[i - 1]
    cdf[-1] = one
    n = len(cdf) - 1
    for i in range(n):
        if cdf[i] == cdf[i + 1]:
            best_freq, best_steal = None, -1
            for j in range(n):
                f = cdf[j + 1] - cdf[j]
                if f > 1 and (best_freq is None or f < best_freq):
                    best_freq, best_steal = f, j
            assert best_steal != -1
            if best_steal < i:
                for j in range(best_steal + 1, i + 1):
                    cdf[j] -= 1
            else:
                for j in range(i + 1, best_steal + 1):
                    cdf[j] += 1
    return cdf


class BufferedRansEncoder:
    def __init__(self):
        self.syms = []

    def encode_with_indexes(self, symbols, indexes, cdfs, cdf_lengths, offsets):
        for s, ci in zip(symbols, indexes):
            cdf = cdfs[ci]
            max_value = cdf_lengths[ci] - 2
            value = s - offsets[ci]
            raw_val = 0
            if value < 0:
                raw_val = -2 * value - 1
                value = max_value
            elif value >= max_value:
                raw_val = 2 * (value - max_value)
                value = max_value
            self.syms.append((cdf[value], cdf[value + 1] - cdf[value], False))
            if value == max_value:
                n_bypass = 0
                while (raw_val >> (n_bypass * BYPASS_PRECISION)) != 0:
                    n_bypass += 1
                val = n_bypass
                while val >= MAX_BYPASS_VAL:
                    self.syms.append((MAX_BYPASS_VAL, MAX_BYPASS_VAL + 1, True))
                    val -= MAX_BYPASS_VAL
                self.syms.append((val, val + 1, True))
                for j in range(n_bypass):
                    v = (raw_val >> (j * BYPASS_PRECISION)) & MAX_BYPASS_VAL
                    self.syms.append((v, v + 1, True))

    def flush(self):
        x = RANS_L
        words = []                       # emitted back to front
        for start, freq, bypass in reversed(self.syms):
            if not bypass:
                x_max = ((RANS_L >> PRECISION) << 32) * freq
                if x >= x_max:
                    words.append(x & MASK32)
                    x >>= 32
                x = ((x // freq) << PRECISION) + (x % freq) + start
            else:
                x_max = ((RANS_L >> 16) << 32) * (1 << (16 - BYPASS_PRECISION))
                if x >= x_max:
                    words.append(x & MASK32)
                    x >>= 32
                x = (x << BYPASS_PRECISION) | start
        words.append(x >> 32)
        words.append(x & MASK32)
        self.syms = []
        return b"".join(w.to_bytes(4, "little") for w in reversed(words))


class RansDecoder:
    def set_stream(self, data):
        self.words = [int.from_bytes(data[i:i + 4], "little") for i in range(0, len(data), 4)]
        self.x = self.words[0] | (self.words[1] << 32)
        self.pos = 2

    def _bits(self, n):
        v = self.x & ((1 << n) - 1)
        self.x >>= n
        if self.x < RANS_L:
            self.x = ((self.x << 32) | self.words[self.pos]) & ((1 << 64) - 1)
            self.pos += 1
        return v

    def decode_stream(self, indexes, cdfs, cdf_lengths, offsets):
        out = []
        for ci in indexes:
            cdf = cdfs[ci]
            size = cdf_lengths[ci]
            max_value = size - 2
            cum = self.x & ((1 << PRECISION) - 1)
            s = next(k for k in range(size) if cdf[k] > cum) - 1
            start, freq = cdf[s], cdf[s + 1] - cdf[s]
            x = freq * (self.x >> PRECISION) + (self.x & ((1 << PRECISION) - 1)) - start
            if x < RANS_L:
                x = (x << 32) | self.words[self.pos]
                self.pos += 1
            self.x = x
            value = s
            if value == max_value:
                val = self._bits(BYPASS_PRECISION)
                n_bypass = val
                while val == MAX_BYPASS_VAL:
                    val = self._bits(BYPASS_PRECISION)
                    n_bypass += val
                raw_val = 0
                for j in range(n_bypass):
                    raw_val |= self._bits(BYPASS_PRECISION) << (j * BYPASS_PRECISION)
                value = raw_val >> 1
                value = -value - 1 if raw_val & 1 else value + max_value
            out.append(value + offsets[ci])
        return out


# ---------------------------------------------------------------- entropy-model tables
def _pmf_to_cdf(pmf, tail_mass, pmf_length, max_length):
    """EntropyModel._pmf_to_cdf -> int32 (n, max_length + 2)."""
    cdf = torch.zeros((len(pmf_length), max_length + 2), dtype=torch.int32)
    for i, p in enumerate(pmf):
        prob = torch.cat((p[:pmf_length[i]], tail_mass[i]), dim=0)
        c = pmf_to_quantized_cdf(prob.tolist())
        cdf[i, :len(c)] = torch.tensor(c, dtype=torch.int32)
    return cdf


def standardized_quantile(q):
    """scipy.stats.norm.ppf(q) (GaussianConditional._standardized_quantile)."""
    from scipy.stats import norm
    return float(norm.ppf(q))


def gc_update(scale_table, tail_mass=1e-9):
    """GaussianConditional.update -> (quantized_cdf, cdf_length, offset)."""
    multiplier = -standardized_quantile(tail_mass / 2)
    pmf_center = torch.ceil(scale_table * multiplier).int()
    pmf_length = 2 * pmf_center + 1
    max_length = int(torch.max(pmf_length).item())
    samples = torch.abs(torch.arange(max_length).int() - pmf_center[:, None]).float()
    samples_scale = scale_table.unsqueeze(1).float()
    upper = ref._std_cumulative((0.5 - samples) / samples_scale)
    lower = ref._std_cumulative((-0.5 - samples) / samples_scale)
    pmf = upper - lower
    tail = 2 * lower[:, :1]
    cdf = _pmf_to_cdf(pmf, tail, pmf_length, max_length)
    return cdf, (pmf_length + 2).int(), (-pmf_center).int()


def eb_update(sd, p="entropy_bottleneck"):
    """EntropyBottleneck.update -> (quantized_cdf, cdf_length, offset)."""
    q = sd[p + ".quantiles"].detach()
    medians = q[:, 0, 1]
    minima = torch.clamp(torch.ceil(medians - q[:, 0, 0]).int(), min=0)
    maxima = torch.clamp(torch.ceil(q[:, 0, 2] - medians).int(), min=0)
    pmf_start = medians - minima
    pmf_length = maxima + minima + 1
    max_length = int(pmf_length.max().item())
    samples = torch.arange(max_length)[None, :] + pmf_start[:, None, None]
    with torch.no_grad():
        lower = ref.eb_logits_cumulative(sd, p, samples - 0.5, stop_gradient=True)
        upper = ref.eb_logits_cumulative(sd, p, samples + 0.5, stop_gradient=True)
    pmf = (torch.sigmoid(upper) - torch.sigmoid(lower))[:, 0, :]
    tail = torch.sigmoid(lower[:, 0, :1]) + torch.sigmoid(-upper[:, 0, -1:])
    cdf = _pmf_to_cdf(pmf, tail, pmf_length, max_length)
    return cdf, (pmf_length + 2).int(), (-minima).int()


def gc_build_indexes(scales, scale_table, bound=0.11):
    s = torch.max(scales, torch.tensor(bound, dtype=torch.float32))
    idx = torch.full(s.shape, len(scale_table) - 1, dtype=torch.int32)
    for t in scale_table[:-1]:
        idx -= (s <= t).int()
    return idx


# ---------------------------------------------------------------- model-level flow
def rgb_compress_symbols(sd, inp, mask, scale_table):
    """AutoEncoderRGB_Journal.py:312-371 up to the coder: returns (z_sym (B,192,h,w) int,
    per-slice y symbols / indexes lists (NCHW order), y_hat (B,80,H,W))."""
    me = ref.supply_mask(mask)
    y = ref.analysis(inp, sd, "Encoder", me[1], me[2])
    z = ref._h_a(y, sd)
    med = ref.eb_medians(sd, "entropy_bottleneck").reshape(1, -1, 1, 1)
    z_sym = torch.round(z - med).int()
    z_hat = z_sym.float() + med
    scales = ref._hyper_s(z_hat, sd, "h_scale_s")
    means = ref._hyper_s(z_hat, sd, "h_mean_s")
    H, W = y.shape[2:]
    hats, syms, idxs = [], [], []
    for i, ysl in enumerate(y.chunk(10, 1)):
        sup = hats[:5]
        ms = torch.cat([means] + sup, dim=1)
        mu = ref._stack3(ms, sd, f"cc_mean_transforms.{i}")[:, :, :H, :W]
        sc = ref._stack3(torch.cat([scales] + sup, dim=1), sd,
                         f"cc_scale_transforms.{i}")[:, :, :H, :W]
        idx = gc_build_indexes(sc, scale_table)
        q = torch.round(ysl - mu)
        syms.append(q.int())
        idxs.append(idx)
        yh = q + mu
        lrp = ref._stack3(torch.cat([ms, yh], dim=1), sd, f"lrp_transforms.{i}")
        hats.append(yh + 0.5 * torch.tanh(lrp))
    return z_sym, syms, idxs, torch.cat(hats, dim=1)
