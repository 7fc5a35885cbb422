"""compressai.ans / compressai._CXX surface over the host rANS coder of librgbac_hip.so.

The reference imports ``BufferedRansEncoder`` and ``RansDecoder`` from compressai.ans
(models/AutoEncoderRGB_Journal.py:5, AutoEncoderMask_Journal.py:6) and uses them at
AutoEncoderRGB_Journal.py:334,367-368 (encode) and :387-388,401 (decode); compressai's
entropy models use ``RansEncoder.encode_with_indexes`` / ``RansDecoder.decode_with_indexes``
and ``_CXX.pmf_to_quantized_cdf``.  Same class / method names and argument meaning; the
coder itself is csrc/rans.cpp (C ABI in include/rgbac.h), byte-compatible with compressai's.
Arguments may be Python lists (as the reference passes them) or numpy / torch int tensors.
"""
import ctypes

import numpy as np
import torch

from . import _lib


def _i32(x):
    if isinstance(x, torch.Tensor):
        x = x.detach().cpu().numpy()
    return np.ascontiguousarray(np.asarray(x, dtype=np.int32).reshape(-1))


class CdfTables:
    """(cdfs, cdf_lengths, offsets) packed once for the C ABI: cdfs as [ncdf][stride] int32."""

    def __init__(self, cdfs, cdf_lengths, offsets):
        if isinstance(cdfs, torch.Tensor):
            tab = cdfs.detach().cpu().numpy().astype(np.int32)
        elif isinstance(cdfs, np.ndarray):
            tab = cdfs.astype(np.int32)
        else:
            rows = [list(r) for r in cdfs]
            width = max(len(r) for r in rows)
            tab = np.zeros((len(rows), width), dtype=np.int32)
            for i, r in enumerate(rows):
                tab[i, :len(r)] = r
        self.cdfs = np.ascontiguousarray(tab.reshape(tab.shape[0], -1))
        self.sizes = _i32(cdf_lengths)
        self.offsets = _i32(offsets)
        n = self.cdfs.shape[0]
        if self.sizes.size != n or self.offsets.size != n:
            raise ValueError("cdfs, cdf_lengths and offsets disagree on the number of tables")

    @classmethod
    def of(cls, cdfs, cdf_lengths=None, offsets=None):
        return cdfs if isinstance(cdfs, CdfTables) else cls(cdfs, cdf_lengths, offsets)

    def args(self):
        return (self.cdfs.ctypes.data, int(self.cdfs.shape[1]), self.sizes.ctypes.data,
                self.offsets.ctypes.data, int(self.cdfs.shape[0]))


def pmf_to_quantized_cdf(pmf, precision=16):
    """compressai._CXX.pmf_to_quantized_cdf -> list of len(pmf)+1 ints."""
    p = np.ascontiguousarray(np.asarray(
        pmf.detach().cpu() if isinstance(pmf, torch.Tensor) else pmf, dtype=np.float32).reshape(-1))
    out = np.zeros(p.size + 1, dtype=np.uint32)
    _lib.call("rgbac_pmf_to_quantized_cdf", p.ctypes.data, int(p.size), int(precision),
              out.ctypes.data)
    return out.astype(np.int64).tolist()


class BufferedRansEncoder:
    """Buffers (symbol, table) records across encode_with_indexes calls; flush() -> bytes."""

    def __init__(self):
        lib = _lib.load()
        self._h = ctypes.c_void_p()
        _lib.call("rgbac_rans_encoder_create", ctypes.byref(self._h))
        self._destroy = lib.rgbac_rans_encoder_destroy

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._destroy(h)
            self._h = None

    def encode_with_indexes(self, symbols, indexes, cdfs, cdf_lengths=None, offsets=None):
        s, i = _i32(symbols), _i32(indexes)
        if s.size != i.size:
            raise ValueError("symbols and indexes differ in length")
        tab = CdfTables.of(cdfs, cdf_lengths, offsets)
        _lib.call("rgbac_rans_encoder_put", self._h, s.ctypes.data, i.ctypes.data, int(s.size),
                  *tab.args())

    def flush(self):
        cap = int(_lib.load().rgbac_rans_encoder_bound(self._h))
        buf = np.empty(max(cap, 8), dtype=np.uint8)
        nb = ctypes.c_int64(0)
        _lib.call("rgbac_rans_encoder_flush", self._h, buf.ctypes.data, int(buf.size),
                  ctypes.byref(nb))
        return buf[:nb.value].tobytes()


class RansEncoder:
    """One-shot encoder: encode_with_indexes(...) -> bytes."""

    def encode_with_indexes(self, symbols, indexes, cdfs, cdf_lengths=None, offsets=None):
        enc = BufferedRansEncoder()
        enc.encode_with_indexes(symbols, indexes, cdfs, cdf_lengths, offsets)
        return enc.flush()


class RansDecoder:
    """set_stream(bytes) + decode_stream(indexes, ...) (stateful, across slices), or the
    one-shot decode_with_indexes(bytes, indexes, ...).  Returns a list of ints, like compressai;
    ``decode_stream_np`` returns the int32 array without the list conversion."""

    def __init__(self):
        _lib.load()
        self._st = _lib.RansDecoderState()
        self._buf = None

    def set_stream(self, encoded):
        self._buf = np.frombuffer(bytes(encoded), dtype=np.uint8).copy()
        _lib.call("rgbac_rans_decoder_init", ctypes.byref(self._st), self._buf.ctypes.data,
                  int(self._buf.size))

    def decode_stream_np(self, indexes, cdfs, cdf_lengths=None, offsets=None):
        if self._buf is None:
            raise RuntimeError("RansDecoder: set_stream() first")
        i = _i32(indexes)
        out = np.empty(i.size, dtype=np.int32)
        tab = CdfTables.of(cdfs, cdf_lengths, offsets)
        _lib.call("rgbac_rans_decode", ctypes.byref(self._st), i.ctypes.data, int(i.size),
                  *tab.args(), out.ctypes.data)
        return out

    def decode_stream(self, indexes, cdfs, cdf_lengths=None, offsets=None):
        return self.decode_stream_np(indexes, cdfs, cdf_lengths, offsets).tolist()

    def decode_with_indexes(self, encoded, indexes, cdfs, cdf_lengths=None, offsets=None):
        self.set_stream(encoded)
        return self.decode_stream(indexes, cdfs, cdf_lengths, offsets)
