"""NHWC executor over the C ABI: feature maps, weight packing, op wrappers.

Data layout in HBM:
  * activations: NHWC, one tensor per feature map, channel stride ``ldc`` =
    round_up(C, 8) (16-byte rows for bf16), padding channels zero;
  * conv weights: packed once per parameter version into
    [nphase][cout_pad][k_pad] with k = tap * cin_pad + cin (K contiguous),
    cout_pad / k_pad zero-padded to the kernel's tile multiples;
  * bias: fp32 [cout_pad].
torch is used here only for device allocation and the (cached) weight
repack; every arithmetic op of the forward runs in librgbac_hip.so.
"""
import math

import torch

from . import _lib
from ._lib import ACT, CONV, CONVT_S2, SUBPEL2


# Optional launch profiler (bench.py's roofline attribution): when set to a
# LaunchProfiler, every launch made through ``launch`` is bracketed by HIP events
# recorded on the launching stream, together with its algorithmic FLOPs/bytes.
PROFILER = None


class LaunchProfiler:
    def __init__(self):
        self.records = []   # (kernel name, flops, bytes, start event, end event)

    def wrap(self, name, flops, nbytes, fn):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        self.records.append((name, flops, nbytes, s, e))

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for name, fl, nb, s, e in self.records:
            d = out.setdefault(name, {"launches": 0, "ms": 0.0, "flops": 0.0, "bytes": 0.0})
            d["launches"] += 1
            d["ms"] += s.elapsed_time(e)
            d["flops"] += fl
            d["bytes"] += nb
        return out


def launch(name, flops, nbytes, fn):
    if PROFILER is None:
        fn()
    else:
        PROFILER.wrap(name, flops, nbytes, fn)


def round_up(x, m):
    return (x + m - 1) // m * m


def pick_cout_pad(cout):
    """Smallest padded row count, preferring the widest N tile (64/32/16)."""
    r16, r32, r64 = round_up(cout, 16), round_up(cout, 32), round_up(cout, 64)
    if r64 == r16:
        return r64
    if r32 == r16:
        return r32
    return r16


class Feat:
    """NHWC feature map: tensor ``t`` of shape (B, H, W, ldc) holding C real channels."""
    __slots__ = ("t", "C")

    def __init__(self, t, C):
        self.t = t
        self.C = C

    @property
    def B(self):
        return self.t.shape[0]

    @property
    def H(self):
        return self.t.shape[1]

    @property
    def W(self):
        return self.t.shape[2]

    @property
    def ldc(self):
        return self.t.shape[3]

    def ptr(self, coff=0):
        return self.t.data_ptr() + coff * self.t.element_size()

    def src(self, coff=0, nch=None):
        """A channel slice usable as a conv source: (feat, coff, padded nch)."""
        if nch is None:
            nch = self.ldc - coff
        return (self, coff, nch)


def new_feat(B, H, W, C, dtype, device, zero=None):
    ldc = round_up(C, 8)
    if zero is None:
        zero = ldc != C
    alloc = torch.zeros if zero else torch.empty
    return Feat(alloc((B, H, W, ldc), dtype=dtype, device=device), C)


def to_nhwc(x, dtype, ldc=None):
    """fp32 NCHW (B,C,H,W) -> Feat."""
    assert x.is_cuda, "rgbac runs on the GPU only"
    x = x.contiguous().float()
    B, C, H, W = x.shape
    f = Feat(torch.empty((B, H, W, ldc or round_up(C, 8)), dtype=dtype, device=x.device), C)
    _lib.call("rgbac_nchw_to_nhwc", _lib.dtype_code(dtype), B, C, H, W, x.data_ptr(),
              f.t.data_ptr(), f.ldc, _lib.stream_ptr(x.device))
    return f


def to_nchw(f):
    out = torch.empty((f.B, f.C, f.H, f.W), dtype=torch.float32, device=f.t.device)
    _lib.call("rgbac_nhwc_to_nchw", _lib.dtype_code(f.t.dtype), f.B, f.C, f.H, f.W,
              f.t.data_ptr(), f.ldc, out.data_ptr(), _lib.stream_ptr(f.t.device))
    return out


# --------------------------------------------------------------------------
# weight packing (cached per parameter version)
# --------------------------------------------------------------------------
def _seg_index(segs, device):
    """Map real input channel j -> padded K column, for sources [(real, padded), ...]."""
    idx, off = [], 0
    for real, padded in segs:
        idx.append(torch.arange(real, device=device) + off)
        off += padded
    return torch.cat(idx), off


class PackedConv:
    """A conv/convT/subpel layer repacked for rgbac_conv2d."""

    def __init__(self, weight, bias, mode, segs, dtype, ksize=None, stride=1, transposed=False):
        dev = weight.device
        w = weight.detach().float()
        idx, cin_pad = _seg_index(segs, dev)
        if transposed and mode == CONV:
            # ConvTranspose2d(k=1, s=1, p=0): a 1x1 conv with W^T
            w = w.transpose(0, 1)
        if mode == CONVT_S2:
            cin, cout, k, _ = w.shape
            assert k == 5 and stride == 2
            phases = []
            for py in (0, 1):
                for px in (0, 1):
                    ky = torch.arange(py, 5, 2, device=dev)
                    kx = torch.arange(px, 5, 2, device=dev)
                    sub = w.index_select(2, ky).index_select(3, kx)       # Cin,Cout,ty,tx
                    phases.append(sub.permute(1, 2, 3, 0).reshape(cout, -1, cin))
            ntaps_max = 9
        else:
            cout, cin, k, _ = w.shape
            phases = [w.permute(0, 2, 3, 1).reshape(cout, k * k, cin)]
            ntaps_max = k * k
        assert cin == idx.numel(), (cin, segs)
        self.mode, self.ksize, self.stride = mode, k, stride
        self.cin, self.cin_pad, self.cout = cin, cin_pad, cout
        self.cout_pad = pick_cout_pad(cout)
        self.k_pad = round_up(ntaps_max * cin_pad, 64)
        wp = torch.zeros((len(phases), self.cout_pad, self.k_pad), device=dev)
        for ph, t in enumerate(phases):
            nt = t.shape[1]
            full = torch.zeros((cout, nt, cin_pad), device=dev)
            full[:, :, idx] = t
            wp[ph, :cout, :nt * cin_pad] = full.reshape(cout, nt * cin_pad)
        self.w = wp.to(dtype).contiguous()
        self.bias = torch.zeros(self.cout_pad, device=dev)
        if bias is not None:
            self.bias[:cout] = bias.detach().float()
        self.segs = list(segs)


def conv(pk, srcs, out=None, out_coff=0, act="none", act_param=0.0, res0=None, res1=None,
         res2=None, sel=None, square=False, bias=True):
    """Run a PackedConv over concatenated sources [(Feat, coff, nch), ...] -> Feat."""
    f0 = srcs[0][0]
    B, H, W = f0.B, f0.H, f0.W
    dtype = f0.t.dtype
    if pk.mode == CONV:
        pad = pk.ksize // 2
        Ho = (H + 2 * pad - pk.ksize) // pk.stride + 1
        Wo = (W + 2 * pad - pk.ksize) // pk.stride + 1
        cstore = pk.cout
    elif pk.mode == CONVT_S2:
        Ho, Wo, cstore = 2 * H, 2 * W, pk.cout
    else:
        Ho, Wo, cstore = 2 * H, 2 * W, pk.cout // 4
    if out is None:
        out = new_feat(B, Ho, Wo, cstore, dtype, f0.t.device)
    a = _lib.ConvArgs()
    a.dtype = _lib.dtype_code(dtype)
    a.mode = pk.mode
    a.batch, a.in_h, a.in_w = B, H, W
    a.ksize, a.stride = pk.ksize, pk.stride
    srcs = [s for s in srcs if s[2] > 0]
    a.nsrc = len(srcs)
    for i, (f, coff, nch) in enumerate(srcs):
        assert f.B == B and f.H == H and f.W == W and f.t.dtype == dtype
        a.src[i].ptr = f.ptr(coff)
        a.src[i].ldc = f.ldc
        a.src[i].channels = nch
    assert sum(s[2] for s in srcs) == pk.cin_pad, (sum(s[2] for s in srcs), pk.cin_pad)
    a.cin_pad, a.k_pad = pk.cin_pad, pk.k_pad
    a.weight = pk.w.data_ptr()
    a.bias = pk.bias.data_ptr() if bias else None
    a.cout, a.cout_pad = pk.cout, pk.cout_pad
    a.out_h, a.out_w = Ho, Wo
    a.out = out.ptr()
    a.out_ldc = out.ldc
    a.out_coff = out_coff
    a.act = ACT[act]
    a.act_param = act_param
    a.square_input = 1 if square else 0
    for name, r in (("res0", res0), ("res1", res1), ("res2", res2)):
        if r is not None:
            assert r.H == Ho and r.W == Wo and r.t.dtype == dtype
            setattr(a, name, r.ptr())
            setattr(a, name + "_ldc", r.ldc)
    a.sel = None if sel is None else sel.data_ptr()
    if PROFILER is None:
        _lib.call("rgbac_conv2d", a, _lib.stream_ptr(f0.t.device))
    else:
        taps = 25 if pk.mode == CONVT_S2 else pk.ksize * pk.ksize
        mgrid = B * (H * W if pk.mode != CONV else Ho * Wo)
        flops = 2.0 * mgrid * pk.cout * pk.cin * taps
        es = f0.t.element_size()
        nbytes = es * (B * H * W * pk.cin + B * Ho * Wo * cstore) + pk.w.numel() * es
        wn = 4 if pk.cout_pad % 64 == 0 else (2 if pk.cout_pad % 32 == 0 else 1)
        name = f"conv_kernel<{'f32' if dtype == torch.float32 else 'bf16'},{wn}>"
        PROFILER.wrap(name, flops, nbytes,
                      lambda: _lib.call("rgbac_conv2d", a, _lib.stream_ptr(f0.t.device)))
    return out


def feat_srcs(f):
    return [(f, 0, f.ldc)]


def packed(m, dtype, segs, mode=CONV, transposed=False, weight=None, bias=None):
    """PackedConv for module ``m`` (Conv2d / ConvTranspose2d / Linear), cached on the
    module and rebuilt when a parameter's version or storage changes."""
    w = m.weight if weight is None else weight
    b = getattr(m, "bias", None) if bias is None else bias
    key = (dtype, tuple(segs), mode, transposed)
    ver = (w._version, w.data_ptr(), None if b is None else (b._version, b.data_ptr()))
    cache = m.__dict__.setdefault("_rgbac_pack", {})
    ent = cache.get(key)
    if ent is None or ent[0] != ver:
        ww = w if w.dim() == 4 else w.reshape(w.shape[0], w.shape[1], 1, 1)
        stride = m.stride[0] if hasattr(m, "stride") else 1
        cache[key] = (ver, PackedConv(ww, b, mode, segs, dtype, stride=stride,
                                      transposed=transposed))
    return cache[key][1]


def segs_of(*srcs):
    """(real, padded) channel segments of conv sources [(Feat, coff, nch), ...]."""
    out = []
    for f, coff, nch in srcs:
        if nch <= 0:
            continue
        real = min(nch, f.C - coff) if coff < f.C else 0
        out.append((real, nch))
    return out


def check_gpu(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("rgbac: this module runs on the GPU (HIP) only; got a CPU tensor. "
                               "There is no CPU fallback in the product path.")
