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
import contextlib
import ctypes
import json
import os

import torch

from . import _lib
from ._lib import ACT, CONV, CONVT_S2, SUBPEL2


# Optional launch profiler (bench.py's roofline attribution): when set to a
# LaunchProfiler, every launch made through ``launch`` is bracketed by HIP events
# recorded on the launching stream, together with its algorithmic FLOPs/bytes.
PROFILER = None

# Bumped by rgbac.optim after every in-place parameter update it makes through raw
# pointers (no autograd version bump): part of every cached weight-pack key.
PARAM_GEN = 0


class _Timer:
    """A fence-free HIP event (rgbac_timer_*): recording it does not write back / invalidate
    the caches, and on a capturing stream it becomes an event node of the HIP graph."""
    __slots__ = ("h",)

    def __init__(self):
        h = ctypes.c_void_p()
        _lib.call("rgbac_timer_create", ctypes.byref(h))
        self.h = h

    def record(self):
        _lib.call("rgbac_timer_record", self.h, _lib.stream_ptr())

    def elapsed_ms(self, end):
        ms = ctypes.c_float()
        _lib.call("rgbac_timer_elapsed_ms", self.h, end.h, ctypes.byref(ms))
        return ms.value

    def __del__(self):
        try:
            _lib.load().rgbac_timer_destroy(self.h)
        except Exception:
            pass


class LaunchProfiler:
    """Per-launch GPU times from fence-free HIP events recorded on the launching stream
    around every launch (works eagerly and inside a HIP-graph capture: read the times after
    a replay of the captured graph)."""

    def __init__(self):
        self.records = []   # (kernel name, flops, bytes, start timer, end timer, desc)

    def wrap(self, name, flops, nbytes, fn, desc=None):
        s, e = _Timer(), _Timer()
        s.record()
        fn()
        e.record()
        self.records.append((name, flops, nbytes, s, e, desc or name))

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for name, fl, nb, s, e, _ in self.records:
            d = out.setdefault(name, {"launches": 0, "ms": 0.0, "flops": 0.0, "bytes": 0.0})
            d["launches"] += 1
            d["ms"] += s.elapsed_ms(e)
            d["flops"] += fl
            d["bytes"] += nb
        return out

    def layers(self):
        """Per-descriptor totals: {desc: [launches, ms, flops, bytes]}."""
        torch.cuda.synchronize()
        out = {}
        for name, fl, nb, s, e, desc in self.records:
            d = out.setdefault(desc, [0, 0.0, 0.0, 0.0])
            d[0] += 1
            d[1] += s.elapsed_ms(e)
            d[2] += fl
            d[3] += nb
        return out


def timed(name, flops, nbytes, fn, desc=None):
    """Run ``fn`` (one non-conv launch), attributed to ``name`` when profiling."""
    if PROFILER is None:
        fn()
    else:
        PROFILER.wrap(name, flops, nbytes, fn, desc)


def round_up(x, m):
    return (x + m - 1) // m * m


# conv tile shapes of csrc/conv.hip (pixels x channels); index = rgbac_conv_args.tile.
# 0..6: streaming K-ring kernel; 7..12: weight-resident persistent kernel (K <= WRES_STAGES
# stages of 64 bf16 / 32 f32 elements, ksplit 1).
TILES = [(128, 128), (128, 64), (64, 64), (128, 32), (64, 32), (128, 16), (64, 16),
         (128, 64), (64, 64), (128, 32), (64, 32), (128, 128), (128, 16),
         (16, 16), (16, 32), (16, 48), (16, 64), (16, 96), (16, 192),
         (256, 32),
         (128, 128), (128, 64), (64, 64), (128, 32), (64, 32), (128, 16), (64, 16),
         (128, 128), (128, 64), (64, 64), (128, 32), (64, 32), (128, 16), (64, 16),
         (32, 96), (32, 32),
         (128, 192), (128, 128), (128, 96), (128, 256), (128, 192), (128, 64),
         (128, 192), (64, 192), (128, 128), (64, 128), (128, 256), (128, 64),
         (128, 64), (128, 128),
         (64, 64),
         (64, 64), (64, 128), (64, 192),
         (32, 192),
         (64, 32),
         (128, 64), (128, 128), (256, 32)]
FIRST_WRES = 7
WRES_STAGES = 6
FIRST_DIRECT = 13        # 13..18: direct kernel (plain conv, K <= DIRECT_STEPS MFMA k-steps)
DIRECT_STEPS = 12
DIRECT_LDS = 65536       # weight panel bytes of a direct tile (dynamic LDS limit)
TILE_SPATIAL = 19        # conv3x3_c32_kernel: 16x16-pixel tiles, 3x3 s1, Cin 32, Cout <= 32, bf16
FIRST_DEEP = 20          # 20..26: tiles 0..6 with 256-byte K stages (KSM = 2, 2..3 in the ring)
FIRST_PERS = 27          # 27..33: tiles 0..6, persistent over output tiles (no GAUSS epilogue)
STREAM_TILES = (tuple(range(FIRST_WRES)) + tuple(range(FIRST_DEEP, FIRST_DEEP + 7)) +
                tuple(range(FIRST_PERS, FIRST_PERS + 7)))
GAUSS_TILES = tuple(range(FIRST_WRES)) + tuple(range(FIRST_DEEP, FIRST_DEEP + 7))
TILE_SMALLK = 34         # conv_smallk_kernel: bf16 1x1 stride-1 conv, one source, cin_pad <= 256
TILE_WSTREAM = 35        # conv_wstream_kernel: bf16 stride-1 1x1/3x3, cout <= 32, K <= 2336
WSTREAM_MAX_STEPS = 146
FIRST_PATCH = 36         # 36..41: conv_patch_kernel (TH x 16 M-grid tile, BN channels, 8 waves)
PATCH_SIG = {36: (8, 192, 2, 4, 3), 37: (8, 128, 2, 4, 3), 38: (8, 96, 4, 2, 3),
             39: (8, 256, 2, 4, 3), 40: (8, 192, 2, 4, 4), 41: (8, 64, 4, 2, 3),
             48: (8, 64, 4, 2, 4), 49: (8, 128, 2, 4, 4)}


def _patch_split_ok(preps):
    """The phase split (ksplit 4 on a conv_patch_kernel tile, csrc/conv.hip): one workgroup
    per (tile, phase) of the 5x5/s2 conv (fp32 phase slabs summed by the split-K epilogue) or
    of the convT (each phase writes its own output pixels; no workspace)."""
    a = preps[0].a
    return (a.mode == CONVT_S2 or (a.mode == CONV and a.ksize == 5 and a.stride == 2)) and \
        a.act not in (ACT["dgelu"], ACT["dlrelu"])
FIRST_FPATCH = 42        # 42..47: conv_fpatch_kernel (fragment-major weight copy, 4 waves)
FPATCH_SIG = {42: (8, 192), 43: (4, 192), 44: (8, 128), 45: (4, 128), 46: (8, 256), 47: (8, 64),
              50: (4, 64), 51: (4, 64), 52: (4, 128), 53: (4, 192),
              56: (8, 64), 57: (8, 128), 58: (16, 32)}
# 51..53: the unrolled-K variants with K split by kernel row (KS = 3, 12 waves): only where
# the unrolled-K variant applies (fpatch_cpt != 0)
FPATCH_KS = {51: 4, 52: 4, 53: 4, 56: 4, 57: 4, 58: 2}    # tile -> N waves (x 3 K parts)
TILE_PW = 54             # conv_pw_kernel: bf16 1x1 stride-1 conv, one source, cin/cout <= 192
TILE_NPATCH = 55         # conv_npatch_kernel: bf16 3x3 stride-1 conv, cout <= 32 (chain tails)
# tiles that read the fragment-major weight copy (frag_weights): forward PackedConv only
FRAG_TILES = frozenset(FPATCH_SIG) | {TILE_NPATCH}
# the fragment-patch kernel's unrolled-K variants (csrc/conv.hip, CPT template argument)
FPATCH_CPT = os.environ.get("RGBAC_FPATCH_CPT", "1") != "0"


def fpatch_cpt(preps):
    """CPT (32-deep k-steps per tap) of the unrolled-K fragment-patch variant the launcher
    picks for these convs, or 0 for the generic loop."""
    if not FPATCH_CPT or preps[0].pk.mode != CONV:
        return 0
    c = {round_up(p.pk.cin_pad, 32) // 32 for p in preps}
    return c.pop() if len(c) == 1 and next(iter(c)) in (3, 4, 7) else 0
def fpatch_cpt_ks(preps, tile):
    """CPT of a K-split fragment-patch tile (51-53, 56-58) for these convs, 0 if it does not
    apply: conv with 3 / 4 / 7 k-steps per tap, and on tiles 51 / 52 also subpel convs and
    8..10 k-steps per tap (csrc/conv.hip launch_conv)."""
    if not FPATCH_CPT:
        return 0
    wide = tile in (51, 52)
    if preps[0].pk.mode != CONV and not (wide and preps[0].pk.mode == SUBPEL2):
        return 0
    c = {round_up(p.pk.cin_pad, 32) // 32 for p in preps}
    if len(c) != 1:
        return 0
    c = c.pop()
    return c if c in (3, 4, 7) or (wide and 8 <= c <= 10) else 0
PATCH = os.environ.get("RGBAC_PATCH", "1") != "0"


def frag_weights(pk):
    """Fragment-major copy of a PackedConv for the conv_fpatch tiles (cached on it):
    [nphase][cout_pad / 16][ntaps_max * cin32 / 32][64 lanes][8] bf16 -- per (phase, 16-row
    N tile, 32-deep k-step) the 64 lanes' 16-byte v_mfma_f32_16x16x32_bf16 A fragments in
    lane order (lane l: row l & 15, k 8 * (l >> 4) .. +7), with K tap-major over the input
    channels padded to 32 per tap (k' = tap * cin32 + ci; zeros in the padding)."""
    f = getattr(pk, "frag", None)
    if f is not None:
        return f
    nph, rows, _ = pk.w.shape
    taps = 9 if pk.mode == CONVT_S2 else pk.ksize * pk.ksize
    cp, c32 = pk.cin_pad, round_up(pk.cin_pad, 32)
    w = pk.w[:, :, :taps * cp].reshape(nph, rows, taps, cp)
    wt = torch.zeros((nph, rows, taps, c32), dtype=pk.w.dtype, device=pk.w.device)
    wt[..., :cp] = w
    nks = taps * c32 // 32
    fr = wt.reshape(nph, rows // 16, 16, nks, 4, 8).permute(0, 1, 3, 4, 2, 5).contiguous()
    pk.frag = fr
    return fr


def _has_frag(pk):
    """A pack the fragment-streamed tiles can read: a forward PackedConv (its fragment-major
    copy built once, frag_weights) or a training pack gathering one every step
    (rgbac.autograd.TPack.enable_frag)."""
    return isinstance(pk, PackedConv) or getattr(pk, "frag", None) is not None


def _patch_tiles(preps):
    """Patch-resident tiles that apply to these (grouped) convs: bf16, the 5x5/s2 convT or a
    3x3 stride-1 conv/subpel, no squared input / GAUSS epilogue, M grid a multiple of 16 wide
    and of the tile height high, whole BN-row weight tiles inside the packed rows."""
    if not PATCH:
        return []
    a = preps[0].a
    if a.dtype != _lib.BF16 or a.square_input or a.act == ACT["gauss"]:
        return []
    s2 = a.mode == CONV and a.ksize == 5 and a.stride == 2
    if a.mode == CONVT_S2:
        hm, wm = a.in_h, a.in_w
    elif a.ksize == 3 and a.stride == 1 and a.mode in (CONV, SUBPEL2):
        hm, wm = a.in_h, a.in_w
    elif s2:
        # the polyphase strided conv (csrc/conv.hip conv_patch_kernel): the output grid
        hm, wm = a.out_h, a.out_w
    else:
        return []
    if wm % 16 or a.batch * a.in_h * a.in_w >= (1 << 24):
        return []
    out = []
    for t, (th, bn, _, _, _) in PATCH_SIG.items():
        if hm % th:
            continue
        if all(p.pk.cout_pad >= -(-p.pk.cout // bn) * bn for p in preps):
            out.append(t)
    # fragment-streamed tiles: PackedConv weights only (the training packs are re-gathered
    # every step in the plain layout) and the whole patch in LDS; no strided conv
    if not s2 and all(_has_frag(p.pk) for p in preps) and \
            a.act not in (ACT["dgelu"], ACT["dlrelu"]):
        c32 = max(round_up(p.pk.cin_pad, 32) for p in preps)
        for t, (th, bn) in FPATCH_SIG.items():
            if hm % th or (th + 2) * 18 * (c32 // 8 + 2) * 16 > 160 * 1024:
                continue
            if t in FPATCH_KS and 2 * (bn // 16) * th * 1024 > 160 * 1024:
                continue
            if t in FPATCH_KS and not fpatch_cpt_ks(preps, t):
                continue
            if all(p.pk.cout_pad >= -(-p.pk.cout // bn) * bn for p in preps):
                out.append(t)
    return out
def _patch_cands(preps):
    """(tile, ksplit) candidates of the patch tiles: every applicable tile unsplit, and the
    conv_patch_kernel tiles with the phase split where it applies."""
    ts = _patch_tiles(preps)
    out = [(t, 1) for t in ts]
    if _patch_split_ok(preps):
        out += [(t, 4) for t in ts if t in PATCH_SIG]
    return out


SMALLK_MAX = 256
KSPLITS = (1, 2, 4, 8)
TUNE = os.environ.get("RGBAC_TUNE", "1") != "0"
# RGBAC_TILE_SET: "stream" (default: streaming K-ring tiles; the weight-resident and
# direct small-K tiles measured slower under graph replay) | "all"
TILE_SET = os.environ.get("RGBAC_TILE_SET", "stream")
_tune_cache = {}          # shape key -> (tile, ksplit)
FORCE = None              # (tile, ksplit) override, used by the tile/split-K tests
STEM_FUSED = os.environ.get("RGBAC_STEM_FUSED", "1") != "0"   # x1 + gdn1 as one launch (bf16)
DSE_FUSED = os.environ.get("RGBAC_DSE_FUSED", "1") != "0"     # DSE as 3 fused launches (bf16)
WINBLOCK_FUSED = os.environ.get("RGBAC_WINBLOCK", "1") != "0"  # ws-8 attention block, 1 launch
WINBLOCK4_FUSED = os.environ.get("RGBAC_WINBLOCK4", "1") != "0"  # ws-4 / C-80 block, 1 launch


_SIDE_STREAMS = {}
# measured slower on the config-2 forward graph (same box, interleaved: 1,796 / 1,794 us with the
# decoder's mask pyramid and x_hat conversion forked off vs 1,772 / 1,775 us without; the
# event waits of the fork / join cost more than the hidden ~18 us): opt-in
SIDE = os.environ.get("RGBAC_SIDE_STREAMS", "0") == "1"


def side_streams(dev):
    """(current stream, this device's side stream) for independent work forked off the
    current stream and joined back (graph-capturable: event waits).  RGBAC_SIDE_STREAMS=0:
    the side stream IS the current stream (no fork)."""
    cur = torch.cuda.current_stream(dev)
    if not SIDE:
        return cur, cur
    st = _SIDE_STREAMS.get(dev)
    if st is None:
        st = _SIDE_STREAMS[dev] = torch.cuda.Stream(device=dev)
    return cur, st


def pick_cout_pad(cout):
    """Packed weight rows per phase: every tile's N blocks stay inside the buffer."""
    return round_up(cout, 128)


def _wstream_ok(preps):
    a = preps[0].a
    if not (a.dtype == _lib.BF16 and a.mode == CONV and a.stride == 1 and a.ksize in (1, 3)):
        return False
    for p in preps:
        if p.pk.cout > 32 or -(-a.ksize * a.ksize * p.a.cin_pad // 16) > WSTREAM_MAX_STEPS:
            return False
        if a.act == ACT["gauss"] and p.pk.cout % 16:
            return False
    return True


def _candidates(M, cout, nst, nks=None, plain=True, spatial=False, smallk=False, wstream=False):
    """(tile, ksplit) pairs worth timing for an M-pixel, cout-channel conv with nst K-stages
    (nks MFMA k-steps; ``plain`` = CONV mode; ``spatial`` = the 3x3/Cin-32 tile applies;
    ``smallk`` = the small-K wave-streaming tile applies)."""
    out = [(TILE_SMALLK, 1)] if smallk else []
    if wstream:
        out.append((TILE_WSTREAM, 1))
    n16 = round_up(cout, 16)
    for t, (bm, bn) in enumerate(TILES):
        if t in (TILE_SMALLK, TILE_WSTREAM) or t >= FIRST_PATCH:
            continue
        if t == TILE_SPATIAL:
            if spatial:
                out.append((t, 1))
            continue
        if TILE_SET == "stream" and t not in STREAM_TILES:
            continue
        if FIRST_DIRECT <= t < FIRST_DEEP:
            if plain and nks is not None and nks <= DIRECT_STEPS and bn >= n16 / 4 \
                    and bn < 2 * n16 + 16 and bn * (4 * nks + 1) * 16 <= DIRECT_LDS:
                out.append((t, 1))
            continue
        if bn > 16 and bn > 2 * n16:
            continue
        if FIRST_WRES <= t < FIRST_DIRECT:
            if nst <= WRES_STAGES:
                out.append((t, 1))
            continue
        blocks = -(-M // bm) * -(-cout // bn)
        for ks in KSPLITS:
            if ks > 1 and (nst // ks < 2 or blocks * ks > 4096 or blocks >= 512):
                continue
            out.append((t, ks))
    return out


def _heuristic(M, cout, nst):
    n16 = round_up(cout, 16)
    if n16 % 128 == 0:
        t = 0
    elif n16 >= 64:
        t = 1
    elif n16 > 16:
        t = 3
    else:
        t = 5
    bm, bn = TILES[t]
    blocks = -(-M // bm) * -(-cout // bn)
    ks = 1
    while ks < 8 and blocks * ks < 256 and nst // (2 * ks) >= 4:
        ks *= 2
    return t, ks


def tune_cache():
    return dict(_tune_cache)


_FIXED = [0]


@contextlib.contextmanager
def fixed_tiles():
    """Within this context every conv launch takes its tile / split-K from the shape rule
    alone (no timing-based autotune, tune cache neither read nor written).  The bitstream
    path needs bit-identical mu / sigma in compress and decompress, whichever process (and
    tuning history) runs them: a different tile or split-K changes the fp32 summation order."""
    _FIXED[0] += 1
    try:
        yield
    finally:
        _FIXED[0] -= 1


def load_tune_cache(path):
    with open(path) as fh:
        for k, v in json.load(fh).items():
            _tune_cache[k] = tuple(v)


def save_tune_cache(path):
    with open(path, "w") as fh:
        json.dump({k: list(v) for k, v in sorted(_tune_cache.items())}, fh, indent=0)


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
        if transposed and mode == SUBPEL2:
            # ConvTranspose2d(5, s=2, p=2, op=1) == conv3x3(4*Cout) + PixelShuffle(2):
            # output parity (py, px) of channel c is conv channel 4c + 2py + px, and its
            # 3x3 tap (a, b) (input offset a-1, b-1) is ConvT tap (py + 4 - 2a, px + 4 - 2b).
            cin_t, cout_t = w.shape[0], w.shape[1]
            ws = torch.zeros((4 * cout_t, cin_t, 3, 3), device=dev)
            for py in (0, 1):
                for px in (0, 1):
                    for ta in range(3):
                        for tb in range(3):
                            ky, kx = py + 4 - 2 * ta, px + 4 - 2 * tb
                            if ky <= 4 and kx <= 4:
                                ws[2 * py + px::4, :, ta, tb] = w[:, :, ky, kx].t()
            w = ws
            if bias is not None:
                bias = bias.detach().float().repeat_interleave(4)
            stride = 1
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
        # zero slack behind the last row: a 256-byte-per-row K stage (KSM = 2 tiles) may read
        # up to 64 elements past k_pad (those lanes multiply zero im2col chunks)
        n = wp.numel()
        flat = torch.zeros(n + 128, dtype=dtype, device=dev)
        flat[:n].copy_(wp.reshape(-1))
        self.w = flat[:n].view(wp.shape)
        self.bias = torch.zeros(self.cout_pad, device=dev)
        if bias is not None:
            self.bias[:cout] = bias.detach().float()
        self.segs = list(segs)


class Prepared:
    """One conv's ABI record plus what the launcher needs (output, tuning key)."""
    __slots__ = ("a", "out", "key", "mgrid", "nphase", "nst", "nks", "pk", "desc", "flops",
                 "nbytes", "partial")


def prepare(pk, srcs, out=None, out_coff=0, act="none", act_param=0.0, res0=None, res1=None,
            res2=None, sel=None, square=False, bias=True, aux0=None, aux1=None, partial=None,
            zout=None):
    """Build the rgbac_conv_args record of one conv over sources [(Feat, coff, nch), ...].

    ``res*`` are Feats on the output grid or (Feat, coff) channel slices."""
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
    if act == "gauss":
        cstore = pk.cout // 2
    if out is None:
        out = new_feat(B, Ho, Wo, cstore, dtype, f0.t.device)
    a = _lib.ConvArgs()
    a.dtype = _lib.dtype_code(dtype)
    a.mode = pk.mode
    a.batch, a.in_h, a.in_w = B, H, W
    a.ksize, a.stride = pk.ksize, pk.stride
    srcs = [sr for sr in srcs if sr[2] > 0]
    a.nsrc = len(srcs)
    for i, (f, coff, nch) in enumerate(srcs):
        assert f.B == B and f.H == H and f.W == W and f.t.dtype == dtype
        a.src[i].ptr = f.ptr(coff)
        a.src[i].ldc = f.ldc
        a.src[i].channels = nch
    assert sum(sr[2] for sr in srcs) == pk.cin_pad, (sum(sr[2] for sr in srcs), pk.cin_pad)
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
            rf, rc = (r, 0) if isinstance(r, Feat) else r
            assert rf.H == Ho and rf.W == Wo and rf.t.dtype == dtype
            setattr(a, name, rf.ptr(rc))
            setattr(a, name + "_ldc", rf.ldc)
    a.sel = None if sel is None else sel.data_ptr()
    a.aux0 = None if aux0 is None else aux0.data_ptr()
    a.aux1 = None if aux1 is None else aux1.data_ptr()
    a.partial = None if partial is None else partial.data_ptr()
    if zout is not None:
        assert zout.H == Ho and zout.W == Wo and zout.t.dtype == dtype
        a.zout, a.zout_ldc = zout.ptr(), zout.ldc
    pr = Prepared()
    pr.a, pr.out, pr.pk = a, out, pk
    pr.partial = partial
    taps = 9 if pk.mode == CONVT_S2 else pk.ksize * pk.ksize
    pr.mgrid = B * (H * W if pk.mode != CONV else Ho * Wo)
    pr.nphase = 4 if pk.mode == CONVT_S2 else 1
    pr.nst = -(-taps * pk.cin_pad // (32 if dtype == torch.float32 else 64))
    pr.nks = -(-taps * pk.cin_pad // (16 if dtype == torch.float32 else 32))
    pr.key = f"{a.dtype}/{pk.mode}/{pk.ksize}/{pk.stride}/{B}x{H}x{W}/{pk.cin_pad}/{pk.cout}/{act == 'gauss'}"
    if act in ("dgelu", "dlrelu"):
        # the folded activation backward runs in other instances and not on the
        # fragment-streamed tiles: its own choice
        pr.key += "/dact"
    pr.flops = 2.0 * pr.mgrid * pk.cout * pk.cin * (25 if pk.mode == CONVT_S2 else taps)
    es = f0.t.element_size()
    pr.nbytes = es * (B * H * W * pk.cin + B * Ho * Wo * cstore) + pk.w.numel() * es
    pr.desc = (f"m{pk.mode} k{pk.ksize}s{pk.stride} {pk.cin}->{pk.cout} {H}x{W}->{Ho}x{Wo} "
               f"B{B} act={act}{' sq' if square else ''}")
    return pr


def _spatial_ok(preps):
    a = preps[0].a
    return (a.dtype == _lib.BF16 and a.mode == CONV and a.ksize == 3 and a.stride == 1 and
            a.in_h % 16 == 0 and a.in_w % 16 == 0 and a.act != ACT["gauss"] and
            all(p.a.nsrc == 1 and p.a.cin_pad == 32 and p.a.src[0].channels == 32 and
                p.a.cout <= 32 for p in preps))


# C++ template arguments (BM, BN, WGM, WGN, NBUF) of the streaming/persistent tiles, so the
# profiler's kernel names are exactly rocprofv3's (csrc/conv.hip launch_conv).
_TILE_SIG = {0: "128, 128, 2, 2, 2", 1: "128, 64, 4, 1, 3", 2: "64, 64, 2, 2, 3",
             3: "128, 32, 4, 1, 3", 4: "64, 32, 2, 2, 3", 5: "128, 16, 4, 1, 3",
             6: "64, 16, 4, 1, 3", 20: "128, 128, 2, 2, 2, 2", 21: "128, 64, 4, 1, 2, 2",
             22: "64, 64, 2, 2, 2, 2", 23: "128, 32, 4, 1, 2, 2", 24: "64, 32, 2, 2, 3, 2",
             25: "128, 16, 4, 1, 2, 2", 26: "64, 16, 4, 1, 3, 2"}
_SMALLK_NKS = {1: 1, 2: 2, 3: 3, 4: 4, 5: 5, 6: 6, 7: 8, 8: 8, 9: 12, 10: 12, 11: 12, 12: 12}


_PW2_ON = os.environ.get("RGBAC_PW2", "1") != "0"
_PW2_ALL = os.environ.get("RGBAC_PW2_ALL", "1") != "0"


def _pw2_admits(preps):
    """Host mirror of csrc/conv.hip pw2_ok (which pointwise kernel a TILE_PW launch runs)."""
    a0 = preps[0].a
    if not _PW2_ON or a0.act in (ACT["tanh_half"], ACT["gauss"]) or a0.mode != CONV:
        return False
    if not _PW2_ALL and -(-preps[0].mgrid // 16) * len(preps) > 8 * 256:
        return False
    for p in preps:
        a = p.a
        if (a.zout and a.zout_ldc % 4) or a.cout % 8 or a.out_coff % 8 or a.out_ldc % 8 or \
                a.cout > 192 or (a.res0 and a.res0_ldc % 4) or (a.res1 and a.res1_ldc % 4) or \
                (a.res2 and a.res2_ldc % 4):
            return False
    return True


_PW3_ON = os.environ.get("RGBAC_PW3", "1") != "0"


def _pw3_admits(preps):
    """Host mirror of csrc/pw3.hip pw3_ok: the two-deep GDN / IGDN forward kernel."""
    a0 = preps[0].a
    gate = a0.act == ACT["gate"] and preps[0].mgrid >= 8192 * 16
    if not _PW3_ON or (a0.act not in (ACT["gdn"], ACT["igdn"]) and not gate) or \
            bool(a0.square_input) == gate or a0.mode != CONV:
        return False
    if not 128 < max(p.a.cin_pad for p in preps) <= 192:
        return False
    for p in preps:
        a = p.a
        if a.res0 or a.zout or a.cout != 192 or a.out_coff % 8 or a.out_ldc % 8 or \
                a.src[0].ldc % 8 or a.k_pad < a.cin_pad:
            return False
        if gate:
            if not a.res1 or not a.res2 or a.res1_ldc % 4 or a.res2_ldc % 4:
                return False
        elif a.res1 != a.src[0].ptr or a.res1_ldc != a.src[0].ldc or a.res2:
            return False
    return True


def kernel_name(tile, preps):
    """rocprofv3-style name (namespace and argument list stripped) of a conv launch."""
    dt = "float" if preps[0].a.dtype == 0 else "bf16_t"
    if tile == TILE_SPATIAL:
        return f"conv3x3_c32_kernel<{dt}>"
    if tile in FPATCH_KS:
        return "conv_fpatch_kernel<%d, %d, %d, 4, %d, 3>" % (FPATCH_SIG[tile] + (FPATCH_KS[tile],
                                                                           fpatch_cpt_ks(preps, tile)))
    if tile in FPATCH_SIG:
        c = fpatch_cpt(preps) if FPATCH_SIG[tile][0] == 4 else 0
        return "conv_fpatch_kernel<%d, %d, 4, 4%s>" % (FPATCH_SIG[tile] + (f", {c}" if c else "",))
    if tile in PATCH_SIG:
        dact = "true" if preps[0].a.act in (ACT["dgelu"], ACT["dlrelu"]) else "false"
        return "conv_patch_kernel<%d, %d, %d, %d, %d, %s>" % (PATCH_SIG[tile] + (dact,))
    if tile == TILE_WSTREAM:
        # the library's wave count choice (csrc/conv.hip launch_wstream)
        nks = max((p.a.ksize * p.a.ksize * p.a.cin_pad + 15) // 16 for p in preps)
        env = os.environ.get("RGBAC_WSTREAM_WAVES", "")
        nw = int(env) if env in ("4", "8") else (8 if nks >= 64 else 4)
        return f"conv_wstream_kernel<8, {nw}>"
    if tile == TILE_NPATCH:
        return f"conv_npatch_kernel<{2 if max(p.pk.cout for p in preps) > 16 else 1}>"
    if tile == TILE_PW:
        cin = max(p.a.cin_pad for p in preps)
        nks = 2 if cin <= 64 else (4 if cin <= 128 else 6)
        # csrc/conv.hip launch_pw: conv_pw2_kernel where pw2_ok admits the launch, else
        # conv_pw_kernel (32-deep k-steps held in LDS: 2 / 4 / 6)
        if _pw3_admits(preps):
            return f"conv_pw3_kernel<6, {preps[0].a.act}>"
        if _pw2_admits(preps):
            return f"conv_pw2_kernel<{nks}>"
        dact = "true" if preps[0].a.act in (ACT["dgelu"], ACT["dlrelu"]) else "false"
        return f"conv_pw_kernel<{nks}, {dact}>"
    if tile == TILE_SMALLK:
        cout = max(p.pk.cout for p in preps)
        nt = 1 if cout <= 32 else (2 if cout <= 64 else 3)
        nks = -(-max(p.a.cin_pad for p in preps) // 16)
        return f"conv_smallk_kernel<{nt}, {_SMALLK_NKS.get(nks, 16)}>"
    if FIRST_DIRECT <= tile < FIRST_DEEP:
        return f"conv_direct_kernel<{dt},{TILES[tile][1] // 16}>"
    if FIRST_WRES <= tile < FIRST_DIRECT:
        bm, bn = TILES[tile]
        return f"conv_wres_kernel<{dt},{bm}x{bn}>"
    if tile >= FIRST_PERS:
        return f"conv_pers_kernel<{dt}, {_TILE_SIG[tile - FIRST_PERS]}>"
    # tiles 0..6 instantiate conv_kernel's KSM = 1 default (rocprofv3 prints it)
    return f"conv_kernel<{dt}, {_TILE_SIG[tile]}{', 1' if tile < FIRST_WRES else ''}>"


# RGBAC_NPATCH_SUBPEL=0: keep subpel convs off the narrow patch tile (A/B against older builds)
NPATCH_SUBPEL = os.environ.get("RGBAC_NPATCH_SUBPEL", "1") != "0"


def _npatch_ok(preps):
    a = preps[0].a
    # subpel convs (the decoder's 3-channel ConvTranspose as conv3x3 + PixelShuffle) take the
    # plain epilogue: bias, optional GELU, shuffled store -- no residual operands
    subpel_ok = (NPATCH_SUBPEL and a.mode == SUBPEL2 and a.act in (ACT["none"], ACT["gelu"]) and
                 all(not (p.a.res0 or p.a.res1 or p.a.res2) for p in preps))
    if not (a.dtype == _lib.BF16 and (a.mode == CONV or subpel_ok) and a.ksize == 3 and
            a.stride == 1 and a.in_w % 16 == 0 and a.in_h % 4 == 0 and
            a.batch * a.in_h * a.in_w < (1 << 24)):
        return False
    if not all(_has_frag(p.pk) for p in preps) or a.act in (ACT["dgelu"], ACT["dlrelu"]):
        return False
    for p in preps:
        if p.pk.cout > 32 or 6 * 18 * (round_up(p.pk.cin_pad, 32) // 8 + 2) * 16 > 128 * 1024:
            return False
        if a.act == ACT["gauss"] and p.pk.cout not in (16, 32):
            return False
    return True


def _pw_ok(preps):
    a = preps[0].a
    return (a.dtype == _lib.BF16 and a.mode == CONV and a.act != ACT["gauss"] and
            a.ksize == 1 and a.stride == 1 and
            all(p.a.nsrc == 1 and p.a.cin_pad <= 192 and p.pk.cout <= 192 for p in preps))


def _smallk_ok(preps):
    a = preps[0].a
    return (a.dtype == _lib.BF16 and a.mode == CONV and a.act != ACT["gauss"] and
            a.ksize == 1 and a.stride == 1 and
            all(p.a.nsrc == 1 and p.a.cin_pad <= SMALLK_MAX for p in preps))


def _gauss_ok(t, cout):
    return TILES[t][1] >= cout


def _choice_valid(t, preps):
    """Whether tile ``t`` accepts these (grouped, non-GAUSS) convs: the special tiles have
    the preconditions their launchers check (csrc/conv.hip RGBAC_REQUIRE); the streaming /
    persistent / weight-resident tiles take any conv."""
    if t == TILE_PW:
        return _pw_ok(preps)
    if t == TILE_NPATCH:
        return _npatch_ok(preps)
    if t == TILE_WSTREAM:
        return _wstream_ok(preps)
    if t == TILE_SMALLK:
        return _smallk_ok(preps)
    if t == TILE_SPATIAL:
        return _spatial_ok(preps)
    if t >= FIRST_PATCH:
        return t in _patch_tiles(preps)
    if FIRST_DIRECT <= t < FIRST_DEEP:
        return preps[0].pk.mode == CONV
    return True


# Split-K tickets for the in-launch reduction (rgbac_conv_args.tile_counters): one zeroed
# int32 buffer per device shared by every launch -- launches on a stream run one after the
# other and the last split block of each tile resets its ticket, so it is zero again between
# launches.  Allocated outside graph capture (the first, eager launch of a shape).
_COUNTERS = {}
_COUNTERS_MIN = 1 << 20
# Off by default: measured slower end-to-end (165.6 -> 157 MPix/s) -- each split block's
# agent-scope release writes back its XCD's L2 -- than the separate reduce launch.
INLAUNCH_SPLITK = os.environ.get("RGBAC_INLAUNCH_SPLITK", "0") == "1"


def _tile_counters(dev, n):
    buf = _COUNTERS.get(dev)
    if buf is None or buf.numel() < n:
        if torch.cuda.is_current_stream_capturing():
            return None                   # never allocate (and zero-fill) inside a capture
        buf = torch.zeros(max(n, _COUNTERS_MIN), dtype=torch.int32, device=dev)
        _COUNTERS[dev] = buf
    return buf


LAST_CHOICE = [None]      # (tile, ksplit) of the most recent launch (debug re-runs)
_FLUSH = {}


def _flush_buffer(dev):
    buf = _FLUSH.get(dev)
    if buf is None:
        buf = _FLUSH[dev] = torch.zeros(16 << 20, dtype=torch.float32, device=dev)   # 64 MB
    return buf


def launch(preps, force=None):
    """Launch prepared convs (same geometry) as ONE grouped kernel; returns their outputs.
    ``force``: (tile, ksplit) to use instead of the tuned / heuristic choice."""
    n = len(preps)
    p0 = preps[0]
    dev = p0.out.t.device
    gauss = p0.a.act == ACT["gauss"]
    key = f"{p0.key}/g{n}"
    keep = []
    arr = (_lib.ConvArgs * n)()
    for i, pr in enumerate(preps):
        arr[i] = pr.a

    def set_choice(t, ks):
        cnt = None
        if ks > 1 and INLAUNCH_SPLITK and (t < FIRST_WRES or FIRST_DEEP <= t < FIRST_PERS):
            bm, bn = TILES[t]
            need = n * p0.nphase * (-(-p0.mgrid // bm)) * (-(-max(pr.pk.cout for pr in preps) // bn))
            buf = _tile_counters(dev, need)
            if buf is not None:
                keep.append(buf)
                cnt = buf.data_ptr()
        for i, pr in enumerate(preps):
            arr[i].tile, arr[i].ksplit = t, ks
            arr[i].tile_counters = cnt
            arr[i].workspace = None
            # the fragment-streamed tiles read the fragment-major weight copy
            arr[i].weight = (frag_weights(pr.pk).data_ptr() if t in FRAG_TILES
                             else pr.pk.w.data_ptr())
            if ks > 1 and not (t in PATCH_SIG and pr.a.mode == CONVT_S2):   # (phase split)
                ws = torch.empty(ks * pr.nphase * pr.mgrid * round_up(pr.pk.cout, 16),
                                 dtype=torch.float32, device=dev)
                keep.append(ws)
                arr[i].workspace = ws.data_ptr()

    def run():
        _lib.call("rgbac_conv2d_grouped", ctypes.addressof(arr), n, _lib.stream_ptr(dev))

    fixed = _FIXED[0] > 0
    choice = None if fixed else (FORCE if (FORCE and not gauss) else _tune_cache.get(key))
    if force is not None:
        choice = tuple(force)
    if choice is None:
        mtot = p0.mgrid * p0.nphase * n
        cout = max(pr.pk.cout for pr in preps)
        nst = max(pr.nst for pr in preps)
        if gauss:
            cands = [(t, 1) for t in GAUSS_TILES if _gauss_ok(t, cout)]
            if _wstream_ok(preps):
                cands.append((TILE_WSTREAM, 1))
            if _npatch_ok(preps):
                cands.append((TILE_NPATCH, 1))
        else:
            cands = _candidates(mtot, cout, nst, max(pr.nks for pr in preps),
                                p0.pk.mode == CONV, _spatial_ok(preps), _smallk_ok(preps),
                                _wstream_ok(preps))
            cands += _patch_cands(preps)
            if _pw_ok(preps):
                cands.append((TILE_PW, 1))
            if _npatch_ok(preps):
                cands.append((TILE_NPATCH, 1))
        if TUNE and not fixed and not torch.cuda.is_current_stream_capturing():
            # each timed run starts with the L2s flushed (a 64 MB write evicts all 8 XCDs'
            # 4 MB): in the forward graph every layer's weights and inputs arrive cold, and a
            # candidate that re-streams its weights per wave from L2 looks 2x faster hot
            flush = _flush_buffer(dev)
            # an output that is also a residual operand (in-place accumulation, the training
            # step's gradient sinks) must not see the repeated timing runs: they write a
            # scratch copy of it, and the chosen tile then runs once on the real one
            outs = [arr[i].out for i in range(n)]
            scratch = []
            for i, pr in enumerate(preps):
                if arr[i].out in (arr[i].res0, arr[i].res1, arr[i].res2):
                    s = pr.out.t.clone()
                    scratch.append(s)
                    arr[i].out = s.data_ptr()
                    for name in ("res0", "res1", "res2"):
                        if getattr(arr[i], name) == outs[i]:
                            setattr(arr[i], name, s.data_ptr())
            best = None
            for cand in cands:
                set_choice(*cand)
                run()                                           # warm-up
                ms = 0.0
                for _ in range(3):
                    flush.add_(1)
                    ev0 = torch.cuda.Event(enable_timing=True)
                    ev1 = torch.cuda.Event(enable_timing=True)
                    ev0.record()
                    run()
                    ev1.record()
                    ev1.synchronize()
                    ms += ev0.elapsed_time(ev1)
                if best is None or ms < best[0]:
                    best = (ms, cand)
            choice = best[1]
            if gauss:
                # every candidate wrote bits partials at ITS M-block granularity: slots the
                # chosen tile does not write must read zero again (the caller zeroed them once)
                for pr in preps:
                    if pr.partial is not None:
                        pr.partial.zero_()
            if scratch:
                for i in range(n):
                    if arr[i].out != outs[i]:
                        s_ptr = arr[i].out
                        arr[i].out = outs[i]
                        for name in ("res0", "res1", "res2"):
                            if getattr(arr[i], name) == s_ptr:
                                setattr(arr[i], name, outs[i])
                torch.cuda.synchronize(dev)
                del scratch
        elif gauss:
            choice = min(cands, key=lambda c: TILES[c[0]][1])
        else:
            choice = _heuristic(mtot, cout, nst)
        if not fixed:
            _tune_cache[key] = choice
    if not gauss and (not _choice_valid(choice[0], preps) or (
            choice[1] > 1 and choice[0] in PATCH_SIG and
            (choice[1] != 4 or not _patch_split_ok(preps)))):
        # a cached / forced tile the C side would refuse for THESE convs: the cache key
        # (dtype / mode / ksize / stride / shape / cin_pad / cout) does not hold the source
        # count, the residual operands, the activation or the pack type, so the same key
        # can come from a conv the special tiles accept (e.g. TILE_PW tuned on a
        # one-source conv, handed a two-source one), or a fragment-streamed tile tuned on a
        # pack with a fragment-major copy handed one without it, or an input-gradient conv
        # with the folded activation backward (not in those tiles) -- take the shape rule
        choice = _heuristic(p0.mgrid * p0.nphase * n, max(pr.pk.cout for pr in preps),
                            max(pr.nst for pr in preps))
    if gauss and not (choice[0] == TILE_WSTREAM and _wstream_ok(preps)) and \
            not (choice[0] == TILE_NPATCH and _npatch_ok(preps)) and (
            choice[0] not in GAUSS_TILES or
            not _gauss_ok(choice[0], max(pr.pk.cout for pr in preps))):
        choice = (min((t for t in GAUSS_TILES if _gauss_ok(t, p0.pk.cout)),
                      key=lambda t: TILES[t][1]), 1)
    set_choice(*choice)
    LAST_CHOICE[0] = tuple(choice)
    if PROFILER is None:
        run()
    else:
        name = kernel_name(choice[0], preps)
        desc = f"{name} ks{choice[1]} g{n} {p0.desc}"
        # main kernel and split-K reduce timed separately (rocprofv3 lists them apart)
        PROFILER.wrap(name, sum(pr.flops for pr in preps), sum(pr.nbytes for pr in preps),
                      lambda: _lib.call("rgbac_conv2d_grouped_part", ctypes.addressof(arr), n, 1,
                                        _lib.stream_ptr(dev)), desc)
        if choice[1] > 1 and not arr[0].tile_counters:
            dts = "float" if p0.a.dtype == 0 else "bf16_t"
            PROFILER.wrap(f"conv_splitk_epilogue<{dts}>", 0.0,
                          sum(4.0 * choice[1] * pr.mgrid * pr.nphase * pr.pk.cout for pr in preps),
                          lambda: _lib.call("rgbac_conv2d_grouped_part", ctypes.addressof(arr), n,
                                            2, _lib.stream_ptr(dev)),
                          f"conv_splitk_epilogue ks{choice[1]} g{n} {p0.desc}")
    return [pr.out for pr in preps]


def conv(pk, srcs, **kw):
    """Run one PackedConv over concatenated sources [(Feat, coff, nch), ...] -> Feat."""
    return launch([prepare(pk, srcs, **kw)])[0]


def feat_srcs(f):
    return [(f, 0, f.ldc)]


def packed(m, dtype, segs, mode=CONV, transposed=False, weight=None, bias=None):
    """PackedConv for module ``m`` (Conv2d / ConvTranspose2d / Linear), cached on the
    module and rebuilt when a parameter's version or storage changes."""
    w = m.weight if weight is None else weight
    b = getattr(m, "bias", None) if bias is None else bias
    key = (dtype, tuple(segs), mode, transposed)
    ver = (PARAM_GEN, w._version, w.data_ptr(),
           None if b is None else (b._version, b.data_ptr()))
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
