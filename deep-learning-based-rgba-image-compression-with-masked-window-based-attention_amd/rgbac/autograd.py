"""Training path: torch.autograd.Function wrappers over the HIP kernels.

SURVEY.md §8b: "The Python torch.autograd.Function wrappers call *_fwd/*_bwd".
Every Function's forward is the same HIP launch the inference path uses (with
the pre-activation saved through ``zout``); its backward is HIP too:

  ConvFn      conv / convT / subpel / Linear / GDN with fused epilogue
              backward = rgbac_act_bwd -> input-gradient conv on the MFMA conv
              engine over a repacked weight (+ SQBWD epilogue for GDN) ->
              rgbac_conv_wgrad + rgbac_wgrad_reduce (weight, bias)
  WinAttnFn   rgbac_winattn_core / rgbac_winattn_core_bwd + rgbac_relpos_bwd
  GaussFn     rgbac_gaussian_slice / rgbac_gaussian_bwd
  EBFn        rgbac_eb_forward / rgbac_eb_bwd
  MSEFn       rgbac_finalize / rgbac_mse_bwd
  CatFn, ToNCHW   channel concat / layout change (rgbac_channel_copy, layout kernels)

Tensors crossing Function boundaries are NHWC (B, H, W, ldc) with zero padding
channels (runtime.Feat).  Weights are repacked each step by ONE gather launch
through an index map computed once per layer (``PackMap``); the map's inverse
scatters the weight-gradient slabs straight into the PyTorch parameter layout.
Parameter-side reparametrisations (GDN beta'/gamma', EntropyBottleneck
softplus/tanh) stay torch autograd on O(#params) tensors.
"""
import ctypes
import os

import torch
from torch.autograd import Function

from . import _lib
from . import runtime as rt
from .runtime import CONV, CONVT_S2, SUBPEL2, Feat, new_feat, round_up

_F32 = torch.float32


def _stream(t):
    return _lib.stream_ptr(t.device)


# --------------------------------------------------------------------------
# index-map weight packing
# --------------------------------------------------------------------------
def _pack_map(idx_w, mode, segs, stride=1, transposed=False):
    """Run runtime.PackedConv over a weight of (flat index + 1) values: the packed
    buffer then holds, per slot, 1 + the source element it takes (0 = zero pad)."""
    pk = rt.PackedConv(idx_w, None, mode, segs, _F32, stride=stride, transposed=transposed)
    idx = (pk.w.round().to(torch.int32) - 1).contiguous()
    return pk, idx


def _inverse(idx, numel, k_pad):
    """param element -> slab position n * k_pad + k of a phase-0 packed map."""
    inv = torch.full((numel,), -1, dtype=torch.int32, device=idx.device)
    flat = idx[0].reshape(-1) if idx.dim() == 3 else idx.reshape(-1)
    pos = torch.nonzero(flat >= 0).squeeze(1)
    inv[flat[pos].long()] = pos.to(torch.int32)
    return inv


class TPack:
    """A packed weight (same fields runtime.prepare reads from a PackedConv),
    refilled from the fp32 parameter by rgbac_weight_gather."""

    def __init__(self, pk, idx, dtype, bias_idx=None):
        self.mode, self.ksize, self.stride = pk.mode, pk.ksize, pk.stride
        self.cin, self.cin_pad, self.cout = pk.cin, pk.cin_pad, pk.cout
        self.cout_pad, self.k_pad = pk.cout_pad, pk.k_pad
        self.idx = idx
        self.bias_idx = bias_idx
        # zero slack behind the last row, as runtime.PackedConv (256-byte K stages)
        n = idx.numel()
        self.w = torch.zeros(n + 128, dtype=dtype, device=idx.device)[:n].view(idx.shape)
        self.bias = torch.zeros(pk.cout_pad, dtype=_F32, device=idx.device)
        self.src = None                # (weight ptr, bias ptr) of the last refresh
        self.token = 0                 # == _PREFETCH[0]: re-gathered by this step's prefetch
        self.gen = -1                  # rt.PARAM_GEN at that prefetch (an optimizer step bumps it)
        self.frag = self.fidx = None   # fragment-major copy (runtime.frag_weights layout)
        self.fcmap = None              # frag 16-byte chunk -> plain-pack chunk (prefetch_packs)
        self._chunks = False           # strided-chunk form of the map (chunk_form), once built

    def enable_frag(self):
        """Also gather the fragment-major copy the conv_fpatch / conv_npatch tiles read
        (runtime.frag_weights' layout, built here from the index map: the same permutation
        of slots), refreshed with the plain pack every step -- so the training convs can take
        the forward's fragment-streamed tiles."""
        nph, rows, _ = self.idx.shape
        taps = 9 if self.mode == CONVT_S2 else self.ksize * self.ksize
        cp, c32 = self.cin_pad, round_up(self.cin_pad, 32)
        w = self.idx[:, :, :taps * cp].reshape(nph, rows, taps, cp)
        wt = torch.full((nph, rows, taps, c32), -1, dtype=torch.int32, device=self.idx.device)
        wt[..., :cp] = w
        nks = taps * c32 // 32
        self.fidx = wt.reshape(nph, rows // 16, 16, nks, 4, 8).permute(0, 1, 3, 4, 2, 5).contiguous()
        self.frag = torch.zeros(self.fidx.shape, dtype=self.w.dtype, device=self.idx.device)
        # the same permutation applied to the PLAIN pack's positions: every 8-element run of
        # the fragment-major copy is one 16-byte chunk of the plain pack (cin_pad and k_pad are
        # multiples of 8), so prefetch_packs copies chunks from the just-gathered plain pack
        pos = torch.arange(self.idx.numel(), dtype=torch.int64, device=self.idx.device)
        pw = pos.reshape(nph, rows, -1)[:, :, :taps * cp].reshape(nph, rows, taps, cp)
        pt = torch.full((nph, rows, taps, c32), -1, dtype=torch.int64, device=self.idx.device)
        pt[..., :cp] = pw
        first = pt.reshape(nph, rows // 16, 16, nks, 4, 8).permute(0, 1, 3, 4, 2, 5)[..., 0]
        self.fcmap = torch.where(first >= 0, first // 8, -1).to(torch.int32).contiguous().reshape(-1)
        self.src = None                # gather both at the next refresh
        return self

    def chunk_form(self):
        """(cmap, stride, fmap) for rgbac_weight_repack_multi, or None when the map is not of
        that form: every 8-element chunk of the bf16 pack is a prefix of 1..8 real elements
        base + j * stride of the parameter (one stride per pack) followed by padding.  fmap:
        plain chunk -> fragment-major chunk (the inverse of fcmap), or None without a frag
        copy."""
        if self._chunks is not False:
            return self._chunks
        self._chunks = None
        if self.w.dtype != torch.bfloat16 or self.idx.numel() % 8:
            return None
        v = self.idx.reshape(-1, 8).to(torch.int64)
        dev = v.device
        valid = v >= 0
        nv = valid.sum(1)
        j = torch.arange(8, device=dev)
        if not bool((valid == (j[None, :] < nv[:, None])).all()):
            return None
        first = v[:, 0]
        multi = nv >= 2
        stride = 1
        if bool(multi.any()):
            d = (v[:, 1] - v[:, 0])[multi]
            stride = int(d[0])
            if stride <= 0 or not bool((d == stride).all()):
                return None
        if not bool(torch.where(valid, v == first[:, None] + j[None, :] * stride, True).all()):
            return None
        if int(first.max()) >= (1 << 28):
            return None
        cmap = torch.where(nv > 0, first | ((nv - 1).clamp(min=0) << 28),
                           torch.full_like(first, -1)).to(torch.int32).contiguous()
        fmap = None
        if self.frag is not None:
            fc = self.fcmap.to(torch.int64)
            sel = fc >= 0
            if int(torch.unique(fc[sel]).numel()) != int(sel.sum()):
                return None
            fmap = torch.full((cmap.numel(),), -1, dtype=torch.int32, device=dev)
            fmap[fc[sel]] = torch.arange(fc.numel(), device=dev, dtype=torch.int32)[sel]
        self._chunks = (cmap, stride, fmap)
        return self._chunks

    def refresh(self, weight, bias=None):
        # re-gathered every training step: the optimizer kernel updates parameters in
        # place through raw pointers (no autograd version bump).  prefetch_packs() does
        # all of a model's packs in one launch at the start of the step's forward; a pack
        # it covered (same source pointers) is not gathered again in that step.
        w = weight.detach()
        assert w.dtype == _F32 and w.is_contiguous()
        src = (w.data_ptr(), None if bias is None else bias.detach().data_ptr())
        if self.token == _PREFETCH[0] and self.gen == rt.PARAM_GEN and self.src == src:
            return self
        self.src = src
        dev = w.device
        _lib.call("rgbac_weight_gather", _lib.dtype_code(self.w.dtype), self.w.numel(),
                  w.data_ptr(), self.idx.data_ptr(), self.w.data_ptr(), _lib.stream_ptr(dev))
        if self.frag is not None:
            _lib.call("rgbac_weight_gather", _lib.dtype_code(self.frag.dtype), self.frag.numel(),
                      w.data_ptr(), self.fidx.data_ptr(), self.frag.data_ptr(),
                      _lib.stream_ptr(dev))
        if bias is not None:
            b = bias.detach()
            _lib.call("rgbac_weight_gather", _lib.F32, self.bias.numel(), b.data_ptr(),
                      self.bias_idx.data_ptr(), self.bias.data_ptr(), _lib.stream_ptr(dev))
        return self


PREFETCH = os.environ.get("RGBAC_PACK_PREFETCH", "1") != "0"
# RGBAC_REPACK_CHUNKS=0: the element gather + chunk copy pair for every pack (A/B switch)
REPACK_CHUNKS = os.environ.get("RGBAC_REPACK_CHUNKS", "1") != "0"
_GATHER_COPY16 = 16          # rgbac_weight_gather_multi task dtype: 16-byte chunk copy
_PREFETCH = [1]              # current prefetch token (TPack.token == it: gathered this step)
_TASKS = {}


def prefetch_packs(model):
    """Re-gather every training weight pack of ``model`` (forward and input-gradient packs
    of all layers, + their biases) in ONE rgbac_weight_gather_multi launch, instead of one
    gather launch per pack (~420 per RGB training step).  Packs appear on the first step
    (its per-layer refreshes record their sources); from then on each step's forward calls
    this first."""
    if not PREFETCH:
        return
    _PREFETCH[0] += 1
    packs = []
    for m in model.modules():
        for tc in m.__dict__.get("_rgbac_train", {}).values():
            packs.extend(tc._fw.values())
            packs.extend(tc._bw.values())
    # only packs of the model's own parameters: a weight computed in the forward (GDN's
    # reparametrised gamma/beta) does not exist yet at this point of the step
    pset = {p.data_ptr() for p in model.parameters()}
    packs = [tp for tp in packs if tp.src is not None and tp.src[0] in pset and
             (tp.src[1] is None or tp.src[1] in pset)]
    if not packs:
        return
    key = tuple((id(tp), tp.src) for tp in packs)
    ent = _TASKS.get(id(model))
    if ent is None or ent[0] != key:
        if torch.cuda.is_current_stream_capturing():
            return                     # no host->device table upload inside a graph capture
        # the bf16 packs whose maps are strided 8-element chunks (all of the RGB model's): ONE
        # rgbac_weight_repack_multi launch writes each plain pack and its fragment-major copy
        # from one int32 per chunk.  The rest (biases, fp32 packs, other maps): element gathers
        # from the fp32 parameters, then the fragment-major copies as 16-byte chunk copies of
        # the plain packs just written.
        rrows, rblk0 = [], [0]
        rows, blk0, crows, cblk0 = [], [0], [], [0]
        keep = []
        for tp in packs:
            cf = tp.chunk_form() if REPACK_CHUNKS else None
            if cf is not None:
                cmap, stride, fmap = cf
                n = cmap.numel()
                rrows.append([tp.src[0], cmap.data_ptr(), tp.w.data_ptr(), n, stride,
                              0 if fmap is None else fmap.data_ptr(),
                              0 if fmap is None else tp.frag.data_ptr(), 0])
                rblk0.append(rblk0[-1] + -(-n // 256))          # 256 chunks per block
                keep.append(cf)
            for dst, idx, sp, dt in ((None if cf is not None else tp.w, tp.idx, tp.src[0],
                                      _lib.dtype_code(tp.w.dtype)),
                                     (tp.bias, tp.bias_idx, tp.src[1], _lib.F32)):
                if sp is None or idx is None or dst is None or dst.numel() == 0:
                    continue
                n = dst.numel()
                rows.append([sp, idx.data_ptr(), dst.data_ptr(), n, dt])
                blk0.append(blk0[-1] + -(-n // 2048))
            if cf is None and tp.frag is not None and tp.frag.numel():
                n = tp.fcmap.numel()
                crows.append([tp.w.data_ptr(), tp.fcmap.data_ptr(), tp.frag.data_ptr(), n,
                              _GATHER_COPY16])
                cblk0.append(cblk0[-1] + -(-n // 2048))
        dev = packs[0].w.device
        launches = []
        for fn, rr, bb in (("rgbac_weight_repack_multi", rrows, rblk0),
                           ("rgbac_weight_gather_multi", rows, blk0),
                           ("rgbac_weight_gather_multi", crows, cblk0)):
            if rr:
                launches.append((fn, torch.tensor(rr, dtype=torch.int64, device=dev),
                                 torch.tensor(bb, dtype=torch.int64, device=dev), len(rr), bb[-1]))
        ent = (key, launches, keep)
        _TASKS[id(model)] = ent
    for fn, tasks, b0, ntask, nblk in ent[1]:
        _lib.call(fn, ntask, tasks.data_ptr(), b0.data_ptr(), nblk, _lib.stream_ptr(tasks.device))
    for tp in packs:
        tp.token, tp.gen = _PREFETCH[0], rt.PARAM_GEN


class TrainConv:
    """Packing maps of one layer for the training path.

    kind: 'conv' (Conv2d / Linear as 1x1), 'convt' (ConvTranspose2d k5 s2 p2 op1 or
    k1), 'subpel' (compressai subpel_conv3x3's conv, PixelShuffle(2) in the store),
    'gdn' (the 1x1 gamma' conv of GDN on x^2).  ``segs``: [(real, padded)] channel
    segments of the sources (conv-like kinds) or of the convT input."""

    def __init__(self, kind, wshape, stride, segs, device):
        self.kind, self.stride, self.segs = kind, stride, list(segs)
        self.wshape = tuple(wshape)
        numel = 1
        for d in wshape:
            numel *= d
        self.numel = numel
        w4 = self.wshape if len(wshape) == 4 else (wshape[0], wshape[1], 1, 1)
        k = w4[2]
        self.ksize = k
        base = (torch.arange(numel, device=device, dtype=_F32) + 1).reshape(w4)
        if kind == "convt":
            cin_t, cout_t = w4[0], w4[1]
            out_segs = [(cout_t, round_up(cout_t, 8))]
            if k == 1:
                self.fwd = _pack_map(base, CONV, segs, transposed=True)
            else:
                assert k == 5 and stride == 2
                self.fwd = _pack_map(base, CONVT_S2, segs, stride=2)
            # input gradient: conv of dY with W_t viewed as (cout = cin_t, cin = cout_t)
            self.bwd = [_pack_map(base, CONV, out_segs, stride=1 if k == 1 else 2)]
            wg = self.bwd[0]
            self.cout = cout_t
            self.rows = cin_t
        else:
            cout, cin = w4[0], w4[1]
            mode = SUBPEL2 if kind == "subpel" else CONV
            self.fwd = _pack_map(base, mode, segs, stride=stride)
            g_segs = [(cout, round_up(cout, 8))]
            self.bwd = []
            col = 0
            for real, padded in segs:
                sub = base[:, col:col + real]
                col += real
                if stride == 1:
                    t = sub.transpose(0, 1).flip(2, 3).contiguous()
                    self.bwd.append(_pack_map(t, CONV, g_segs))
                else:
                    # stride-2 conv: input gradient = ConvTranspose(k5, s2, p2, op1); a 3x3
                    # (pad 1) kernel is embedded in the 5x5 frame (same output geometry)
                    if k == 3:
                        t = torch.zeros((cout, real, 5, 5), device=device)
                        t[:, :, 1:4, 1:4] = sub
                        sub = t
                    assert sub.shape[2] == 5
                    self.bwd.append(_pack_map(sub.contiguous(), CONVT_S2, g_segs, stride=2))
            wg = self.fwd
            self.cout = cout
            self.rows = cout
        pkw, idxw = wg
        self.wg_kpad = pkw.k_pad
        self.wg_map = _inverse(idxw, numel, pkw.k_pad)      # param element -> slab slot
        self.wg_fmap = idxw[0].contiguous()                  # slab slot -> param element
        self.bias_idx = {}
        self._fw = {}
        self._bw = {}

    def _bidx(self, pk, nreal):
        key = (pk.cout_pad, nreal)
        if key not in self.bias_idx:
            b = torch.full((pk.cout_pad,), -1, dtype=torch.int32, device=self.wg_map.device)
            b[:nreal] = torch.arange(nreal, dtype=torch.int32, device=b.device)
            self.bias_idx[key] = b
        return self.bias_idx[key]

    def fwd_pack(self, dtype, weight, bias):
        tp = self._fw.get(dtype)
        if tp is None:
            pk, idx = self.fwd
            nb = self.cout if self.kind != "subpel" else pk.cout
            tp = TPack(pk, idx, dtype, self._bidx(pk, nb))
            if _frag_eligible(tp):
                tp.enable_frag()
            self._fw[dtype] = tp
        return tp.refresh(weight, bias)

    def bwd_pack(self, i, dtype, weight):
        tp = self._bw.get((i, dtype))
        if tp is None:
            pk, idx = self.bwd[i]
            tp = TPack(pk, idx, dtype)
            if _frag_eligible(tp):
                tp.enable_frag()
            self._bw[(i, dtype)] = tp
        return tp.refresh(weight, None)


# RGBAC_TRAIN_FRAG=0: training packs without the fragment-major copy (plain-layout tiles only)
TRAIN_FRAG = os.environ.get("RGBAC_TRAIN_FRAG", "1") != "0"


def _frag_eligible(tp):
    """Packs the fragment-streamed tiles can take: bf16, 3x3 stride-1 conv / subpel conv, or
    the 5x5/s2 ConvTranspose (runtime._patch_tiles, _npatch_ok)."""
    return (TRAIN_FRAG and tp.w.dtype == torch.bfloat16 and
            ((tp.mode in (CONV, SUBPEL2) and tp.ksize == 3 and tp.stride == 1) or
             tp.mode == CONVT_S2))


def train_conv_of(m, kind, wshape, stride, segs, device):
    key = (kind, tuple(segs), tuple(wshape))
    cache = m.__dict__.setdefault("_rgbac_train", {})
    tc = cache.get(key)
    if tc is None:
        tc = TrainConv(kind, wshape, stride, segs, device)
        cache[key] = tc
    return tc


# --------------------------------------------------------------------------
# weight gradient (rgbac_conv_wgrad + rgbac_wgrad_reduce)
# --------------------------------------------------------------------------
_SLAB_FLOATS = 16 << 20         # cap of nsplit * n_pad * k_pad (64 MiB of fp32 partials)


WGRAD_BIG = os.environ.get("RGBAC_WGRAD_BIG", "1") != "0"


def wgrad_tile(dtype, n_pad, k_pad, square):
    """(output tiles per pixel split, workgroups wanted in flight) of rgbac_conv_wgrad -- the
    tile rule of csrc/train.hip: 128 x 256 tiles (512 threads, one workgroup per CU) when bf16,
    no squared input, n_pad >= 128 and k_pad >= 512; otherwise counted in 64 x 64 units with
    ~1024 workgroups wanted (the 64 x 64 / 64 x 128 tiles run two workgroups per CU)."""
    if dtype == torch.bfloat16 and not square and n_pad >= 128 and k_pad >= 512 and WGRAD_BIG:
        return -(-k_pad // 256) * -(-n_pad // 128), _WG_TARGET_BIG
    return (k_pad // 64) * (n_pad // 64), _WG_TARGET


# workgroups wanted per weight-gradient launch (A/B knobs: fewer = fewer fp32 slabs to write
# and reduce, more = more CUs busy)
_WG_TARGET_BIG = int(os.environ.get("RGBAC_WGRAD_TARGET_BIG", "256"))
_WG_TARGET = int(os.environ.get("RGBAC_WGRAD_TARGET", "1024"))
_WG_CEIL = os.environ.get("RGBAC_WGRAD_CEIL", "0") == "1"
_HALO_WG = int(os.environ.get("RGBAC_WGRAD_HALO_WG", "512"))   # stride-1 halo kernel target
_PATCH_PIX = int(os.environ.get("RGBAC_WGRAD_PATCH_PIX", "256"))  # min pixels per patch workgroup


WGRAD_PATCH = os.environ.get("RGBAC_WGRAD_PATCH", "1") != "0"


def wgrad_patch_ok(dtype, gch, S, ksize, stride, pad, square, grid_h, grid_w):
    """csrc/train.hip wgrad_patch_ok: the 8 x 32-pixel patch kernel's shapes (bf16, 3x3
    stride 1 pad 1, one source of whole 32-channel blocks, <= 32 output channels)."""
    s0 = S[0]
    return (WGRAD_PATCH and dtype == torch.bfloat16 and not square and ksize == 3 and
            stride == 1 and pad == 1 and len(S) == 1 and gch <= 32 and s0.ldc % 32 == 0 and
            grid_w % 32 == 0 and grid_h % 8 == 0 and s0.H == grid_h and s0.W == grid_w)


WGRAD_HALO = os.environ.get("RGBAC_WGRAD_HALO", "1") != "0"
WGRAD_S2 = os.environ.get("RGBAC_WGRAD_S2", "1") != "0"


def wgrad_halo_ok(dtype, gch, S, ksize, stride, pad, square, grid_h, grid_w):
    """csrc/train.hip wgrad_halo_ok: 2 / 1 when the halo-staged kernel takes the shape (bf16;
    5x5 stride 2 pad 2, or 3x3 stride 1 pad 1 with more than 32 outputs; the grid 4 x 32-pixel
    patches of the source grid, or of half of it), else 0."""
    s0 = S[0]
    if not (WGRAD_HALO and dtype == torch.bfloat16 and not square and grid_w % 32 == 0 and
            grid_h % 4 == 0):
        return 0
    if (WGRAD_S2 and ksize == 5 and stride == 2 and pad == 2 and s0.H == 2 * grid_h and
            s0.W == 2 * grid_w):
        return 2
    if ksize == 3 and stride == 1 and pad == 1 and gch > 32 and s0.H == grid_h and s0.W == grid_w:
        return 1
    return 0


def _nsplit(tiles, M, slab, target=1024):
    """Pixel splits: enough workgroups to fill the chip (``target``), each split >= 512
    pixels, and the fp32 partial slabs bounded (their write + reduce read is pure overhead)."""
    # floor: never a nearly empty extra round of workgroups (RGBAC_WGRAD_CEIL=1: the ceiling, A/B)
    want = max(1, -(-target // tiles) if _WG_CEIL else target // tiles)
    cap = max(1, _SLAB_FLOATS // slab)
    return int(max(1, min(want, -(-M // 512), cap, 1024)))


# Weight-gradient reductions that add into param.grad (DIRECT_GRAD) are queued and issued
# eight at a time by rgbac_wgrad_reduce_multi -- a reduce launch is a few microseconds of
# mostly fixed cost, ~195 per training step.  The queue is flushed when it is full, before any
# reduction whose result autograd reads (not accumulated into .grad), at the end of the
# backward pass (an engine callback), and by the data-parallel bucket hooks before they
# all-reduce (rgbac.parallel).  Measured neutral on config 3 (49.30 vs 49.25 MPix/s: the
# reductions are bound by their slab reads, not launch cost), so RGBAC_REDUCE_BATCH=1 opts in.
REDUCE_BATCH = os.environ.get("RGBAC_REDUCE_BATCH", "0") == "1"   # measured neutral: off
_PENDING = []                   # (task int64 x 11, keep-alive tensors)
_PENDING_CB = [False]


def flush_reductions():
    """Issue every queued weight-gradient reduction (one launch per 8)."""
    while _PENDING:
        part = _PENDING[:8]
        del _PENDING[:8]
        desc = (ctypes.c_int64 * (11 * len(part)))()
        for i, (task, _) in enumerate(part):
            desc[11 * i: 11 * i + 11] = task
        dev = part[0][1][0].device
        _lib.call("rgbac_wgrad_reduce_multi", len(part), ctypes.addressof(desc),
                  _lib.stream_ptr(dev))


def _end_of_backward():
    _PENDING_CB[0] = False
    flush_reductions()


def _reduce(nslot, fmap, part, nsplit, slab, dw, nbias, bpart, n_pad, db, acc, st):
    # queued reductions are flushed by a callback of the running backward pass: outside one
    # (a weight gradient computed directly, e.g. a test or a custom loop) there is no engine
    # to run the callback, so the reduction goes out immediately
    if not (REDUCE_BATCH and acc) or torch._C._current_graph_task_id() < 0:
        flush_reductions()
        _lib.call("rgbac_wgrad_reduce", nslot, None if fmap is None else fmap.data_ptr(),
                  None if part is None else part.data_ptr(), nsplit, slab,
                  None if dw is None else dw.data_ptr(), nbias,
                  None if bpart is None else bpart.data_ptr(), n_pad,
                  None if db is None else db.data_ptr(), 1 if acc else 0, st)
        return
    keep = [t for t in (part, bpart, fmap, dw, db) if t is not None]
    task = [nslot, 0 if fmap is None else fmap.data_ptr(), 0 if part is None else part.data_ptr(),
            nsplit, slab, 0 if dw is None else dw.data_ptr(), nbias,
            0 if bpart is None else bpart.data_ptr(), n_pad, 0 if db is None else db.data_ptr(), 1]
    _PENDING.append((task, keep))
    if not _PENDING_CB[0]:
        torch.autograd.Variable._execution_engine.queue_callback(_end_of_backward)
        _PENDING_CB[0] = True
    if len(_PENDING) >= 8:
        flush_reductions()


def wgrad(G, S, ksize, stride, pad, square, k_pad, fmap, numel, nbias=0, bias_from_g=True,
          acc_dw=None, acc_db=None):
    """dW (fp32, flat param layout) and optional db from G (Feat on the M grid) and
    sources S [Feat] sampled with (ksize, stride, pad).  ``acc_dw`` / ``acc_db`` (both or
    neither): fp32 tensors the sums are ADDED into instead (param.grad), returned as is."""
    dev = G.t.device
    n_pad = round_up(G.ldc, 64)
    M = G.B * G.H * G.W
    hs = wgrad_halo_ok(G.t.dtype, G.ldc, S, ksize, stride, pad, square, G.H, G.W)
    if hs:
        # workgroups over (32-channel source block, 64-channel output block) pairs: one per CU
        # for stride 2 (136 KiB of LDS), two for stride 1 (58 KiB); each at least 2 patches of
        # 4 x 32 pixels (floor: a workgroup past a full round would run a nearly empty one)
        tiles = -(-sum(f.ldc for f in S) // 32) * -(-G.ldc // 64)
        ns = int(max(1, min((256 if hs == 2 else _HALO_WG) // tiles, M // 256,
                            _SLAB_FLOATS // (n_pad * k_pad))))
    elif wgrad_patch_ok(G.t.dtype, G.ldc, S, ksize, stride, pad, square, G.H, G.W):
        # one workgroup per (32-channel block, run of 8 x 32-pixel patches): <= 512 in flight
        # (two per CU); small grids (32^2 latents) take one patch per workgroup -- more
        # workgroups beat the double-buffered staging overlap there (RGBAC_WGRAD_PATCH_PIX A/B)
        tiles = S[0].ldc // 32
        ns = int(max(1, min(512 // tiles, M // _PATCH_PIX, _SLAB_FLOATS // (n_pad * k_pad))))
    else:
        tiles, target = wgrad_tile(G.t.dtype, n_pad, k_pad, square)
        ns = _nsplit(tiles, M, n_pad * k_pad, target)
    part = torch.empty(ns * n_pad * k_pad, dtype=_F32, device=dev)
    bpart = None
    if nbias and bias_from_g:
        bpart = torch.empty(ns * n_pad, dtype=_F32, device=dev)
    a = _lib.WgradArgs()
    a.dtype = _lib.dtype_code(G.t.dtype)
    a.batch, a.grid_h, a.grid_w = G.B, G.H, G.W
    a.g, a.g_ldc, a.g_channels = G.ptr(), G.ldc, G.ldc
    s0 = S[0]
    a.in_h, a.in_w, a.ksize, a.stride, a.pad = s0.H, s0.W, ksize, stride, pad
    a.nsrc = len(S)
    cin = 0
    for i, f in enumerate(S):
        assert f.t.dtype == G.t.dtype and f.B == G.B
        a.src[i].ptr, a.src[i].ldc, a.src[i].channels = f.ptr(), f.ldc, f.ldc
        cin += f.ldc
    a.cin_pad = cin
    a.square_input = 1 if square else 0
    a.n_pad, a.k_pad, a.nsplit = n_pad, k_pad, ns
    a.partial = part.data_ptr()
    a.bias_partial = None if bpart is None else bpart.data_ptr()
    st = _stream(G.t)
    # the launched form's rocprof name (the C side's choice, restated), so the bench's
    # per-kernel table and training roofline keep the forms apart
    if hs:
        kname = f"wgrad_halo_kernel<{hs}>"
    elif wgrad_patch_ok(G.t.dtype, G.ldc, S, ksize, stride, pad, square, G.H, G.W):
        kname = f"wgrad_patch_kernel<{2 if G.ldc > 16 else 1}>"
    elif G.t.dtype == torch.bfloat16 and not square and n_pad >= 128 and k_pad >= 512 and \
            WGRAD_BIG:
        kname = "wgrad_ring_kernel<4, 4, 3, 2, 4>"
    elif G.t.dtype == torch.bfloat16 and not square:
        kname = "wgrad_ring_kernel"
    else:
        kname = "wgrad_kernel"
    rt.timed(kname, 2.0 * M * G.ldc * ksize * ksize * cin,
             G.t.element_size() * M * (G.ldc + cin * ksize * ksize // max(1, stride * stride)),
             lambda: _lib.call("rgbac_conv_wgrad", ctypes.byref(a), st),
             f"{kname} k{ksize}s{stride} G{G.ldc}@{G.H}x{G.W} S{cin}@{s0.H}x{s0.W} "
             f"B{G.B} split{ns}{' sq' if square else ''}")
    acc = acc_dw is not None
    dw = acc_dw if acc else torch.empty(numel, dtype=_F32, device=dev)
    db = acc_db if acc else (torch.empty(nbias, dtype=_F32, device=dev) if nbias else None)
    assert not acc or (dw.numel() == numel and dw.is_contiguous() and
                       (not nbias or (db is not None and db.numel() == nbias)))
    if nbias and not bias_from_g:
        raise ValueError("use colsum for biases not on G")
    nslot = min(fmap.shape[0], n_pad) * k_pad
    _reduce(nslot, fmap, part, ns, n_pad * k_pad, dw, nbias if bpart is not None else 0, bpart,
            n_pad, db, acc, st)
    return dw, db


def colsum(f, C, acc=None):
    """Per-channel sum over pixels of Feat ``f`` (first C channels) -> fp32 (C,) (added into
    ``acc`` instead when given)."""
    dev = f.t.device
    npix = f.B * f.H * f.W
    ns = int(max(1, min(1024, -(-npix // 256))))
    part = torch.empty(ns * C, dtype=_F32, device=dev)
    st = _stream(f.t)
    _lib.call("rgbac_colsum", _lib.dtype_code(f.t.dtype), npix, C, f.ptr(), f.ldc, ns,
              part.data_ptr(), st)
    db = acc if acc is not None else torch.empty(C, dtype=_F32, device=dev)
    _reduce(0, None, None, ns, 1, None, C, part, C, db, acc is not None, st)
    return db


# --------------------------------------------------------------------------
# ConvFn
# --------------------------------------------------------------------------
_NEEDS_Z = {"gelu", "relu", "lrelu", "tanh_half", "gate", "gdn", "igdn"}


class ConvCall:
    """Non-tensor description of one training conv (ctx of ConvFn).  ``defer``: the conv
    returns (z, act(z)) and leaves its activation backward to its consumer; ``src_act`` /
    ``src_param``: this conv's source is such a deferred output -- its input-gradient conv
    applies the producer's activation backward in its epilogue (DGELU / DLRELU)."""
    __slots__ = ("tc", "src_C", "act", "act_param", "square", "defer", "src_act", "src_param",
                 "sink", "src_sinks", "res_sinks", "zsink")

    def __init__(self, tc, src_C, act, act_param, square=False, defer=False, src_act=None,
                 src_param=0.0):
        self.tc, self.src_C, self.act, self.act_param = tc, list(src_C), act, act_param
        self.square, self.defer, self.src_act, self.src_param = square, defer, src_act, src_param
        # gradient sinks: of this conv's output, of its sources / residual operands / folded
        # producer (rgbac.autograd.Sink)
        self.sink, self.src_sinks, self.res_sinks, self.zsink = None, (), (None,) * 3, None


class ActFeat(Feat):
    """Output of a deferred-activation conv (``conv_t(..., defer=True)``): ``t`` = act(z)
    (not autograd-tracked), ``pre`` = z (tracked).  Only a single-source ``conv_t`` may
    consume it: that conv routes the gradient to ``pre`` through its input-gradient
    epilogue, so the act_bwd pass (dy and z read, dL/dz written) never runs."""
    __slots__ = ("pre", "dact", "dparam")

    def __init__(self, t, C, pre, dact, dparam):
        super().__init__(t, C)
        self.pre, self.dact, self.dparam = pre, dact, dparam


# the DGELU epilogue takes act_bwd's bf16 derivative (the fast form); RGBAC_GELU_BWD_EXACT=1
# (act_bwd's exact-erfc A/B switch) therefore also keeps the activation backward unfolded
DEFER_ACT = (os.environ.get("RGBAC_DEFER_ACT", "1") != "0" and
             os.environ.get("RGBAC_GELU_BWD_EXACT", "0") in ("", "0"))
_DEFERRABLE = {"gelu": "dgelu", "relu": "dlrelu", "lrelu": "dlrelu"}


def _act_bwd(act, slope, dy, z, r1, sel, C, want_r1):
    dev = dy.t.device
    dz = Feat(torch.empty_like(dy.t), C)
    dr1 = Feat(torch.empty_like(dy.t), C) if want_r1 else None
    npix = dy.B * dy.H * dy.W
    _lib.call("rgbac_act_bwd", _lib.dtype_code(dy.t.dtype), _lib.ACT[act], slope, npix, C,
              dy.ptr(), dy.ldc, None if z is None else z.ptr(), 0 if z is None else z.ldc,
              None if r1 is None else r1.ptr(), 0 if r1 is None else r1.ldc,
              _lib.ptr(sel), dz.ptr(), dz.ldc, None if dr1 is None else dr1.ptr(),
              0 if dr1 is None else dr1.ldc, _lib.stream_ptr(dev))
    return dz, dr1


DIRECT_GRAD = [True]


def _direct_grad(p):
    """p.grad when weight-gradient sums may be added into it in place: a leaf parameter
    whose .grad is an attached fp32 contiguous tensor of its shape."""
    if not DIRECT_GRAD[0] or p is None or not p.is_leaf or not p.requires_grad:
        return None
    g = p.grad
    if g is None or g.dtype != _F32 or not g.is_contiguous() or g.shape != p.shape:
        return None
    return g


class GdnReparamFn(torch.autograd.Function):
    """GDN / IGDN beta' = LowerBound(beta, beta_bound)^2 - pedestal and gamma' likewise
    (layers/GDN.py:9-23, 71-78) as one HIP launch forward (rgbac_gdn_reparam) and one
    backward (rgbac_gdn_reparam_bwd, LowerBound's pass-through rule), bit-identical to the
    torch graph of the reference's LowerBound Function, ``** 2`` and ``- pedestal``.  With an
    attached fp32 .grad (AdamClamp) the backward adds into it and hands autograd None (as the
    conv weight gradients do, DIRECT_GRAD)."""

    @staticmethod
    def forward(ctx, beta, gamma, beta_bound, gamma_bound, pedestal):
        b, g = beta.detach(), gamma.detach()
        assert b.dtype == _F32 and g.dtype == _F32 and b.is_contiguous() and g.is_contiguous()
        bo, go = torch.empty_like(b), torch.empty_like(g)
        _lib.call("rgbac_gdn_reparam", b.numel(), g.numel(), b.data_ptr(), g.data_ptr(),
                  float(beta_bound), float(gamma_bound), float(pedestal), bo.data_ptr(),
                  go.data_ptr(), _lib.stream_ptr(b.device))
        ctx.save_for_backward(beta, gamma)
        ctx.bounds = (float(beta_bound), float(gamma_bound))
        return bo, go

    @staticmethod
    def backward(ctx, dbo, dgo):
        beta, gamma = ctx.saved_tensors
        need_b, need_g = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        acc_b = _direct_grad(beta) if need_b else None
        acc_g = _direct_grad(gamma) if need_g else None
        direct = acc_b is not None and acc_g is not None
        db = acc_b if direct else torch.empty_like(beta)
        dg = acc_g if direct else torch.empty_like(gamma)
        dbo = None if dbo is None else dbo.contiguous()
        dgo = None if dgo is None else dgo.contiguous()
        _lib.call("rgbac_gdn_reparam_bwd", beta.numel(), gamma.numel(), beta.data_ptr(),
                  gamma.data_ptr(), ctx.bounds[0], ctx.bounds[1], _lib.ptr(dbo), _lib.ptr(dgo),
                  db.data_ptr(), dg.data_ptr(), 1 if direct else 0, _lib.stream_ptr(beta.device))
        if direct:
            return None, None, None, None, None
        return (db if need_b else None), (dg if need_g else None), None, None, None


class EbParamsFn(torch.autograd.Function):
    """The EntropyBottleneck parameter block of rgbac_eb_forward / rgbac_eb_bwd ([C][64]:
    softplus(_matrix0..4) | _bias0..4 | tanh(_factor0..3) | median | 0 pad; compressai
    EntropyBottleneck, filters (3, 3, 3, 3)) from the 15 raw parameters in one HIP launch
    (rgbac_eb_params), and its backward in one (rgbac_eb_params_bwd: softplus / tanh
    derivatives, added straight into attached fp32 .grad tensors as DIRECT_GRAD does)."""

    @staticmethod
    def forward(ctx, C, *params):
        ps = [t.detach() for t in params]
        assert len(ps) == 15 and all(t.dtype == _F32 and t.is_contiguous() for t in ps)
        out = torch.empty((C, 64), dtype=_F32, device=ps[0].device)
        arr = (ctypes.c_void_p * 15)(*[t.data_ptr() for t in ps])
        _lib.call("rgbac_eb_params", C, ctypes.cast(arr, ctypes.c_void_p), out.data_ptr(),
                  _lib.stream_ptr(out.device))
        ctx.C = C
        ctx.save_for_backward(*params)
        return out

    @staticmethod
    def backward(ctx, dout):
        params = ctx.saved_tensors
        if dout is None:
            return (None,) * 16
        accs = [_direct_grad(t) if ctx.needs_input_grad[1 + i] else None
                for i, t in enumerate(params)]
        direct = all(a is not None for a in accs)
        if direct:
            grads = accs
        else:
            grads = [torch.empty_like(t) for t in params[:14]] + [torch.zeros_like(params[14])]
        dout = dout.contiguous()
        pa = (ctypes.c_void_p * 15)(*[t.data_ptr() for t in params])
        ga = (ctypes.c_void_p * 15)(*[g.data_ptr() for g in grads])
        _lib.call("rgbac_eb_params_bwd", ctx.C, ctypes.cast(pa, ctypes.c_void_p), dout.data_ptr(),
                  ctypes.cast(ga, ctypes.c_void_p), 1 if direct else 0, _lib.stream_ptr(dout.device))
        if direct:
            return (None,) * 16
        return (None, *[g if ctx.needs_input_grad[1 + i] else None for i, g in enumerate(grads)])


class Sink:
    """Gradient buffer of one autograd-tracked training activation (a ConvFn / CatFn output).
    Consumers that know the protocol (ConvFn sources and residual operands, CatFn parts) add
    their gradient here and hand autograd None; the producer's backward takes the buffer (plus
    whatever ordinary gradient autograd still delivers from other consumers).  A multiply-used
    activation -- the slice supports used by up to 11 concatenations, every residual-unit and
    attention-block input -- then costs no autograd add: the first deposit adopts the tensor,
    later ones accumulate inside the input-gradient conv's epilogue (res0 = the buffer) or the
    concatenation split's copy (rgbac_channel_copy_multi_ex).  autograd still runs the
    producer after every consumer (its dependency count does not depend on the values)."""
    __slots__ = ("buf", "own", "slices")

    def __init__(self):
        # slices: the buffer holds only disjoint channel slices written so far (GaussFn),
        # so another slice may be written into it without an add
        self.buf, self.own, self.slices = None, False, False


GRAD_SINKS = os.environ.get("RGBAC_GRAD_SINKS", "1") != "0"


def _sink(t):
    return getattr(t, "_rgbac_sink", None) if (GRAD_SINKS and t is not None) else None


def _deposit(sink, g, own):
    """sink += g.  own: g is a fresh tensor nobody else holds (adoptable, accumulable)."""
    sink.slices = False
    if sink.buf is None:
        sink.buf, sink.own = g, own
    elif sink.own:
        sink.buf.add_(g)
    else:
        sink.buf, sink.own = sink.buf + g, True


def _take(sink, g):
    """The producer's output gradient: its sink plus the gradient autograd delivered."""
    if sink is None or sink.buf is None:
        return g
    if g is None:
        return sink.buf
    return sink.buf + g


class ConvFn(Function):
    @staticmethod
    def forward(ctx, call, weight, bias, res0, res1, res2, sel, zsrc, *srcs):
        tc = call.tc
        dt = srcs[0].dtype
        feats = [Feat(t, c) for t, c in zip(srcs, call.src_C)]
        pk = tc.fwd_pack(dt, weight.contiguous(), bias)
        f0 = feats[0]
        if tc.kind == "convt" and tc.ksize == 5:
            Ho, Wo, Cs = 2 * f0.H, 2 * f0.W, tc.cout
        elif tc.kind == "subpel":
            Ho, Wo, Cs = 2 * f0.H, 2 * f0.W, tc.cout // 4
        else:
            s = tc.stride
            p = tc.ksize // 2
            Ho = (f0.H + 2 * p - tc.ksize) // s + 1
            Wo = (f0.W + 2 * p - tc.ksize) // s + 1
            Cs = tc.cout
        out = new_feat(f0.B, Ho, Wo, Cs, dt, f0.t.device)
        z = new_feat(f0.B, Ho, Wo, Cs, dt, f0.t.device) if call.act in _NEEDS_Z else None

        def rf(r):
            return None if r is None else Feat(r, Cs)
        pr = rt.prepare(pk, [f.src() for f in feats], out=out, act=call.act,
                        act_param=call.act_param, res0=rf(res0), res1=rf(res1), res2=rf(res2),
                        sel=sel, square=call.square, bias=bias is not None, zout=z)
        rt.launch([pr])
        ctx.call = call
        ctx.bias_param = bias if (bias is not None and bias.is_leaf) else None
        ctx.has = (bias is not None, res0 is not None, res1 is not None, res2 is not None)
        ctx.shape = (f0.B, Ho, Wo, Cs)
        keep_r1 = res1 if call.act in ("gate", "gdn", "igdn") else None
        ctx.save_for_backward(weight, None if (z is None or call.defer) else z.t, keep_r1, sel,
                              zsrc, *srcs)
        if sel is not None:
            ctx.mark_non_differentiable(sel)
        ctx.set_materialize_grads(False)
        if call.defer:
            ctx.mark_non_differentiable(out.t)
            return z.t, out.t
        return out.t

    @staticmethod
    def backward(ctx, dy_t, *_):
        call = ctx.call
        tc = call.tc
        weight, z_t, r1_t, sel, zsrc, *srcs = ctx.saved_tensors
        has_b, has0, has1, has2 = ctx.has
        B, Ho, Wo, Cs = ctx.shape
        dy_t = _take(call.sink, dy_t)
        if dy_t is None:                              # no consumer contributed a gradient
            return (None,) * (8 + len(srcs))
        dy = Feat(dy_t.contiguous(), Cs)
        dt = dy.t.dtype
        act = call.act
        z = None if z_t is None else Feat(z_t, Cs)
        r1 = None if r1_t is None else Feat(r1_t, Cs)
        if act == "none" or call.defer:
            # deferred: dy_t is already dL/dz (the consumer's input-gradient epilogue applied
            # this conv's activation backward)
            dz, dr1 = dy, None
        else:
            dz, dr1 = _act_bwd(act, call.act_param, dy, z, r1, sel, Cs,
                               act in ("gate", "gdn", "igdn"))
        g_res0 = dz.t if has0 else None
        g_res1 = None
        if has1:
            if act in ("tanh_half", "masksel"):
                g_res1 = dy.t
            elif act in ("gate", "igdn", "gdn") and not call.square:
                g_res1 = dr1.t
        g_res2 = dy.t if has2 else None
        # residual gradients into their operands' sinks; a tensor is adopted by at most one
        # sink, and dy (autograd's or this conv's own sink buffer) never
        adopted = set()
        res_g = [g_res0, g_res1, g_res2]
        for j, sk in enumerate(call.res_sinks):
            if sk is not None and res_g[j] is not None:
                g = res_g[j]
                own = g is not dy.t and id(g) not in adopted
                if own:
                    adopted.add(id(g))
                _deposit(sk, g, own)
                res_g[j] = None
        g_res0, g_res1, g_res2 = res_g
        feats = [Feat(t, c) for t, c in zip(srcs, call.src_C)]
        # the conv's own output-gradient grid
        if tc.kind == "subpel":
            f0 = feats[0]
            G = new_feat(B, f0.H, f0.W, tc.cout, dt, dy.t.device)
            _lib.call("rgbac_pixel_shuffle", _lib.dtype_code(dt), 1, B, f0.H, f0.W, Cs,
                      dz.ptr(), dz.ldc, G.ptr(), G.ldc, _lib.stream_ptr(dy.t.device))
        else:
            G = dz
        need = ctx.needs_input_grad
        # ---- input gradients (one grouped launch over the sources)
        g_srcs = [None] * len(srcs)
        g_zsrc = None
        preps = []
        idxs = []
        sinks_in = []
        targeted = set()            # sinks this launch already accumulates into in place
        for i, f in enumerate(feats):
            folded = call.src_act is not None and i == 0
            if not (need[7] if folded else need[8 + i]):
                continue
            sk = call.zsink if folded else (call.src_sinks[i] if call.src_sinks else None)
            pk = tc.bwd_pack(i, dt, weight.detach().contiguous())
            if call.square:
                o = new_feat(f.B, f.H, f.W, f.C, dt, f.t.device)   # zero-filled iff padded
                preps.append(rt.prepare(pk, [G.src()], out=o, act="sqbwd", res0=dr1,
                                        res1=f, bias=False))
            elif folded:
                # dL/dz of the producer = (W^T G) * act'(z): its activation backward here
                o = new_feat(f.B, f.H, f.W, f.C, dt, f.t.device)
                preps.append(rt.prepare(pk, [G.src()], out=o, act=call.src_act,
                                        act_param=call.src_param, res0=Feat(zsrc, f.C),
                                        bias=False))
            elif sk is not None and sk.buf is not None and id(sk) not in targeted:
                # accumulate in the epilogue: out = W^T G + buffer (in place when the buffer
                # is ours -- every element is read and written by the same lane -- and not an
                # operand of this very launch).  Only ONE group of a launch may target a sink:
                # a tensor used as two sources of one conv would otherwise have two groups
                # read-modify-write the same buffer concurrently; later ones take the plain
                # branch (fresh output, deposited after the launch)
                targeted.add(id(sk))
                prev = Feat(sk.buf, f.C)
                inplace = sk.own and all(sk.buf is not t for t in (G.t, dz.t, dy.t))
                o = prev if inplace else new_feat(f.B, f.H, f.W, f.C, dt, f.t.device)
                preps.append(rt.prepare(pk, [G.src()], out=o, res0=prev, bias=False))
                sk.buf, sk.own, sk.slices = o.t, True, False
                sk = None                               # deposited by the launch itself
            else:
                o = new_feat(f.B, f.H, f.W, f.C, dt, f.t.device)
                preps.append(rt.prepare(pk, [G.src()], out=o, bias=False))
            idxs.append(i)
            sinks_in.append(sk)
        if preps:
            outs = rt.launch(preps)
            for i, o, sk in zip(idxs, outs, sinks_in):
                folded = call.src_act is not None and i == 0
                if folded or call.src_sinks:
                    target = call.zsink if folded else call.src_sinks[i]
                    if target is not None:
                        if sk is not None:
                            _deposit(sk, o.t, True)
                        continue                          # (accumulated in place otherwise)
                if folded:
                    g_zsrc = o.t
                else:
                    g_srcs[i] = o.t
        # ---- weight / bias gradients
        g_w = g_b = None
        if need[1] or (has_b and need[2]):
            nb = tc.rows if (has_b and tc.kind != "convt") else 0
            # parameters with an attached fp32 .grad (rgbac.optim.AdamClamp's flat-buffer
            # views): the reduce adds straight into .grad, and autograd gets None -- no
            # per-parameter accumulate launch (DIRECT_GRAD).  autograd still runs the
            # parameter's AccumulateGrad node (with no gradient) once every use of it has
            # been back-propagated, so its post-accumulate hook -- which launches the
            # data-parallel bucket all-reduces (rgbac/parallel.py) -- fires after these adds
            bias_p = ctx.bias_param
            acc_w = _direct_grad(weight) if need[1] else None
            acc_b = _direct_grad(bias_p) if (has_b and need[2]) else None
            direct = acc_w is not None and (not has_b or not need[2] or acc_b is not None)
            if not direct:
                acc_w = acc_b = None
            if tc.kind == "convt":
                # G = the convT input, S = dL/dv on the output grid
                dw, _ = wgrad(feats[0], [dz], tc.ksize, tc.stride if tc.ksize == 5 else 1,
                              tc.ksize // 2, False, tc.wg_kpad, tc.wg_fmap, tc.numel,
                              acc_dw=None if acc_w is None else acc_w.view(-1),
                              acc_db=None)
                db = colsum(dz, tc.cout, acc=acc_b) if has_b else None
            else:
                p = tc.ksize // 2
                dw, db = wgrad(G, feats, tc.ksize, tc.stride, p, call.square, tc.wg_kpad,
                               tc.wg_fmap, tc.numel, nbias=nb,
                               acc_dw=None if acc_w is None else acc_w.view(-1),
                               acc_db=acc_b if nb else None)
            if not direct:
                g_w = dw.view(weight.shape)
                g_b = db
        return (None, g_w, g_b, g_res0, g_res1, g_res2, None, g_zsrc, *g_srcs)


def conv_t(m, srcs, act="none", act_param=0.0, res0=None, res1=None, res2=None, sel=None,
           kind=None, weight=None, bias=None, square=False, defer=False):
    """Training conv of module ``m`` over Feat sources -> Feat (autograd-tracked).
    ``defer=True`` (GELU / (Leaky)ReLU, no post-activation residual): return an ActFeat whose
    only consumer is the next single-source conv_t, which folds this activation's backward
    into its input-gradient conv (RGBAC_DEFER_ACT=0 turns the folding off)."""
    import torch.nn as nn
    dev = srcs[0].t.device
    src_act, src_param, zsrc = None, 0.0, None
    if any(isinstance(f, ActFeat) for f in srcs):
        assert len(srcs) == 1 and not square, "a deferred activation feeds one plain conv"
        f = srcs[0]
        src_act, zsrc = f.dact, f.pre
        src_param = f.dparam
    defer = defer and DEFER_ACT
    if defer:
        assert act in _DEFERRABLE and res1 is None and res2 is None and sel is None \
            and not square and kind != "gdn", "deferrable: GELU / ReLU / LeakyReLU epilogue only"
    segs = [(f.C, f.ldc) for f in srcs]
    w = m.weight if weight is None else weight
    b = getattr(m, "bias", None) if bias is None else bias
    if kind is None:
        if isinstance(m, nn.ConvTranspose2d):
            kind = "convt"
        else:
            kind = "conv"
    stride = m.stride[0] if hasattr(m, "stride") else 1
    if kind == "convt":
        stride = m.stride[0]
    wshape = tuple(w.shape) if w.dim() == 4 else (w.shape[0], w.shape[1], 1, 1)
    tc = train_conv_of(m, kind, wshape, stride, segs, dev)
    call = ConvCall(tc, [f.C for f in srcs], act, act_param, square, defer, src_act, src_param)
    if GRAD_SINKS:
        call.sink = Sink()
        call.src_sinks = tuple(None if isinstance(f, ActFeat) else _sink(f.t) for f in srcs)
        call.res_sinks = tuple(None if r is None else _sink(r.t) for r in (res0, res1, res2))
        call.zsink = _sink(zsrc)
    # the weight goes in with its own shape (ConvFn reads it flat through the pack maps): a
    # Linear's 2-D leaf then takes the DIRECT_GRAD path like a conv's, instead of its reshaped
    # view's gradient reaching .grad through an autograd-engine add
    out = ConvFn.apply(call, w, b, None if res0 is None else res0.t,
                       None if res1 is None else res1.t, None if res2 is None else res2.t,
                       sel, zsrc, *[f.t for f in srcs])
    C = tc.cout // 4 if kind == "subpel" else tc.cout
    if defer:
        z_t, o_t = out
        if call.sink is not None:
            z_t._rgbac_sink = call.sink
        return ActFeat(o_t, C, z_t, _DEFERRABLE[act], act_param if act == "lrelu" else 0.0)
    if call.sink is not None:
        out._rgbac_sink = call.sink
    return Feat(out, C)


# --------------------------------------------------------------------------
# window attention core
# --------------------------------------------------------------------------
_CSR = {}


def _relpos_csr(index, ntab):
    """(offsets, flat (i, j) list) grouping relative_position_index by table row."""
    key = (index.data_ptr(), ntab)
    if key not in _CSR:
        flat = index.reshape(-1).long()
        order = torch.argsort(flat, stable=True)
        counts = torch.bincount(flat, minlength=ntab)
        off = torch.zeros(ntab + 1, dtype=torch.int64, device=index.device)
        off[1:] = torch.cumsum(counts, 0)
        _CSR[key] = (off.to(torch.int32).contiguous(), order.to(torch.int32).contiguous())
    return _CSR[key]


class WinAttnFn(Function):
    """Attention core; ``amask``: explicit additive (nW, N, N) fp32 mask or None
    (WindowAttention.forward(x, mask))."""

    @staticmethod
    def forward(ctx, spec, qkv_t, table, alpha, amask=None):
        C, heads, ws, shift, masked, scale, index = spec
        B, H, W, ldq = qkv_t.shape
        dt = qkv_t.dtype
        dev = qkv_t.device
        with torch.no_grad():
            N = ws * ws
            dense = table.detach()[index.reshape(-1)].reshape(N, N, -1).permute(2, 0, 1)
            dense = dense.contiguous().float()
        o = new_feat(B, H, W, C, dt, dev)
        sel = torch.empty((B, H, W), dtype=torch.uint8, device=dev) if masked else None
        al = alpha.contiguous().float() if masked else None
        am = None if amask is None else amask.detach().contiguous().float()
        _lib.call("rgbac_winattn_core_ex", _lib.dtype_code(dt), B, H, W, C, heads, ws, shift,
                  1 if masked else 0, scale, qkv_t.data_ptr(), ldq, _lib.ptr(al),
                  dense.data_ptr(), o.ptr(), o.ldc, _lib.ptr(sel), _lib.ptr(am),
                  0 if am is None else am.shape[0], 1, _lib.stream_ptr(dev))
        ctx.spec = spec
        ctx.save_for_backward(qkv_t, dense, al, table, am)
        if sel is None:
            sel = torch.empty(0, dtype=torch.uint8, device=dev)
        ctx.mark_non_differentiable(sel)
        return o.t, sel

    @staticmethod
    def backward(ctx, do_t, _dsel):
        C, heads, ws, shift, masked, scale, index = ctx.spec
        qkv_t, dense, al, table, am = ctx.saved_tensors
        B, H, W, ldq = qkv_t.shape
        dt = qkv_t.dtype
        dev = qkv_t.device
        do_t = do_t.contiguous()
        # both backward kernels write every q/k/v channel of every pixel (zeros in inactive
        # windows); only row padding past 3C would stay unwritten
        dqkv = (torch.empty_like if ldq == 3 * C else torch.zeros_like)(qkv_t)
        N = ws * ws
        groups = -(-(B * (H // ws) * (W // ws)) // (64 // N))
        nblk = int(min(groups, 64))
        part = torch.empty(nblk * heads * N * N, dtype=_F32, device=dev)
        st = _lib.stream_ptr(dev)
        rt.timed(f"winattn_bwd_kernel<{'f32' if dt == _F32 else 'bf16'},{ws}>",
                 8.0 * B * H * W * N * C, qkv_t.element_size() * B * H * W * 8 * C,
                 lambda: _lib.call("rgbac_winattn_core_bwd_ex", _lib.dtype_code(dt), B, H, W,
                                   C, heads, ws, shift, 1 if masked else 0, scale,
                                   qkv_t.data_ptr(), ldq, _lib.ptr(al), dense.data_ptr(),
                                   do_t.data_ptr(), do_t.shape[3], dqkv.data_ptr(), ldq, nblk,
                                   part.data_ptr(), _lib.ptr(am),
                                   0 if am is None else am.shape[0], st))
        dtab = None
        if ctx.needs_input_grad[2]:
            off, ij = _relpos_csr(index, table.shape[0])
            dense_g = torch.empty(heads * N * N, dtype=_F32, device=dev)
            dtab = torch.empty(table.shape, dtype=_F32, device=dev)
            _lib.call("rgbac_relpos_bwd", nblk, heads, ws, part.data_ptr(), off.data_ptr(),
                      ij.data_ptr(), dense_g.data_ptr(), dtab.data_ptr(), st)
        return None, dqkv, dtab, None, None


# --------------------------------------------------------------------------
# channel concat / layout
# --------------------------------------------------------------------------
def _copy(dst, dcoff, src, scoff, C):
    _lib.call("rgbac_channel_copy", _lib.dtype_code(src.t.dtype), src.B * src.H * src.W, C,
              src.ptr(), src.ldc, scoff, dst.ptr(), dst.ldc, dcoff, _lib.stream_ptr(src.t.device))


# RGBAC_CAT_MULTI=0: one rgbac_channel_copy launch per part (A/B)
_CAT_MULTI = os.environ.get("RGBAC_CAT_MULTI", "1") != "0"


def _copy_multi(pairs, npix, accs=None):
    """[(dst Feat, dst channel offset, src Feat, src channel offset, channels)] -> one
    rgbac_channel_copy_multi launch per 16 copies; ``accs``: per pair, add into dst instead."""
    if accs is not None and any(accs):
        for k in range(0, len(pairs), 16):
            part, acc = pairs[k:k + 16], accs[k:k + 16]
            desc = (ctypes.c_int64 * (8 * len(part)))()
            for i, ((dst, dcoff, src, scoff, C), a) in enumerate(zip(part, acc)):
                desc[8 * i: 8 * i + 8] = [src.ptr(), src.ldc, scoff, C, dst.ptr(), dst.ldc, dcoff,
                                          1 if a else 0]
            src0 = part[0][2]
            _lib.call("rgbac_channel_copy_multi_ex", _lib.dtype_code(src0.t.dtype), npix,
                      len(part), ctypes.addressof(desc), _lib.stream_ptr(src0.t.device))
        return
    if not _CAT_MULTI:
        for dst, dcoff, src, scoff, C in pairs:
            _copy(dst, dcoff, src, scoff, C)
        return
    for k in range(0, len(pairs), 16):
        part = pairs[k:k + 16]
        desc = (ctypes.c_int64 * (7 * len(part)))()
        for i, (dst, dcoff, src, scoff, C) in enumerate(part):
            desc[7 * i: 7 * i + 7] = [src.ptr(), src.ldc, scoff, C, dst.ptr(), dst.ldc, dcoff]
        src0 = part[0][2]
        _lib.call("rgbac_channel_copy_multi", _lib.dtype_code(src0.t.dtype), npix, len(part),
                  ctypes.addressof(desc), _lib.stream_ptr(src0.t.device))


class CatFn(Function):
    """torch.cat(parts, dim=1) of NHWC Feats (the slice supports of
    AutoEncoderRGB_Journal.py:249-262): all parts in one copy launch, and the backward split
    likewise."""

    @staticmethod
    def forward(ctx, meta, *ts):
        Cs, sink, part_sinks = meta
        fs = [Feat(t, c) for t, c in zip(ts, Cs)]
        f0 = fs[0]
        out = new_feat(f0.B, f0.H, f0.W, sum(Cs), f0.t.dtype, f0.t.device)
        pairs, off = [], 0
        for f in fs:
            pairs.append((out, off, f, 0, f.C))
            off += f.C
        _copy_multi(pairs, f0.B * f0.H * f0.W)
        ctx.meta = meta
        ctx.shapes = [t.shape for t in ts]
        ctx.set_materialize_grads(False)
        return out.t

    @staticmethod
    def backward(ctx, g):
        Cs, sink, part_sinks = ctx.meta
        g = _take(sink, g)
        if g is None:
            return (None,) * (1 + len(Cs))
        g = Feat(g.contiguous(), sum(Cs))
        outs, pairs, accs = [], [], []
        off = 0
        for c, shp, sk in zip(Cs, ctx.shapes, part_sinks):
            if sk is not None and sk.buf is not None:
                # add this part's slice into the producer's gradient buffer
                if not sk.own:
                    sk.buf, sk.own = sk.buf.clone(), True
                sk.slices = False
                pairs.append((Feat(sk.buf, c), 0, g, off, c))
                accs.append(True)
                outs.append(None)
            else:
                # the copy writes channels [0, c) of every pixel: only channel padding
                # (ldc > c) needs the zero fill (the slice supports are unpadded)
                alloc = torch.empty if shp[-1] == c else torch.zeros
                o = Feat(alloc(shp, dtype=g.t.dtype, device=g.t.device), c)
                pairs.append((o, 0, g, off, c))
                accs.append(False)
                if sk is not None:
                    sk.buf, sk.own, sk.slices = o.t, True, False
                    outs.append(None)
                else:
                    outs.append(o.t)
            off += c
        _copy_multi(pairs, g.B * g.H * g.W, accs)
        return (None, *outs)


def cat_t(feats):
    if len(feats) == 1:
        return feats[0]
    Cs = [f.C for f in feats]
    sink = Sink() if GRAD_SINKS else None
    part_sinks = tuple(_sink(f.t) for f in feats)
    out = CatFn.apply((Cs, sink, part_sinks), *[f.t for f in feats])
    if sink is not None:
        out._rgbac_sink = sink
    return Feat(out, sum(Cs))


class SliceFn(Function):
    """Channels [coff, coff + C) of a Feat as a new Feat."""

    @staticmethod
    def forward(ctx, t, Cin, coff, C):
        f = Feat(t, Cin)
        out = new_feat(f.B, f.H, f.W, C, t.dtype, t.device)
        _copy(out, 0, f, coff, C)
        ctx.meta = (t.shape, Cin, coff, C)
        return out.t

    @staticmethod
    def backward(ctx, g):
        shp, Cin, coff, C = ctx.meta
        alloc = torch.empty if (coff == 0 and C == shp[-1]) else torch.zeros
        o = Feat(alloc(shp, dtype=g.dtype, device=g.device), Cin)
        _copy(o, coff, Feat(g.contiguous(), C), 0, C)
        return o.t, None, None, None


def slice_t(f, coff, C):
    return Feat(SliceFn.apply(f.t, f.C, coff, C), C)


class ToNCHWFn(Function):
    @staticmethod
    def forward(ctx, t, C):
        ctx.meta = (t.shape, t.dtype, C)
        return rt.to_nchw(Feat(t, C))

    @staticmethod
    def backward(ctx, g):
        shp, dt, C = ctx.meta
        g = g.contiguous().float()
        B, _, H, W = g.shape
        out = torch.empty(shp, dtype=dt, device=g.device)
        _lib.call("rgbac_nchw_to_nhwc", _lib.dtype_code(dt), B, C, H, W, g.data_ptr(),
                  out.data_ptr(), shp[3], _lib.stream_ptr(g.device))
        return out, None


def to_nchw_t(f):
    return ToNCHWFn.apply(f.t, f.C)


class ToNHWCFn(Function):
    """fp32 NCHW -> NHWC Feat tensor of ``dtype`` (rgbac_nchw_to_nhwc), with its inverse as
    the backward."""

    @staticmethod
    def forward(ctx, x, dtype):
        f = rt.to_nhwc(x, dtype)
        ctx.meta = (x.shape, f.C)
        return f.t

    @staticmethod
    def backward(ctx, g):
        shp, C = ctx.meta
        g = g.contiguous()
        B, _, H, W = shp
        out = torch.empty(shp, dtype=torch.float32, device=g.device)
        _lib.call("rgbac_nhwc_to_nchw", _lib.dtype_code(g.dtype), B, C, H, W, g.data_ptr(),
                  g.shape[3], out.data_ptr(), _lib.stream_ptr(g.device))
        return out, None


def to_nhwc_t(x, dtype=torch.float32):
    """Autograd-tracked NCHW (B, C, H, W) -> Feat."""
    return Feat(ToNHWCFn.apply(x.contiguous().float(), dtype), x.shape[1])


# --------------------------------------------------------------------------
# entropy models and loss
# --------------------------------------------------------------------------
class GaussFn(Function):
    """One latent slice: (hat = ste_round(y - mu) + mu, sum of clamped bits)."""

    @staticmethod
    def forward(ctx, y_t, Cy, coff, cs, mu_t, sc_t, noise, sinks=None):
        y = Feat(y_t, Cy)
        mu, sc = Feat(mu_t, cs), Feat(sc_t, cs)
        dev = y_t.device
        npix = y.B * y.H * y.W
        hat = new_feat(y.B, y.H, y.W, cs, y_t.dtype, dev)
        nb = _lib.load().rgbac_reduce_blocks(npix * cs)
        part = torch.empty(nb, dtype=torch.float64, device=dev)
        _lib.call("rgbac_gaussian_slice", _lib.dtype_code(y_t.dtype), npix, cs, y.ptr(coff), y.ldc,
                  mu.ptr(), mu.ldc, sc.ptr(), sc.ldc, _lib.ptr(noise), hat.ptr(), hat.ldc, None,
                  part.data_ptr(), _lib.stream_ptr(dev))
        bits = torch.empty(1, dtype=_F32, device=dev)
        _lib.call("rgbac_sum_partials", 1, nb, part.data_ptr(), bits.data_ptr(),
                  _lib.stream_ptr(dev))
        ctx.meta = (Cy, coff, cs, sinks)
        ctx.save_for_backward(y_t, mu_t, sc_t, noise)
        ctx.set_materialize_grads(False)
        return hat.t, bits.reshape(())

    @staticmethod
    def backward(ctx, dhat, dbits):
        Cy, coff, cs, sinks = ctx.meta
        ysink, hsink = sinks if sinks is not None else (None, None)
        dhat = _take(hsink, dhat)
        y_t, mu_t, sc_t, noise = ctx.saved_tensors
        y = Feat(y_t, Cy)
        mu, sc = Feat(mu_t, cs), Feat(sc_t, cs)
        dev = y_t.device
        npix = y.B * y.H * y.W
        # dL/dy of this slice's channels: written straight into y's gradient sink while it
        # holds only other slices' disjoint channels (the ten slices' backward run before
        # y's other consumer); else into a zero-filled tensor as before
        direct = ysink is not None and (ysink.buf is None or (ysink.slices and ysink.own))
        if direct and ysink.buf is None:
            ysink.buf, ysink.own, ysink.slices = torch.zeros_like(y_t), True, True
        dy = Feat(ysink.buf if direct else torch.zeros_like(y_t), Cy)
        # rgbac_gaussian_bwd writes every (pixel, channel < cs) element: no zero fill unless
        # the tensors carry pad channels
        dmu = Feat(torch.empty_like(mu_t) if mu_t.shape[-1] == cs else torch.zeros_like(mu_t), cs)
        dsc = Feat(torch.empty_like(sc_t) if sc_t.shape[-1] == cs else torch.zeros_like(sc_t), cs)
        gb = (dbits if dbits is not None else torch.zeros((), device=dev)).float().reshape(1)
        dh = None if dhat is None else Feat(dhat.contiguous(), cs)
        _lib.call("rgbac_gaussian_bwd", _lib.dtype_code(y_t.dtype), npix, cs, y.ptr(coff), y.ldc,
                  mu.ptr(), mu.ldc, sc.ptr(), sc.ldc, _lib.ptr(noise), gb.data_ptr(),
                  None if dh is None else dh.ptr(), 0 if dh is None else dh.ldc, dy.ptr(coff),
                  dy.ldc, dmu.ptr(), dmu.ldc, dsc.ptr(), dsc.ldc, _lib.stream_ptr(dev))
        if direct:
            return None, None, None, None, dmu.t, dsc.t, None, None
        if ysink is not None:
            _deposit(ysink, dy.t, True)
            return None, None, None, None, dmu.t, dsc.t, None, None
        return dy.t, None, None, None, dmu.t, dsc.t, None, None


def gauss_t(y, coff, mu, sc, noise):
    """GaussianConditional + ste_round of y[..., coff:coff+cs] -> (hat Feat, bits scalar).
    A gradient-sink consumer of y (its slice gradient goes into y's buffer) and producer of
    hat (whose consumers -- the lrp support concatenation, the lrp update's residual --
    deposit into hat's buffer)."""
    ysink = _sink(y.t)
    hsink = Sink() if GRAD_SINKS else None
    hat, bits = GaussFn.apply(y.t, y.C, coff, mu.C, mu.t, sc.t, noise, (ysink, hsink))
    if hsink is not None:
        hat._rgbac_sink = hsink
    return Feat(hat, mu.C), bits


class EBFn(Function):
    """EntropyBottleneck forward (noise / dequantize) + z_hat STE + bits."""

    @staticmethod
    def forward(ctx, z_t, C, params, noise):
        z = Feat(z_t, C)
        dev = z_t.device
        npix = z.B * z.H * z.W
        zh = new_feat(z.B, z.H, z.W, C, z_t.dtype, dev)
        nb = _lib.load().rgbac_reduce_blocks(npix * C)
        part = torch.empty(nb, dtype=torch.float64, device=dev)
        p = params.detach().contiguous()
        _lib.call("rgbac_eb_forward", _lib.dtype_code(z_t.dtype), npix, C, z.ptr(), z.ldc,
                  p.data_ptr(), _lib.ptr(noise), zh.ptr(), zh.ldc, None, part.data_ptr(),
                  _lib.stream_ptr(dev))
        bits = torch.empty(1, dtype=_F32, device=dev)
        _lib.call("rgbac_sum_partials", 1, nb, part.data_ptr(), bits.data_ptr(),
                  _lib.stream_ptr(dev))
        ctx.C = C
        ctx.save_for_backward(z_t, p, noise)
        return zh.t, bits.reshape(())

    @staticmethod
    def backward(ctx, dzh, dbits):
        C = ctx.C
        z_t, p, noise = ctx.saved_tensors
        z = Feat(z_t, C)
        dev = z_t.device
        npix = z.B * z.H * z.W
        dz = Feat(torch.zeros_like(z_t), C)
        dp = torch.zeros_like(p)
        gb = (dbits if dbits is not None else torch.zeros((), device=dev)).float().reshape(1)
        dh = None if dzh is None else Feat(dzh.contiguous(), C)
        _lib.call("rgbac_eb_bwd", _lib.dtype_code(z_t.dtype), npix, C, z.ptr(), z.ldc,
                  p.data_ptr(), _lib.ptr(noise), gb.data_ptr(), None if dh is None else dh.ptr(),
                  0 if dh is None else dh.ldc, dz.ptr(), dz.ldc, dp.data_ptr(),
                  _lib.stream_ptr(dev))
        return dz.t, None, dp, None


class MSEFn(Function):
    """reconstruct_error (mode 0) / plain MSE (mode 1) of NHWC x_hat vs NCHW x."""

    @staticmethod
    def forward(ctx, xh_t, C, x, mask, mode):
        xh = Feat(xh_t, C)
        dev = xh_t.device
        B, cx, H, W = x.shape
        scratch = torch.empty(_lib.finalize_scratch_doubles(B, H, W), dtype=torch.float64,
                              device=dev)
        zero = torch.zeros(1, dtype=torch.float64, device=dev)
        out = torch.empty(4, dtype=_F32, device=dev)
        _lib.call("rgbac_finalize", _lib.dtype_code(xh_t.dtype), mode, B, cx, H, W, x.data_ptr(),
                  xh.ptr(), xh.ldc, _lib.ptr(mask), zero.data_ptr(), 1, zero.data_ptr(), 1,
                  scratch.data_ptr(), out.data_ptr(), _lib.stream_ptr(dev))
        ctx.meta = (C, mode)
        ctx.save_for_backward(xh_t, x, mask, scratch)
        return out[0]

    @staticmethod
    def backward(ctx, g):
        C, mode = ctx.meta
        xh_t, x, mask, scratch = ctx.saved_tensors
        B, cx, H, W = x.shape
        dev = xh_t.device
        dxh = torch.empty_like(xh_t)
        gm = g.float().reshape(1).contiguous()
        _lib.call("rgbac_mse_bwd", _lib.dtype_code(xh_t.dtype), mode, B, cx, H, W, x.data_ptr(),
                  xh_t.data_ptr(), xh_t.shape[3], _lib.ptr(mask), scratch.data_ptr(),
                  gm.data_ptr(), dxh.data_ptr(), dxh.shape[3], _lib.stream_ptr(dev))
        return dxh, None, None, None, None
