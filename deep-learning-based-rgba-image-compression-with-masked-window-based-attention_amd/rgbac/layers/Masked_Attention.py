"""Win_noShift_Attention block (reference: layers/Masked_Attention.py:143-189).

out = conv_a(x) * sigmoid(conv_b(attn(x, mask))) + x, with every conv on the
MFMA engine and the elementwise tails fused into conv epilogues:
  ResidualUnit:  1x1+GELU -> 3x3+GELU -> 1x1 (+identity, GELU in the epilogue)
  gate:          conv_b[3] epilogue computes a * sigmoid(v) + x directly.
(The name is the reference's: the shift IS applied, shift_size = ws/2.)"""
import ctypes
import os

import torch
import torch.nn as nn

from .. import _lib
from .. import runtime as rt
from ._blocks import conv1x1, conv3x3
from .masked_win_attention import WinBasedAttention, needs_grad


class ResidualUnit(nn.Module):
    """Masked_Attention.py:150-169 (nested class there; same state_dict keys)."""

    def __init__(self, N):
        super().__init__()
        self.conv = nn.Sequential(conv1x1(N, N // 2), nn.GELU(), conv3x3(N // 2, N // 2),
                                  nn.GELU(), conv1x1(N // 2, N))
        self.relu = nn.GELU()

    def nhwc(self, x):
        return run_residual_units([(self, x)])[0]

    def forward(self, x):
        rt.check_gpu(x)
        if needs_grad(self, x):
            from ..train_forward import layer_t, residual_unit_t
            return layer_t(lambda f: residual_unit_t(self, f), x)
        with torch.no_grad():
            return rt.to_nchw(self.nhwc(rt.to_nhwc(x, torch.float32)))


FUSED = os.environ.get("RGBAC_FUSED_RU", "1") != "0"
# C = 192 units on fragment-major packs (ru_stream_kernel); "0" keeps the chunk-ring kernel
STREAM = os.environ.get("RGBAC_RU_STREAM", "1") != "0"


def _fused_ok(pairs):
    x = pairs[0][1]
    return (FUSED and x.t.dtype == torch.bfloat16 and x.C in (192, 80) and x.H % 8 == 0 and
            x.W % 8 == 0 and len(pairs) <= 4 and x.ldc % 8 == 0)


def small_unit_packs(c1, c2, c3):
    """Fragment-major bf16 packs of a C = 80 bottleneck (1x1 80->40, 3x3 40->40, 1x1 40->80)
    for rgbac_residual_unit_ex: w1 [3][3][64][8], w2 [3][18][64][8], w3 [5][2][64][8] (16
    rows x 32 k per fragment; lane l holds row 16t + l%16, k 32ks + 8(l/16) .. +8; zero
    padded), biases fp32 [48], [48], [80].  Cached on conv1 per parameter version."""
    ps = [c1.weight, c1.bias, c2.weight, c2.bias, c3.weight, c3.bias]
    key = (rt.PARAM_GEN,) + tuple((t._version, t.data_ptr()) for t in ps)
    ent = c1.__dict__.get("_rgbac_small_ru")
    if ent is None or ent[0] != key:
        with torch.no_grad():
            dev = c1.weight.device
            ar = lambda k: torch.arange(k, device=dev)

            def pack(w, nt, nks, kfn):
                # w: (rows, K) fp32 in the pack's k order; kfn: (ks, lane, e) -> k index
                t, ks = ar(nt)[:, None, None, None], ar(nks)[None, :, None, None]
                l, e = ar(64)[None, None, :, None], ar(8)[None, None, None, :]
                row = 16 * t + (l & 15)
                k = kfn(ks, l, e)
                ok = (row < w.shape[0]) & (k >= 0) & (k < w.shape[1])
                row, k, ok = torch.broadcast_tensors(row, k, ok)
                v = w[row.clamp(max=w.shape[0] - 1), k.clamp(0, w.shape[1] - 1)]
                return torch.where(ok, v, torch.zeros((), device=dev)).to(torch.bfloat16).contiguous()

            w1 = c1.weight.float().reshape(40, 80)
            p1 = pack(w1, 3, 3, lambda ks, l, e: 32 * ks + 8 * (l >> 4) + e)
            # w2: k = tap * 64 + ci (ci < 40 real), k-step kk = 2 * tap + half
            w2 = torch.zeros((40, 9, 64), device=dev)
            w2[:, :, :40] = c2.weight.float().permute(0, 2, 3, 1).reshape(40, 9, 40)
            p2 = pack(w2.reshape(40, 9 * 64), 3, 18, lambda ks, l, e: 32 * ks + 8 * (l >> 4) + e)
            w3 = c3.weight.float().reshape(80, 40)
            p3 = pack(w3, 5, 2, lambda ks, l, e: 32 * ks + 8 * (l >> 4) + e)
            b1 = torch.zeros(48, device=dev)
            b1[:40] = c1.bias.float()
            b2 = torch.zeros(48, device=dev)
            b2[:40] = c2.bias.float()
            b3 = c3.bias.float().contiguous()
        c1.__dict__["_rgbac_small_ru"] = (key, (p1, p2, p3, b1, b2, b3))
        ent = c1.__dict__["_rgbac_small_ru"]
    return ent[1]


def wide_unit_packs(c1, c2, c3):
    """Fragment-major bf16 packs of a C = 192 bottleneck (1x1 192->96, 3x3 96->96, 1x1 96->192)
    for ru_stream_kernel: w1 [6][6][64][8], w2 [6][27][64][8] (k = tap * 96 + ci), w3
    [12][3][64][8] (16 rows x 32 k per fragment; lane l holds row 16t + l%16, k 32ks +
    8(l/16) .. +8), biases fp32 [96], [96], [192].  Cached on conv1 per parameter version."""
    ps = [c1.weight, c1.bias, c2.weight, c2.bias, c3.weight, c3.bias]
    key = (rt.PARAM_GEN,) + tuple((t._version, t.data_ptr()) for t in ps)
    ent = c1.__dict__.get("_rgbac_wide_ru")
    if ent is None or ent[0] != key:
        with torch.no_grad():
            kfn = lambda ks, l, e: 32 * ks + 8 * (l >> 4) + e
            p1 = _frag_pack(c1.weight.float().reshape(96, 192), 6, 6, kfn)
            w2 = c2.weight.float().permute(0, 2, 3, 1).reshape(96, 9 * 96)
            p2 = _frag_pack(w2, 6, 27, kfn)
            p3 = _frag_pack(c3.weight.float().reshape(192, 96), 12, 3, kfn)
            bs = tuple(c.bias.float().contiguous().clone() for c in (c1, c2, c3))
        c1.__dict__["_rgbac_wide_ru"] = (key, (p1, p2, p3) + bs)
        ent = c1.__dict__["_rgbac_wide_ru"]
    return ent[1]


def _frag_pack(w, nt, nks, kfn):
    """(rows, K) fp32 -> [nt][nks][64 lanes][8] bf16 MFMA A fragments (zero padded)."""
    dev = w.device
    ar = lambda k: torch.arange(k, device=dev)
    t, ks = ar(nt)[:, None, None, None], ar(nks)[None, :, None, None]
    l, e = ar(64)[None, None, :, None], ar(8)[None, None, None, :]
    row = 16 * t + (l & 15)
    k = kfn(ks, l, e)
    ok = (row < w.shape[0]) & (k >= 0) & (k < w.shape[1])
    row, k, ok = torch.broadcast_tensors(row, k, ok)
    v = w[row.clamp(max=w.shape[0] - 1), k.clamp(0, w.shape[1] - 1)]
    return torch.where(ok, v, torch.zeros((), device=dev)).to(torch.bfloat16).contiguous()


def run_bottlenecks_fused(units, kind):
    """Bottleneck residual blocks [((conv1, conv2, conv3), x), ...] of one geometry as ONE
    rgbac_residual_unit_ex launch (csrc/fused.hip; kind 0 = ResidualUnit, 1 = ResBlock):
    both intermediates stay in LDS, one read of x and one write of y per pixel."""
    x0 = units[0][1]
    C = x0.C
    stream = C == 192 and STREAM and x0.W % 16 == 0
    arr = (_lib.RuArgs * len(units))()
    outs, keep = [], []
    for i, ((c1, c2, c3), x) in enumerate(units):
        o = rt.new_feat(x.B, x.H, x.W, x.C, x.t.dtype, x.t.device)
        a = arr[i]
        a.dtype, a.channels, a.batch, a.h, a.w = _lib.BF16, x.C, x.B, x.H, x.W
        a.x, a.x_ldc = x.ptr(), x.ldc
        if C == 80 or stream:
            p1, p2, p3, b1, b2, b3 = (small_unit_packs if C == 80 else wide_unit_packs)(c1, c2, c3)
            a.w1, a.w2, a.w3 = p1.data_ptr(), p2.data_ptr(), p3.data_ptr()
            a.w1_kpad = a.w2_kpad = a.w3_kpad = 0
            a.b1, a.b2, a.b3 = b1.data_ptr(), b2.data_ptr(), b3.data_ptr()
            keep.append((p1, p2, p3, b1, b2, b3))
        else:
            segs = [(x.C, x.ldc)]
            p1 = rt.packed(c1, x.t.dtype, segs)
            p2 = rt.packed(c2, x.t.dtype, [(p1.cout, rt.round_up(p1.cout, 8))])
            p3 = rt.packed(c3, x.t.dtype, [(p2.cout, rt.round_up(p2.cout, 8))])
            a.w1, a.w2, a.w3 = p1.w.data_ptr(), p2.w.data_ptr(), p3.w.data_ptr()
            a.w1_kpad, a.w2_kpad, a.w3_kpad = p1.k_pad, p2.k_pad, p3.k_pad
            a.b1, a.b2, a.b3 = p1.bias.data_ptr(), p2.bias.data_ptr(), p3.bias.data_ptr()
            keep.append((p1, p2, p3))
        a.out, a.out_ldc = o.ptr(), o.ldc
        outs.append(o)
    npix = x0.B * x0.H * x0.W
    flops = 2.0 * npix * len(units) * (C * C // 2 * 2 + 9 * (C // 2) ** 2)
    # the launched template's rocprof name (csrc/fused.hip rgbac_residual_unit_ex's choice,
    # restated): C 80 takes two tiles per workgroup on multi-round launches
    if C == 80:
        tiles = x0.B * (x0.H // 8) * (x0.W // 8)
        ncu = torch.cuda.get_device_properties(x0.t.device).multi_processor_count
        dual_env = os.environ.get("RGBAC_RU_SMALL_DUAL", "")
        dual = (tiles > max(1, ncu // len(units)) and dual_env != "0") or dual_env == "2"
        kname = f"ru_small_kernel<{kind}, {2 if dual else 1}>"
    elif stream:
        kname = f"ru_stream_kernel<{kind}, 8, false>"     # (rocprofv3 name)
    else:
        kname = f"ru_fused_kernel<{C}, {C // 2}>"
    rt.timed(kname, flops, 2 * npix * len(units) * 2 * C,
             lambda: _lib.call("rgbac_residual_unit_ex", ctypes.addressof(arr), len(units), kind,
                               _lib.stream_ptr(x0.t.device)),
             f"{kname} kind{kind} g{len(units)} C{C} {x0.H}x{x0.W} B{x0.B}")
    return outs


# the last unit pair + gate of a C = 192 block as one launch (rgbac_residual_unit_gate);
# RGBAC_GATE_FUSED=0: the unit-pair launch, then the gate conv launch
GATE_FUSED = os.environ.get("RGBAC_GATE_FUSED", "1") != "0"


def gate_pack(conv):
    """conv_b[3] (1x1, 192 -> 192) as the fragment-major [12][6][64][8] bf16 pack and its fp32
    bias, cached on the module per parameter version."""
    key = (rt.PARAM_GEN, conv.weight._version, conv.weight.data_ptr(), conv.bias._version,
           conv.bias.data_ptr())
    ent = conv.__dict__.get("_rgbac_gate_pack")
    if ent is None or ent[0] != key:
        with torch.no_grad():
            kfn = lambda ks, l, e: 32 * ks + 8 * (l >> 4) + e
            pw = _frag_pack(conv.weight.float().reshape(192, 192), 12, 6, kfn)
            pb = conv.bias.float().contiguous().clone()
        conv.__dict__["_rgbac_gate_pack"] = (key, (pw, pb))
        ent = conv.__dict__["_rgbac_gate_pack"]
    return ent[1]


_FLAGS = {}


def gate_flags(dev, n):
    """One zeroed int32 buffer per device for the gated launch's per-tile hand-off words (each
    launch leaves them zero; launches on a stream run one after the other); its last word is
    the timeout word.  Allocated outside graph capture only."""
    buf = _FLAGS.get(dev)
    if buf is None or buf.numel() < n:
        if torch.cuda.is_current_stream_capturing():
            return None
        buf = torch.zeros(max(n, 1 << 16), dtype=torch.int32, device=dev)
        _FLAGS[dev] = buf
    return buf


def gated_ok(block, a, b, x):
    return (GATE_FUSED and STREAM and _fused_ok([(block.conv_a[2], a), (block.conv_b[2], b)]) and
            a.C == 192 and a.W % 16 == 0 and x.ldc % 8 == 0 and
            block.conv_b[3].weight.shape == (192, 192, 1, 1))


def run_last_units_gated(block, a, b, x):
    """conv_a[2] on a, conv_b[2] on b and the gate a3 * sigmoid(conv_b[3](b3)) + x as ONE launch
    (rgbac_residual_unit_gate): the b3 tile never leaves LDS, a3 is handed over in-launch.
    Returns the block output, or None when the hand-off words are not available (first use
    inside a graph capture)."""
    ntiles = a.B * (a.H // 8) * (a.W // 16)
    flags = gate_flags(a.t.device, ntiles + 1)
    if flags is None:
        return None
    arr = (_lib.RuArgs * 2)()
    keep = []
    outs = []
    for i, (u, t) in enumerate(((block.conv_a[2], a), (block.conv_b[2], b))):
        c1, c2, c3 = u.conv[0], u.conv[2], u.conv[4]
        p1, p2, p3, b1, b2, b3 = wide_unit_packs(c1, c2, c3)
        o = rt.new_feat(t.B, t.H, t.W, t.C, t.t.dtype, t.t.device)
        r = arr[i]
        r.dtype, r.channels, r.batch, r.h, r.w = _lib.BF16, t.C, t.B, t.H, t.W
        r.x, r.x_ldc = t.ptr(), t.ldc
        r.w1, r.w2, r.w3 = p1.data_ptr(), p2.data_ptr(), p3.data_ptr()
        r.w1_kpad = r.w2_kpad = r.w3_kpad = 0
        r.b1, r.b2, r.b3 = b1.data_ptr(), b2.data_ptr(), b3.data_ptr()
        r.out, r.out_ldc = o.ptr(), o.ldc
        keep.append((p1, p2, p3, b1, b2, b3))
        outs.append(o)
    gw, gb = gate_pack(block.conv_b[3])
    npix = a.B * a.H * a.W
    C = 192
    flops = 2.0 * npix * (2 * (C * C // 2 * 2 + 9 * (C // 2) ** 2) + C * C)
    rt.timed("ru_stream_kernel<0, 8, true>", flops, 2 * npix * 6 * C,
             lambda: _lib.call("rgbac_residual_unit_gate", ctypes.addressof(arr), gw.data_ptr(),
                               gb.data_ptr(), x.ptr(), x.ldc, flags.data_ptr(), flags.numel(),
                               _lib.stream_ptr(a.t.device)),
             f"ru_stream_kernel<0, 8, true> gate C{C} {a.H}x{a.W} B{a.B}")
    return outs[1]


def run_residual_units_fused(pairs):
    """The same units as ONE fused launch (both intermediates in LDS)."""
    return run_bottlenecks_fused([((u.conv[0], u.conv[2], u.conv[4]), x) for u, x in pairs], 0)


def run_residual_units(pairs):
    """Independent ResidualUnits [(unit, x), ...] of equal shape as grouped launches:
    1x1+GELU, 3x3+GELU, 1x1 (+identity, GELU) -- three launches for all units
    (or one fused launch for bf16 C = 192)."""
    if _fused_ok(pairs):
        return run_residual_units_fused(pairs)
    return run_residual_units_unfused(pairs)


def run_residual_units_unfused(pairs):
    from .TransformRGB import prep_conv
    ts = rt.launch([prep_conv(u.conv[0], [x.src()], act="gelu") for u, x in pairs])
    ts = rt.launch([prep_conv(u.conv[2], [t.src()], act="gelu") for (u, _), t in zip(pairs, ts)])
    return rt.launch([prep_conv(u.conv[4], [t.src()], act="gelu", res0=x)
                      for (u, x), t in zip(pairs, ts)])


class Win_noShift_Attention(nn.Module):
    """Window-based self-attention module."""

    def __init__(self, dim, num_heads=8, window_size=8, shift_size=0):
        super().__init__()
        N = dim
        self.conv_a = nn.Sequential(ResidualUnit(N), ResidualUnit(N), ResidualUnit(N))
        self.attn = WinBasedAttention(dim=dim, num_heads=num_heads, window_size=window_size,
                                      shift_size=shift_size)
        self.conv_b = nn.Sequential(ResidualUnit(N), ResidualUnit(N), ResidualUnit(N),
                                    conv1x1(N, N))

    def nhwc(self, x, mask):
        # the trunk (conv_a) and the attention branch (attn -> conv_b) are independent
        # until the gate: their residual units run pairwise as 2-group launches
        b = self.attn.nhwc(x, mask)
        a = x
        for k in range(2):
            a, b = run_residual_units([(self.conv_a[k], a), (self.conv_b[k], b)])
        if gated_ok(self, a, b, x):
            out = run_last_units_gated(self, a, b, x)
            if out is not None:
                return out
        a, b = run_residual_units([(self.conv_a[2], a), (self.conv_b[2], b)])
        pk = rt.packed(self.conv_b[3], x.t.dtype, rt.segs_of(b.src()))
        return rt.conv(pk, [b.src()], act="gate", res1=a, res2=x)

    def forward(self, x, mask):
        rt.check_gpu(x, mask)
        if needs_grad(self, x):
            from ..train_forward import attention_block_t, layer_t
            return layer_t(lambda f: attention_block_t(self, f, mask), x)
        with torch.no_grad():
            return rt.to_nchw(self.nhwc(rt.to_nhwc(x, torch.float32), mask))
