"""Masked shifted-window attention (reference: layers/masked_win_attention.py).

HIP paths per WinBasedAttention call (no permuted copies, no host sync):

* inference, bf16, the model's two shapes -- ONE fused launch per block:
  ``winblock_kernel`` (ws 8, C 192: rgbac_winattn_block) and ``winblock4_kernel``
  (ws 4, C 80: rgbac_winattn_block_ws4) gather the shifted window with the
  partition / window drop folded into index math, run qkv Linear, scores + rel-pos
  bias + region mask, softmax, P.V and the proj Linear on MFMA with the attention
  chain in registers, and store x + proj(o) on pixels of active windows, x elsewhere
  (result[~window_mask] = 0 then shortcut + x, :235-249);
* every other case (fp32 parity mode, other shapes, training) -- the 3-launch
  pipeline: qkv = rgbac_conv2d 1x1 [B,H,W,3C]; core = rgbac_winattn_core (shift +
  partition + window drop + scores + bias + region mask + softmax + P.V + reverse +
  unshift); out = rgbac_conv2d 1x1 (proj) with the MASKSEL epilogue.  Training runs
  it through rgbac.autograd (WinAttnFn, HIP backward).
"""
import os

import torch
import torch.nn as nn

from .. import _lib
from .. import runtime as rt

# Heads per workgroup of the MFMA attention core (rgbac_winattn_core_ex's hpb; values that do
# not divide num_heads fall back to 1).  Read per call: RGBAC_WINATTN_HPB or HPB[0].
HPB = [None]


def heads_per_block():
    if HPB[0] is not None:
        return int(HPB[0])
    try:
        return int(os.environ.get("RGBAC_WINATTN_HPB", "1"))
    except ValueError:
        return 1


def needs_grad(module, *tensors):
    """True when a forward must build an autograd graph: grad mode on and an input or a
    parameter of ``module`` requires grad (the layer then runs the autograd Functions of
    rgbac/autograd.py, whose backward is HIP; it never detaches silently)."""
    if not torch.is_grad_enabled():
        return False
    if any(t is not None and t.requires_grad for t in tensors):
        return True
    return any(p.requires_grad for p in module.parameters())


def _to_2tuple(x):
    return tuple(x) if isinstance(x, (tuple, list)) else (x, x)


def _trunc_normal_(t, std=0.02):
    # timm.models.layers.trunc_normal_(t, std) == nn.init.trunc_normal_(t, 0, std, -2, 2)
    return nn.init.trunc_normal_(t, mean=0.0, std=std, a=-2.0, b=2.0)


def window_partition(x, window_size=8):
    """(B,H,W,C) -> (B*nW, ws, ws, C)   (:6-18; index permutation)."""
    B, H, W, C = x.shape
    x = x.reshape(B, H // window_size, window_size, W // window_size, window_size, C)
    return x.permute(0, 1, 3, 2, 4, 5).reshape(-1, window_size, window_size, C)


def window_reverse(windows, window_size, H, W):
    """(B*nW, ws, ws, C) -> (B,H,W,C)   (:20-33)."""
    B = int(windows.shape[0] / (H * W / window_size / window_size))
    x = windows.reshape(B, H // window_size, W // window_size, window_size, window_size, -1)
    return x.permute(0, 1, 3, 2, 4, 5).reshape(B, H, W, -1)


def remove_zero_windows(x, alpha):
    """(:35-47) keep windows whose alpha sums to non-zero.  The fused kernel computes
    the same decision in-place; this helper is kept for API compatibility."""
    mask = alpha.sum(dim=(1, 2, 3)) != 0
    return x[mask], mask


class WindowAttention(nn.Module):
    """W-MSA with relative position bias; parameters as masked_win_attention.py:62-94."""

    def __init__(self, dim=192, window_size=(8, 8), num_heads=8, qkv_bias=True, qk_scale=None,
                 attn_drop=0., proj_drop=0.):
        super().__init__()
        self.dim = dim
        self.window_size = _to_2tuple(window_size)
        self.num_heads = num_heads
        head_dim = dim // num_heads
        self.scale = qk_scale or head_dim ** -0.5
        wh, ww = self.window_size
        assert wh == ww, "square windows only"
        self.relative_position_bias_table = nn.Parameter(
            torch.zeros((2 * wh - 1) * (2 * ww - 1), num_heads))
        ys, xs = torch.meshgrid(torch.arange(wh), torch.arange(ww), indexing="ij")
        pts = torch.stack([ys.flatten(), xs.flatten()])
        rel = (pts[:, :, None] - pts[:, None, :]).permute(1, 2, 0).contiguous()
        rel[:, :, 0] += wh - 1
        rel[:, :, 1] += ww - 1
        rel[:, :, 0] *= 2 * ww - 1
        self.register_buffer("relative_position_index", rel.sum(-1))
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(dim, dim)
        self.proj_drop = nn.Dropout(proj_drop)
        _trunc_normal_(self.relative_position_bias_table, std=.02)
        self.softmax = nn.Softmax(dim=-1)

    def dense_bias(self):
        """[heads][N][N] fp32 relative position bias (:109-111), cached per version."""
        t = self.relative_position_bias_table
        key = (rt.PARAM_GEN, t._version, t.data_ptr())
        ent = self.__dict__.get("_rgbac_bias")
        if ent is None or ent[0] != key:
            N = self.window_size[0] * self.window_size[1]
            with torch.no_grad():
                b = t[self.relative_position_index.reshape(-1)].reshape(N, N, -1)
                b = b.permute(2, 0, 1).contiguous().float()
            self.__dict__["_rgbac_bias"] = (key, b)
            ent = self.__dict__["_rgbac_bias"]
        return ent[1]

    def block_packs(self):
        """Fragment-major bf16 packs for the fused block kernels, cached per parameter version.
        ws 8 / C 192 (rgbac_winattn_block): wq [4 pairs][54][64 lanes][8] (q | k | v of heads
        2p, 2p+1: 3 x 3 16-row tiles x 6 32-deep k-steps), wp [2][12][3][64][8]: proj input
        channels 96u .. 96u + 95 (head pairs 2u, 2u + 1) as 3 k-steps in the kernel's
        accumulator-operand order -- element e of lane l in k-step s is input channel
        96u + 32s + 4(l >> 4) + (e & 3) + 16(e >> 2); biases as one fp32 [5][256] pack (bproj |
        per head pair: the q, k, v bias rows of its two heads) and the bias table per head
        pair, [4][1024] = [var][head][225] in log2 units (the kernel stages whole 1 KiB
        pieces).
        ws 4 / C 80 (rgbac_winattn_block_ws4): wq [15 tiles][3 k-steps][64][8] (k >= 80 zero),
        wp [5][5][64][4] 16x16x16 fragments (lane l: row 16m + (l & 15), input channels
        16kt + 4(l >> 4) .. +3) in a 13 KiB buffer (the kernel DMAs whole KiB)."""
        ps = (self.qkv.weight, self.qkv.bias, self.proj.weight, self.proj.bias,
              self.relative_position_bias_table)
        key = (rt.PARAM_GEN,) + tuple((t._version, t.data_ptr()) for t in ps)
        ent = self.__dict__.get("_rgbac_block")
        if ent is None or ent[0] != key:
            with torch.no_grad():
                dev = self.qkv.weight.device
                ar = lambda k: torch.arange(k, device=dev)
                Wq = self.qkv.weight.float()
                Wp = self.proj.weight.float()
                if self.window_size[0] == 8:
                    p, f, l = ar(4)[:, None, None], ar(54)[None, :, None], ar(64)[None, None, :]
                    row = (f // 18) * 192 + 48 * p + 16 * ((f % 18) // 6) + (l & 15)
                    col = (32 * (f % 6) + 8 * (l >> 4))[..., None] + ar(8)
                    rowb, colb = torch.broadcast_tensors(row[..., None], col)
                    wq = Wq[rowb, colb].to(torch.bfloat16).contiguous()
                    u = ar(2).view(2, 1, 1, 1, 1)
                    m = ar(12).view(1, 12, 1, 1, 1)
                    s = ar(3).view(1, 1, 3, 1, 1)
                    l4 = ar(64).view(1, 1, 1, 64, 1)
                    e = ar(8).view(1, 1, 1, 1, 8)
                    rowp = (16 * m + (l4 & 15)).expand(2, 12, 3, 64, 8)
                    colp = (96 * u + 32 * s + 4 * (l4 >> 4) + (e & 3) +
                            16 * (e >> 2)).expand(2, 12, 3, 64, 8)
                    wp = Wp[rowp, colp].to(torch.bfloat16).contiguous()
                    bq = self.qkv.bias.float()
                    bias = torch.zeros((5, 256), dtype=torch.float32, device=dev)
                    bias[0, :192] = self.proj.bias.float()
                    for pr in range(4):
                        for part in range(3):
                            bias[1 + pr, 48 * part:48 * part + 48] = bq[192 * part + 48 * pr:
                                                                      192 * part + 48 * pr + 48]
                    # per head pair [var][head][225] in log2 units (softmax runs on exp2):
                    # var 0 = table * log2 e, var 1 = (table - 100) * log2 e (the shift
                    # mask folded in), fp32 ops in the kernel's order
                    log2e = torch.tensor(1.4426950408889634, dtype=torch.float32)
                    tb = self.relative_position_bias_table.float().t()        # [8][225]
                    table = torch.zeros((4, 1024), dtype=torch.float32, device=dev)
                    for pr in range(4):
                        h2 = tb[2 * pr:2 * pr + 2]
                        table[pr, :450] = (h2 * log2e.to(dev)).reshape(-1)
                        table[pr, 450:900] = ((h2 + -100.0) * log2e.to(dev)).reshape(-1)
                    ent = (wq, bias, wp, None, table)
                    self.__dict__["_rgbac_block"] = (key, ent)
                    return ent
                else:
                    C = self.dim
                    t, ks = ar(3 * C // 16).view(-1, 1, 1, 1), ar(3).view(1, 3, 1, 1)
                    l4, e = ar(64).view(1, 1, 64, 1), ar(8).view(1, 1, 1, 8)
                    row = (16 * t + (l4 & 15)).expand(-1, 3, 64, 8)
                    col = (32 * ks + 8 * (l4 >> 4) + e).expand(3 * C // 16, 3, 64, 8)
                    wq = torch.where(col < C, Wq[row, col.clamp(max=C - 1)],
                                     torch.zeros((), device=dev)).to(torch.bfloat16).contiguous()
                    m, kt = ar(C // 16).view(-1, 1, 1, 1), ar(C // 16).view(1, -1, 1, 1)
                    l4, e = ar(64).view(1, 1, 64, 1), ar(4).view(1, 1, 1, 4)
                    rowp = (16 * m + (l4 & 15)).expand(C // 16, C // 16, 64, 4)
                    colp = (16 * kt + 4 * (l4 >> 4) + e).expand(C // 16, C // 16, 64, 4)
                    wp = torch.zeros(13 * 512, dtype=torch.bfloat16, device=dev)
                    wp[:rowp.numel()] = Wp[rowp, colp].to(torch.bfloat16).reshape(-1)
                bqkv = self.qkv.bias.float().contiguous()
                bproj = self.proj.bias.float().contiguous()
                table = self.relative_position_bias_table.float().contiguous()
            self.__dict__["_rgbac_block"] = (key, (wq, bqkv, wp, bproj, table))
            ent = self.__dict__["_rgbac_block"]
        return ent[1]

    def block_fused_ok(self, x, residual, amask):
        if not (rt.WINBLOCK_FUSED and residual and amask is None and
                x.t.dtype == torch.bfloat16 and self.num_heads == 8 and
                self.qkv.bias is not None and x.ldc % 8 == 0):
            return False
        ws = self.window_size[0]
        if ws == 8 and self.dim == 192:
            return x.H % 8 == 0 and x.W % 8 == 0
        return (ws == 4 and self.dim == 80 and x.H % 4 == 0 and x.W % 4 == 0 and
                rt.WINBLOCK4_FUSED)

    def block_workspace(self, B, H, W, device):
        """Device workspace of the ws-8 block (rgbac_winattn_block_workspace bytes): per-window
        arrival counters (zero here, and left zero by every launch), alpha flags and the O^T
        hand-off slots.  Kept per module and device, grown when a larger frame comes."""
        need = int(_lib.load().rgbac_winattn_block_workspace(B, H, W))
        if need < 0:
            raise RuntimeError(f"rgbac_winattn_block_workspace({B}, {H}, {W}) failed")
        cache = self.__dict__.setdefault("_rgbac_ws", {})
        buf = cache.get(device)
        if buf is None or buf.numel() < need:
            buf = torch.zeros(need, dtype=torch.uint8, device=device)
            cache[device] = buf
        return buf

    def run_block(self, x, alpha, shift, masked):
        """The whole block (qkv + attention + proj + MASKSEL residual) as one
        rgbac_winattn_block(_ws4) call: x + attn(x) on active windows, x elsewhere."""
        packs = self.block_packs()
        out = rt.new_feat(x.B, x.H, x.W, x.C, x.t.dtype, x.t.device)
        if masked:
            alpha = alpha.contiguous().float()
        npix = x.B * x.H * x.W
        C, ws = self.dim, self.window_size[0]
        scale = float(torch.tensor(self.scale, dtype=torch.float32))
        aptr = _lib.ptr(alpha) if masked else None
        stream = _lib.stream_ptr(x.t.device)
        if ws == 8:
            wq, bias, wp, _, table = packs
            work = self.block_workspace(x.B, x.H, x.W, x.t.device)
            # the C side's form (rgbac_winattn_block, restated for the timer's name): the
            # round-3 kernel below 2,048 windows, the head-pair kernels from there on
            nwin = x.B * (x.H // 8) * (x.W // 8)
            form = os.environ.get("RGBAC_WINBLOCK_FORM", "")
            v2 = form == "2" or (form != "3" and nwin < 2048)
            kname = "winblock_v2_kernel" if v2 else "winblock_kernel"
            run = lambda: _lib.call(
                "rgbac_winattn_block", x.B, x.H, x.W, shift, 1 if masked else 0, scale,
                x.ptr(), x.ldc, aptr, wq.data_ptr(), bias.data_ptr(), wp.data_ptr(),
                table.data_ptr(), out.ptr(), out.ldc, work.data_ptr(), work.numel(), stream)
        else:
            wq, bqkv, wp, bproj, table = packs
            kname = "winblock4_kernel"
            run = lambda: _lib.call(
                "rgbac_winattn_block_ws4", x.B, x.H, x.W, shift, 1 if masked else 0, scale,
                x.ptr(), x.ldc, aptr, wq.data_ptr(), bqkv.data_ptr(), wp.data_ptr(),
                bproj.data_ptr(), table.data_ptr(), out.ptr(), out.ldc, stream)
        rt.timed(kname, 2.0 * npix * (3 * C * C + 2 * ws * ws * C + C * C),
                 2.0 * npix * 2 * x.ldc, run, f"{kname} ws{ws} C{C} {x.H}x{x.W} B{x.B} shift{shift}")
        return out

    def run_nhwc(self, x, alpha, shift, masked, residual=True, amask=None):
        """x: Feat (B,H,W,C), alpha: fp32 (B,1,H,W) or None -> Feat x + attn(x)
        (or attn(x) alone when ``residual`` is False); ``amask``: explicit additive mask
        fp32 (nW, N, N) for window w = mask[w % nW] (WindowAttention.forward's ``mask``)."""
        if self.block_fused_ok(x, residual, amask):
            return self.run_block(x, alpha, shift, masked)
        C, ws = self.dim, self.window_size[0]
        dt = x.t.dtype
        qkv = rt.conv(rt.packed(self.qkv, dt, [(C, x.ldc)]), [x.src()])
        o = rt.new_feat(x.B, x.H, x.W, C, dt, x.t.device)
        sel = None
        if masked:
            sel = torch.empty((x.B, x.H, x.W), dtype=torch.uint8, device=x.t.device)
            alpha = alpha.contiguous().float()
        npix = x.B * x.H * x.W
        dh = C // self.num_heads
        tname = "float" if dt == torch.float32 else "bf16_t"
        kname = (f"winattn_mfma_kernel<{tname}, {ws}, {dh}>" if (ws, dh) in ((8, 24), (4, 10))
                 else f"winattn_core_kernel<{tname}, {ws}>")    # rocprofv3's kernel names
        rt.timed(kname,
                  4.0 * npix * ws * ws * C, qkv.t.element_size() * npix * 4 * C,
                  lambda: _lib.call(
                      "rgbac_winattn_core_ex", _lib.dtype_code(dt), x.B, x.H, x.W, C,
                      self.num_heads, ws, shift, 1 if masked else 0,
                      float(torch.tensor(self.scale, dtype=torch.float32)), qkv.ptr(), qkv.ldc,
                      _lib.ptr(alpha) if masked else None, self.dense_bias().data_ptr(), o.ptr(),
                      o.ldc, _lib.ptr(sel), _lib.ptr(amask),
                      0 if amask is None else amask.shape[0], heads_per_block(),
                      _lib.stream_ptr(x.t.device)))
        pk = rt.packed(self.proj, dt, [(C, o.ldc)])
        if not residual:
            return rt.conv(pk, [o.src()])
        if masked:
            return rt.conv(pk, [o.src()], act="masksel", res1=x, sel=sel)
        return rt.conv(pk, [o.src()], res0=x)

    def forward(self, x, mask=None):
        """:96-131.  x: (num_windows*B, N, C) windows, N = ws*ws; mask: additive
        (num_windows, N, N) (0 / -100 or -inf) or None -- window b adds mask[b % nW].
        Each window is handled as a one-window image (shift 0, no window drop), so the
        per-window gather of the fused core is the identity here."""
        rt.check_gpu(x, mask)
        Bw, N, C = x.shape
        ws = self.window_size[0]
        if N != ws * ws or C != self.dim:
            raise RuntimeError(f"WindowAttention: expected (B_, {ws * ws}, {self.dim}), "
                               f"got {tuple(x.shape)}")
        amask = None
        if mask is not None:
            nw = mask.shape[0]
            if nw == 0:
                # :115-118: an empty mask prints "nW error!"; the reference's broadcast then
                # yields no windows, which only has a consistent shape when B_ == 0
                print("nW error!")
                if Bw == 0:
                    return x.new_zeros((0, N, C))
                raise RuntimeError("WindowAttention: empty mask (nW = 0) with B_ > 0 windows")
            if Bw % nw:
                raise RuntimeError(f"WindowAttention: B_={Bw} is not a multiple of nW={nw}")
            amask = mask.detach().contiguous().float().reshape(nw, N, N)
        if Bw == 0:
            return x.new_zeros((0, N, C))
        if needs_grad(self, x):
            from ..train_forward import window_attention_t
            return window_attention_t(self, x, amask)
        with torch.no_grad():
            f = rt.Feat(_window_feat(x, ws), C)
            o = self.run_nhwc(f, None, 0, False, residual=False, amask=amask)
            return o.t[..., :C].reshape(Bw, N, C).float()


def _window_feat(x, ws):
    """(B_, N, C) windows -> NHWC (B_, ws, ws, round_up(C, 8)) fp32 tensor (zero pad)."""
    Bw, N, C = x.shape
    t = x.float().reshape(Bw, ws, ws, C)
    ldc = rt.round_up(C, 8)
    if ldc != C:
        t = torch.nn.functional.pad(t, (0, ldc - C))
    return t.contiguous()


class WinBasedAttention(nn.Module):
    """Masked Swin block: x + scatter(W-MSA(windows with alpha != 0))  (:134-251)."""
    masked = True

    def __init__(self, dim=192, num_heads=8, window_size=8, shift_size=0, qkv_bias=True,
                 qk_scale=None, drop=0., attn_drop=0., drop_path=0.):
        super().__init__()
        self.dim = dim
        self.num_heads = num_heads
        self.window_size = window_size
        self.shift_size = shift_size
        assert 0 <= self.shift_size < self.window_size, "shift_size must in 0-window_size"
        self.attn = WindowAttention(dim, window_size=_to_2tuple(window_size), num_heads=num_heads,
                                    qkv_bias=qkv_bias, qk_scale=qk_scale, attn_drop=attn_drop,
                                    proj_drop=drop)
        assert drop_path == 0.0, "DropPath is the identity in every reference configuration"
        self.drop_path = nn.Identity()

    def nhwc(self, x, img_alpha):
        return self.attn.run_nhwc(x, img_alpha, self.shift_size, self.masked)

    def forward(self, x, img_alpha):
        rt.check_gpu(x, img_alpha)
        if needs_grad(self, x):
            from ..train_forward import win_attention_t, layer_t
            return layer_t(lambda f: win_attention_t(self, f, img_alpha), x)
        with torch.no_grad():
            return rt.to_nchw(self.nhwc(rt.to_nhwc(x, torch.float32), img_alpha))
