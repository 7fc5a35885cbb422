"""Autograd-tracked forward of the RGB codec for the training step
(reference: trainRGB.py:178-198 -> models/AutoEncoderRGB_Journal.py:203-296).

Same arithmetic and op order as the inference path (runtime/_latent), expressed
with the Functions of ``autograd.py`` so ``rd_loss.backward()`` runs the HIP
backward kernels.  Differences from the inference path are structural only:
  * one launch per conv (no grouping), concatenations materialised by
    rgbac_channel_copy (CatFn) so every conv input is one autograd tensor;
  * the (mu | sigma) heads are two convs + rgbac_gaussian_slice (no fused
    GAUSS epilogue), so mu and sigma exist as tensors for their gradients;
  * ConvTranspose2d(192 -> 3) runs as 4 output phases (CONVT_S2) rather than the
    inference-only conv3x3 + PixelShuffle form.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import autograd as ag
from . import runtime as rt
from .layers.SupplyMask import mask_pyramid
from .layers.TransformRGB import _act_of
from .runtime import Feat

conv_t = ag.conv_t


def gdn_t(g, x):
    """GDN.py:64-94: beta'/gamma' through the reference's LowerBound (torch autograd on
    the O(C^2) parameters), the norm pool + division as one ConvFn (square input)."""
    beta, gamma = g.effective_params()
    C = x.C
    return conv_t(g, [x], act="igdn" if g.inverse else "gdn", res1=x, kind="gdn",
                  weight=gamma.reshape(C, C, 1, 1), bias=beta, square=True)


def residual_unit_t(u, x):
    """Masked_Attention.py:150-169."""
    t = conv_t(u.conv[0], [x], act="gelu", defer=True)
    t = conv_t(u.conv[2], [t], act="gelu", defer=True)
    return conv_t(u.conv[4], [t], act="gelu", res0=x)


def win_attention_t(blk, x, alpha):
    """masked_win_attention.py:169-251 (or win_attention.py:153-207 when unmasked)."""
    wa = blk.attn
    C, ws = wa.dim, wa.window_size[0]
    masked = type(blk).masked
    qkv = conv_t(wa.qkv, [x])
    scale = float(torch.tensor(wa.scale, dtype=torch.float32))
    spec = (C, wa.num_heads, ws, blk.shift_size, masked, scale, wa.relative_position_index)
    o_t, sel = ag.WinAttnFn.apply(spec, qkv.t, wa.relative_position_bias_table,
                                  alpha if masked else None, None)
    o = Feat(o_t, C)
    if masked:
        return conv_t(wa.proj, [o], act="masksel", res1=x, sel=sel)
    return conv_t(wa.proj, [o], res0=x)


def window_attention_t(wa, x, amask=None):
    """WindowAttention.forward(x, mask) (masked_win_attention.py:96-131) with autograd:
    x (B_, N, C) windows, each run as a one-window image (shift 0), ``amask`` the additive
    (nW, N, N) mask or None.  -> (B_, N, C) fp32."""
    Bw, N, C = x.shape
    ws = wa.window_size[0]
    t = x.float().reshape(Bw, ws, ws, C)
    ldc = rt.round_up(C, 8)
    if ldc != C:
        t = F.pad(t, (0, ldc - C))
    f = Feat(t.contiguous(), C)
    qkv = conv_t(wa.qkv, [f])
    scale = float(torch.tensor(wa.scale, dtype=torch.float32))
    spec = (C, wa.num_heads, ws, 0, False, scale, wa.relative_position_index)
    o_t, _ = ag.WinAttnFn.apply(spec, qkv.t, wa.relative_position_bias_table, None, amask)
    out = conv_t(wa.proj, [Feat(o_t, C)])
    return out.t[..., :C].reshape(Bw, N, C)


def layer_t(fn, x, dtype=torch.float32):
    """Run an NHWC training-path function on an NCHW fp32 tensor with autograd:
    NCHW -> NHWC (ToNHWCFn) -> fn(Feat) -> NCHW (ToNCHWFn).  The L3 layers' forward uses
    this when grad is needed, so composing them under autograd back-propagates through the
    HIP kernels (reference layers are ordinary differentiable modules)."""
    return ag.to_nchw_t(fn(ag.to_nhwc_t(x, dtype)))


def attention_block_t(blk, x, mask):
    """Win_noShift_Attention.forward (Masked_Attention.py:182-189)."""
    b = win_attention_t(blk.attn, x, mask)
    a = x
    for k in range(3):
        a = residual_unit_t(blk.conv_a[k], a)
        b = residual_unit_t(blk.conv_b[k], b)
    return conv_t(blk.conv_b[3], [b], act="gate", res1=a, res2=x)


def enhancement_t(e, x, post=None):
    act, slope = _act_of(e.relu)
    t = conv_t(e.conv1, [x], act=act, act_param=slope, defer=act != "none")
    return conv_t(e.conv2, [t], res0=x, res2=post)


def dse_t(d, x):
    first = conv_t(d.input_conv, [x])
    t = enhancement_t(d.enh1, first)
    t = enhancement_t(d.enh2, t)
    t = enhancement_t(d.enh3, t, post=first)
    return conv_t(d.output_conv, [t], res0=x)


def analysis_t(E, x, me2, me3):
    """TransformRGB.py:65-75."""
    y = gdn_t(E.gdn1, conv_t(E.x1, [x]))
    y = gdn_t(E.gdn2, conv_t(E.x2, [y]))
    y = attention_block_t(E.attention1, y, me2)
    y = gdn_t(E.gdn3, conv_t(E.x3, [y]))
    y = conv_t(E.x4, [y])
    return attention_block_t(E.attention2, y, me3)


def synthesis_t(D, y, md2, md3):
    """TransformRGB.py:90-100."""
    t = attention_block_t(D.attention1, y, md3)
    t = gdn_t(D.igdn1, conv_t(D.x1, [t]))
    t = gdn_t(D.igdn2, conv_t(D.x2, [t]))
    t = attention_block_t(D.attention2, t, md2)
    t = gdn_t(D.igdn3, conv_t(D.x3, [t]))
    t = conv_t(D.x4, [t])
    return dse_t(D.dse, t)


def _seq_t(seq, x):
    """conv / GELU / ... / conv (the hyper transforms and slice stacks).  A GELU followed by
    another conv of the stack is deferred into that conv's input-gradient epilogue."""
    mods = list(seq)
    t = x
    i = 0
    while i < len(mods):
        m = mods[i]
        act = "none"
        if i + 1 < len(mods) and isinstance(mods[i + 1], nn.GELU):
            act = "gelu"
        step = 2 if act != "none" else 1
        defer = act != "none" and i + step < len(mods)
        if isinstance(m, nn.Sequential):            # compressai subpel_conv3x3
            assert isinstance(m[1], nn.PixelShuffle) and m[1].upscale_factor == 2
            t = conv_t(m[0], [t], act=act, kind="subpel", defer=defer)
        else:
            t = conv_t(m, [t], act=act, defer=defer)
        i += step
    return t


def resblock_t(b, x):
    """AutoEncoderMask_Journal.py:96-110: conv1x1+ReLU, conv3x3+ReLU, conv1x1, + x."""
    t = conv_t(b.conv1, [x], act="relu", defer=True)
    t = conv_t(b.conv2, [t], act="relu", defer=True)
    return conv_t(b.conv3, [t], res0=x)


def simplified_attention_t(sa, x):
    """AutoEncoderMask_Journal.py:112-136: x + sigmoid(conv1(att(x))) * trunk(x)."""
    tr, at = x, x
    for k in (1, 2, 3):
        tr = resblock_t(getattr(sa, f"trunk_ResBlock{k}"), tr)
        at = resblock_t(getattr(sa, f"attention_ResBlock{k}"), at)
    return conv_t(sa.conv1, [at], act="gate", res1=tr, res2=x)


def mask_seq_t(seq, x):
    """EncoderMask / DecoderMask (AutoEncoderMask_Journal.py:153-176) with autograd."""
    from .layers.GDN import GDN
    from .models.AutoEncoderMask_Journal import DSE as MaskDSE
    from .models.AutoEncoderMask_Journal import SimplifiedAttention
    t = x
    for m in seq:
        if isinstance(m, GDN):
            t = gdn_t(m, t)
        elif isinstance(m, SimplifiedAttention):
            t = simplified_attention_t(m, t)
        elif isinstance(m, MaskDSE):
            t = dse_t(m, t)
        elif isinstance(m, (nn.Conv2d, nn.ConvTranspose2d)):
            t = conv_t(m, [t])
        else:
            raise TypeError(type(m))
    return t


def eb_params_t(eb):
    """The [C][64] param block of rgbac_eb_forward with autograd to the raw parameters: one
    HIP launch each way (rgbac.autograd.EbParamsFn) for compressai's filters (3, 3, 3, 3);
    other filter sets chain softplus / tanh in torch."""
    C = eb.channels
    if tuple(eb.filters) == (3, 3, 3, 3):
        ps = ([getattr(eb, f"_matrix{i}") for i in range(5)] +
              [getattr(eb, f"_bias{i}") for i in range(5)] +
              [getattr(eb, f"_factor{i}") for i in range(4)] + [eb.quantiles])
        if all(t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() for t in ps):
            return ag.EbParamsFn.apply(C, *ps)
    parts = [F.softplus(getattr(eb, f"_matrix{i}")).reshape(C, -1) for i in range(5)]
    parts += [getattr(eb, f"_bias{i}").reshape(C, -1) for i in range(5)]
    parts += [torch.tanh(getattr(eb, f"_factor{i}")).reshape(C, -1) for i in range(4)]
    parts.append(eb._get_medians().reshape(C, 1))
    return F.pad(torch.cat(parts, dim=1), (0, 64 - 59)).contiguous()


def latent_t(model, y, training, noise_z=None, noise_y=None):
    """Hyperprior + 10-slice channel-conditional model (AutoEncoderRGB_Journal.py:222-271)
    -> (y_hat Feat, sum of y bits, sum of z bits)."""
    dev = y.t.device
    ns, msup = model.num_slices, model.max_support_slices
    cs = y.C // ns
    z = _seq_t(model.h_a, y)
    nz = None
    draw = None
    if training and (noise_z is None or noise_y is None):
        # every drawn noise tensor of the step (z, then the ns y slices) from ONE uniform_
        # launch; each is a contiguous view of it
        zn = z.B * z.H * z.W * z.C if noise_z is None else 0
        sn = y.B * y.H * y.W * cs if noise_y is None else 0
        draw = (torch.empty(zn + ns * sn, device=dev).uniform_(-0.5, 0.5), zn, sn)
    if training:
        nz = (noise_z.contiguous().float() if noise_z is not None else
              draw[0][:draw[1]].view(z.B, z.H, z.W, z.C))
    zh_t, zbits = ag.EBFn.apply(z.t, z.C, eb_params_t(model.entropy_bottleneck), nz)
    z_hat = Feat(zh_t, z.C)
    scales = _seq_t(model.h_scale_s, z_hat)
    means = _seq_t(model.h_mean_s, z_hat)
    yh, ybits = [], []
    for i in range(ns):
        sup = yh if msup < 0 else yh[:msup]
        ms = ag.cat_t([means] + sup)
        ss = ag.cat_t([scales] + sup)
        mu = _seq_t(model.cc_mean_transforms[i], ms)
        sc = _seq_t(model.cc_scale_transforms[i], ss)
        nyi = None
        if training:
            o = draw[1] + i * draw[2] if noise_y is None else 0
            nyi = (noise_y[..., i * cs:(i + 1) * cs].contiguous().float() if noise_y is not None
                   else draw[0][o:o + draw[2]].view(y.B, y.H, y.W, cs))
        hat, bits = ag.gauss_t(y, i * cs, mu, sc, nyi)
        lrp = model.lrp_transforms[i]
        lsup = ag.cat_t([ms, hat])
        t = conv_t(lrp[0], [lsup], act="gelu", defer=True)
        t = conv_t(lrp[2], [t], act="gelu", defer=True)
        yh.append(conv_t(lrp[4], [t], act="tanh_half", res1=hat))
        ybits.append(bits)
    # the slices' bits summed in one reduction (torch.stack + sum) instead of nine adds
    return ag.cat_t(yh), torch.stack(ybits).sum(), zbits


def rgb_forward_train(model, input, mask, reconmask, me2, me3, noise_z=None, noise_y=None):
    """AutoEncoderRGB_Journal.forward with autograd -> (x_hat, mse, bpp, y_bpp, z_bpp)."""
    ag.prefetch_packs(model)                 # every weight pack of the step: one launch
    B, _, H, W = input.shape
    dt = model.compute_dtype
    x = input.contiguous().float()
    with torch.no_grad():
        xf = rt.to_nhwc(x, dt)
        _, md = mask_pyramid(reconmask, 4, round255=True)                      # :212-215
    y = analysis_t(model.Encoder, xf, me2, me3)                                 # :217
    yh, ybits, zbits = latent_t(model, y, model.training, noise_z, noise_y)
    xh = synthesis_t(model.Decoder, yh, md[1], md[2])                          # :273
    mse = ag.MSEFn.apply(xh.t, xh.C, x, mask.contiguous().float(), 0)          # :285
    npix = float(B * H * W)
    y_bpp = ybits / npix                                                       # :290-295
    z_bpp = zbits / npix
    return ag.to_nchw_t(xh), mse, y_bpp + z_bpp, y_bpp, z_bpp


def mask_forward_train(model, mask, noise_z=None, noise_y=None):
    """AutoEncoderMask_Journal.forward with autograd (trainmask.py:165-198: net(mask) ->
    rd_loss.backward()) -> (x_hat, mse, bpp, y_bpp, z_bpp)."""
    ag.prefetch_packs(model)
    B, _, H, W = mask.shape
    dt = model.compute_dtype
    m = mask.contiguous().float()
    with torch.no_grad():
        mf = rt.to_nhwc(m, dt)
    y = mask_seq_t(model.EncoderMask, mf)                                       # :250
    yh, ybits, zbits = latent_t(model, y, model.training, noise_z, noise_y)    # :251-298
    xh = mask_seq_t(model.DecoderMask, yh)                                      # :300
    mse = ag.MSEFn.apply(xh.t, xh.C, m, None, 1)                               # :309
    npix = float(B * H * W)
    y_bpp = ybits / npix
    z_bpp = zbits / npix
    return ag.to_nchw_t(xh), mse, y_bpp + z_bpp, y_bpp, z_bpp
