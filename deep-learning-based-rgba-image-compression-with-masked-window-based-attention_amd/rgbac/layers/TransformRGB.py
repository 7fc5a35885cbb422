"""Analysis / synthesis transforms (reference: layers/TransformRGB.py:16-100).

Every conv is one rgbac_conv2d launch; the 5x5 stride-2 ConvTranspose2d layers
run as four output-parity phases of one launch; GDN/IGDN is one launch each
(see GDN.py); residual adds are conv epilogues."""
import torch
import torch.nn as nn

from .. import runtime as rt
from .GDN import GDN
from .Masked_Attention import Win_noShift_Attention
from .masked_win_attention import needs_grad
from ._blocks import conv3x3, subpel_conv3x3  # noqa: F401  (re-exported like the reference)


def _act_of(m):
    if isinstance(m, nn.LeakyReLU):
        return "lrelu", float(m.negative_slope)
    if isinstance(m, nn.ReLU):
        return "relu", 0.0
    if isinstance(m, nn.GELU):
        return "gelu", 0.0
    raise TypeError(f"unsupported activation {type(m)}")


def _layer_forward(module, nhwc_fn, train_fn, x):
    """forward() of a conv block: the fused no-grad NHWC path, or -- when grad is needed --
    the autograd Function ``train_forward.<train_fn>`` (HIP backward)."""
    rt.check_gpu(x)
    if needs_grad(module, x):
        from .. import train_forward as tf
        fn = getattr(tf, train_fn)
        return tf.layer_t(lambda f: fn(module, f), x)
    with torch.no_grad():
        return rt.to_nchw(nhwc_fn(rt.to_nhwc(x, torch.float32)))


def run_conv(m, srcs, **kw):
    """Run nn.Conv2d / nn.ConvTranspose2d ``m`` over concatenated Feat sources."""
    return rt.launch([prep_conv(m, srcs, **kw)])[0]


def prep_conv(m, srcs, **kw):
    """rt.Prepared record of ``m`` over ``srcs`` (for grouped launches)."""
    dt = srcs[0][0].t.dtype
    segs = rt.segs_of(*srcs)
    if isinstance(m, nn.ConvTranspose2d):
        k, s = m.kernel_size[0], m.stride[0]
        if k == 1 and s == 1:
            pk = rt.packed(m, dt, segs, rt.CONV, transposed=True)
        elif m.out_channels <= 4:
            # tiny Cout: one conv3x3 with 4*Cout rows + PixelShuffle store beats 4 phases
            assert k == 5 and s == 2 and m.padding[0] == 2 and m.output_padding[0] == 1
            pk = rt.packed(m, dt, segs, rt.SUBPEL2, transposed=True)
        else:
            assert k == 5 and s == 2 and m.padding[0] == 2 and m.output_padding[0] == 1
            pk = rt.packed(m, dt, segs, rt.CONVT_S2)
    else:
        assert m.padding[0] == m.kernel_size[0] // 2 and m.dilation[0] == 1 and m.groups == 1
        pk = rt.packed(m, dt, segs)
    return rt.prepare(pk, srcs, **kw)


def prep_subpel(seq, srcs, act="none"):
    """compressai subpel_conv3x3 = Sequential(conv3x3(C, r^2 C), PixelShuffle(r)), r = 2."""
    assert isinstance(seq[1], nn.PixelShuffle) and seq[1].upscale_factor == 2
    dt = srcs[0][0].t.dtype
    pk = rt.packed(seq[0], dt, rt.segs_of(*srcs), rt.SUBPEL2)
    return rt.prepare(pk, srcs, act=act)


def run_subpel(seq, srcs, act="none"):
    return rt.launch([prep_subpel(seq, srcs, act)])[0]


class EnhancementBlock(nn.Module):
    def __init__(self, num_filters=32):
        super().__init__()
        self.conv1 = nn.Conv2d(num_filters, num_filters, 3, stride=1, padding=1)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(num_filters, num_filters, 3, stride=1, padding=1)

    def nhwc(self, x, post=None):
        act, slope = _act_of(self.relu)
        t = run_conv(self.conv1, [x.src()], act=act, act_param=slope)
        return run_conv(self.conv2, [t.src()], res0=x, res2=post)

    def forward(self, input):
        """TransformRGB.py:16-28: conv2(relu(conv1(x))) + x."""
        return _layer_forward(self, lambda f: self.nhwc(f), "enhancement_t", input)


def dse_fused_ok(dse, x):
    """The 3-launch fused DSE (rgbac_dse_block) applies: bf16, 32 filters, ReLU or LeakyReLU
    blocks (one slope), a DSE input of 1 or 3 channels at ldc % 8 == 0."""
    if not (rt.DSE_FUSED and x.t.dtype == torch.bfloat16 and x.C in (1, 3) and x.ldc % 8 == 0):
        return False
    if dse.input_conv.out_channels != 32:
        return False
    slopes = set()
    for e in (dse.enh1, dse.enh2, dse.enh3):
        if type(e.relu) not in (nn.ReLU, nn.LeakyReLU) or e.conv1.in_channels != 32 or \
                e.conv1.kernel_size != (3, 3):
            return False
        slopes.add(_act_of(e.relu)[1])
    return len(slopes) == 1


def dse_fused(dse, x, only=None):
    """DSE.forward (TransformRGB.py:39-49 / AutoEncoderMask_Journal.py:39-48) as three
    rgbac_dse_block launches: in_conv fused into block 1, blocks 1-3 each one launch with
    the ReLU map on chip, (+ x_first, out_conv, + identity) fused into block 3."""
    dt, dev = x.t.dtype, x.t.device
    c32 = [(32, 32)]
    pin = rt.packed(dse.input_conv, dt, rt.segs_of(x.src()))
    pout = rt.packed(dse.output_conv, dt, c32)
    packs = [(rt.packed(e.conv1, dt, c32), rt.packed(e.conv2, dt, c32))
             for e in (dse.enh1, dse.enh2, dse.enh3)]
    slope = _act_of(dse.enh1.relu)[1]
    # block 3 writes the x.C real channels; every consumer of the DSE output (mse_partial,
    # nhwc_to_nchw) reads only those, so the pad channels are not zero-filled
    out = rt.new_feat(x.B, x.H, x.W, x.C, dt, dev, zero=False)
    t = None
    st = rt._lib.stream_ptr(dev)
    npx = x.B * x.H * x.W
    for mode, (p1, p2) in enumerate(packs):
        dst = out if mode == 2 else rt.new_feat(x.B, x.H, x.W, 32, dt, dev)
        args = (mode, x.B, x.H, x.W, x.C, slope, x.ptr(), x.ldc,
                0 if t is None else t.ptr(), 0 if t is None else t.ldc,
                pin.w.data_ptr(), pin.k_pad, pin.bias.data_ptr(),
                p1.w.data_ptr(), p1.k_pad, p1.bias.data_ptr(),
                p2.w.data_ptr(), p2.k_pad, p2.bias.data_ptr(),
                pout.w.data_ptr(), pout.k_pad, pout.bias.data_ptr(), dst.ptr(), dst.ldc, st)
        if only is not None and mode != only:         # (tools/dse_probe.py: one launch)
            t = dst
            continue
        rt.timed("dse_block_kernel", 2.0 * npx * 32 * 288 * 2,
                 2.0 * npx * ((8 if mode == 0 else 32) + (x.ldc if mode == 2 else 32)),
                 lambda a=args: rt._lib.call("rgbac_dse_block", *a),
                 f"dse_block_kernel mode{mode} 32ch {x.H}x{x.W} B{x.B}")
        t = dst
    return out


class DSE(nn.Module):
    def __init__(self, num_filters=32):
        super().__init__()
        self.input_conv = nn.Conv2d(3, num_filters, 1, stride=1)
        self.enh1 = EnhancementBlock(num_filters)
        self.enh2 = EnhancementBlock(num_filters)
        self.enh3 = EnhancementBlock(num_filters)
        self.output_conv = nn.Conv2d(num_filters, 3, 1, stride=1)

    def nhwc(self, x):
        if dse_fused_ok(self, x):
            return dse_fused(self, x)
        first = run_conv(self.input_conv, [x.src()])
        t = self.enh1.nhwc(first)
        t = self.enh2.nhwc(t)
        t = self.enh3.nhwc(t, post=first)          # (enh3(t) + x_first)
        return run_conv(self.output_conv, [t.src()], res0=x)

    def forward(self, input):
        return _layer_forward(self, lambda f: self.nhwc(f), "dse_t", input)


class Analysis_transform(nn.Module):
    def __init__(self, N=192, M=320):
        super().__init__()
        self.x1 = nn.Conv2d(3, N, 5, stride=2, padding=2)
        self.gdn1 = GDN(N)
        self.x2 = nn.Conv2d(N, N, 5, stride=2, padding=2)
        self.gdn2 = GDN(N)
        self.attention1 = Win_noShift_Attention(dim=N, num_heads=8, window_size=8, shift_size=4)
        self.x3 = nn.Conv2d(N, N, 5, stride=2, padding=2)
        self.gdn3 = GDN(N)
        self.x4 = nn.Conv2d(N, M, 1, stride=1, padding=0)
        self.attention2 = Win_noShift_Attention(dim=M, num_heads=8, window_size=4, shift_size=2)

    def _stem(self, x):
        """x1 -> gdn1 (TransformRGB.py:66).  bf16 with the reference's 5x5/s2 3 -> 192 stem:
        one fused launch (rgbac_stem_gdn) that never writes the stem output to HBM."""
        m = self.x1
        if (x.t.dtype == torch.bfloat16 and x.ldc == 8 and m.out_channels == 192 and
                m.kernel_size == (5, 5) and m.stride == (2, 2) and m.padding == (2, 2) and
                not self.gdn1.inverse and rt.STEM_FUSED):
            pk1 = rt.packed(m, x.t.dtype, rt.segs_of(x.src()))
            pk2 = self.gdn1._pack(x.t.dtype, 192)
            out = rt.new_feat(x.B, (x.H + 1) // 2, (x.W + 1) // 2, 192, x.t.dtype, x.t.device)
            rt.timed("stem_gdn_kernel", 2.0 * out.B * out.H * out.W * 192 * (75 + 192),
                     2.0 * (x.B * x.H * x.W * 8 + out.B * out.H * out.W * 192),
                     lambda: rt._lib.call("rgbac_stem_gdn", x.B, x.H, x.W, x.ptr(), x.ldc,
                                          pk1.w.data_ptr(), pk1.k_pad, pk1.bias.data_ptr(),
                                          pk2.w.data_ptr(), pk2.k_pad, pk2.bias.data_ptr(), 0,
                                          out.ptr(), out.ldc, rt._lib.stream_ptr(x.t.device)),
                     f"stem_gdn_kernel 3->192 {x.H}x{x.W} B{x.B}")
            return out
        return self.gdn1.nhwc(run_conv(m, [x.src()]))

    def nhwc(self, x, me2, me3):
        y = self._stem(x)
        y = self.gdn2.nhwc(run_conv(self.x2, [y.src()]))
        y = self.attention1.nhwc(y, me2)
        y = self.gdn3.nhwc(run_conv(self.x3, [y.src()]))
        y = run_conv(self.x4, [y.src()])
        return self.attention2.nhwc(y, me3)

    def forward(self, input, mask, me1, me2, me3, me4):
        rt.check_gpu(input, me2, me3)
        if needs_grad(self, input):
            from ..train_forward import analysis_t, layer_t
            return layer_t(lambda f: analysis_t(self, f, me2, me3), input)
        with torch.no_grad():
            return rt.to_nchw(self.nhwc(rt.to_nhwc(input, torch.float32), me2, me3))


class Synthesis_transform(nn.Module):
    def __init__(self, N=196, M=320):
        super().__init__()
        self.attention1 = Win_noShift_Attention(dim=M, num_heads=8, window_size=4, shift_size=2)
        self.x1 = nn.Conv2d(M, N, 1, stride=1, padding=0)
        self.igdn1 = GDN(N, inverse=True)
        self.x2 = nn.ConvTranspose2d(N, N, 5, stride=2, padding=2, output_padding=1)
        self.igdn2 = GDN(N, inverse=True)
        self.attention2 = Win_noShift_Attention(N, num_heads=8, window_size=8, shift_size=4)
        self.x3 = nn.ConvTranspose2d(N, N, 5, stride=2, padding=2, output_padding=1)
        self.igdn3 = GDN(N, inverse=True)
        self.x4 = nn.ConvTranspose2d(N, 3, 5, stride=2, padding=2, output_padding=1)
        self.dse = DSE(32)

    def nhwc(self, y, md2, md3):
        t = self.attention1.nhwc(y, md3)
        t = self.igdn1.nhwc(run_conv(self.x1, [t.src()]))
        t = self.igdn2.nhwc(run_conv(self.x2, [t.src()]))
        t = self.attention2.nhwc(t, md2)
        t = self.igdn3.nhwc(run_conv(self.x3, [t.src()]))
        # x4's 3-channel output (ldc 8): the fused DSE reads only its real channels (channel 7
        # carries the kernel's in-image mark), so it skips the zero fill of the pad channels
        # (a 16.8 MB memset at 256^2 B8); any other consumer gets them zeroed
        x4o = rt.new_feat(t.B, 2 * t.H, 2 * t.W, self.x4.out_channels, t.t.dtype, t.t.device,
                          zero=False)
        if not dse_fused_ok(self.dse, x4o):
            x4o.t.zero_()
        t = run_conv(self.x4, [t.src()], out=x4o)
        return self.dse.nhwc(t)

    def forward(self, input, reconmask, md1, md2, md3, md4):
        rt.check_gpu(input, md2, md3)
        if needs_grad(self, input):
            from ..train_forward import layer_t, synthesis_t
            return layer_t(lambda f: synthesis_t(self, f, md2, md3), input)
        with torch.no_grad():
            return rt.to_nchw(self.nhwc(rt.to_nhwc(input, torch.float32), md2, md3))
