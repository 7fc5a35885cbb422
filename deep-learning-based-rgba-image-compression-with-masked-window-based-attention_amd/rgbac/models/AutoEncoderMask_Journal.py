"""Alpha codec (reference: models/AutoEncoderMask_Journal.py), MI355X hot path.

``AutoEncoder().forward(mask)`` -> ``(x_hat, mse_loss, total_bpp, y_bpp, z_bpp)``
(:248-316), same module tree / state_dict keys as the reference."""
import torch
import torch.nn as nn

from .. import runtime as rt
from ..entropy import EntropyBottleneck, GaussianConditional
from ..layers.GDN import GDN
from ..layers.Masked_Attention import _fused_ok, run_bottlenecks_fused
from ..layers.TransformRGB import _act_of, _layer_forward, dse_fused, dse_fused_ok, prep_conv, run_conv
from ..layers._blocks import conv, conv3x3, deconv, subpel_conv3x3  # noqa: F401
from ._latent import latent_path
from .AutoEncoderRGB_Journal import (_CompressionModelMixin, _hyper_analysis, _hyper_synthesis,
                                     _stack3, check_geometry, finalize, get_scale_table,  # noqa: F401
                                     ste_round)


class EnhancementBlock(nn.Module):
    def __init__(self, num_filters=32):
        super().__init__()
        self.conv1 = nn.Conv2d(num_filters, num_filters, 3, stride=1, padding=1)
        self.relu = nn.LeakyReLU(inplace=True)
        self.conv2 = nn.Conv2d(num_filters, num_filters, 3, stride=1, padding=1)

    def nhwc(self, x, post=None):
        act, slope = _act_of(self.relu)
        t = run_conv(self.conv1, [x.src()], act=act, act_param=slope)
        return run_conv(self.conv2, [t.src()], res0=x, res2=post)

    def forward(self, input):
        """:23-28"""
        return _layer_forward(self, lambda f: self.nhwc(f), "enhancement_t", input)


class DSE(nn.Module):
    def __init__(self, in_ch=1, num_filters=32):
        super().__init__()
        self.input_conv = nn.Conv2d(in_ch, num_filters, 1, stride=1)
        self.enh1 = EnhancementBlock(num_filters)
        self.enh2 = EnhancementBlock(num_filters)
        self.enh3 = EnhancementBlock(num_filters)
        self.output_conv = nn.Conv2d(num_filters, in_ch, 1, stride=1)

    def nhwc(self, x):
        if dse_fused_ok(self, x):
            return dse_fused(self, x)
        first = run_conv(self.input_conv, [x.src()])
        t = self.enh1.nhwc(first)
        t = self.enh2.nhwc(t)
        t = self.enh3.nhwc(t, post=first)
        return run_conv(self.output_conv, [t.src()], res0=x)

    def forward(self, input):
        """:39-48"""
        return _layer_forward(self, lambda f: self.nhwc(f), "dse_t", input)


def _resblock_fused_ok(pairs):
    return _fused_ok(pairs) and all(type(b.relu1) is nn.ReLU and type(b.relu2) is nn.ReLU
                                    for b, _ in pairs)


class ResBlock(nn.Module):
    def __init__(self, num_filters=128):
        super().__init__()
        self.conv1 = nn.Conv2d(num_filters, num_filters // 2, 1, stride=1)
        self.relu1 = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(num_filters // 2, num_filters // 2, 3, stride=1, padding=1)
        self.relu2 = nn.ReLU(inplace=True)
        self.conv3 = nn.Conv2d(num_filters // 2, num_filters, 1, stride=1)

    def nhwc(self, x):
        return run_resblocks([(self, x)])[0]

    def forward(self, x):
        """:105-110"""
        return _layer_forward(self, lambda f: self.nhwc(f), "resblock_t", x)


def run_resblocks(pairs):
    """Independent ResBlocks [(block, x), ...] of equal shape: one fused launch (bf16, C 192
    or 80, ReLU blocks) or three grouped conv launches."""
    if _resblock_fused_ok(pairs):
        return run_bottlenecks_fused([((b.conv1, b.conv2, b.conv3), x) for b, x in pairs], 1)
    ts = rt.launch([prep_conv(b.conv1, [x.src()], act="relu") for b, x in pairs])
    ts = rt.launch([prep_conv(b.conv2, [t.src()], act="relu") for (b, _), t in zip(pairs, ts)])
    return rt.launch([prep_conv(b.conv3, [t.src()], res0=x) for (b, x), t in zip(pairs, ts)])


class SimplifiedAttention(nn.Module):
    """x + sigmoid(conv1(attention_branch)) * trunk_branch  (:112-136)."""

    def __init__(self, num_filters=128):
        super().__init__()
        self.conv1 = nn.Conv2d(num_filters, num_filters, 1, stride=1)
        self.sigmoid = nn.Sigmoid()
        self.trunk_ResBlock1 = ResBlock(num_filters)
        self.trunk_ResBlock2 = ResBlock(num_filters)
        self.trunk_ResBlock3 = ResBlock(num_filters)
        self.attention_ResBlock1 = ResBlock(num_filters)
        self.attention_ResBlock2 = ResBlock(num_filters)
        self.attention_ResBlock3 = ResBlock(num_filters)

    def nhwc(self, x):
        # trunk and attention branches are independent: ResBlock pairs as 2-group launches
        tr, at = x, x
        for k in (1, 2, 3):
            tr, at = run_resblocks([(getattr(self, f"trunk_ResBlock{k}"), tr),
                                    (getattr(self, f"attention_ResBlock{k}"), at)])
        return run_conv(self.conv1, [at.src()], act="gate", res1=tr, res2=x)

    def forward(self, x):
        """:124-136"""
        return _layer_forward(self, lambda f: self.nhwc(f), "simplified_attention_t", x)


def _run_seq(seq, x):
    t = x
    for m in seq:
        if isinstance(m, GDN):
            t = m.nhwc(t)
        elif isinstance(m, (SimplifiedAttention, DSE)):
            t = m.nhwc(t)
        elif isinstance(m, (nn.Conv2d, nn.ConvTranspose2d)):
            t = run_conv(m, [t.src()])
        else:
            raise TypeError(type(m))
    return t


class AutoEncoder(_CompressionModelMixin, nn.Module):
    def __init__(self):
        super().__init__()
        self.maskN = 192
        self.maskM = 80
        N, M = self.maskN, self.maskM
        self.EncoderMask = nn.Sequential(
            nn.Conv2d(1, N, 5, stride=2, padding=2), GDN(N),
            nn.Conv2d(N, N, 5, stride=2, padding=2), GDN(N),
            SimplifiedAttention(N),
            nn.Conv2d(N, N, 5, stride=2, padding=2), GDN(N),
            nn.Conv2d(N, M, 1, stride=1, padding=0),
            SimplifiedAttention(M))
        self.DecoderMask = nn.Sequential(
            SimplifiedAttention(M),
            nn.ConvTranspose2d(M, N, 1, stride=1, padding=0, output_padding=0),
            GDN(N, inverse=True),
            nn.ConvTranspose2d(N, N, 5, stride=2, padding=2, output_padding=1),
            GDN(N, inverse=True),
            SimplifiedAttention(N),
            nn.ConvTranspose2d(N, N, 5, stride=2, padding=2, output_padding=1),
            GDN(N, inverse=True),
            nn.ConvTranspose2d(N, 1, 5, stride=2, padding=2, output_padding=1),
            DSE(in_ch=1, num_filters=32))
        self.num_slices = 5
        self.max_support_slices = 5
        self.h_a = _hyper_analysis(M)
        self.h_mean_s = _hyper_synthesis(M)
        self.h_scale_s = _hyper_synthesis(M)
        ns, cs = self.num_slices, M // self.num_slices
        self.cc_mean_transforms = nn.ModuleList(
            _stack3(M + cs * min(i, 5), cs) for i in range(ns))
        self.cc_scale_transforms = nn.ModuleList(
            _stack3(M + cs * min(i, 5), cs) for i in range(ns))
        self.lrp_transforms = nn.ModuleList(
            _stack3(M + cs * min(i + 1, 6), cs) for i in range(ns))
        self.entropy_bottleneck = EntropyBottleneck(192)
        self.gaussian_conditional = GaussianConditional(None)
        self.compute_dtype = torch.float32

    def set_compute_dtype(self, dtype):
        assert dtype in (torch.float32, torch.bfloat16)
        self.compute_dtype = dtype
        return self

    def forward(self, mask, *, noise_z=None, noise_y=None, debug=None):
        rt.check_gpu(mask)
        B, _, H, W = mask.shape
        check_geometry(H, W)
        if debug is None and torch.is_grad_enabled() and \
                any(p.requires_grad for p in self.parameters()):
            # training step (trainmask.py:165-198): autograd graph over the HIP kernels
            from ..train_forward import mask_forward_train
            return mask_forward_train(self, mask, noise_z, noise_y)
        dt = self.compute_dtype
        with torch.no_grad():
            m = mask.contiguous().float()
            y = _run_seq(self.EncoderMask, rt.to_nhwc(m, dt))
            yh, ypart, zpart = latent_path(self, y, self.training, noise_z, noise_y, debug)
            xh = _run_seq(self.DecoderMask, yh)
            # x_hat's NCHW copy written by the loss pass (was a separate rgbac_nhwc_to_nchw)
            x_hat = torch.empty((B, xh.C, H, W), dtype=torch.float32, device=m.device)
            out = finalize(1, m, xh, None, ypart, zpart, x_hat_nchw=x_hat)
        if debug is not None:
            debug.update(y=y)
        return x_hat, out[0], out[1], out[2], out[3]
