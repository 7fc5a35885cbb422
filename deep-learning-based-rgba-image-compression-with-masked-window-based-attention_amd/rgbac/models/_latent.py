"""Hyperprior + channel-conditional slice loop shared by both models
(reference: models/AutoEncoderRGB_Journal.py:222-271,
models/AutoEncoderMask_Journal.py:251-298), on the HIP path.

Concatenations are never materialised: the slice stacks read up to three
channel sources (latent means/scales, the y_hat prefix, the current
pre-lrp slice) directly.  y_hat slices are written into one NHWC buffer YH
that is the decoder input.  The lrp update ``y_hat += 0.5*tanh(lrp)`` is the
last lrp conv's epilogue."""
import torch
import torch.nn as nn

from .. import runtime as rt
from ..entropy import eb_forward_hip, gaussian_slice_hip, reduce_blocks
from ..layers.TransformRGB import run_conv, run_subpel


def _hyper_a(h_a, y):
    t = y
    for idx in (0, 2, 4, 6, 8):
        t = run_conv(h_a[idx], [t.src()], act="gelu" if idx != 8 else "none")
    return t


def _hyper_s(h_s, z_hat):
    t = z_hat
    for idx in (0, 2, 4, 6, 8):
        act = "gelu" if idx != 8 else "none"
        if isinstance(h_s[idx], nn.Sequential):
            t = run_subpel(h_s[idx], [t.src()], act=act)
        else:
            t = run_conv(h_s[idx], [t.src()], act=act)
    return t


def _stack(seq, srcs, out=None, out_coff=0, **last_kw):
    t = run_conv(seq[0], srcs, act="gelu")
    t = run_conv(seq[2], [t.src()], act="gelu")
    return run_conv(seq[4], [t.src()], out=out, out_coff=out_coff, **last_kw)


def latent_path(model, y, training=False, noise_z=None, noise_y=None, debug=None):
    """y: Feat (B,h,w,M) -> (YH Feat, ybits fp64 partials, zbits fp64 partials)."""
    dev, dt = y.t.device, y.t.dtype
    ns, msup = model.num_slices, model.max_support_slices
    M = y.C
    cs = M // ns
    z = _hyper_a(model.h_a, y)
    eb = model.entropy_bottleneck
    z_hat = rt.new_feat(z.B, z.H, z.W, z.C, dt, dev)
    zpart = torch.empty(reduce_blocks(z.B * z.H * z.W * z.C), dtype=torch.float64, device=dev)
    zlik = None
    if debug is not None:
        zlik = torch.empty((z.B, z.H, z.W, z.C), dtype=torch.float32, device=dev)
    nz = None
    if training:
        nz = noise_z if noise_z is not None else torch.rand((z.B, z.H, z.W, z.C), device=dev) - 0.5
    eb_forward_hip(eb, z, z_hat, eb.packed_params_cached(), nz, zpart, zlik)
    scales = _hyper_s(model.h_scale_s, z_hat)
    means = _hyper_s(model.h_mean_s, z_hat)

    B, h, w = y.B, y.H, y.W
    npix = B * h * w
    YH = rt.new_feat(B, h, w, M, dt, dev)
    pre = rt.new_feat(B, h, w, cs, dt, dev)
    nb = reduce_blocks(npix * cs)
    ypart = torch.empty((ns, nb), dtype=torch.float64, device=dev)
    liks, mus, sigmas = [], [], []
    for i in range(ns):
        nsup = cs * min(i, msup)
        msrc = [means.src(), YH.src(0, nsup)]
        ssrc = [scales.src(), YH.src(0, nsup)]
        mu = _stack(model.cc_mean_transforms[i], msrc)
        sc = _stack(model.cc_scale_transforms[i], ssrc)
        lik = None
        if debug is not None:
            lik = torch.empty((B, h, w, cs), dtype=torch.float32, device=dev)
            liks.append(lik)
            mus.append(mu)
            sigmas.append(sc)
        ny = None
        if training:
            ny = (noise_y[..., i * cs:(i + 1) * cs].contiguous() if noise_y is not None
                  else torch.rand((B, h, w, cs), device=dev) - 0.5)
        gaussian_slice_hip(y, i * cs, cs, mu, sc, pre, ny, ypart[i], lik)
        _stack(model.lrp_transforms[i], msrc + [pre.src()], out=YH, out_coff=i * cs,
               act="tanh_half", res1=pre)
    if debug is not None:
        debug.update(z=z, z_hat=z_hat, z_lik=zlik, y_lik=liks, mu=mus, sigma=sigmas,
                     latent_means=means, latent_scales=scales, y_hat=YH)
    return YH, ypart, zpart
