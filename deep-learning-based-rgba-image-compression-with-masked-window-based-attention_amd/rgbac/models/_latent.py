"""Hyperprior + channel-conditional slice loop shared by both models
(reference: models/AutoEncoderRGB_Journal.py:222-271,
models/AutoEncoderMask_Journal.py:251-298), on the HIP path.

Restructured for the GPU without changing the arithmetic:
  * concatenations are never materialised: the slice stacks read up to three
    channel sources (latent means/scales, the y_hat prefix, the pre-lrp
    slice) directly, and y_hat slices land in one NHWC buffer YH (the
    decoder input); ``y_hat += 0.5*tanh(lrp)`` is the last lrp conv's epilogue;
  * cc_mean and cc_scale stacks of a slice (and h_mean_s / h_scale_s) are
    independent and run as 2-group launches;
  * the last mean and scale convs form one block-diagonal conv producing
    (mu | sigma) whose epilogue is the Gaussian conditional + quantiser + bits
    (ACT_GAUSS): no mu/sigma round trip through HBM;
  * slices i >= max_support_slices all see the same support
    [latent, y_hat_0 .. y_hat_{msup-1}] (:241), so they are mutually
    independent and run together as one wave of grouped launches.
"""
import ctypes
import os

import torch
import torch.nn as nn

from .. import _lib
from .. import runtime as rt
from ..entropy import eb_forward_hip, reduce_blocks
from ..layers.TransformRGB import prep_conv, prep_subpel, run_conv


def _hyper_a(h_a, y):
    t = y
    for idx in (0, 2, 4, 6, 8):
        t = run_conv(h_a[idx], [t.src()], act="gelu" if idx != 8 else "none")
    return t


def _hyper_s_pair(hs, z_hat):
    """h_scale_s and h_mean_s (identical shapes, same input) as 2-group launches."""
    ts = [z_hat] * len(hs)
    for idx in (0, 2, 4, 6, 8):
        act = "gelu" if idx != 8 else "none"
        preps = []
        for h, t in zip(hs, ts):
            if isinstance(h[idx], nn.Sequential):
                preps.append(prep_subpel(h[idx], [t.src()], act=act))
            else:
                preps.append(prep_conv(h[idx], [t.src()], act=act))
        ts = rt.launch(preps)
    return ts


def _musigma_pack(mconv, sconv, dtype, cin):
    """Block-diagonal (mu | sigma) conv from the last cc_mean / cc_scale convs."""
    key = (dtype, cin, rt.PARAM_GEN) + tuple((p._version, p.data_ptr()) for p in
                               (mconv.weight, mconv.bias, sconv.weight, sconv.bias))
    ent = mconv.__dict__.get("_rgbac_musigma")
    if ent is None or ent[0] != key:
        with torch.no_grad():
            cs, k = mconv.out_channels, mconv.kernel_size[0]
            w = torch.zeros((2 * cs, 2 * cin, k, k), device=mconv.weight.device)
            w[:cs, :cin] = mconv.weight.float()
            w[cs:, cin:] = sconv.weight.float()
            b = torch.cat([mconv.bias.float(), sconv.bias.float()])
            pk = rt.PackedConv(w, b, rt.CONV, [(cin, cin), (cin, cin)], dtype)
        mconv.__dict__["_rgbac_musigma"] = (key, pk)
        ent = mconv.__dict__["_rgbac_musigma"]
    return ent[1]


# bf16 inference: the latent-means/scales half of a slice's first cc / lrp conv can be
# computed on a side stream (the convs are linear in their input channels:
# conv([means, y_hat_<i]) = conv_means(means) + conv_yhat(y_hat_<i)), overlapping the
# latency-bound slice chain; the chain's first convs then only read the y_hat channels and add
# the precomputed partial in their epilogue (res0).  fp32 parity mode keeps the reference's
# single-conv summation.  Modes (RGBAC_SLICE_PRECOMPUTE):
#   "all"  every slice (round 1: 156 vs 166 MPix/s -- the chain's first convs stay
#          launch-bound at K = 9 * 8i, while 30 precompute GEMMs compete for the CUs);
#   "tail" only the slices >= max_support_slices: their stacks run as ONE wide wave after the
#          sequential slices, whose latency-bound launches leave most CUs idle -- the side
#          stream fills them with the means half of the wide wave's cc1 (g10) and lrp1 (g5)
#          convs (2/3 of their K), so the wide wave's own first convs shrink to the y_hat part.
PRECOMPUTE = {"1": "all", "all": "all", "tail": "tail"}.get(
    os.environ.get("RGBAC_SLICE_PRECOMPUTE", "0"), None)
_SIDE = {}


def _side_stream(dev):
    st = _SIDE.get(dev)
    if st is None:
        st = _SIDE[dev] = torch.cuda.Stream(device=dev)
    return st


def _part_prepare(m, srcs, c0, c1, bias, **kw):
    """rt.Prepared record of conv ``m`` restricted to input channels [c0, c1) (weight
    columns), with or without its bias, over sources ``srcs`` (packs cached on the module)."""
    dt = srcs[0][0].t.dtype
    segs = rt.segs_of(*srcs)
    key = (dt, tuple(segs), c0, c1, bias, rt.PARAM_GEN, m.weight._version, m.weight.data_ptr(),
           m.bias._version, m.bias.data_ptr())
    cache = m.__dict__.setdefault("_rgbac_part", {})
    pk = cache.get((c0, c1, bias, tuple(segs), dt))
    if pk is None or pk[0] != key:
        with torch.no_grad():
            w = m.weight[:, c0:c1].float()
            b = m.bias.float() if bias else torch.zeros_like(m.bias, dtype=torch.float32)
            pk = (key, rt.PackedConv(w, b, rt.CONV, segs, dt))
        cache[(c0, c1, bias, tuple(segs), dt)] = pk
    return rt.prepare(pk[1], srcs, **kw)


def ypart_slots(model, B, h, w):
    """(slices, slots per slice) of latent_path's fp64 bits partials for a B x h x w latent."""
    return model.num_slices, -(-(B * h * w) // 32)


def latent_path(model, y, training=False, noise_z=None, noise_y=None, debug=None, ypart=None):
    """y: Feat (B,h,w,M) -> (YH Feat, ybits fp64 partials, zbits fp64 partials).
    ``ypart``: a zeroed fp64 (slices, slots) buffer (ypart_slots) for the bits partials, e.g.
    zero-filled by the forward's prologue launch; allocated and zeroed here when None."""
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
    scales, means = _hyper_s_pair((model.h_scale_s, model.h_mean_s), z_hat)

    B, h, w = y.B, y.H, y.W
    npix = B * h * w
    YH = rt.new_feat(B, h, w, M, dt, dev)
    # one fp64 bits partial per M block of the GAUSS conv (64-pixel LDS-ring tiles or
    # 32-pixel wave tiles); unused slots stay zero
    if ypart is None:
        ypart = torch.zeros(ypart_slots(model, B, h, w), dtype=torch.float64, device=dev)
    assert tuple(ypart.shape) == ypart_slots(model, B, h, w) and ypart.dtype == torch.float64
    liks = [None] * ns
    musig = [None] * ns
    waves = [[i] for i in range(min(msup, ns))]
    if ns > msup:
        waves.append(list(range(msup, ns)))
    Cm = means.C
    pre_ok = (PRECOMPUTE is not None and not training and debug is None and
              dt == torch.bfloat16 and ns > 1 and not torch.is_grad_enabled())
    # slices whose first convs read precomputed partials: cc from p0c, lrp from p0l
    p0c, p0l = (1, 0) if PRECOMPUTE == "all" else (msup, msup)
    if pre_ok and PRECOMPUTE == "tail" and ns <= msup:
        pre_ok = False
    if pre_ok:
        main = torch.cuda.current_stream(dev)
        side = _side_stream(dev)
        side.wait_stream(main)
        Wc = model.cc_mean_transforms[0][0].out_channels
        Wl = model.lrp_transforms[0][0].out_channels
        Plrp = rt.new_feat(B, h, w, (ns - p0l) * Wl, dt, dev)
        Pm = rt.new_feat(B, h, w, (ns - p0c) * Wc, dt, dev)
        Ps = rt.new_feat(B, h, w, (ns - p0c) * Wc, dt, dev)
        for f in (Plrp, Pm, Ps):
            f.t.record_stream(side)
        ev_lrp, ev_cc = torch.cuda.Event(), torch.cuda.Event()
        with torch.cuda.stream(side):
            if PRECOMPUTE == "tail":
                # the wide wave's cc1 partials first (it needs them first), mean and scale
                # stacks as one grouped launch
                rt.launch([_part_prepare(model.cc_mean_transforms[i][0], [means.src()], 0, Cm,
                                         True, out=Pm, out_coff=Wc * (i - p0c))
                           for i in range(p0c, ns)] +
                          [_part_prepare(model.cc_scale_transforms[i][0], [scales.src()], 0, Cm,
                                         True, out=Ps, out_coff=Wc * (i - p0c))
                           for i in range(p0c, ns)])
                ev_cc.record(side)
                rt.launch([_part_prepare(model.lrp_transforms[i][0], [means.src()], 0, Cm, True,
                                         out=Plrp, out_coff=Wl * (i - p0l))
                           for i in range(p0l, ns)])
                ev_lrp.record(side)
            else:
                rt.launch([_part_prepare(model.lrp_transforms[i][0], [means.src()], 0, Cm, True,
                                         out=Plrp, out_coff=Wl * (i - p0l))
                           for i in range(p0l, ns)])
                ev_lrp.record(side)
                rt.launch([_part_prepare(model.cc_mean_transforms[i][0], [means.src()], 0, Cm,
                                         True, out=Pm, out_coff=Wc * (i - p0c))
                           for i in range(p0c, ns)])
                rt.launch([_part_prepare(model.cc_scale_transforms[i][0], [scales.src()], 0, Cm,
                                         True, out=Ps, out_coff=Wc * (i - p0c))
                           for i in range(p0c, ns)])
                ev_cc.record(side)
    waited = set()
    _slice_waves(model, waves, y, YH, means, scales, Cm, cs, B, h, w, dt, dev, training,
                 noise_y, debug, liks, musig, ypart, pre_ok, p0c, p0l, waited,
                 (main, ev_cc, ev_lrp, Pm, Ps, Plrp) if pre_ok else None)
    if pre_ok:
        main.wait_stream(side)                 # join the side stream (graph capture needs it)
    if debug is not None:
        debug.update(z=z, z_hat=z_hat, z_lik=zlik, y_lik=liks, latent_means=means,
                     latent_scales=scales, y_hat=YH, musigma=musig)
    return YH, ypart, zpart


def _slice_waves(model, waves, y, YH, means, scales, Cm, cs, B, h, w, dt, dev, training,
                 noise_y, debug, liks, musig, ypart, pre_ok, p0c, p0l, waited, side):
    """The slice waves of latent_path: per wave the cc stacks, the (mu | sigma) Gaussian
    launch and the lrp stacks (grouped launches)."""
    msup = model.max_support_slices
    Wc = model.cc_mean_transforms[0][0].out_channels
    Wl = model.lrp_transforms[0][0].out_channels
    if side is not None:
        main, ev_cc, ev_lrp, Pm, Ps, Plrp = side
    for wave in waves:
        sup = [cs * min(i, msup) for i in wave]
        # cc_mean / cc_scale stacks of every slice in the wave, as one grouped launch per layer
        if pre_ok and wave[0] >= p0c:
            if "cc" not in waited:
                main.wait_event(ev_cc)
                waited.add("cc")
            t1 = rt.launch(
                [_part_prepare(model.cc_mean_transforms[i][0], [YH.src(0, n)], Cm, Cm + n, False,
                               act="gelu", res0=(Pm, Wc * (i - p0c))) for i, n in zip(wave, sup)] +
                [_part_prepare(model.cc_scale_transforms[i][0], [YH.src(0, n)], Cm, Cm + n,
                               False, act="gelu", res0=(Ps, Wc * (i - p0c)))
                 for i, n in zip(wave, sup)])
        else:
            t1 = rt.launch(
                [prep_conv(model.cc_mean_transforms[i][0], [means.src(), YH.src(0, n)], act="gelu")
                 for i, n in zip(wave, sup)] +
                [prep_conv(model.cc_scale_transforms[i][0], [scales.src(), YH.src(0, n)],
                           act="gelu")
                 for i, n in zip(wave, sup)])
        k = len(wave)
        t2 = rt.launch(
            [prep_conv(model.cc_mean_transforms[i][2], [t1[j].src()], act="gelu")
             for j, i in enumerate(wave)] +
            [prep_conv(model.cc_scale_transforms[i][2], [t1[k + j].src()], act="gelu")
             for j, i in enumerate(wave)])
        # (mu | sigma) conv + GaussianConditional + ste_round + bits (one launch)
        pres, preps = [], []
        for j, i in enumerate(wave):
            pre = rt.new_feat(B, h, w, cs, dt, dev)
            pres.append(pre)
            pk = _musigma_pack(model.cc_mean_transforms[i][4], model.cc_scale_transforms[i][4],
                               dt, t2[j].ldc)
            nyi = None
            if training:
                nyi = (noise_y[..., i * cs:(i + 1) * cs].contiguous() if noise_y is not None
                       else torch.rand((B, h, w, cs), device=dev) - 0.5)
            if debug is not None:
                liks[i] = torch.empty((B, h, w, cs), dtype=torch.float32, device=dev)
            preps.append(rt.prepare(pk, [t2[j].src(), t2[k + j].src()], out=pre, act="gauss",
                                    res1=(y, i * cs), aux0=nyi, aux1=liks[i], partial=ypart[i]))
        rt.launch(preps)
        gauss_choice = rt.LAST_CHOICE[0]
        if debug is not None:
            # the (mu | sigma) the GAUSS epilogue consumed, re-run without the epilogue (the
            # checker's view of the integer symbols round(y - mu), :255-257)
            for j, i in enumerate(wave):
                pk = _musigma_pack(model.cc_mean_transforms[i][4],
                                   model.cc_scale_transforms[i][4], dt, t2[j].ldc)
                musig[i] = rt.launch([rt.prepare(pk, [t2[j].src(), t2[k + j].src()],
                                                 out=rt.new_feat(B, h, w, 2 * cs, dt, dev))],
                                     force=gauss_choice)[0]
        # lrp stacks: y_hat_i = pre_i + 0.5 * tanh(lrp([means, y_hat_<i, pre_i]))
        if pre_ok and wave[0] >= p0l:
            if "lrp" not in waited:
                main.wait_event(ev_lrp)
                waited.add("lrp")
            l1 = rt.launch([_part_prepare(model.lrp_transforms[i][0],
                                          [YH.src(0, n), pres[j].src()], Cm, Cm + n + cs, False,
                                          act="gelu", res0=(Plrp, Wl * (i - p0l)))
                            for j, (i, n) in enumerate(zip(wave, sup))])
        else:
            l1 = rt.launch([prep_conv(model.lrp_transforms[i][0],
                                      [means.src(), YH.src(0, n), pres[j].src()], act="gelu")
                            for j, (i, n) in enumerate(zip(wave, sup))])
        l2 = rt.launch([prep_conv(model.lrp_transforms[i][2], [l1[j].src()], act="gelu")
                        for j, i in enumerate(wave)])
        rt.launch([prep_conv(model.lrp_transforms[i][4], [l2[j].src()], out=YH,
                             out_coff=i * cs, act="tanh_half", res1=pres[j])
                   for j, i in enumerate(wave)])


def debug_views(debug):
    """CPU NCHW fp32 copies of a ``debug=`` forward's latent tensors (parity tooling):
    y, per-slice mu (the first half of the (mu | sigma) the GAUSS epilogue consumed) and
    likelihoods, y_hat (decoder input), z and z_hat.  In bf16 mode the stored mu is rounded to
    bf16 (the epilogue used fp32), so symbol accounting is meaningful in fp32 mode only."""
    y = rt.to_nchw(debug["y"]).cpu()
    mus = [rt.to_nchw(ms).cpu()[:, :ms.C // 2] for ms in debug["musigma"]]
    cs = mus[0].shape[1]
    return {"y": [y[:, i * cs:(i + 1) * cs] for i in range(len(mus))], "mu": mus,
            "lik": [t.permute(0, 3, 1, 2).cpu() for t in debug["y_lik"]],
            "y_hat": rt.to_nchw(debug["y_hat"]).cpu(), "z": rt.to_nchw(debug["z"]).cpu(),
            "z_hat": rt.to_nchw(debug["z_hat"]).cpu()}
