"""Symbol-flip accounting for the north_star parity bar -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s parity / cpu_baseline leg may
import this module, and only as the checker.

The bar is "bpp bit-exact after integer quantisation, PSNR / MS-SSIM within 1e-4"
(BASELINE.json north_star).  Two fp32 implementations that sum in different orders agree on
the integer symbols round(y - mu) (AutoEncoderRGB_Journal.py:255-257, compressai
GaussianConditional.quantize) except where y - mu lies within their rounding disagreement of
a half-integer (a "near-tie"): there neither answer is more right than the other.  A flip in
slice i also changes every later slice's support (:241) and the decoder input, so comparing
two free-running forwards blames later symbols on the first flip.

This module separates the two:

* ``teacher_forced`` runs the oracle (oracle/ref_model.py) with the DEVICE path's z_hat and
  y_hat slices as the hyper-synthesis input / slice supports / decoder input, so every
  symbol and every output pixel is computed from the same inputs on both sides;
* ``symbol_accounting`` compares the device symbols with the teacher-forced oracle's, slice by
  slice: a flip is attributed to a near-tie when the device / oracle disagreement on y - mu
  (|d_dev - d_ref|) at that symbol is no larger than the disagreement seen on the symbols
  that did NOT flip (the measured fp32 noise floor of the whole latent), i.e. the half-integer
  lies inside the fp32 noise band.  Anything else is ``far`` -- a real arithmetic difference.
"""
import math

import torch

from oracle import ref_model as ref


def _noise_and_flips(pairs):
    """pairs: [(d_dev, d_ref)] -> (flip masks, |d_dev - d_ref| per pair, noise floor)."""
    flips, dds, noise = [], [], 0.0
    for d_dev, d_ref in pairs:
        f = torch.round(d_dev) != torch.round(d_ref)
        dd = (d_dev - d_ref).abs()
        flips.append(f)
        dds.append(dd)
        if (~f).any():
            noise = max(noise, dd[~f].max().item())
    return flips, dds, noise


def _bits(lik):
    """AutoEncoderRGB_Journal.py:280-281, per element (fp64 for the comparison sums)."""
    return torch.clamp(-1.0 * torch.log(lik.double() + 1e-10) / math.log(2.0), 0, 50)


def symbol_accounting(y_dev, mu_dev, y_ref, mu_ref, z_dev=None, z_ref=None, z_med=None,
                      lik_dev=None, lik_ref=None):
    """Per-slice symbol comparison.

    y_dev / mu_dev / y_ref / mu_ref: lists (one per slice) of NCHW fp32 CPU tensors: the device
    path's y slice and the mu its fused Gaussian epilogue consumed; the teacher-forced oracle's
    y slice and mu.  z_dev / z_ref (NCHW) and z_med (C,1,1): the hyper latent and the
    EntropyBottleneck medians (symbols round(z - med), compressai EntropyBottleneck.forward).
    lik_dev / lik_ref (per slice, NCHW): the y likelihoods -- bits are compared over the
    symbols that did not flip (a flipped symbol's likelihood is a different number).
    """
    pairs = [(yd - md, yr - mr) for yd, md, yr, mr in zip(y_dev, mu_dev, y_ref, mu_ref)]
    zpair = None
    if z_dev is not None:
        med = z_med.reshape(1, -1, 1, 1)
        zpair = (z_dev - med, z_ref - med)
    flips, dds, noise = _noise_and_flips(pairs + ([zpair] if zpair else []))
    rep = {"symbols": 0, "nonzero_symbols": 0, "flips": 0, "near_tie_flips": 0, "far_flips": 0,
           "per_slice_flips": [], "noise_floor": noise, "max_flip_dd": 0.0}
    for i, (d_dev, d_ref) in enumerate(pairs):
        f, dd = flips[i], dds[i]
        near = f & (dd <= noise)
        rep["symbols"] += f.numel()
        rep["nonzero_symbols"] += int((torch.round(d_ref) != 0).sum())
        rep["flips"] += int(f.sum())
        rep["near_tie_flips"] += int(near.sum())
        rep["far_flips"] += int((f & ~near).sum())
        rep["per_slice_flips"].append(int(f.sum()))
        if f.any():
            rep["max_flip_dd"] = max(rep["max_flip_dd"], dd[f].max().item())
        if lik_dev is not None:
            bd, br = _bits(lik_dev[i]), _bits(lik_ref[i])
            rep["bits_dev"] = rep.get("bits_dev", 0.0) + bd.sum().item()
            rep["bits_ref"] = rep.get("bits_ref", 0.0) + br.sum().item()
            rep["bits_dev_unflipped"] = rep.get("bits_dev_unflipped", 0.0) + bd[~f].sum().item()
            rep["bits_ref_unflipped"] = rep.get("bits_ref_unflipped", 0.0) + br[~f].sum().item()
    if lik_dev is not None:
        rep["bits_unflipped_rel"] = (abs(rep["bits_dev_unflipped"] - rep["bits_ref_unflipped"]) /
                                     max(rep["bits_ref_unflipped"], 1e-30))
    if zpair is not None:
        f, dd = flips[-1], dds[-1]
        rep["z_symbols"] = f.numel()
        rep["z_flips"] = int(f.sum())
        rep["z_far_flips"] = int((f & (dd > noise)).sum())
    return rep


def teacher_forced(sd, kind, inp, y_hat_dev, z_hat_dev, mask=None, reconmask=None):
    """The oracle forward with the device path's y_hat / z_hat forced in (see module doc).

    kind "rgb": AutoEncoderRGB_Journal (inp = masked RGB, mask / reconmask = alpha);
    kind "mask": AutoEncoderMask_Journal (inp = the alpha tile).
    -> (outputs 5-tuple, dbg dict with per-slice y / mu / scale and z, z_med)."""
    dbg = {}
    with torch.no_grad():
        if kind == "rgb":
            me = ref.supply_mask(mask)
            out = ref.rgb_forward(sd, inp, mask, reconmask, *me[:4], dbg=dbg,
                                  force_hats=y_hat_dev, force_zhat=z_hat_dev)
        else:
            out = ref.mask_forward(sd, inp, dbg=dbg, force_hats=y_hat_dev, force_zhat=z_hat_dev)
    return out, dbg


def psnr_db(mse):
    return 10 * math.log10(1.0 / mse) if mse > 0 else None


def north_star_report(sd, kind, inp, mask, dev, dev_out):
    """Teacher-forced parity of one device forward (fp32 mode).

    inp / mask: the CPU NCHW inputs the device forward got (mask unused for kind "mask");
    dev: ``rgbac.models._latent.debug_views`` of that forward; dev_out: its (x_hat NCHW CPU,
    mse, bpp, y_bpp, z_bpp).  -> symbol accounting + the teacher-forced output deltas:
    x_hat, PSNR of the model's MSE (trainRGB.py:305) and MS-SSIM of the clamped x_hat
    (:308-311), both sides from the same y_hat."""
    from oracle import ref_metrics
    tf, dbg = teacher_forced(sd, kind, inp, dev["y_hat"], dev["z_hat"], mask, mask)
    rep = symbol_accounting(dev["y"], dev["mu"], dbg["y"], dbg["mu"], dev["z"], dbg["z"],
                            dbg["z_med"], dev["lik"], dbg["lik"])
    xd, xr = dev_out[0], tf[0]
    rep["tf_max_abs_dx_hat"] = (xd - xr).abs().max().item()
    pd, pr = psnr_db(float(dev_out[1])), psnr_db(tf[1].item())
    rep["tf_d_psnr_db"] = None if pd is None or pr is None else abs(pd - pr)
    rep["tf_d_ms_ssim"] = None
    if min(inp.shape[-2:]) > 160:                # ms_ssim_torch.py:158-160 (5 levels, win 11)
        with torch.no_grad():
            msd = ref_metrics.ms_ssim(inp, xd.clamp(0, 1), data_range=1.0).item()
            msr = ref_metrics.ms_ssim(inp, xr.clamp(0, 1), data_range=1.0).item()
        rep["tf_d_ms_ssim"] = abs(msd - msr)
    rep["tf_rel_d_bpp"] = abs(float(dev_out[2]) - tf[2].item()) / max(abs(tf[2].item()), 1e-30)
    return rep
