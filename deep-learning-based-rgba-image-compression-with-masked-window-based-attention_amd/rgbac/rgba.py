"""RGBA evaluation pipeline (reference: trainRGB.py:98-111 `constraint`, :284-306 test loop).

The alpha codec's reconstruction feeds the RGB codec as one GPU pipeline: alpha forward ->
clamp/round(.*255)/255/constraint (one HIP launch, `rgbac_alpha_recon`) -> mask pyramid ->
RGB forward -> clamp of the RGB reconstruction and the bpp/PSNR scalars (one HIP launch,
`rgbac_rgba_finish`).  No host synchronisation: the reference's `torch.all(mask == 1.0)`
(:300) becomes a device flag raised by the alpha launch, so the whole chain can be captured
in a HIP graph.
"""
import torch

from . import _lib
from . import runtime as rt
from .layers.SupplyMask import mask_pyramid


def _recon(x, quantise, true_mask=None, flag=None):
    rt.check_gpu(x)
    if x.dim() != 4 or x.shape[1] != 1:
        raise ValueError("alpha planes are (B, 1, H, W)")
    src = x.contiguous().float()
    out = torch.empty_like(src)
    tm = None
    if true_mask is not None:
        tm = true_mask.contiguous().float()
        if tm.shape != src.shape:
            raise ValueError("true mask shape must match the reconstruction")
    B, _, H, W = src.shape
    _lib.call("rgbac_alpha_recon", B, H, W, 1 if quantise else 0, src.data_ptr(),
              out.data_ptr(), _lib.ptr(tm), _lib.ptr(flag), _lib.stream_ptr(src.device))
    return out


def constraint(tensor):
    """trainRGB.py:98-111: isolated zeros (all 8 neighbours 1) -> 1, isolated non-zeros
    (all 8 neighbours 0) -> 0, zero padding at the border.  In place, returns `tensor`."""
    out = _recon(tensor, quantise=False)
    tensor.copy_(out.view_as(tensor))
    return tensor


def recon_alpha(x_hat_mask):
    """trainRGB.py:285-287: constraint(round(clamp(x_hat_mask, 0, 1) * 255) / 255)."""
    return _recon(x_hat_mask, quantise=True)


@torch.no_grad()
def rgba_forward(masknet, net, masked_input, mask, msssim=False):
    """One evaluation pass of trainRGB.py:282-306 for an RGBA batch on the GPU.

    masked_input: (B,3,H,W) RGB (where(alpha>0, rgb, alpha), MYdataset.py:113), mask: (B,1,H,W)
    true alpha.  Returns (clipped_recon_image, clipped_recon_mask, mse_loss, bpp, psnr, out_mask)
    where bpp already includes the alpha codec's bpp unless the mask is all ones (:300-303),
    psnr = 10*log10(1/mse) (:306), and out_mask is the alpha codec's own 5-tuple.  With
    msssim=True a 7th element is ms_ssim(masked_input, clipped image, data_range=1) (:311),
    computed by the HIP metric kernels."""
    rt.check_gpu(masked_input, mask)
    mask = mask.contiguous().float()
    levels = mask_pyramid(mask, 6)[1]                        # EncMakeMask(mask)  (:283)
    out_mask = masknet(mask)                                  # masknet(mask)      (:284)
    flag = torch.empty((1,), dtype=torch.int32, device=mask.device)
    recon_mask = _recon(out_mask[0], True, mask, flag)        # :285-287 (+ :300 flag)
    x_hat, mse, bpp = net(masked_input, mask, recon_mask, *levels[:4])[:3]   # :289
    img = torch.empty_like(x_hat)
    bpp_total = torch.empty((), dtype=torch.float32, device=x_hat.device)
    psnr = torch.empty((), dtype=torch.float32, device=x_hat.device)
    bpp_f, bppm_f, mse_f = bpp.float(), out_mask[2].float(), mse.float()
    _lib.call("rgbac_rgba_finish", x_hat.numel(), x_hat.data_ptr(), img.data_ptr(),
              bpp_f.data_ptr(), bppm_f.data_ptr(), flag.data_ptr(), mse_f.data_ptr(),
              bpp_total.data_ptr(), psnr.data_ptr(), _lib.stream_ptr(x_hat.device))
    if msssim:
        from .metrics.ms_ssim_torch import ms_ssim
        return (img, recon_mask, mse, bpp_total, psnr, out_mask,
                ms_ssim(masked_input, img, data_range=1.0, size_average=True))
    return img, recon_mask, mse, bpp_total, psnr, out_mask
