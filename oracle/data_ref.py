"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the reference's training-data transform,
the checker for rgbac/data.py + csrc/augment.hip.  Only tests/ may import it.

Follows my_datasets/MYdataset.py:71-115 (COCOP3MDataset.__getitem__) for given random
parameters: ToTensor (/255) of RGB and alpha -> cat -> RandomResizedCrop = torchvision
`F.resized_crop` on a tensor, i.e. a crop followed by
`torch.nn.functional.interpolate(mode="bilinear", align_corners=False, antialias=...)`
(torchvision/transforms/functional.py resize -> _functional_tensor.resize) -> hflip -> vflip
-> RandomApply(FillImage) on alpha -> where(alpha > 0, img, alpha).  torchvision is absent in
this image; its resize is restated as the torch call it makes, which is the same CPU kernel
the reference runs.  Parity pinned against torch's CPU interpolate, not against reference
outputs (the reference cannot be run here: SURVEY.md §8c).
"""
import numpy as np
import torch
import torch.nn.functional as F


def augment_one(u8, params, height=256, width=256, antialias=True):
    """u8: (H, W, 4) uint8 RGBA; params: (i, j, h, w, hflip, vflip, fill)."""
    i, j, h, w, fh, fv, fill = params
    t = torch.from_numpy(np.ascontiguousarray(u8)).permute(2, 0, 1).float().div(255)  # ToTensor
    crop = t[:, i:i + h, j:j + w]
    rgba = F.interpolate(crop[None], size=(height, width), mode="bilinear",
                         align_corners=False, antialias=antialias)[0]
    if fh:
        rgba = rgba.flip(-1)
    if fv:
        rgba = rgba.flip(-2)
    img, alpha = rgba[:3], rgba[3:4]
    if fill:
        alpha = torch.ones_like(alpha)
    masked = torch.where(alpha > 0, img, alpha)
    return masked, alpha, img, alpha, torch.cat([img, alpha], 0)
