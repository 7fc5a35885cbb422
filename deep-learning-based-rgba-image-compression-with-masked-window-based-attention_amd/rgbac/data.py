"""Training-data pipeline on the GPU (reference: my_datasets/MYdataset.py:55-115, COCOP3MDataset).

The reference decodes each PNG with PIL, converts to tensors and runs RandomResizedCrop,
random flips and the alpha "fill" on the CPU per item.  Here the host keeps only the PNG
decode and the random draws -- made with the SAME RNG calls in the SAME order as the
reference (torch RNG for the crop box and the fill, Python `random` for the flips), so a
seeded run draws identical parameters -- and one `rgbac_rgba_augment` launch does the pixel
work for a whole batch on the GPU (csrc/augment.hip), writing the reference's 5-tuple
`(masked_image, alpha, img, alpha, images_with_alpha)` directly.

Crop + resize follow torchvision's `resized_crop` on a tensor: crop, then
`F.interpolate(mode="bilinear", align_corners=False, antialias=True)` (torchvision >= 0.17;
`antialias=False` gives the older tensor behaviour).  torchvision is not installed here; the
semantics are restated from its published source and pinned against torch's own CPU
`F.interpolate` in tests/test_gpu_data.py.
"""
import ctypes
import glob
import math
import os
import random

import numpy as np
import torch

from . import _lib

SCALE = (0.08, 1.0)
RATIO = (3.0 / 4.0, 4.0 / 3.0)
MAX_DOWNSCALE = 31          # filter window cap of the kernel (64 taps)


def random_resized_crop_params(height, width, scale=SCALE, ratio=RATIO):
    """torchvision RandomResizedCrop.get_params (transforms.py), same torch RNG calls."""
    area = height * width
    log_ratio = torch.log(torch.tensor(ratio))
    for _ in range(10):
        target_area = area * torch.empty(1).uniform_(scale[0], scale[1]).item()
        aspect_ratio = torch.exp(torch.empty(1).uniform_(log_ratio[0], log_ratio[1])).item()
        w = int(round(math.sqrt(target_area * aspect_ratio)))
        h = int(round(math.sqrt(target_area / aspect_ratio)))
        if 0 < w <= width and 0 < h <= height:
            i = torch.randint(0, height - h + 1, size=(1,)).item()
            j = torch.randint(0, width - w + 1, size=(1,)).item()
            return i, j, h, w
    in_ratio = float(width) / float(height)
    if in_ratio < min(ratio):
        w = width
        h = int(round(w / min(ratio)))
    elif in_ratio > max(ratio):
        h = height
        w = int(round(h * max(ratio)))
    else:
        w, h = width, height
    return (height - h) // 2, (width - w) // 2, h, w


def draw_params(height, width, fill_mix_ratio=0.25):
    """All random draws of one COCOP3MDataset.__getitem__ (MYdataset.py:86-108), in order:
    crop box (torch), hflip, vflip (python random), fill (RandomApply: torch.rand(1))."""
    i, j, h, w = random_resized_crop_params(height, width)
    flip_h = random.random() < 0.5
    flip_v = random.random() < 0.5
    fill = not (fill_mix_ratio < torch.rand(1))
    return i, j, h, w, flip_h, flip_v, bool(fill)


class _Desc(ctypes.Structure):
    _fields_ = [("src", ctypes.c_void_p), ("h", ctypes.c_int32), ("w", ctypes.c_int32),
                ("ci", ctypes.c_int32), ("cj", ctypes.c_int32), ("ch", ctypes.c_int32),
                ("cw", ctypes.c_int32), ("flags", ctypes.c_int32), ("pad", ctypes.c_int32)]


def augment_batch(images, params, height=256, width=256, antialias=True, device="cuda"):
    """images: list of (H, W, 4) uint8 arrays / tensors (decoded RGBA); params: list of
    draw_params() tuples.  Returns the reference's tuple (masked_image, alpha, img, alpha,
    images_with_alpha) as (B, C, height, width) fp32 GPU tensors."""
    B = len(images)
    if B == 0 or len(params) != B:
        raise ValueError("augment_batch: one parameter tuple per image")
    dev = torch.device(device)
    srcs = []
    for im in images:
        t = torch.as_tensor(im)
        if t.dtype != torch.uint8 or t.dim() != 3 or t.shape[2] != 4:
            raise ValueError(f"augment_batch: expected (H, W, 4) uint8 RGBA, got {tuple(t.shape)} {t.dtype}")
        srcs.append(t.to(dev, non_blocking=True).contiguous())
    arr = (_Desc * B)()
    for k, (t, (i, j, h, w, fh, fv, fill)) in enumerate(zip(srcs, params)):
        H, W = t.shape[0], t.shape[1]
        if not (0 <= i and 0 <= j and 0 < h and 0 < w and i + h <= H and j + w <= W):
            raise ValueError(f"augment_batch: crop {(i, j, h, w)} outside the {H}x{W} image")
        if h > MAX_DOWNSCALE * height or w > MAX_DOWNSCALE * width:
            raise ValueError("augment_batch: crop downscale factor above 31 is not supported")
        arr[k] = _Desc(t.data_ptr(), H, W, i, j, h, w, int(fh) | (int(fv) << 1) | (int(fill) << 2), 0)
    descs = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(dev)
    masked = torch.empty((B, 3, height, width), device=dev)
    alpha = torch.empty((B, 1, height, width), device=dev)
    img = torch.empty((B, 3, height, width), device=dev)
    rgba = torch.empty((B, 4, height, width), device=dev)
    _lib.call("rgbac_rgba_augment", B, descs.data_ptr(), height, width, 1 if antialias else 0,
              masked.data_ptr(), alpha.data_ptr(), img.data_ptr(), rgba.data_ptr(),
              _lib.stream_ptr(dev))
    # the sources and descriptors may be freed now: the caching allocator orders their reuse
    # after this launch on the same stream
    return masked, alpha, img, alpha, rgba


def decode_rgba(path):
    """PNG -> (H, W, 4) uint8 (MYdataset.py:73-79: PIL decode; non-RGBA files get alpha 255)."""
    from PIL import Image, ImageFile
    ImageFile.LOAD_TRUNCATED_IMAGES = True
    img = Image.open(path)
    if img.mode != "RGBA":
        img = img.convert("RGBA")
    return np.asarray(img, dtype=np.uint8)


class COCOP3MDataset(torch.utils.data.Dataset):
    """Drop-in for my_datasets.MYdataset.COCOP3MDataset (same ctor, len, item tuple).  Items
    are augmented on the GPU one at a time; for the batched path use `decode_item` in the
    DataLoader workers and `collate_gpu` as the collate function (one launch per batch)."""

    def __init__(self, coco_path="P3Mdata/COCOdata", p3m_path="P3Mdata/MASKpatches", height=256,
                 width=256, fill_mix_ratio=0.25, device="cuda"):
        self.images = (glob.glob(os.path.join(coco_path, "*.png")) +
                       glob.glob(os.path.join(p3m_path, "*.png")))
        self.height, self.width = height, width
        self.fill_mix_ratio = fill_mix_ratio
        self.device = device

    def __len__(self):
        return len(self.images)

    def decode_item(self, index):
        u8 = decode_rgba(self.images[index])
        return u8, draw_params(u8.shape[0], u8.shape[1], self.fill_mix_ratio)

    def collate_gpu(self, items):
        imgs, params = zip(*items)
        return augment_batch(list(imgs), list(params), self.height, self.width,
                             device=self.device)

    def __getitem__(self, index):
        out = self.collate_gpu([self.decode_item(index)])
        return tuple(t[0] for t in out)
