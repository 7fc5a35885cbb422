"""Training-data pipeline on the GPU (reference: my_datasets/MYdataset.py:55-115, COCOP3MDataset;
my_datasets/MYprepare.py:7-10, prepare_dataset_train_COCOP3M).

The reference decodes each PNG with PIL, converts to tensors and runs RandomResizedCrop,
random flips and the alpha "fill" on the CPU per item, inside `DataLoader(num_workers=4,
pin_memory=True)` worker processes.  Here the split is:

* worker processes (`COCOP3MDataset.__getitem__`, CPU only -- no GPU context is ever created
  in a forked worker): PNG decode, the random draws -- the SAME RNG calls in the SAME order as
  the reference (torch RNG for the crop box and the fill, Python `random` for the flips), so a
  seeded run draws identical parameters -- and the crop box cut out as uint8 (the only source
  pixels the resize reads);
* `collate_rgba` (also in the workers): the batch's variable-size crops packed into ONE flat
  uint8 tensor + a descriptor tensor, which `pin_memory=True` pins as usual;
* the main process (`GPUAugmentLoader`): one non-blocking H2D copy of the packed crops and ONE
  `rgbac_rgba_augment` launch per batch (csrc/augment.hip: antialiased bilinear resize, flips,
  fill, masking), yielding the reference's 5-tuple `(masked_image, alpha, img, alpha,
  images_with_alpha)` as (B, C, H, W) fp32 GPU tensors.

`prepare_dataset_train_COCOP3M` has MYprepare's signature and returns (loader, dataset).

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
    return _launch_augment(arr, B, height, width, antialias, dev, keep=srcs)


def _launch_augment(arr, B, height, width, antialias, dev, keep=None):
    descs = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(dev)
    masked = torch.empty((B, 3, height, width), device=dev)
    alpha = torch.empty((B, 1, height, width), device=dev)
    img = torch.empty((B, 3, height, width), device=dev)
    rgba = torch.empty((B, 4, height, width), device=dev)
    _lib.call("rgbac_rgba_augment", B, descs.data_ptr(), height, width, 1 if antialias else 0,
              masked.data_ptr(), alpha.data_ptr(), img.data_ptr(), rgba.data_ptr(),
              _lib.stream_ptr(dev))
    # the sources (``keep``) and descriptors may be freed now: the caching allocator orders
    # their reuse after this launch on the same stream
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
    """my_datasets.MYdataset.COCOP3MDataset (same constructor arguments, same file list, same
    length).  ``__getitem__`` runs in DataLoader workers and touches no GPU: it returns
    (crop, params) -- the crop box of the decoded RGBA image as a CPU (h, w, 4) uint8 tensor and
    an int32 tensor (i, j, h, w, hflip, vflip, fill, index); the pixel transform happens batched
    on the GPU in the main process (`collate_rgba` + `GPUAugmentLoader`, or `augment_items`)."""

    def __init__(self, coco_path="P3Mdata/COCOdata", p3m_path="P3Mdata/MASKpatches", height=256,
                 width=256, fill_mix_ratio=0.25):
        self.images = (glob.glob(os.path.join(coco_path, "*.png")) +
                       glob.glob(os.path.join(p3m_path, "*.png")))
        self.height, self.width = height, width
        self.fill_mix_ratio = fill_mix_ratio

    def __len__(self):
        return len(self.images)

    def __getitem__(self, index):
        u8 = decode_rgba(self.images[index])                         # MYdataset.py:73-79
        i, j, h, w, fh, fv, fill = draw_params(u8.shape[0], u8.shape[1], self.fill_mix_ratio)
        crop = torch.from_numpy(np.ascontiguousarray(u8[i:i + h, j:j + w]))
        return crop, torch.tensor([i, j, h, w, fh, fv, fill, index], dtype=torch.int32)


def collate_rgba(items):
    """DataLoader collate_fn: a list of dataset items (crop, params) -> {"pixels": one flat
    uint8 tensor holding every crop, "desc": int64 (B, 8) [byte offset, h, w, flags, i, j,
    dataset index, 0]} -- plain CPU tensors: pin_memory pins them, and they cross the worker
    queue as two buffers."""
    sizes = [int(c.numel()) for c, _ in items]
    pixels = torch.empty(sum(sizes), dtype=torch.uint8)
    desc = torch.zeros((len(items), 8), dtype=torch.int64)
    off = 0
    for k, ((crop, p), n) in enumerate(zip(items, sizes)):
        pixels[off:off + n].copy_(crop.reshape(-1))
        p = [int(v) for v in p]
        idx = p[7] if len(p) > 7 else -1
        desc[k] = torch.tensor([off, crop.shape[0], crop.shape[1],
                                p[4] | (p[5] << 1) | (p[6] << 2), p[0], p[1], idx, 0])
        off += n
    return {"pixels": pixels, "desc": desc}


def augment_packed(batch, height=256, width=256, antialias=True, device="cuda"):
    """A `collate_rgba` batch -> the reference's 5-tuple on ``device`` (one H2D copy, one
    launch).  The copy is non-blocking from pinned memory; the launch follows it on the same
    stream."""
    dev = torch.device(device)
    pix = batch["pixels"].to(dev, non_blocking=True)
    desc = batch["desc"]
    B = desc.shape[0]
    if B == 0:
        raise ValueError("augment_packed: empty batch")
    arr = (_Desc * B)()
    base = pix.data_ptr()
    for k in range(B):
        off, h, w, flags = (int(v) for v in desc[k, :4])
        if h < 1 or w < 1 or off + h * w * 4 > pix.numel():
            raise ValueError(f"augment_packed: bad crop descriptor {desc[k].tolist()}")
        if h > MAX_DOWNSCALE * height or w > MAX_DOWNSCALE * width:
            raise ValueError("augment_packed: crop downscale factor above 31 is not supported")
        arr[k] = _Desc(base + off, h, w, 0, 0, h, w, flags, 0)
    return _launch_augment(arr, B, height, width, antialias, dev, keep=pix)


def augment_items(items, height=256, width=256, antialias=True, device="cuda"):
    """`COCOP3MDataset` items (e.g. ``[ds[k] for k in idx]``) -> the batched 5-tuple."""
    return augment_packed(collate_rgba(items), height, width, antialias, device)


class GPUAugmentLoader:
    """Wraps a DataLoader whose collate_fn is `collate_rgba`: every batch it yields is augmented
    on the GPU in THIS (main) process and comes out as the reference's 5-tuple, so the training
    loop reads it exactly like the reference's loader (trainRGB.py:165-177; the tensors are
    already on ``device``, and `.to(device)` on them is a no-op)."""

    def __init__(self, loader, height=256, width=256, device="cuda", antialias=True):
        self.loader = loader
        self.dataset = loader.dataset
        self.batch_size = loader.batch_size
        self.height, self.width = height, width
        self.device, self.antialias = device, antialias

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        for batch in self.loader:
            yield augment_packed(batch, self.height, self.width, self.antialias, self.device)


def prepare_dataset_train_COCOP3M(batch_size=1, COCOrootpath="../P3Mdata/COCOdata",
                                  P3Mrootpath="../P3Mdata/MASKpatches", height=256, width=256,
                                  fill_mix_ratio=0.25, num_workers=4, device="cuda"):
    """my_datasets/MYprepare.py:7-10 -> (train_dataloader, train_dataset): the same
    DataLoader(shuffle=True, pin_memory=True, num_workers=4) over COCOP3MDataset, with the
    pixel transform moved to one GPU launch per batch in the main process."""
    ds = COCOP3MDataset(coco_path=COCOrootpath, p3m_path=P3Mrootpath, height=height,
                        width=width, fill_mix_ratio=fill_mix_ratio)
    dl = torch.utils.data.DataLoader(ds, batch_size=batch_size, shuffle=True, pin_memory=True,
                                     num_workers=num_workers, collate_fn=collate_rgba)
    return GPUAugmentLoader(dl, height, width, device), ds
