"""GPU: the batched augmentation kernel (csrc/augment.hip via rgbac/data.py) against the CPU
restatement of COCOP3MDataset.__getitem__'s pixel path (oracle/data_ref.py, which runs
torch's own CPU bilinear/antialias interpolate -- the call torchvision's resized_crop makes).
Bar: 2e-6 absolute on values in [0, 1] (fp32, same window/weight formulas; only the
summation order's rounding differs); the alpha > 0 selection is exact except where the two
alphas straddle 0 within that tolerance (none occur with these inputs)."""
import random

import numpy as np
import pytest
import torch

from oracle import data_ref

pytestmark = pytest.mark.gpu

CASES = [
    # (H, W, params, antialias)
    (480, 640, (98, 42, 376, 439, False, False, False), True),      # downscale, no flips
    (480, 640, (0, 0, 480, 640, True, True, True), True),           # whole image, both flips, fill
    (300, 200, (17, 5, 61, 77, True, False, False), True),          # upscale, odd crop
    (300, 200, (0, 0, 300, 200, False, True, False), False),        # plain bilinear (no aa)
    (1000, 1300, (3, 9, 997, 1201, False, False, True), True),      # 4-5x downscale
    (64, 64, (10, 20, 1, 1, True, True, False), True),              # 1x1 crop -> constant
    (256, 256, (0, 0, 256, 256, False, False, False), True),        # identity size
]


def _image(H, W, seed, alpha_zero_frac=0.4):
    g = np.random.default_rng(seed)
    u8 = g.integers(0, 256, size=(H, W, 4), dtype=np.uint8)
    # blocky alpha with exact zeros, like matting masks
    blk = g.random(((H + 15) // 16, (W + 15) // 16)) < alpha_zero_frac
    zero = np.kron(blk, np.ones((16, 16), bool))[:H, :W]
    u8[..., 3][zero] = 0
    return u8


@pytest.mark.parametrize("idx", range(len(CASES)))
def test_augment_matches_oracle(device, idx):
    from rgbac import data
    H, W, params, aa = CASES[idx]
    u8 = _image(H, W, idx)
    out = data.augment_batch([u8], [params], 256, 256, antialias=aa, device=device)
    ref = data_ref.augment_one(u8, params, 256, 256, antialias=aa)
    for k, (g, r) in enumerate(zip(out, ref)):
        assert g.shape[1:] == r.shape, k
        err = (g[0].cpu() - r).abs().max().item()
        assert err <= 2e-6, (k, err)


def test_augment_batch_mixed_sizes(device):
    """One launch over a batch of differently sized sources and random parameters drawn the
    reference's way (torch + python RNG), rectangular output size."""
    from rgbac import data
    torch.manual_seed(5)
    random.seed(5)
    shapes = [(480, 640), (333, 500), (640, 427), (97, 131), (1024, 768), (256, 256)]
    imgs = [_image(h, w, 100 + k) for k, (h, w) in enumerate(shapes)]
    params = [data.draw_params(h, w, 0.25) for h, w in shapes]
    out = data.augment_batch(imgs, params, 192, 160, device=device)
    for b, (u8, p) in enumerate(zip(imgs, params)):
        ref = data_ref.augment_one(u8, p, 192, 160)
        for k in range(5):
            err = (out[k][b].cpu() - ref[k]).abs().max().item()
            assert err <= 2e-6, (b, k, p, err)


def test_augment_rejects_bad_input(device):
    from rgbac import data
    u8 = _image(64, 64, 1)
    with pytest.raises(ValueError):
        data.augment_batch([u8], [(0, 0, 65, 64, False, False, False)], device=device)
    with pytest.raises(ValueError):
        data.augment_batch([u8[..., :3]], [(0, 0, 64, 64, False, False, False)], device=device)


def test_prepare_dataset_loader_workers_pinned(device, tmp_path):
    """MYprepare.prepare_dataset_train_COCOP3M's loader shape, unchanged: DataLoader(shuffle,
    pin_memory=True, num_workers=4) over COCOP3MDataset -- decode / draws / crop in the forked
    workers (no GPU there), one H2D copy + one augment launch per batch in this process -- and
    every image equal to the CPU restatement of __getitem__ for the parameters it drew.
    Also reports the pipeline's images/s (the DP config needs 16 per rank per step)."""
    import os
    import sys
    import time
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_data_loader import _write_pngs
    from rgbac import data
    coco, p3m = _write_pngs(str(tmp_path), 24, seed=7)
    loader, ds = data.prepare_dataset_train_COCOP3M(batch_size=4, COCOrootpath=coco,
                                                    P3Mrootpath=p3m, height=64, width=64,
                                                    num_workers=4, device=device)
    n = 0
    for batch in loader.loader:
        assert batch["pixels"].is_pinned()
        out = data.augment_packed(batch, 64, 64, device=device)
        for b, (off, h, w, flags, i, j, idx, _) in enumerate(batch["desc"].tolist()):
            u8 = data.decode_rgba(ds.images[idx])
            ref = data_ref.augment_one(u8, (i, j, h, w, bool(flags & 1), bool(flags & 2),
                                            bool(flags & 4)), 64, 64)
            for k in range(5):
                err = (out[k][b].cpu() - ref[k]).abs().max().item()
                assert err <= 2e-6, (idx, k, err)
            n += 1
    assert n == 24
    # the drop-in iterator: the reference's 5-tuple, already on the GPU
    got = next(iter(loader))
    assert len(got) == 5 and got[0].shape == (4, 3, 64, 64) and got[4].shape == (4, 4, 64, 64)
    assert all(t.is_cuda for t in got)
    # throughput at the training size (256x256 from ~480x640 sources)
    big = str(tmp_path / "big")
    from PIL import Image
    g = np.random.default_rng(3)
    os.makedirs(big, exist_ok=True)
    for k in range(64):
        Image.fromarray(g.integers(0, 256, size=(480, 640, 4), dtype=np.uint8), "RGBA").save(
            os.path.join(big, f"b{k:03d}.png"))
    loader, _ = data.prepare_dataset_train_COCOP3M(batch_size=16, COCOrootpath=big,
                                                   P3Mrootpath=big + "/none", num_workers=4,
                                                   device=device)
    for _ in loader:                                 # warm the workers / page cache
        pass
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(2):
        for _ in loader:
            pass
    torch.cuda.synchronize()
    ips = 128 / (time.perf_counter() - t0)
    print(f"data pipeline: {ips:.0f} images/s (480x640 PNG -> 256x256, batch 16, 4 workers)")
    assert ips > 16
