"""CPU: the worker side of the GPU data pipeline through a REAL DataLoader with worker
processes (my_datasets/MYprepare.py:7-10: DataLoader(shuffle=True, pin_memory=True,
num_workers=4) over COCOP3MDataset).  __getitem__ and collate_rgba run in the workers and must
touch no GPU; each packed crop must be exactly the drawn crop box of the decoded PNG."""
import os

import numpy as np
import pytest
import torch

from rgbac import data


def _write_pngs(root, n, seed=0):
    from PIL import Image
    g = np.random.default_rng(seed)
    os.makedirs(os.path.join(root, "coco"), exist_ok=True)
    os.makedirs(os.path.join(root, "p3m"), exist_ok=True)
    shapes = []
    for k in range(n):
        h, w = int(g.integers(40, 200)), int(g.integers(40, 200))
        u8 = g.integers(0, 256, size=(h, w, 4), dtype=np.uint8)
        u8[: h // 3, :, 3] = 0
        sub = "coco" if k % 2 == 0 else "p3m"
        mode = "RGBA" if k % 5 else "RGB"                 # non-RGBA files get alpha 255
        img = Image.fromarray(u8 if mode == "RGBA" else u8[..., :3], mode)
        img.save(os.path.join(root, sub, f"img{k:03d}.png"))
        shapes.append((h, w))
    return os.path.join(root, "coco"), os.path.join(root, "p3m")


def test_items_are_cpu_crops(tmp_path):
    coco, p3m = _write_pngs(str(tmp_path), 6)
    ds = data.COCOP3MDataset(coco_path=coco, p3m_path=p3m, height=64, width=48)
    assert len(ds) == 6
    torch.manual_seed(0)
    for k in range(len(ds)):
        crop, p = ds[k]
        assert crop.device.type == "cpu" and crop.dtype == torch.uint8 and crop.shape[2] == 4
        u8 = data.decode_rgba(ds.images[k])
        i, j, h, w = (int(v) for v in p[:4])
        assert tuple(crop.shape[:2]) == (h, w) and int(p[7]) == k
        assert torch.equal(crop, torch.from_numpy(u8[i:i + h, j:j + w].copy()))


@pytest.mark.parametrize("workers", [0, 2])
def test_dataloader_with_workers(tmp_path, workers):
    coco, p3m = _write_pngs(str(tmp_path), 10, seed=1)
    loader, ds = data.prepare_dataset_train_COCOP3M(batch_size=4, COCOrootpath=coco,
                                                    P3Mrootpath=p3m, height=64, width=64,
                                                    num_workers=workers)
    assert len(loader) == 3 and loader.batch_size == 4
    seen = []
    for batch in loader.loader:                     # the workers' output, before the GPU step
        pix, desc = batch["pixels"], batch["desc"]
        assert pix.dtype == torch.uint8 and desc.shape[1] == 8
        for off, h, w, flags, i, j, idx, _ in desc.tolist():
            u8 = data.decode_rgba(ds.images[idx])
            want = torch.from_numpy(u8[i:i + h, j:j + w].copy()).reshape(-1)
            assert torch.equal(pix[off:off + h * w * 4], want)
            assert 0 <= flags < 8
            seen.append(idx)
    assert sorted(seen) == list(range(10))          # shuffle=True: a permutation
