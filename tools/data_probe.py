"""Time the batched augmentation launch (rgbac/data.py) on COCO-sized sources resident in HBM,
and the reference-style CPU transform (torch CPU crop+interpolate+flip, oracle/data_ref.py)
on the same items.  Prints one JSON line.  ``--pipeline``: the whole input pipeline of a DP
step (worker-side PNG decode + crop, main-process collate + H2D + augment launch) at 16 and
128 images."""
import json
import os
import random
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-learning-based-rgba-image-compression-with-masked-window-based-attention_amd")]
from rgbac import data, _lib          # noqa: E402
from oracle import data_ref           # noqa: E402


def main(B=8, iters=50):
    torch.manual_seed(0)
    random.seed(0)
    g = np.random.default_rng(0)
    shapes = [(480, 640), (427, 640), (640, 480), (500, 375)] * (B // 4)
    imgs = [g.integers(0, 256, size=(h, w, 4), dtype=np.uint8) for h, w in shapes]
    params = [data.draw_params(h, w) for h, w in shapes]
    dev = torch.device("cuda:0")
    srcs = [torch.from_numpy(u).to(dev) for u in imgs]
    arr = (data._Desc * B)()
    for k, (t, p) in enumerate(zip(srcs, params)):
        i, j, h, w, fh, fv, fill = p
        arr[k] = data._Desc(t.data_ptr(), t.shape[0], t.shape[1], i, j, h, w,
                            int(fh) | (int(fv) << 1) | (int(fill) << 2), 0)
    descs = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(dev)
    outs = [torch.empty((B, c, 256, 256), device=dev) for c in (3, 1, 3, 4)]

    def launch():
        _lib.call("rgbac_rgba_augment", B, descs.data_ptr(), 256, 256, 1,
                  *[o.data_ptr() for o in outs], _lib.stream_ptr(dev))
    for _ in range(5):
        launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        launch()
    e1.record()
    torch.cuda.synchronize()
    gpu_ms = e0.elapsed_time(e1) / iters
    # algorithmic bytes: each covered source pixel read once (4 B) + 44 B written per output px
    src_bytes = sum(p[2] * p[3] * 4 for p in params)
    dst_bytes = B * 256 * 256 * 44
    t0 = time.perf_counter()
    for u, p in zip(imgs, params):
        data_ref.augment_one(u, p)
    cpu_ms = (time.perf_counter() - t0) * 1e3
    print(json.dumps({"batch": B, "gpu_ms_per_batch": round(gpu_ms, 4),
                      "gpu_items_per_s": round(B / gpu_ms * 1e3, 1),
                      "gbps": round((src_bytes + dst_bytes) / gpu_ms / 1e6, 1),
                      "cpu_ms_per_batch": round(cpu_ms, 2), "cpu_threads": torch.get_num_threads()}))


def pipeline(per_rank=16, ranks=8, n_png=32, iters=20):
    """The whole input pipeline of a DP step at BASELINE config 5 (16 images per rank, 128 per
    step on 8 GPUs): worker side = COCOP3MDataset.__getitem__ (PNG decode + parameter draw +
    crop) per item on one core, on synthetic 640x480 / 427x640 RGBA PNGs (random pixels:
    they compress worse than photos, so decode is pessimistic); main process = collate_rgba
    (pinned) + augment_packed (one H2D copy + one launch) per rank batch.  Prints one JSON line
    with the rates against the training step's need."""
    import tempfile
    from PIL import Image
    g = np.random.default_rng(1)
    tmp = tempfile.mkdtemp(prefix="rgbac_png_")
    shapes = [(480, 640), (427, 640), (640, 480), (500, 375)]
    for k in range(n_png):
        h, w = shapes[k % 4]
        a = g.integers(0, 256, size=(h, w, 4), dtype=np.uint8)
        a[..., 3] = np.where(g.random((h, w)) < 0.3, 0, 255)
        Image.fromarray(a, "RGBA").save(os.path.join(tmp, f"{k:04d}.png"))
    ds = data.COCOP3MDataset(coco_path=tmp, p3m_path=tmp + "_none")
    t0 = time.perf_counter()
    items = [ds[k % len(ds)] for k in range(n_png * 2)]
    worker_ms = (time.perf_counter() - t0) * 1e3 / len(items)
    dev = torch.device("cuda:0")
    res = {"png_items": len(items), "worker_ms_per_item_1core": round(worker_ms, 3)}
    for B in (per_rank, per_rank * ranks):
        batch_items = [items[k % len(items)] for k in range(B)]
        data.collate_rgba(batch_items)          # warm-up (torch's first CPU copy pays a one-off)
        t0 = time.perf_counter()
        for _ in range(iters):
            batch = data.collate_rgba(batch_items)
        collate_ms = (time.perf_counter() - t0) * 1e3 / iters
        batch = {k: v.pin_memory() for k, v in batch.items()}
        for _ in range(3):
            data.augment_packed(batch, device=dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            out = data.augment_packed(batch, device=dev)
        torch.cuda.synchronize()
        main_ms = (time.perf_counter() - t0) * 1e3 / iters
        res[f"B{B}"] = {"collate_ms": round(collate_ms, 3), "h2d_augment_ms": round(main_ms, 3),
                        "main_process_img_per_s": round(B / (collate_ms + main_ms) * 1e3, 1)}
    res["need_img_per_s_per_rank"] = "16 per training step: 16 / 25 ms = 640 img/s (config 3 graph step)"
    res["workers_needed_per_rank"] = round(640 * worker_ms / 1e3, 2)
    print(json.dumps(res))


if __name__ == "__main__":
    if sys.argv[1:] == ["--pipeline"]:
        pipeline()
    else:
        main()
