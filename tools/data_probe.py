"""Time the batched augmentation launch (rgbac/data.py) on COCO-sized sources resident in HBM,
and the reference-style CPU transform (torch CPU crop+interpolate+flip, oracle/data_ref.py)
on the same items.  Prints one JSON line."""
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


if __name__ == "__main__":
    main()
