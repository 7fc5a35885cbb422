"""Time one conv layer shape across tile shapes / split-K (diagnostics, GPU only).

python tools/conv_probe.py --cin 96 --cout 192 --k 1 --hw 64 --batch 8 --groups 2 [--act gelu --res]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-learning-based-rgba-image-compression-with-masked-window-based-attention_amd")]

from rgbac import runtime as rt  # noqa: E402
from rgbac.layers.TransformRGB import prep_conv  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cin", type=int, default=96)
    ap.add_argument("--cout", type=int, default=192)
    ap.add_argument("--k", type=int, default=1)
    ap.add_argument("--stride", type=int, default=1)
    ap.add_argument("--hw", type=int, default=64)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--groups", type=int, default=1)
    ap.add_argument("--act", default="gelu")
    ap.add_argument("--res", action="store_true")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--only", default=None, help="tile,ksplit to run repeatedly (for rocprof)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    torch.manual_seed(0)
    mods = [torch.nn.Conv2d(a.cin, a.cout, a.k, stride=a.stride, padding=a.k // 2).to(dev)
            for _ in range(a.groups)]
    xs = [rt.to_nhwc(torch.randn(a.batch, a.cin, a.hw, a.hw, device=dev), dt) for _ in mods]
    ho = (a.hw + 2 * (a.k // 2) - a.k) // a.stride + 1
    res = [rt.to_nhwc(torch.randn(a.batch, a.cout, ho, ho, device=dev), dt) for _ in mods] \
        if a.res else [None] * a.groups
    preps = [prep_conv(m, [x.src()], act=a.act, res0=r) for m, x, r in zip(mods, xs, res)]
    flops = sum(p.flops for p in preps)
    nbytes = sum(p.nbytes for p in preps)
    cands = rt._candidates(preps[0].mgrid * a.groups, a.cout, preps[0].nst, preps[0].nks, True)
    if a.only:
        cands = [tuple(int(v) for v in a.only.split(","))]
    for cand in cands:
        rt.FORCE = cand
        rt.launch(preps)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            rt.launch(preps)
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) / a.iters * 1e3
        print(f"tile {cand[0]:2d} {rt.TILES[cand[0]]} ks {cand[1]}: {us:8.2f} us  {flops / us / 1e6:7.1f} TF/s  "
              f"{nbytes / us / 1e3:7.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
