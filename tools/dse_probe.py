"""Time the fused DSE launches (rgbac_dse_block, modes first / mid / last) against the
unfused DSE at 256x256 B8 (bf16).  python tools/dse_probe.py [--reps N] [--mode M]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-learning-based-rgba-image-compression-with-"
                                         "masked-window-based-attention_amd")]

from rgbac import runtime as rt  # noqa: E402
from rgbac.layers.TransformRGB import DSE, dse_fused  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--unfused", action="store_true")
    ap.add_argument("--mode", type=int, default=None, help="only this fused launch (0/1/2)")
    args = ap.parse_args()
    torch.manual_seed(0)
    m = DSE(32).cuda().eval()
    x = rt.to_nhwc(torch.rand((args.batch, 3, args.size, args.size), device="cuda"),
                   torch.bfloat16)
    prof = rt.LaunchProfiler()
    with torch.no_grad():
        rt.DSE_FUSED = not args.unfused
        run = (lambda: m.nhwc(x)) if args.unfused else (lambda: dse_fused(m, x, only=args.mode))
        run()
        torch.cuda.synchronize()
        rt.PROFILER = prof
        for _ in range(args.reps):
            run()
        rt.PROFILER = None
    for desc, (n, ms, fl, nb) in sorted(prof.layers().items()):
        us = ms / n * 1e3
        print(f"{us:9.2f} us  {fl / n / us / 1e6:8.1f} TF/s  {nb / n / us / 1e3:8.1f} GB/s  {desc}")


if __name__ == "__main__":
    main()
