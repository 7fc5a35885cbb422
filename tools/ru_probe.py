"""Time the fused ResidualUnit kernel (csrc/fused.hip) on one shape (bench helper)."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deep-learning-based-rgba-image-compression-with-masked-window-based-attention_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--hw", type=int, default=64)
    ap.add_argument("--groups", type=int, default=2)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--kind", type=int, default=0,
                    help="0: ResidualUnit (GELU epilogues); 1: the same kernel shape with ReLU "
                         "epilogues (ResBlock) -- the difference is the GELU cost")
    a = ap.parse_args()
    from rgbac import runtime as rt
    from rgbac.layers.Masked_Attention import ResidualUnit, run_bottlenecks_fused
    dev = torch.device("cuda:0")
    us = [ResidualUnit(192).to(dev) for _ in range(a.groups)]
    xs = [rt.to_nhwc(torch.randn((a.batch, 192, a.hw, a.hw), device=dev), torch.bfloat16)
          for _ in range(a.groups)]
    with torch.no_grad():
        def run():
            return run_bottlenecks_fused([((u.conv[0], u.conv[2], u.conv[4]), x)
                                          for u, x in zip(us, xs)], a.kind)
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            run()
        e1.record()
        e1.synchronize()
    us_per = e0.elapsed_time(e1) / a.iters * 1e3
    print(f"ru_fused kind {a.kind} g{a.groups} B{a.batch} {a.hw}x{a.hw}: {us_per:.1f} us")


if __name__ == "__main__":
    main()
