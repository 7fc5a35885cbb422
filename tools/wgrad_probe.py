"""Time the weight-gradient kernel (rgbac.autograd.wgrad: rgbac_conv_wgrad + slab reduce) on one
conv shape, e.g. the slice-stack 3x3 224->128 at 32x32, B16 (bench helper / PMC driver).

  python tools/wgrad_probe.py --cin 224 --cout 128 --hw 32 --batch 16 --ksize 3 --iters 50
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deep-learning-based-rgba-image-compression-with-masked-window-based-attention_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cin", type=int, default=224)
    ap.add_argument("--cout", type=int, default=128)
    ap.add_argument("--hw", type=int, default=32)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--ksize", type=int, default=3)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--stride", type=int, default=1, help="2: the source at twice --hw")
    a = ap.parse_args()
    from rgbac import runtime as rt
    from rgbac.autograd import wgrad
    dev = torch.device("cuda:0")
    G = rt.to_nhwc(torch.randn((a.batch, a.cout, a.hw, a.hw), device=dev), torch.bfloat16)
    sh = a.hw * a.stride
    S = rt.to_nhwc(torch.randn((a.batch, a.cin, sh, sh), device=dev), torch.bfloat16)
    n_pad = rt.round_up(G.ldc, 64)
    k_pad = rt.round_up(a.ksize * a.ksize * S.ldc, 64)
    fmap = torch.arange(n_pad * k_pad, dtype=torch.int32, device=dev).view(n_pad, k_pad)
    numel = n_pad * k_pad
    run = lambda: wgrad(G, [S], a.ksize, a.stride, a.ksize // 2, False, k_pad, fmap,  # noqa: E731
                        numel)
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        run()
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) / a.iters * 1e3
    flop = 2.0 * a.batch * a.hw * a.hw * a.cout * a.ksize * a.ksize * a.cin
    print(f"wgrad k{a.ksize}s{a.stride} {a.cin}->{a.cout} {a.hw}x{a.hw} B{a.batch}: {us:.1f} us "
          f"(kernel + reduce), {flop / us / 1e6:.1f} TF/s")


if __name__ == "__main__":
    main()
