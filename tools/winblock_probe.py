"""Time the fused window-attention block (rgbac_winattn_block) against the unfused
qkv GEMM + core + MASKSEL proj at 64x64 B8 (bf16).  python tools/winblock_probe.py"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-learning-based-rgba-image-compression-with-"
                                         "masked-window-based-attention_amd")]

from rgbac import runtime as rt  # noqa: E402
from rgbac.layers.masked_win_attention import WinBasedAttention  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--shift", type=int, default=4)
    ap.add_argument("--unfused", action="store_true")
    ap.add_argument("--alpha", default="half", choices=["half", "ones"])
    args = ap.parse_args()
    torch.manual_seed(0)
    m = WinBasedAttention(192, 8, 8, args.shift).cuda().eval()
    S = args.size
    x = rt.to_nhwc(torch.randn((args.batch, 192, S, S), device="cuda"), torch.bfloat16)
    alpha = torch.ones((args.batch, 1, S, S), device="cuda")
    if args.alpha == "half":
        alpha[1::2, :, :, : S // 2] = 0
    # active windows (judged in the shifted frame, masked_win_attention.py:178-190)
    ar = torch.roll(alpha, (-args.shift, -args.shift), (2, 3)).cpu()
    nact = int((ar.reshape(args.batch, S // 8, 8, S // 8, 8).abs().sum((2, 4)) > 0).sum())
    nwin = args.batch * (S // 8) ** 2
    prof = rt.LaunchProfiler()
    rt.WINBLOCK_FUSED = not args.unfused
    with torch.no_grad():
        m.nhwc(x, alpha)
        torch.cuda.synchronize()
        rt.PROFILER = prof
        for _ in range(args.reps):
            m.nhwc(x, alpha)
        rt.PROFILER = None
    tot = 0.0
    for desc, (n, ms, fl, nb) in sorted(prof.layers().items()):
        us = ms / n * 1e3
        tot += us
        print(f"{us:9.2f} us  {fl / n / us / 1e6:8.1f} TF/s  {nb / n / us / 1e3:8.1f} GB/s  {desc}")
    print(f"{tot:9.2f} us  total ({'unfused' if args.unfused else 'fused'})")
    fl = nact * 64 * 2.0 * (576 * 192 + 2 * 64 * 192 + 192 * 192)
    print(f"active windows {nact}/{nwin}: {fl / tot / 1e6:.1f} TF/s on active-window FLOPs "
          f"({fl / tot / 1e6 / 2500 * 100:.1f} % of 2.5 PF dense bf16)")


if __name__ == "__main__":
    main()
