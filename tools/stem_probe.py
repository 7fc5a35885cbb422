"""Time the fused stem+GDN launch vs the unfused pair at 8x256x256 (diagnostics, GPU only)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-learning-based-rgba-image-compression-with-masked-window-based-attention_amd")]

from rgbac import runtime as rt  # noqa: E402
from rgbac.layers.TransformRGB import Analysis_transform  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    enc = Analysis_transform(192, 80).to(dev)
    x = rt.to_nhwc(torch.rand((8, 3, 256, 256), device=dev), torch.bfloat16)
    for fused in (True, False):
        rt.STEM_FUSED = fused
        with torch.no_grad():
            for _ in range(3):
                enc._stem(x)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                enc._stem(x)
            e1.record()
            e1.synchronize()
        print(f"fused={fused}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us", flush=True)


if __name__ == "__main__":
    main()
