"""Time the C = 80 ResidualUnit kernel (ru_small_kernel, csrc/fused.hip) on the latent shapes of
config 2 (B 8, 32^2) and config 4 (B 4, 128^2): GELU vs ReLU epilogues (kind 0 / 1: the
difference is the GELU cost) and one vs two 4-wave halves per workgroup (RGBAC_RU_SMALL_DUAL)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deep-learning-based-rgba-image-compression-with-masked-window-based-attention_amd"))


def main():
    from rgbac import runtime as rt
    from rgbac.layers.Masked_Attention import ResidualUnit, run_bottlenecks_fused
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    for batch, hw in ((8, 32), (4, 128)):
        us = [ResidualUnit(80).to(dev) for _ in range(2)]
        xs = [rt.to_nhwc(torch.randn((batch, 80, hw, hw), device=dev), torch.bfloat16)
              for _ in range(2)]
        for dual in ("0", "2"):
            os.environ["RGBAC_RU_SMALL_DUAL"] = dual
            for kind in (0, 1):
                with torch.no_grad():
                    def run():
                        return run_bottlenecks_fused([((u.conv[0], u.conv[2], u.conv[4]), x)
                                                      for u, x in zip(us, xs)], kind)
                    for _ in range(3):
                        run()
                    torch.cuda.synchronize()
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(50):
                        run()
                    e1.record()
                    e1.synchronize()
                t = e0.elapsed_time(e1) / 50 * 1e3
                fl = 2 * batch * hw * hw * 2 * (80 * 40 + 9 * 40 * 40 + 40 * 80)
                print(f"B{batch} {hw}x{hw} dual={dual} kind={kind}: {t:7.1f} us/launch "
                      f"({fl / t / 1e6:6.1f} TF/s)", flush=True)


if __name__ == "__main__":
    main()
