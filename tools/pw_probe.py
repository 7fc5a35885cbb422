"""Time the forward pointwise launches of config 2 (GDN / IGDN at 64^2 and 128^2, the attention
gate at 64^2; B = 8, C = 192, bf16) on the pointwise tile, events around 50 back-to-back
launches per shape (one HIP graph replay).  Run twice to A/B the kernels:  RGBAC_PW2=0 python tools/pw_probe.py"""
import os
import sys

import torch
import torch.nn as nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-learning-based-rgba-image-compression-with-masked-window-based-attention_amd")]


def main():
    from rgbac import runtime as rt
    dev = torch.device("cuda:0")
    dt = torch.bfloat16
    g = torch.Generator().manual_seed(0)
    rows = []
    for kind, H in (("gdn", 64), ("igdn", 64), ("gate", 64), ("igdn", 128)):
        B, C = 8, 192
        m = nn.Conv2d(C, C, 1)
        with torch.no_grad():
            m.weight.copy_(0.1 * torch.rand(C, C, 1, 1, generator=g))
            m.bias.copy_(0.5 + torch.rand(C, generator=g))
        md = m.to(dev)
        fx = rt.to_nhwc(torch.randn((B, C, H, H), generator=g).to(dev), dt)
        fa = rt.to_nhwc(torch.randn((B, C, H, H), generator=g).to(dev), dt)
        fr = rt.to_nhwc(torch.randn((B, C, H, H), generator=g).to(dev), dt)
        pk = rt.packed(md, dt, [(C, C)])
        out = rt.new_feat(B, H, H, C, dt, dev)
        rt.FORCE = (rt.TILE_PW, 1)

        def run():
            if kind == "gate":
                rt.conv(pk, [fx.src()], act="gate", res1=fa, res2=fr, out=out)
            else:
                rt.conv(pk, [fx.src()], square=True, act=kind, res1=fx, out=out)
        with torch.no_grad():
            for _ in range(5):
                run()
            torch.cuda.synchronize()
            # 50 launches captured in a HIP graph: the replay times the GPU, not the host
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                for _ in range(50):
                    run()
            graph.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            graph.replay()
            e1.record()
            torch.cuda.synchronize()
        rt.FORCE = None
        us = e0.elapsed_time(e1) / 50 * 1e3
        nbytes = B * H * H * C * 2 * (4 if kind == "gate" else 2)
        rows.append(f"{kind:5s} {H:4d}^2  {us:7.2f} us  {nbytes / us / 1e3:7.1f} GB/s (algorithmic "
                    f"{nbytes / 1e6:.1f} MB)")
    tag = os.environ.get("RGBAC_PW2", "1") + ("all" if os.environ.get("RGBAC_PW2_ALL") == "1" else "")
    for r in rows:
        print(f"PW2={tag} {r}", flush=True)


if __name__ == "__main__":
    main()
