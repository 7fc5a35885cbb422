"""Every tile the autotuner would consider, timed like the tuner (L2s flushed by a 64 MB write
before each run, 3 runs summed) on the model's conv shapes: which tile wins per shape and by
how much.  python tools/tile_probe.py [--only SUBSTR]"""
import argparse
import os
import sys

import torch
import torch.nn as nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-learning-based-rgba-image-compression-with-"
                                         "masked-window-based-attention_amd")]

from rgbac import runtime as rt  # noqa: E402
from rgbac.layers.TransformRGB import prep_conv, prep_subpel  # noqa: E402
from rgbac.layers._blocks import subpel_conv3x3  # noqa: E402

# name, cin list, cout, k, H, W, B, groups, kind ("conv" | "gdn" | "gate")
SHAPES = [
    ("igdn 192 128^2", [192], 192, 1, 128, 128, 8, 1, "igdn"),
    ("gdn 192 64^2", [192], 192, 1, 64, 64, 8, 1, "gdn"),
    ("gate 192 64^2", [192], 192, 1, 64, 64, 8, 1, "gate"),
    ("igdn 192 32^2", [192], 192, 1, 32, 32, 8, 1, "igdn"),
    ("1x1 80->192 32^2", [80], 192, 1, 32, 32, 8, 1, "conv"),
    ("cc2 224->128 g2", [224], 128, 3, 32, 32, 8, 2, "conv"),
    ("lrp2 224->128 g1", [224], 128, 3, 32, 32, 8, 1, "conv"),
    ("cc1 88->224 g2", [80, 8], 224, 3, 32, 32, 8, 2, "conv"),
    ("cc1 120->224 g10", [80, 40], 224, 3, 32, 32, 8, 10, "conv"),
    ("lrp1 128->224 g5", [80, 40, 8], 224, 3, 32, 32, 8, 5, "conv"),
    ("cc2 224->128 g10", [224], 128, 3, 32, 32, 8, 10, "conv"),
    ("hs 256->288 g2 16x16", [256], 288, 3, 16, 16, 8, 2, "conv"),
    ("hs subpel 288->80 g2 16x16", [288], 80, 3, 16, 16, 8, 2, "subpel"),
    ("ha 320->288 16x16", [320], 288, 3, 16, 16, 8, 1, "conv"),
    # the strided analysis / synthesis convs (5x5 stride 2; TransformRGB.py:57-58, 83-84)
    ("5x5s2 E.x2 192 128^2", [192], 192, 5, 128, 128, 8, 1, "s2"),
    ("5x5s2 E.x3 192 64^2", [192], 192, 5, 64, 64, 8, 1, "s2"),
    ("5x5s2 D.x2 convT 192 32^2", [192], 192, 5, 32, 32, 8, 1, "convT"),
    ("5x5s2 D.x3 convT 192 64^2", [192], 192, 5, 64, 64, 8, 1, "convT"),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda")
    dt = torch.bfloat16
    flush = torch.zeros(16 << 20, device=dev)
    for name, cins, cout, k, H, W, B, G, kind in SHAPES:
        if args.only and args.only not in name:
            continue
        preps = []
        for gi in range(G):
            torch.manual_seed(gi)
            if kind == "subpel":
                m = subpel_conv3x3(sum(cins), cout, 2)
            elif kind == "convT":
                m = nn.ConvTranspose2d(sum(cins), cout, k, stride=2, padding=k // 2,
                                       output_padding=1)
            else:
                m = nn.Conv2d(sum(cins), cout, k, stride=2 if kind == "s2" else 1,
                              padding=k // 2)
            m = m.to(dev)
            if kind in ("gdn", "igdn"):
                with torch.no_grad():
                    m.weight.uniform_(0, 0.01)
                    m.bias.uniform_(0.5, 1.0)
            fs = [rt.to_nhwc(torch.randn((B, c, H, W), device=dev), dt) for c in cins]
            srcs = [f.src() for f in fs]
            if kind in ("gdn", "igdn"):
                pk = rt.packed(m, dt, [(cins[0], rt.round_up(cins[0], 8))])
                preps.append(rt.prepare(pk, srcs, square=True, act=kind, res1=fs[0]))
            elif kind == "gate":
                r1 = rt.to_nhwc(torch.randn((B, cout, H, W), device=dev), dt)
                pk = rt.packed(m, dt, [(cins[0], rt.round_up(cins[0], 8))])
                preps.append(rt.prepare(pk, srcs, act="gate", res1=r1, res2=r1))
            elif kind == "subpel":
                preps.append(prep_subpel(m, srcs))
            else:
                preps.append(prep_conv(m, srcs, act="gelu"))
        p0 = preps[0]
        cands = rt._candidates(p0.mgrid * p0.nphase * G, cout, max(p.nst for p in preps),
                               max(p.nks for p in preps), p0.pk.mode == rt.CONV,
                               rt._spatial_ok(preps), rt._smallk_ok(preps), rt._wstream_ok(preps))
        cands += [(t, 1) for t in rt._patch_tiles(preps)]
        if rt._pw_ok(preps):
            cands.append((rt.TILE_PW, 1))
        if rt._npatch_ok(preps):
            cands.append((rt.TILE_NPATCH, 1))
        flops = sum(p.flops for p in preps)
        res = []
        with torch.no_grad():
            for c in cands:
                try:
                    rt.launch(preps, force=c)
                except RuntimeError as e:
                    res.append((float("inf"), c, str(e)[:60]))
                    continue
                torch.cuda.synchronize()
                us = 0.0
                for _ in range(3):
                    flush.add_(1)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    rt.launch(preps, force=c)
                    e1.record()
                    e1.synchronize()
                    us += e0.elapsed_time(e1) * 1e3 / 3
                res.append((us, c, rt.kernel_name(c[0], preps)))
        res.sort(key=lambda r: r[0])
        print(f"== {name}: {flops / 1e9:.2f} GFLOP", flush=True)
        for us, c, kn in res[:8]:
            print(f"   {us:8.1f} us {flops / max(us, 1e-9) / 1e6:7.1f} TF/s  {c}  {kn}", flush=True)


if __name__ == "__main__":
    main()
