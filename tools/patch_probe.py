"""Time the conv tiles on the model's conv shapes (bf16): im2col ring tiles vs the
patch-resident tiles.  python tools/patch_probe.py [--reps N]"""
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

SHAPES = [  # name, kind, cin, cout, H, W, B, groups
    ("convT x3 192 64->128", "convt", 192, 192, 64, 64, 8, 1),
    ("convT x2 192 32->64", "convt", 192, 192, 32, 32, 8, 1),
    ("x3 s2 192 64->32", "s2", 192, 192, 64, 64, 8, 1),
    ("x2 s2 192 128->64", "s2", 192, 192, 128, 128, 8, 1),
    ("cc1 120->224 g10", "conv", 120, 224, 32, 32, 8, 10),
    ("cc2 224->128 g2", "conv", 224, 128, 32, 32, 8, 2),
    ("cc2 224->128 g10", "conv", 224, 128, 32, 32, 8, 10),
    ("cc1 88->224 g2", "conv", 88, 224, 32, 32, 8, 2),
    ("lrp2 224->128 g1", "conv", 224, 128, 32, 32, 8, 1),
    ("lrp1 96->224 g1", "conv", 96, 224, 32, 32, 8, 1),
    ("ru 40->40 g2", "conv", 40, 40, 32, 32, 8, 2),
    ("x4 subpel 192->12", "subpel", 192, 12, 128, 128, 8, 1),
    ("hs 256->288 g2 16x16", "conv", 256, 288, 16, 16, 8, 2),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--shape", default=None, help="substring of a shape name: only that shape")
    ap.add_argument("--tile", type=int, default=None, help="only this tile (for rocprofv3)")
    args = ap.parse_args()
    dev = torch.device("cuda")
    dt = torch.bfloat16
    for name, kind, cin, cout, H, W, B, G in SHAPES:
        if args.shape and args.shape not in name:
            continue
        preps = []
        for gi in range(G):
            torch.manual_seed(gi)
            if kind == "convt":
                m = nn.ConvTranspose2d(cin, cout, 5, 2, 2, 1).to(dev)
            elif kind == "conv":
                m = nn.Conv2d(cin, cout, 3, padding=1).to(dev)
            elif kind == "s2":
                m = nn.Conv2d(cin, cout, 5, 2, 2).to(dev)
            else:
                m = subpel_conv3x3(cin, cout, 2).to(dev)
            x = rt.to_nhwc(torch.randn((B, cin, H, W), device=dev), dt)
            preps.append(prep_subpel(m, [x.src()]) if kind == "subpel"
                         else prep_conv(m, [x.src()], act="none" if kind in ("s2", "convt") else "gelu"))
        flops = sum(p.flops for p in preps)
        cands = rt._candidates(preps[0].mgrid * preps[0].nphase * G, cout, preps[0].nst,
                               preps[0].nks, preps[0].pk.mode == rt.CONV, False, False, False)
        cands += rt._patch_cands(preps)
        if args.tile is not None:
            cands = [(args.tile, 1)]
        res = []
        ref = None
        diffs = {}
        for c in cands:
            with torch.no_grad():
                outs = rt.launch(preps, force=c)
                torch.cuda.synchronize()
                # outputs against the first candidate's (the split / 16-row tiles' parity)
                o = torch.cat([t.t.float().flatten() for t in outs])
                if ref is None:
                    ref = o.clone()
                diffs[c] = (o - ref).abs().max().item() / max(ref.abs().max().item(), 1e-30)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    rt.launch(preps, force=c)
                e1.record()
                e1.synchronize()
            us = e0.elapsed_time(e1) / args.reps * 1e3
            res.append((us, c))
        res.sort()
        old = [r for r in res if r[1][0] < rt.FIRST_PATCH]
        best_old = min(old) if old else (float("nan"), None)
        best_new = [r for r in res if r[1][0] >= rt.FIRST_PATCH]
        line = f"{name:24s} {flops / 1e9:7.2f} GF | best im2col {best_old[1]} {best_old[0]:8.1f} us " \
               f"{flops / best_old[0] / 1e6:7.1f} TF/s"
        for us, c in sorted(best_new, key=lambda r: r[1]):
            line += (f" | {rt.kernel_name(c[0], preps)[18:]}/ks{c[1]} {us:7.1f} us "
                     f"{flops / us / 1e6:6.1f} TF/s rel {diffs[c]:.1e}")
        print(line, flush=True)


if __name__ == "__main__":
    main()
