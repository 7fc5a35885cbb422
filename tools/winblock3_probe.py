"""Time the ws-8 window-attention block: the head-pair kernel (winblock_kernel + winflag_kernel,
round 6, RGBAC_WINBLOCK_FORM=3) against the round-3 kernel (=2), each as N calls captured in one HIP
graph and replayed, on the bench's alpha pyramid level at the block's resolution (config 2:
B 8, 64^2; config 4: B 4, 256^2).  Prints us per call and TF/s on active-window FLOPs.
python tools/winblock3_probe.py [--configs 2,4] [--calls 50] [--reps 5]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-learning-based-rgba-image-compression-with-"
                                         "masked-window-based-attention_amd")]

from bench import synth_inputs  # noqa: E402
from rgbac import runtime as rt  # noqa: E402
from rgbac.layers.SupplyMask import mask_pyramid  # noqa: E402
from rgbac.layers.masked_win_attention import WinBasedAttention  # noqa: E402

FLOP_PER_TOKEN = 2.0 * (576 * 192 + 2 * 64 * 192 + 192 * 192)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="2,4")
    ap.add_argument("--calls", type=int, default=50)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variants", default="v3,v2,v3,v2")
    args = ap.parse_args()
    torch.manual_seed(0)
    m = WinBasedAttention(192, 8, 8, 0).cuda().eval()
    with torch.no_grad():
        m.attn.relative_position_bias_table.normal_(0, 0.5)
    for cfg in args.configs.split(","):
        B, S = {"2": (8, 256), "4": (4, 1024)}[cfg]
        _, a = synth_inputs(B, S, S)
        a = a.cuda()
        _, me = mask_pyramid(a, 4)
        alpha = me[1]                                  # the block's resolution (S / 4)
        s = S // 4
        x = rt.to_nhwc(torch.randn((B, 192, s, s), device="cuda"), torch.bfloat16)
        nact = int((alpha.reshape(B, s // 8, 8, s // 8, 8).abs().sum((2, 4)) > 0).sum())
        nwin = B * (s // 8) ** 2
        fl = nact * 64 * FLOP_PER_TOKEN
        for var in args.variants.split(","):
            if var == "v2":
                os.environ["RGBAC_WINBLOCK_FORM"] = "2"
            else:
                os.environ["RGBAC_WINBLOCK_FORM"] = "3"
            with torch.no_grad():
                for _ in range(3):
                    m.nhwc(x, alpha)
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                st = torch.cuda.Stream()
                st.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(st):
                    m.nhwc(x, alpha)
                torch.cuda.current_stream().wait_stream(st)
                with torch.cuda.graph(g):
                    for _ in range(args.calls):
                        m.nhwc(x, alpha)
            g.replay()
            torch.cuda.synchronize()
            ts = []
            for _ in range(args.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                g.replay()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3 / args.calls)
            us = sorted(ts)[len(ts) // 2]
            print(f"config {cfg} B{B} {s}x{s} {var}: {us:8.2f} us/call  active {nact}/{nwin}  "
                  f"{fl / us / 1e6:7.1f} TF/s active-window ({fl / us / 1e6 / 25:.1f} % of 2.5 PF)",
                  flush=True)
            del g
    os.environ.pop("RGBAC_WINBLOCK_FORM", None)


if __name__ == "__main__":
    main()
