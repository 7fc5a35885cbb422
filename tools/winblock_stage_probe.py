"""Per-phase cycle breakdown of winblock_kernel (csrc/winblock.hip built with -DRGBAC_WB_TIMING
into rgbac/librgbac_wbprof.so): clock64() stamps of wave 0 of every workgroup at each head
pair's start (after the pair's barrier), qkv done, exchange barrier passed, attention (+ proj)
done.  python tools/winblock_stage_probe.py [--batch B --size S --alpha ones|half]"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deep-learning-based-rgba-image-compression-with-masked-window-based-attention_amd")
os.environ["RGBAC_LIB_PATH"] = os.path.join(PKG, "rgbac", "librgbac_wbprof.so")
sys.path.insert(0, PKG)
import numpy as np   # noqa: E402
import torch         # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--alpha", default="ones", choices=["ones", "half"])
    args = ap.parse_args()
    from rgbac import _lib, runtime as rt
    from rgbac.layers.masked_win_attention import WinBasedAttention
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = WinBasedAttention(192, 8, 8, 4).to(dev).eval()
    B, S = args.batch, args.size
    x = rt.to_nhwc(torch.randn((B, 192, S, S), device=dev), torch.bfloat16)
    alpha = torch.ones((B, 1, S, S), device=dev)
    if args.alpha == "half":
        alpha[1::2, :, :, : S // 2] = 0
    with torch.no_grad():
        for _ in range(5):
            m.nhwc(x, alpha)
        torch.cuda.synchronize()
    nblk = min(8192, (B * (S // 8) ** 2 + 1) // 2)
    buf = (ctypes.c_ulonglong * (nblk * 20))()
    assert _lib.load().rgbac_debug_wb_times(buf, nblk) == 0
    a = np.frombuffer(buf, dtype=np.uint64).astype(np.int64)
    t = a[:nblk * 18].reshape(nblk, 18)
    wc = a[nblk * 18:].reshape(nblk, 2)
    live = t[:, 17] > t[:, 0]                       # both-transparent workgroups exit early
    t, wc = t[live], wc[live]
    print(f"B{B} {S}x{S} alpha {args.alpha}: {live.sum()} computing workgroups of {nblk}")
    print(f"  total        median {np.median(t[:, 17] - t[:, 0]):8.0f} cycles")
    print(f"  setup        median {np.median(t[:, 1] - t[:, 0]):8.0f}  (gather, weights + x, tables)")
    names = ["qkv", "barrier A", "attention(+proj)", "barrier B"]
    for p in range(4):
        seg = [(t[:, 2 + 4 * p] - t[:, 1 + 4 * p]), (t[:, 3 + 4 * p] - t[:, 2 + 4 * p]),
               (t[:, 4 + 4 * p] - t[:, 3 + 4 * p])]
        if p < 3:
            seg.append(t[:, 5 + 4 * p] - t[:, 4 + 4 * p])
        print(f"  pair {p}: " + "  ".join(f"{n} {np.median(d):6.0f}" for n, d in zip(names, seg)))
    print(f"  epilogue     median {np.median(t[:, 17] - t[:, 16]):8.0f}")
    t0 = wc[:, 0].min()
    st, en = (wc[:, 0] - t0) / 100.0, (wc[:, 1] - t0) / 100.0
    print(f"wall: span {en.max():.1f} us; workgroup duration median {np.median(en - st):.1f} us; "
          f"start p50 {np.median(st):.1f} p90 {np.percentile(st, 90):.1f} us")
    cyc = np.median(t[:, 17] - t[:, 0]) / np.median(en - st)
    print(f"shader clock ~ {cyc / 1e3:.2f} GHz")


if __name__ == "__main__":
    main()
