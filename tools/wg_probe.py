"""Per-workgroup phase timing of the slice-chain conv kernels (csrc/conv.hip built with
-DRGBAC_WG_TIMING into rgbac/librgbac_wgprof.so: `make -C csrc wgprof`): one cold launch per
shape (L2s flushed by a 64 MB write first, as in the forward graph), then the 100-MHz
wall-clock stamps of every workgroup -- start, operands staged / K loop entered, K loop done,
end -- as the kernel span, the dispatch spread and the median phase durations."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deep-learning-based-rgba-image-compression-with-masked-window-based-attention_amd")
os.environ["RGBAC_LIB_PATH"] = os.path.join(PKG, "rgbac", "librgbac_wgprof.so")
sys.path[:0] = [ROOT, PKG]
import numpy as np   # noqa: E402
import torch         # noqa: E402
import torch.nn as nn  # noqa: E402

# name, cin (list of source widths), cout, act, groups, tile
SHAPES = [
    ("cc1 88->224 g2 fpatch", [80, 8], 224, "gelu", 2, 45),
    ("cc2 224->128 g2 KS3", [224], 128, "gelu", 2, 52),
    ("cc2 224->128 g2 fpatch", [224], 128, "gelu", 2, 45),
    ("lrp1 96->224 g1", [80, 8, 8], 224, "gelu", 1, 45),
    ("lrp2 224->128 g1 KS3", [224], 128, "gelu", 1, 51),
    ("lrp3 128->8 wstream", [128], 8, "none", 1, 35),
    ("mu|sigma 256->16 wstream", [128, 128], 16, "none", 1, 35),
    ("cc2 224->128 g10 KS3", [224], 128, "gelu", 10, 52),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", type=int, default=32)
    args = ap.parse_args()
    from rgbac import _lib, runtime as rt
    from rgbac.layers.TransformRGB import prep_conv
    lib = _lib.load()
    lib.rgbac_debug_wg_times.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda:0")
    B, H = args.batch, args.size
    flush = torch.zeros(16 << 20, device=dev)
    for name, cins, cout, act, G, tile in SHAPES:
        preps = []
        for gi in range(G):
            torch.manual_seed(gi)
            m = nn.Conv2d(sum(cins), cout, 3, padding=1).to(dev)
            srcs = [rt.to_nhwc(torch.randn((B, c, H, H), device=dev), torch.bfloat16).src()
                    for c in cins]
            preps.append(prep_conv(m, srcs, act=act))
        with torch.no_grad():
            for _ in range(3):
                rt.launch(preps, force=(tile, 1))
            torch.cuda.synchronize()
            spans = []
            rows = []
            for rep in range(5):
                flush.add_(1)
                assert lib.rgbac_debug_wg_reset() == 0
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                rt.launch(preps, force=(tile, 1))
                e1.record()
                torch.cuda.synchronize()
                n = 16384
                buf = (ctypes.c_ulonglong * (n * 4))()
                assert lib.rgbac_debug_wg_times(buf, n) == 0
                t = np.frombuffer(buf, dtype=np.uint64).astype(np.int64).reshape(n, 4)
                t = t[t[:, 0] > 0]
                t0 = t[:, 0].min()
                st = (t[:, 0] - t0) / 100.0
                en = (t[:, 3] - t0) / 100.0
                ph = np.diff(t, axis=1) / 100.0
                spans.append(e0.elapsed_time(e1) * 1e3)
                rows.append((len(t), en.max(), np.median(en - st), np.percentile(en - st, 90),
                             np.median(st), st.max(), *np.median(ph, axis=0)))
        r = np.median(np.array(rows), axis=0)
        print(f"{name:26s} event {np.median(spans):6.1f} us | {int(r[0]):5d} WGs span {r[1]:6.1f} "
              f"WG dur p50 {r[2]:5.1f} p90 {r[3]:5.1f} | start p50 {r[4]:5.1f} max {r[5]:5.1f} | "
              f"phases: stage {r[6]:5.1f} K {r[7]:5.1f} epi {r[8]:5.1f} us", flush=True)


if __name__ == "__main__":
    main()
