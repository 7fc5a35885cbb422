"""Per-stage cycle breakdown of ru_stream_kernel (csrc/fused.hip built with -DRGBAC_RU_TIMING
into rgbac/librgbac_ruprof.so): clock64() stamps of waves 0 and 3 of every workgroup at the
stage boundaries; prints median / p10 / p90 of each stage's cycles."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deep-learning-based-rgba-image-compression-with-masked-window-based-attention_amd")
os.environ["RGBAC_LIB_PATH"] = os.path.join(PKG, "rgbac", "librgbac_ruprof.so")
sys.path.insert(0, PKG)
import numpy as np   # noqa: E402
import torch         # noqa: E402

NAMES = ["s1 load+mfma", "s1 epilogue", "barrier1", "s2 mfma", "s2 epilogue", "barrier2",
         "s3 mfma+epi"]


def main():
    from rgbac import _lib, runtime as rt
    from rgbac.layers.Masked_Attention import ResidualUnit, run_residual_units_fused
    dev = torch.device("cuda:0")
    B, H = 8, 64
    us = [ResidualUnit(192).to(dev) for _ in range(2)]
    xs = [rt.to_nhwc(torch.randn((B, 192, H, H), device=dev), torch.bfloat16) for _ in range(2)]
    with torch.no_grad():
        for _ in range(5):
            run_residual_units_fused(list(zip(us, xs)))
        torch.cuda.synchronize()
    nblk = B * (H // 8) * (H // 16)
    buf = (ctypes.c_ulonglong * (nblk * 18))()
    assert _lib.load().rgbac_debug_ru_times(buf, nblk) == 0
    a = np.frombuffer(buf, dtype=np.uint64).astype(np.int64)
    t = a[:nblk * 16].reshape(nblk, 2, 8)
    wc = a[nblk * 16:].reshape(nblk, 2)
    for w in range(2):
        d = np.diff(t[:, w, :], axis=1)
        print(f"wave {'0' if w == 0 else '3'}: total median {np.median(t[:, w, 7] - t[:, w, 0]):.0f} cycles")
        for k, name in enumerate(NAMES):
            print(f"  {name:14s} median {np.median(d[:, k]):8.0f}  p10 {np.percentile(d[:, k], 10):8.0f}"
                  f"  p90 {np.percentile(d[:, k], 90):8.0f}")
    t0 = wc[:, 0].min()
    st, en = (wc[:, 0] - t0) / 100.0, (wc[:, 1] - t0) / 100.0     # us (100 MHz wall clock)
    print(f"wall: kernel span {en.max():.1f} us; workgroup duration median {np.median(en - st):.1f} us; "
          f"start times p50 {np.median(st):.1f} p90 {np.percentile(st, 90):.1f} max {st.max():.1f} us")
    cyc = np.median(t[:, 0, 7] - t[:, 0, 0]) / np.median(en - st)
    print(f"shader clock ~ {cyc / 1e3:.2f} GHz")

if __name__ == "__main__":
    main()
