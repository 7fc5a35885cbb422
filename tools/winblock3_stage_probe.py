"""Per-phase cycle breakdown of the head-pair window block (winblock_kernel, csrc/winblock.hip
built with -DRGBAC_WB_TIMING into rgbac/librgbac_wbprof.so: make -C <pkg>/csrc wbprof).
clock64() stamps of wave 0 of every workgroup: 0 start, 1 lists built, 2 panel + first x
landed, per window j (j = 0, 1, last): GEMM done, exchange barrier passed, attention (+ the
previous window's proj) done, end-of-window barrier passed; 15 loop end, 17 exit.
python tools/winblock3_stage_probe.py [--config 2|4]"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "deep-learning-based-rgba-image-compression-with-masked-window-based-attention_amd")
os.environ["RGBAC_LIB_PATH"] = os.path.join(PKG, "rgbac", "librgbac_wbprof.so")
sys.path[:0] = [ROOT, PKG]
import numpy as np   # noqa: E402
import torch         # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="2")
    args = ap.parse_args()
    from bench import synth_inputs
    from rgbac import _lib, runtime as rt
    from rgbac.layers.SupplyMask import mask_pyramid
    from rgbac.layers.masked_win_attention import WinBasedAttention
    assert _lib.LIB_PATH.endswith("librgbac_wbprof.so"), _lib.LIB_PATH
    B, S = {"2": (8, 256), "4": (4, 1024)}[args.config]
    torch.manual_seed(0)
    m = WinBasedAttention(192, 8, 8, 0).cuda().eval()
    _, a = synth_inputs(B, S, S)
    _, me = mask_pyramid(a.cuda(), 4)
    s = S // 4
    x = rt.to_nhwc(torch.randn((B, 192, s, s), device="cuda"), torch.bfloat16)
    with torch.no_grad():
        for _ in range(5):
            m.nhwc(x, me[1])
        torch.cuda.synchronize()
    nblk = 256
    buf = (ctypes.c_ulonglong * (nblk * 20))()
    assert _lib.load().rgbac_debug_wb_times(buf, nblk) == 0
    arr = np.frombuffer(buf, dtype=np.uint64).astype(np.int64)
    t = arr[:nblk * 18].reshape(nblk, 18)
    wc = arr[nblk * 18:].reshape(nblk, 2)
    names = {1: "lists", 2: "panel+x", 3: "p0 gemm", 4: "p0 B1", 5: "p0 attn", 6: "p0 B2",
             7: "p1 gemm", 8: "p1 B1", 9: "p1 attn", 10: "p1 B2",
             11: "pl gemm", 12: "pl B1", 13: "pl attn", 14: "pl B2", 15: "loop end",
             17: "exit"}
    tot = t[:, 17] - t[:, 0]
    print(f"config {args.config}: total median {np.median(tot):.0f} cycles, max {tot.max()}")
    prev = 0
    for k in sorted(names):
        d = t[:, k] - t[:, prev]
        ok = t[:, k] > 0
        if ok.sum() == 0:
            continue
        print(f"  {names[k]:>14}: median {np.median(d[ok]):8.0f}  p90 {np.percentile(d[ok], 90):8.0f}")
        prev = k
    t0 = wc[:, 0].min()
    st, en = (wc[:, 0] - t0) / 100.0, (wc[:, 1] - t0) / 100.0
    print(f"wall: span {en.max():.1f} us; workgroup duration median {np.median(en - st):.1f} us; "
          f"start p50 {np.median(st):.1f} p90 {np.percentile(st, 90):.1f} max {st.max():.1f} us")
    print(f"shader clock ~ {np.median(tot) / np.median(en - st) / 1e3:.2f} GHz")


if __name__ == "__main__":
    main()
