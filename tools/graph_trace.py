"""Forward HIP-graph replays delimited by a spin kernel, for rocprofv3 --kernel-trace.

  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gt -o t -- python tools/graph_trace.py
  python tools/graph_trace.py --analyze gpurun_out/gt/t_kernel_trace.csv

The analysis takes the dispatches between consecutive spin kernels (one replay each) and reports
per-position mean durations, the sum of kernel durations and the replay span (gaps included)."""
import argparse
import csv
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-learning-based-rgba-image-compression-with-masked-window-based-attention_amd")]


def run(args):
    import torch
    import bench
    from rgbac.layers.SupplyMask import mask_pyramid
    from rgbac.models.AutoEncoderRGB_Journal import AutoEncoder
    dev = torch.device("cuda:0")
    net = bench.rgb_net().to(dev).set_compute_dtype(torch.bfloat16)   # the bench's codec
    x, a = bench.synth_inputs(args.batch, args.size, args.size, seed=0)
    x, a = x.to(dev), a.to(dev)
    _, me = mask_pyramid(a, 4)

    def step():
        with torch.no_grad():
            return net(x, a, a, *me)
    from rgbac import runtime as rt
    cache = os.environ.get("RGBAC_TUNE_CACHE") or os.path.join(
        ROOT, "profiles", f"tune_fwd_bf16_b{args.batch}_{args.size}.json")
    if os.path.exists(cache):
        rt.load_tune_cache(cache)        # no autotuning dispatches in the trace
    step()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    for _ in range(args.reps):
        torch.cuda._sleep(2_000_000)
        g.replay()
    torch.cuda._sleep(2_000_000)
    torch.cuda.synchronize()
    print("done", flush=True)


def analyze(path):
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if "sleep" in r[2].lower() or "spin" in r[2].lower()]
    reps = []
    for a, b in zip(marks, marks[1:]):
        seg = rows[a + 1:b]
        if seg:
            reps.append(seg)
    n = min(len(r) for r in reps)
    reps = [r for r in reps if len(r) == n]
    dur = defaultdict(float)
    span = sum(r[-1][1] - r[0][0] for r in reps) / len(reps)
    busy = sum(sum(e - s for s, e, _ in r) for r in reps) / len(reps)
    print(f"replays {len(reps)}  kernels/replay {n}  span {span / 1e3:.1f} us  "
          f"sum of kernel durations {busy / 1e3:.1f} us  gaps {(span - busy) / 1e3:.1f} us")
    by_name = defaultdict(lambda: [0, 0.0])
    for i in range(n):
        d = sum(r[i][1] - r[i][0] for r in reps) / len(reps)
        gap = sum(r[i][0] - r[i - 1][1] for r in reps) / len(reps) if i else 0.0
        nm = reps[0][i][2]
        short = nm.split("(")[0].replace("void ", "").replace("rgbac::", "")[:70]
        print(f"{i:4d} {d / 1e3:9.2f} us  gap {gap / 1e3:6.2f}  {short}")
        by_name[short][0] += 1
        by_name[short][1] += d
    print("\nby kernel:")
    for k, (c, d) in sorted(by_name.items(), key=lambda kv: -kv[1][1]):
        print(f"  {d / 1e3:9.1f} us  {100 * d / busy:5.1f}%  n={c:3d}  {k}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--analyze", default=None)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    if a.analyze:
        analyze(a.analyze)
    else:
        run(a)
