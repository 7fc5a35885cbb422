"""Per-kernel floor in HIP-graph replay: N back-to-back tiny kernels (torch elementwise on
a 1-element / 1 MB tensor) captured in one graph; reports microseconds per kernel."""
import torch


def floor(numel, n=200, reps=20):
    x = torch.zeros(numel, device="cuda")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            x.add_(1.0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(n):
            x.add_(1.0)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps / n * 1e3


if __name__ == "__main__":
    for numel in (1, 1 << 18, 1 << 22):
        print(f"{numel * 4 / 1e6:8.3f} MB tensor: {floor(numel):6.2f} us per kernel in graph replay")
