"""Which Python lines of the training step dispatch ATen kernels (the glue around the HIP
kernels): one eager bf16 config-3 step under torch.profiler (CPU activity, stacks), ATen ops
that launch device work grouped by op and by the innermost rgbac / bench frame.
python tools/aten_origins.py [--batch 16]"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-learning-based-rgba-image-compression-with-"
                                         "masked-window-based-attention_amd")]
import torch  # noqa: E402

from bench import synth_inputs  # noqa: E402

KERNEL_OPS = ("aten::add", "aten::add_", "aten::fill_", "aten::zero_", "aten::copy_",
              "aten::mul", "aten::mul_", "aten::sub", "aten::rand", "aten::uniform_",
              "aten::softplus", "aten::tanh", "aten::sigmoid", "aten::clamp", "aten::where",
              "aten::max", "aten::maximum", "aten::pow", "aten::div", "aten::neg", "aten::sum",
              "aten::cat", "aten::index", "aten::mean", "aten::log", "aten::exp", "aten::abs",
              "aten::sign", "aten::lt", "aten::ge", "aten::bitwise_or", "aten::masked_fill")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    args = ap.parse_args()
    from rgbac.layers.SupplyMask import mask_pyramid
    from rgbac.models.AutoEncoderRGB_Journal import AutoEncoder
    from rgbac.optim import AdamClamp
    from rgbac.parallel import DataParallelTrainer
    dev = torch.device("cuda:0")
    torch.manual_seed(234)
    net = AutoEncoder().train().to(dev).set_compute_dtype(torch.bfloat16)
    opt = AdamClamp(net.parameters(), lr=1e-4, clip=5.0)
    trainer = DataParallelTrainer(net, opt)
    x, a = synth_inputs(args.batch, 256, 256)
    x, a = x.to(dev), a.to(dev)
    _, me = mask_pyramid(a, 4)

    def step():
        out = net(x, a, a, *me)
        trainer.step(4096.0 * out[1] + out[2])

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    import traceback
    from torch.utils._python_dispatch import TorchDispatchMode

    by_site = collections.Counter()
    by_op = collections.Counter()

    class Spy(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args_=(), kwargs=None):
            name = str(func.overloadpacket)
            out = func(*args_, **(kwargs or {}))
            dev_args = [t for t in list(args_) + list((kwargs or {}).values())
                        if isinstance(t, torch.Tensor) and t.is_cuda]
            if dev_args and not any(k in name for k in ("view", "detach", "empty", "as_strided",
                                                          "_unsafe", "alias", "t.default",
                                                          "reshape", "expand", "select",
                                                          "slice", "permute", "unsqueeze",
                                                          "squeeze", "transpose", "_to_copy")):
                site = "?"
                for fr in reversed(traceback.extract_stack()[:-1]):
                    f = fr.filename
                    if ("rgbac" in f or "bench.py" in f) and "aten_origins" not in f:
                        site = f"{os.path.basename(f)}:{fr.lineno} {fr.name}"
                        break
                if site == "?":              # the autograd engine's own ops: name the operand
                    t0 = dev_args[0]
                    site = f"? {tuple(t0.shape)} {str(t0.dtype).replace('torch.', '')}"
                by_site[(name, site)] += 1
                by_op[name] += 1
            return out

    with Spy():
        step()
        torch.cuda.synchronize()
    print("by op:", dict(by_op.most_common()))
    for (op, site), n in by_site.most_common(80):
        print(f"{n:4d}  {op:28s} {site}")


if __name__ == "__main__":
    main()
