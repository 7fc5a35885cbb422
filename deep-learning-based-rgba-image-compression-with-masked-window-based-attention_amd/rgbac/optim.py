"""Optimizer of the training step (trainRGB.py:187-198):

    optimizer.zero_grad(); rd_loss.backward()
    clip_gradient(optimizer, 5)        # param.grad.data.clamp_(-5, 5)
    optimizer.step()                   # torch.optim.Adam(net.parameters(), lr)

``AdamClamp`` is the drop-in for that pair: the parameters are re-homed into ONE
flat fp32 buffer (each ``p.data`` becomes a view), their gradients into another
(``p.grad`` views that autograd accumulates into in place), and one
rgbac_adam_clamp launch clamps every gradient element and applies the Adam update
with torch.optim.Adam's exact formula.  The flat gradient buffer is also what
the data-parallel all-reduce works on (rgbac/parallel.py).
"""
import torch

from . import _lib
from . import runtime as rt


class AdamClamp:
    def __init__(self, params, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, clip=5.0):
        params = [p for p in params]
        if not params:
            raise ValueError("no parameters")
        dev = params[0].device
        if dev.type != "cuda":
            raise RuntimeError("rgbac.optim.AdamClamp runs on the GPU (HIP) only")
        for p in params:
            if p.dtype != torch.float32 or p.device != dev:
                raise ValueError("AdamClamp needs fp32 parameters on one device")
        self.params = params
        self.defaults = dict(lr=lr, betas=tuple(betas), eps=eps, clip=clip)
        self.param_groups = [dict(params=params, lr=lr, betas=tuple(betas), eps=eps)]
        n = sum(p.numel() for p in params)
        self.numel = n
        self.flat = torch.empty(n, dtype=torch.float32, device=dev)
        self.flat_grad = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, device=dev)
        self.offsets = []
        off = 0
        with torch.no_grad():
            for p in params:
                k = p.numel()
                self.flat[off:off + k].copy_(p.detach().reshape(-1))
                p.data = self.flat[off:off + k].view_as(p)
                self.offsets.append((off, k))
                off += k
        self._attach_grads()
        self.step_count = 0
        self.grad_scale = 1.0
        self.step_dev = None           # device step counter (graph-replayable step)

    def use_device_step(self):
        """Keep the step count in device memory from now on, so a training step captured in
        a HIP graph replays the Adam bias corrections correctly (rgbac_adam_clamp_dstep)."""
        if self.step_dev is None:
            self.step_dev = torch.tensor([self.step_count], dtype=torch.int64,
                                         device=self.flat.device)
        return self

    def _sync_step(self):
        if self.step_dev is not None:
            self.step_count = int(self.step_dev.item())

    def _attach_grads(self):
        for p, (off, k) in zip(self.params, self.offsets):
            view = self.flat_grad[off:off + k].view_as(p)
            if p.grad is None:
                p.grad = view
            elif p.grad.data_ptr() != view.data_ptr():
                view.copy_(p.grad)
                p.grad = view

    def zero_grad(self, set_to_none=False):
        """Zeros the flat gradient buffer in place (``set_to_none`` is ignored: the
        views must survive so autograd keeps accumulating into the flat buffer)."""
        self.flat_grad.zero_()
        self._attach_grads()

    def state_dict(self):
        self._sync_step()
        return dict(step=self.step_count, exp_avg=self.exp_avg, exp_avg_sq=self.exp_avg_sq,
                    param_groups=[{k: v for k, v in g.items() if k != "params"}
                                  for g in self.param_groups])

    def load_state_dict(self, sd):
        self.step_count = int(sd["step"])
        if self.step_dev is not None:
            self.step_dev.fill_(self.step_count)
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        for g, s in zip(self.param_groups, sd["param_groups"]):
            g.update(s)

    def step(self):
        self._attach_grads()           # adopt gradients someone replaced / set to None
        self.step_count += 1
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        if self.step_dev is not None:
            _lib.call("rgbac_adam_clamp_dstep", self.numel, self.flat.data_ptr(),
                      self.flat_grad.data_ptr(), self.exp_avg.data_ptr(),
                      self.exp_avg_sq.data_ptr(), float(g["lr"]), float(b1), float(b2),
                      float(g["eps"]), self.step_dev.data_ptr(),
                      float(self.defaults["clip"] or 0.0), float(self.grad_scale),
                      _lib.stream_ptr(self.flat.device))
            rt.PARAM_GEN += 1
            return
        _lib.call("rgbac_adam_clamp", self.numel, self.flat.data_ptr(), self.flat_grad.data_ptr(),
                  self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(), float(g["lr"]), float(b1),
                  float(b2), float(g["eps"]), self.step_count, float(self.defaults["clip"] or 0.0),
                  float(self.grad_scale), _lib.stream_ptr(self.flat.device))
        rt.PARAM_GEN += 1
