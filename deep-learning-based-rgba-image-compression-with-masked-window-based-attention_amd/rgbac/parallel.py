"""Data-parallel training (trainRGB.py:178-198 across ranks).

One process per GPU (torchrun); every rank runs the full model on its shard of
the global batch.  The only exchange is the gradient all-reduce: the flat fp32
gradient buffer of rgbac.optim.AdamClamp is cut into ~25 MB buckets in REVERSE
parameter order (the order backward produces them), and each bucket's
all-reduce (backend "nccl" = RCCL over xGMI) is launched from the parameters'
post-accumulate-grad hooks as soon as its last gradient lands -- overlapped with
the rest of backward on RCCL's own stream.  ``finish()`` waits for all buckets
and hands the 1/world mean to the optimizer kernel, which applies it before the
per-element clamp (the reference clamps the global-batch gradient).
"""
import torch
import torch.distributed as dist


class GradBuckets:
    """Bucketed all-reduce of the flat gradient buffer, launched from post-accumulate-grad
    hooks.  A bucket is a set of parameters whose flat ranges are all-reduced (one collective
    per contiguous run) as soon as the last of them has accumulated its gradient.

    Parameters that receive no gradient in a step (EntropyBottleneck.quantiles: only the aux
    loss, which trainRGB.py never back-propagates, reaches it) would hold their bucket back
    until ``finish()``, losing its overlap with backward.  After the first step the buckets
    are re-cut: such parameters move to a tail bucket reduced in ``finish()`` (zeros unless
    they do receive a gradient later, which stays correct since the tail always waits for
    the end of backward)."""

    def __init__(self, params, flat_grad, bucket_bytes=25 << 20, group=None):
        self.params = list(params)
        self.flat = flat_grad
        self.group = group
        self.world = dist.get_world_size(group)
        # param i occupies [off_i, off_i + n_i) of the flat buffer (AdamClamp layout)
        self.offs, off = [], 0
        for p in self.params:
            self.offs.append((off, p.numel()))
            off += p.numel()
        assert off == flat_grad.numel()
        self.per = max(1, bucket_bytes // flat_grad.element_size())
        self._cut(list(range(len(self.params) - 1, -1, -1)), [])
        self.fired = [False] * len(self.params)
        self.learned = False
        self.active = False
        self.hooks = [p.register_post_accumulate_grad_hook(self._hook(i))
                      for i, p in enumerate(self.params)]

    def _runs(self, idx):
        """Contiguous flat ranges covering params ``idx``."""
        rs = sorted(self.offs[i] for i in idx)
        out = []
        for lo, n in rs:
            if out and out[-1][1] == lo:
                out[-1][1] = lo + n
            else:
                out.append([lo, lo + n])
        return [tuple(r) for r in out]

    def _cut(self, order, tail):
        """Buckets of ~per elements over ``order`` (backward order), plus a tail bucket."""
        self.buckets = []                  # [ranges, [param idx]]
        cur, size = [], 0
        for i in order:
            cur.append(i)
            size += self.offs[i][1]
            if size >= self.per:
                self.buckets.append([self._runs(cur), cur])
                cur, size = [], 0
        if cur:
            self.buckets.append([self._runs(cur), cur])
        self.tail = None
        if tail:
            self.tail = len(self.buckets)
            self.buckets.append([self._runs(tail), list(tail)])
        self.owner = {}
        for b, (_, idx) in enumerate(self.buckets):
            for i in idx:
                self.owner[i] = b
        self.pending = [0] * len(self.buckets)
        self.works = [None] * len(self.buckets)

    def _hook(self, i):
        def fn(_p):
            if not self.active:
                return
            self.fired[i] = True
            b = self.owner[i]
            if b == self.tail:
                return
            self.pending[b] -= 1
            if self.pending[b] == 0:
                self._launch(b)
        return fn

    def _launch(self, b):
        self.works[b] = [dist.all_reduce(self.flat[lo:hi], op=dist.ReduceOp.SUM,
                                         group=self.group, async_op=True)
                         for lo, hi in self.buckets[b][0]]

    def begin(self):
        """Call before loss.backward()."""
        for b, (_, idx) in enumerate(self.buckets):
            self.pending[b] = len(idx)
            self.works[b] = None
        self.fired = [False] * len(self.params)
        self.active = True

    def finish(self):
        """Call after loss.backward(): all-reduce what backward did not launch (parameters
        without a gradient this step), wait for every bucket; returns 1/world."""
        self.active = False
        for b in range(len(self.buckets)):
            if self.works[b] is None:
                self._launch(b)
        for ws in self.works:
            for w in ws:
                w.wait()
        if not self.learned and any(self.fired):
            self.learned = True
            # every rank must cut the same buckets (else ranks would issue all-reduces of
            # different ranges and counts): a parameter counts as fired if it fired anywhere
            fired = torch.tensor(self.fired, dtype=torch.int32, device=self.flat.device)
            dist.all_reduce(fired, op=dist.ReduceOp.MAX, group=self.group)
            self.fired = [bool(f) for f in fired.tolist()]
            quiet = [i for i, f in enumerate(self.fired) if not f]
            if quiet:
                order = [i for i in range(len(self.params) - 1, -1, -1) if self.fired[i]]
                self._cut(order, quiet)
        return 1.0 / self.world

    def remove(self):
        for h in self.hooks:
            h.remove()


class DataParallelTrainer:
    """net + AdamClamp + GradBuckets: ``step(loss)`` = backward with overlapped all-reduce,
    clamp, Adam (one launch)."""

    def __init__(self, net, optimizer, bucket_bytes=25 << 20):
        self.net, self.opt = net, optimizer
        self.buckets = None
        # optional exposed-communication probe: a list receiving (end of backward, gradients
        # reduced) event pairs recorded on the compute stream -- the all-reduce time backward
        # did not hide
        self.comm_events = None
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            self.buckets = GradBuckets(optimizer.params, optimizer.flat_grad, bucket_bytes)
            # the bucket all-reduces are launched from post-accumulate-grad hooks: keep
            # autograd's per-parameter accumulation (no in-place weight-gradient adds)
            from . import autograd as ag
            ag.DIRECT_GRAD[0] = False

    def step(self, loss):
        self.opt.zero_grad()
        if self.buckets is not None:
            self.buckets.begin()
        loss.backward()
        if self.buckets is not None:
            ev = None
            if self.comm_events is not None:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
            self.opt.grad_scale = self.buckets.finish()
            if ev is not None:
                ev[1].record()
                self.comm_events.append(ev)
        self.opt.step()
