"""CPU (gloo, world_size 2): the data-parallel gradient exchange of rgbac/parallel.py.

Each rank back-propagates a different shard through the same toy model whose
gradients live in one flat buffer (the AdamClamp layout).  The first step is the
learning step (notification counts per parameter, every bucket reduced in
finish()); from the second step on, with small buckets, several all-reduces are
launched from the gradient-landed notifications during backward.  After finish()
every rank holds the SUM of both ranks' gradients (the 1/world mean is returned
for the optimizer kernel)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(6, 16), torch.nn.GELU(), torch.nn.Linear(16, 5),
                               torch.nn.GELU(), torch.nn.Linear(5, 3))


def _shard_grads(rank):
    m = _model()
    x = torch.randn((4, 6), generator=torch.Generator().manual_seed(100 + rank))
    m(x).pow(2).sum().backward()
    return torch.cat([p.grad.reshape(-1) for p in m.parameters()])


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rgbac.parallel import GradBuckets
        m = _model()
        params = list(m.parameters())
        flat = torch.zeros(sum(p.numel() for p in params))
        off = 0
        for p in params:
            p.grad = flat[off:off + p.numel()].view_as(p)
            off += p.numel()
        gb = GradBuckets(params, flat, bucket_bytes=64)
        assert len(gb.buckets) > 2
        want = sum(_shard_grads(r) for r in range(world))
        res = []
        for step in range(2):
            flat.zero_()
            x = torch.randn((4, 6), generator=torch.Generator().manual_seed(100 + rank))
            gb.begin()
            m(x).pow(2).sum().backward()
            launched_in_backward = gb.launched_in_backward()
            scale = gb.finish()
            ok = torch.allclose(flat, want, rtol=1e-6, atol=1e-6)
            res.append((ok, scale, launched_in_backward, len(gb.buckets)))
        out.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_grad_buckets_allreduce_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, steps in res:
        (ok0, sc0, l0, nb0), (ok1, sc1, l1, nb1) = steps
        assert ok0 and ok1, rank
        assert sc0 == sc1 == 0.5
        assert l0 == 0                 # learning step: every bucket reduced in finish()
        assert l1 == nb1               # then every bucket goes out during backward


def _quiet_worker(rank, world, port, out):
    """A parameter without a gradient (like EntropyBottleneck.quantiles) is found in the
    learning step; afterwards it sits in the tail bucket and every other bucket launches
    from a hook during backward.  Sums stay exact in both steps."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rgbac.parallel import GradBuckets
        m = _model()
        quiet = torch.nn.Parameter(torch.zeros(7))
        params = list(m.parameters())
        params.insert(2, quiet)                    # in the middle of the flat buffer
        flat = torch.zeros(sum(p.numel() for p in params))
        off = 0
        for p in params:
            p.grad = flat[off:off + p.numel()].view_as(p)
            off += p.numel()
        gb = GradBuckets(params, flat, bucket_bytes=64)
        res = []
        for step in range(2):
            flat.zero_()
            x = torch.randn((4, 6), generator=torch.Generator().manual_seed(100 + rank))
            gb.begin()
            m(x).pow(2).sum().backward()
            launched = gb.launched_in_backward()
            nb, tail = len(gb.buckets), gb.tail
            gb.finish()
            want = sum(_shard_grads(r) for r in range(world))
            q0 = sum(p.numel() for p in params[:2])
            got = torch.cat([flat[:q0], flat[q0 + quiet.numel():]])
            ok = torch.allclose(got, want, rtol=1e-6, atol=1e-6) and \
                bool((flat[q0:q0 + quiet.numel()] == 0).all())
            res.append((ok, launched, nb, tail))
        out.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_grad_buckets_quiet_param_moves_to_tail():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_quiet_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, steps in res:
        (ok0, l0, nb0, tail0), (ok1, l1, nb1, tail1) = steps
        assert ok0 and ok1, rank
        assert tail0 is None and l0 == 0       # step 1: learning, all reduced in finish()
        assert tail1 == nb1 - 1 and l1 == nb1 - 1   # step 2: all but the tail from hooks


class _DirectAdd(torch.autograd.Function):
    """y = x * w (elementwise) whose backward ADDS dL/dw straight into w.grad and returns
    None for w -- the shape of rgbac.autograd.ConvFn's direct weight-gradient path."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return x * w

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        w.grad.add_((g * x).sum(0))
        return g * w, None


def _direct_worker(rank, world, port, out):
    """One parameter reaches its gradient twice through the direct-add path (two uses), one
    once, one through autograd: each hook fires once per step (autograd runs a parameter's
    AccumulateGrad node after its last use even when every use returned None), so the
    buckets launch only once every use has landed, and the sums equal the autograd
    reference."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rgbac.parallel import GradBuckets
        torch.manual_seed(3)
        w2 = torch.nn.Parameter(torch.randn(5))      # used twice, direct
        w1 = torch.nn.Parameter(torch.randn(5))      # used once, direct
        lin = torch.nn.Linear(5, 5)                  # autograd (post-accumulate hook)
        params = [w2, w1, lin.weight, lin.bias]
        flat = torch.zeros(sum(p.numel() for p in params))
        off = 0
        for p in params:
            p.grad = flat[off:off + p.numel()].view_as(p)
            off += p.numel()

        def loss_of(x, direct=True):
            f = _DirectAdd.apply if direct else (lambda a, b: a * b)
            h = f(lin(f(x, w2)), w1)
            return f(h, w2).pow(2).sum()

        def ref():
            tot = None
            for r in range(world):
                xr = torch.randn((3, 5), generator=torch.Generator().manual_seed(7 + r))
                ps = [q.detach().clone().requires_grad_(True) for q in params]
                ws, wo, lw, lb = ps
                h = torch.nn.functional.linear(xr * ws, lw, lb) * wo
                (h * ws).pow(2).sum().backward()
                g = torch.cat([q.grad.reshape(-1) for q in ps])
                tot = g if tot is None else tot + g
            return tot
        want = ref()
        gb = GradBuckets(params, flat, bucket_bytes=16)   # 4 floats: one bucket per param
        x = torch.randn((3, 5), generator=torch.Generator().manual_seed(7 + rank))
        res = []
        for step in range(2):
            flat.zero_()
            gb.begin()
            loss_of(x).backward()
            launched = gb.launched_in_backward()
            gb.finish()
            res.append((torch.allclose(flat, want, rtol=1e-5, atol=1e-5), launched,
                        len(gb.buckets)))
        out.put((rank, res, list(gb.expect)))
        gb.remove()
    finally:
        dist.destroy_process_group()


def test_grad_buckets_direct_notifications_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_direct_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, steps, expect in res:
        assert expect == [1, 1, 1, 1], expect
        (ok0, l0, _), (ok1, l1, nb1) = steps
        assert ok0 and ok1, rank
        assert l0 == 0 and l1 == nb1
