"""CPU (gloo, world_size 2): the data-parallel gradient exchange of rgbac/parallel.py.

Each rank back-propagates a different shard through the same toy model whose
gradients live in one flat buffer (the AdamClamp layout); with small buckets
several all-reduces are launched from the post-accumulate hooks during
backward.  After finish() every rank holds the SUM of both ranks' gradients
(the 1/world mean is returned for the optimizer kernel)."""
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
        x = torch.randn((4, 6), generator=torch.Generator().manual_seed(100 + rank))
        gb.begin()
        m(x).pow(2).sum().backward()
        launched_in_backward = sum(w is not None for w in gb.works)
        scale = gb.finish()
        want = sum(_shard_grads(r) for r in range(world))
        ok = torch.allclose(flat, want, rtol=1e-6, atol=1e-6)
        out.put((rank, ok, scale, launched_in_backward, len(gb.buckets)))
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
    for rank, ok, scale, launched, nb in res:
        assert ok, rank
        assert scale == 0.5
        assert launched == nb          # every bucket went out from a hook during backward


def _quiet_worker(rank, world, port, out):
    """A parameter without a gradient (like EntropyBottleneck.quantiles) holds its bucket
    back only in the first step; afterwards it sits in the tail bucket and every other
    bucket launches from a hook during backward.  Sums stay exact in both steps."""
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
            launched = sum(w is not None for w in gb.works)
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
        assert tail0 is None and l0 < nb0      # step 1: the quiet param's bucket waits
        assert tail1 == nb1 - 1 and l1 == nb1 - 1   # step 2: all but the tail from hooks
