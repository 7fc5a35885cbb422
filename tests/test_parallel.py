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
