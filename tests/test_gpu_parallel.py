"""GPU, world size 2 (BASELINE config 5 in miniature): the real RGB codec + AdamClamp +
DataParallelTrainer across two rank processes sharing cuda:0, gradients exchanged by the
bucketed hook-launched all-reduce (gloo here: RCCL cannot put two ranks on one GPU; the
driver's 8-GPU run uses backend "nccl" = RCCL with the same code path).

Checked against one process running the concatenated batch (same noise):
  * the all-reduced gradient / world == the single-process gradient (fp32, 1e-4 norm-wise);
  * after clamp + Adam every rank holds bit-identical parameters;
  * in step 2 every bucket was launched from a hook during backward (overlapped).
The reference loss is a per-batch mean (masked MSE averaged over images, bpp over B*H*W),
so equal shards give exactly the global-batch gradient."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

B_RANK, H, W = 1, 64, 64


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(world):
    g = torch.Generator().manual_seed(21)
    B = B_RANK * world
    x = torch.round(torch.rand((B, 3, H, W), generator=g) * 255) / 255
    a = torch.ones((B, 1, H, W))
    a[1::2, :, :, : W // 2] = 0
    x = torch.where(a > 0, x, a)
    nz = torch.rand((B, 1, 1, 192), generator=g) - 0.5
    ny = torch.rand((B, 8, 8, 80), generator=g) - 0.5
    return x, a, nz, ny


def _net():
    from rgbac.models.AutoEncoderRGB_Journal import AutoEncoder
    torch.manual_seed(234)
    return AutoEncoder().train().cuda()


def _step(net, trainer, x, a, nz, ny):
    from rgbac.layers.SupplyMask import mask_pyramid
    _, me = mask_pyramid(a, 4)
    out = net(x, a, a, *me, noise_z=nz, noise_y=ny)
    trainer.step(4096.0 * out[1] + out[2])


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "deep-learning-based-rgba-image-compression-with-"
                                             "masked-window-based-attention_amd")]
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rgbac.optim import AdamClamp
        from rgbac.parallel import DataParallelTrainer
        net = _net()
        opt = AdamClamp(net.parameters(), lr=1e-4)
        tr = DataParallelTrainer(net, opt, bucket_bytes=4 << 20)
        x, a, nz, ny = _batch(world)
        sl = slice(rank * B_RANK, (rank + 1) * B_RANK)
        args = [t[sl].cuda() for t in (x, a, nz, ny)]
        # step 1, with the optimizer's update held back to read the reduced gradient
        real_step = opt.step
        opt.step = lambda: None
        _step(net, tr, *args)
        grad1 = (opt.flat_grad * opt.grad_scale).cpu()
        opt.step = real_step
        opt.step()
        tail = tr.buckets.tail
        # step 2: quiet parameters in the tail bucket, the rest launched during backward
        opt.zero_grad()
        tr.buckets.begin()
        from rgbac.layers.SupplyMask import mask_pyramid
        _, me = mask_pyramid(args[1], 4)
        out = net(args[0], args[1], args[1], *me, noise_z=args[2], noise_y=args[3])
        (4096.0 * out[1] + out[2]).backward()
        launched = tr.buckets.launched_in_backward()
        nb = len(tr.buckets.buckets)
        opt.grad_scale = tr.buckets.finish()
        opt.step()
        torch.cuda.synchronize()
        # numpy, not torch tensors: a torch CPU tensor travels as a shared-memory handle
        # served by this process, which exits right after
        q.put((rank, grad1.numpy(), opt.flat.cpu().numpy(), tail, launched, nb))
    finally:
        dist.destroy_process_group()


def test_dp_world2_matches_single_process(device):
    from rgbac.optim import AdamClamp
    from rgbac.parallel import DataParallelTrainer
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    env_keep = os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert env_keep == os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")
    # single process on the concatenated batch, same noise
    net = _net()
    opt = AdamClamp(net.parameters(), lr=1e-4)
    tr = DataParallelTrainer(net, opt)
    x, a, nz, ny = [t.cuda() for t in _batch(world)]
    real_step = opt.step
    opt.step = lambda: None
    _step(net, tr, x, a, nz, ny)
    want = opt.flat_grad.cpu().clone()
    opt.step = real_step
    (_, g0, p0, tail0, l0, nb0), (_, g1, p1, _, _, _) = res
    g0, g1, p0, p1 = (torch.from_numpy(t) for t in (g0, g1, p0, p1))
    e = ((g0 - want).double().norm() / want.double().norm()).item()
    print("DP world 2: reduced-gradient rel err", e, "buckets", nb0, "launched in backward", l0)
    assert e < 1e-4, e
    assert torch.equal(g0, g1)                       # every rank reduced the same sum
    assert torch.equal(p0, p1)                       # replicas stay bit-identical
    # every bucket's all-reduce went out from a hook during backward: no parameter of the
    # codec is quiet (quantiles receives the medians' STE gradient, zero but accumulated,
    # :227-229) -- and had one been, it would sit in a tail bucket (tests/test_parallel.py)
    tail_n = 0 if tail0 is None else 1
    assert l0 == nb0 - tail_n, (l0, nb0, tail0)


def _nccl_world1_worker(q):
    """Child process: the plain 1-GPU step (no process group) vs DataParallelTrainer under a
    one-rank RCCL process group with the buckets forced on -- 2 eager steps, then the step
    captured in a HIP graph (the hook-launched RCCL all-reduces inside it) and replayed."""
    import faulthandler
    import sys
    # a hang shows up as this child's Python stacks on stderr (and ends it) before the
    # parent's queue timeout
    faulthandler.dump_traceback_later(120, exit=True)

    def say(msg):
        print(f"[dp nccl world 1] {msg}", file=sys.stderr, flush=True)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "deep-learning-based-rgba-image-compression-with-"
                                             "masked-window-based-attention_amd")]
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    say("child up")
    from bench import capture_train
    from rgbac import runtime as rt
    from rgbac.optim import AdamClamp
    from rgbac.parallel import DataParallelTrainer
    x, a, nz, ny = [t.cuda() for t in _batch(2)]
    out = {}
    with rt.fixed_tiles():
        net0 = _net()
        opt0 = AdamClamp(net0.parameters(), lr=1e-4).use_device_step()
        tr0 = DataParallelTrainer(net0, opt0)
        assert tr0.buckets is None
        ref = []
        for _ in range(6):
            _step(net0, tr0, x, a, nz, ny)
            ref.append(opt0.flat.clone())
        say("reference steps done")
        dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1,
                                device_id=dev)
        say("process group up")
        try:
            net1 = _net()
            opt1 = AdamClamp(net1.parameters(), lr=1e-4).use_device_step()
            tr1 = DataParallelTrainer(net1, opt1, bucket_bytes=4 << 20, force_buckets=True)
            assert tr1.buckets is not None
            assert tr1.buckets.comm is not None              # RCCL called directly
            _step(net1, tr1, x, a, nz, ny)                       # learning step
            out["launched1"] = tr1.buckets.launched_in_backward()
            say("learning step done")
            _step(net1, tr1, x, a, nz, ny)
            out["launched2"] = tr1.buckets.launched_in_backward()
            out["nb"] = len(tr1.buckets.buckets)
            out["tail"] = tr1.buckets.tail
            torch.cuda.synchronize()
            out["eq2"] = torch.equal(opt1.flat, ref[1])

            def step():
                _step(net1, tr1, x, a, nz, ny)
                return opt1.flat
            # capture_train: 2 warm steps (3, 4) on a side stream, capture, 2 replays (5, 6)
            say("eager DP steps done")
            run, graph, _ = capture_train(step, opt1, dev, False)
            say("captured and replayed")
            out["launched_capture"] = tr1.buckets.launched_in_backward()
            torch.cuda.synchronize()
            out["eq6"] = torch.equal(opt1.flat, ref[5])
            out["diff6"] = (opt1.flat - ref[5]).abs().max().item()
            run()
            torch.cuda.synchronize()
            out["moved7"] = not torch.equal(opt1.flat, ref[5])
            del run, graph
        finally:
            dist.destroy_process_group()
    q.put(out)


def test_dp_nccl_world1_buckets_bitexact(device):
    """the config-5 code path on RCCL -- buckets forced on at world 1 so
    the post-accumulate-grad hooks issue RCCL all-reduces (ncclAllReduce on the comm stream,
    rgbac.parallel.RcclComm) during backward (direct weight-gradient adds kept on: the same
    backward as the 1-GPU step), eager and captured in a HIP graph; the parameters equal the
    plain step's bit for bit (a one-rank SUM is the identity and the 1/world scale is 1)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_world1_worker, args=(q,))
    p.start()
    try:
        out = q.get(timeout=170)
    finally:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert p.exitcode == 0
    print("DP nccl world 1:", out)
    assert out["launched1"] == 0                         # learning step: all in finish()
    tail_n = 0 if out["tail"] is None else 1
    assert out["launched2"] == out["nb"] - tail_n > 1    # then from the hooks, in backward
    assert out["launched_capture"] == out["nb"] - tail_n
    assert out["eq2"], "eager DP step differs from the plain step"
    assert out["eq6"], out["diff6"]
    assert out["moved7"]
