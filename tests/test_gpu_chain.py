"""The slice-chain engine (csrc/chain.hip, rgbac.runtime.Chain): the channel-conditional slice
loop of both codecs (models/AutoEncoderRGB_Journal.py:240-266,
AutoEncoderMask_Journal.py:268-298) as ONE persistent launch with in-launch dependency
counters, against the same stages launched one per kernel.  Same arithmetic in the same order:
x_hat, bpp and mse must be bit-identical, and the launch's give-up word must stay 0 (no
dependency wait timed out).  Bench inputs (bench.synth_inputs: every alpha pattern) and the
bench's codec (non-zero latent symbols)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(net, x, a, me, chain):
    from rgbac import runtime as rt
    prev = rt.CHAIN
    rt.CHAIN = chain
    try:
        with torch.no_grad():
            out = net(x, a, a, *me)
        torch.cuda.synchronize()
    finally:
        rt.CHAIN = prev
    err = None
    if chain:
        err = int(rt.LAST_CHAIN[0][-1].item())
    return [o.detach().clone() for o in out[:3]], err


def _check(net, B, S, device):
    import bench
    from rgbac.layers.SupplyMask import mask_pyramid
    x, a = bench.synth_inputs(B, S, S, seed=3)
    x, a = x.to(device), a.to(device)
    _, me = mask_pyramid(a, 4)
    ref, _ = _run(net, x, a, me, False)
    got, err = _run(net, x, a, me, True)
    assert err == 0, "a chain dependency wait gave up"
    assert torch.equal(got[0], ref[0]), (got[0] - ref[0]).abs().max().item()
    assert got[1].item() == ref[1].item() and got[2].item() == ref[2].item(), \
        (got[1].item(), ref[1].item(), got[2].item(), ref[2].item())


@pytest.mark.parametrize("B,S", [(2, 128), (8, 256), (1, 256)])
def test_chain_rgb_bitexact(device, B, S):
    import bench
    net = bench.rgb_net().to(device).set_compute_dtype(torch.bfloat16)
    _check(net, B, S, device)


def test_chain_rgb_graph_replay(device):
    """The chain captured in a HIP graph (descriptor table uploaded by a memcpy node, counters
    reset by a memset node) and replayed twice: identical to the eager per-stage forward."""
    import bench
    from rgbac import runtime as rt
    from rgbac.layers.SupplyMask import mask_pyramid
    net = bench.rgb_net().to(device).set_compute_dtype(torch.bfloat16)
    x, a = bench.synth_inputs(4, 128, 128, seed=5)
    x, a = x.to(device), a.to(device)
    _, me = mask_pyramid(a, 4)
    ref, _ = _run(net, x, a, me, False)
    assert rt.CHAIN
    with torch.no_grad():
        net(x, a, a, *me)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            net(x, a, a, *me)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = net(x, a, a, *me)
        for _ in range(2):
            g.replay()
            torch.cuda.synchronize()
            assert int(rt.LAST_CHAIN[0][-1].item()) == 0
            assert torch.equal(out[0], ref[0])
            assert out[2].item() == ref[2].item()


def test_chain_alpha_bitexact(device):
    import bench
    from rgbac.layers.SupplyMask import mask_pyramid
    net = bench.mask_net().to(device).set_compute_dtype(torch.bfloat16)
    x, a = bench.synth_inputs(2, 256, 256, seed=7)
    a = a.to(device)
    _, me = mask_pyramid(a, 4)
    from rgbac import runtime as rt

    def run(chain):
        prev = rt.CHAIN
        rt.CHAIN = chain
        try:
            with torch.no_grad():
                out = net(a, *me)
            torch.cuda.synchronize()
        finally:
            rt.CHAIN = prev
        return [o.detach().clone() for o in out[:3]]
    ref, got = run(False), run(True)
    assert int(rt.LAST_CHAIN[0][-1].item()) == 0
    assert torch.equal(got[0], ref[0])
    assert got[2].item() == ref[2].item()


def test_chain_stage_outputs_bitexact(device):
    """Every stage output of one recorded slice loop (the same Prepared records and buffers):
    chain launch vs one launch per stage -- localises a mismatch to its stage and group."""
    import bench
    from rgbac import runtime as rt
    from rgbac.layers.SupplyMask import mask_pyramid
    from rgbac.models import _latent
    net = bench.rgb_net().to(device).set_compute_dtype(torch.bfloat16)
    x, a = bench.synth_inputs(2, 128, 128, seed=3)
    x, a = x.to(device), a.to(device)
    _, me = mask_pyramid(a, 4)
    rec = {}
    orig = _latent._slice_waves

    def spy(*args):
        with rt.chain_recording() as ch:
            orig(*args)
        rec["ch"], rec["ypart"] = ch, args[18]
    prev = rt.CHAIN
    rt.CHAIN = False
    _latent._slice_waves = spy
    try:
        with torch.no_grad():
            net(x, a, a, *me)
    finally:
        _latent._slice_waves = orig
        rt.CHAIN = prev
    ch, ypart = rec["ch"], rec["ypart"]
    # the written channels of every stage output (an output may be a channel slice of YH)
    views = [pr.out.t[..., pr.a.out_coff:pr.a.out_coff + (pr.pk.cout // 2 if pr.a.act == rt.ACT["gauss"]
                                                          else pr.pk.cout)]
             for st in ch.stages for pr in st]
    for v in views:
        v.zero_()
    torch.cuda.synchronize()
    ch.launch_each()
    torch.cuda.synchronize()
    ref = [v.clone() for v in views]
    ref_bits = ypart.clone()
    for v in views:
        v.fill_(float("nan"))
    ypart.zero_()
    assert ch.run()
    torch.cuda.synchronize()
    assert int(rt.LAST_CHAIN[0][-1].item()) == 0
    k = 0
    for si, st in enumerate(ch.stages):
        for gi, pr in enumerate(st):
            same = torch.equal(views[k].view(torch.int16), ref[k].view(torch.int16))
            assert same, (si, gi, pr.desc, (views[k].float() - ref[k].float()).abs().max().item())
            k += 1
    assert torch.equal(ypart, ref_bits), (ypart.sum().item(), ref_bits.sum().item())
