"""End-to-end GPU parity of both codecs against the CPU oracle (fp32 parity mode),
plus stage-wise (teacher-forced) checks that isolate quantisation flips."""
import pytest
import torch

from oracle import ref_model as ref

pytestmark = pytest.mark.gpu


def cpu_sd(net):
    return {k: v.detach().cpu() for k, v in net.state_dict().items()}


def rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


def _inputs(B, H, W, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.round(torch.rand((B, 3, H, W), generator=g) * 255) / 255
    a = torch.ones((B, 1, H, W))
    kinds = ["ones", "half", "blob", "zero"]
    for b in range(B):
        k = kinds[b % 4]
        if k == "half":
            a[b, :, :, : W // 2] = 0
        elif k == "blob":
            yy, xx = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
            r = ((yy - H / 2) ** 2 + (xx - W / 2) ** 2).float().sqrt()
            a[b, 0] = torch.clamp((H / 3 - r) / 8, 0, 1)
            a[b, 0] = torch.round(a[b, 0] * 255) / 255
        elif k == "zero":
            a[b].zero_()
    xm = torch.where(a > 0, x, a)
    return xm, a


@pytest.fixture(scope="module")
def rgb_net():
    from rgbac.models.AutoEncoderRGB_Journal import AutoEncoder
    torch.manual_seed(234)
    return AutoEncoder().eval()


def test_rgb_forward_fp32(device, rgb_net):
    x, a = _inputs(4, 64, 128)
    me = ref.supply_mask(a)
    sd = cpu_sd(rgb_net)
    with torch.no_grad():
        want = ref.rgb_forward(sd, x, a, a, *me[:4])
    net = rgb_net.to(device)
    dbg = {}
    got = net(x.to(device), a.to(device), a.to(device), *[m.to(device) for m in me[:4]], debug=dbg)
    with torch.no_grad():
        y_ref = ref.analysis(x, sd, "Encoder", me[1], me[2])
    from rgbac import runtime as rt
    assert rel(rt.to_nchw(dbg["y"]), y_ref) < 1e-4
    assert got[0].shape == want[0].shape
    print("x_hat rel", rel(got[0], want[0]), "bpp", got[2].item(), want[2].item())
    assert rel(got[0], want[0]) < 1e-3
    for i in (1, 2, 3, 4):
        assert abs(got[i].item() - want[i].item()) <= 1e-4 * max(abs(want[i].item()), 1e-6)


def test_rgb_forward_bf16(device, rgb_net):
    x, a = _inputs(2, 64, 64, seed=1)
    me = ref.supply_mask(a)
    with torch.no_grad():
        want = ref.rgb_forward(cpu_sd(rgb_net), x, a, a, *me[:4])
    net = rgb_net.to(device).set_compute_dtype(torch.bfloat16)
    try:
        got = net(x.to(device), a.to(device), a.to(device), *[m.to(device) for m in me[:4]])
    finally:
        net.set_compute_dtype(torch.float32)
    assert torch.isfinite(got[0]).all()
    # bf16 storage: reconstruction within 5e-2 of the fp32 oracle's range, bpp within 5 %
    assert rel(got[0], want[0]) < 5e-2
    assert abs(got[2].item() - want[2].item()) < 0.05 * want[2].item()


def test_mask_forward_fp32(device):
    from rgbac.models.AutoEncoderMask_Journal import AutoEncoder
    torch.manual_seed(234)
    net = AutoEncoder().eval()
    _, a = _inputs(2, 64, 64, seed=3)
    with torch.no_grad():
        want = ref.mask_forward(cpu_sd(net), a)
    got = net.to(device)(a.to(device))
    print("alpha x_hat rel", rel(got[0], want[0]))
    assert rel(got[0], want[0]) < 1e-3
    for i in (1, 2, 3, 4):
        assert abs(got[i].item() - want[i].item()) <= 1e-4 * max(abs(want[i].item()), 1e-6)


def test_rgb_bf16_slice_precompute_matches(device, rgb_net):
    """bf16 inference with the side-stream precompute of the slice convs' latent-means/scales
    half (rgbac.models._latent.PRECOMPUTE: every slice, or only the wide tail wave) and with
    the single-conv path: all within the bf16 bar of the fp32 oracle, and the same bpp within
    bf16 noise."""
    from rgbac.models import _latent
    x, a = _inputs(4, 64, 64, seed=3)
    me = ref.supply_mask(a)
    with torch.no_grad():
        want = ref.rgb_forward(cpu_sd(rgb_net), x, a, a, *me[:4])
    net = rgb_net.to(device).set_compute_dtype(torch.bfloat16)
    outs, saved = {}, _latent.PRECOMPUTE
    try:
        for flag in (None, "all", "tail"):
            _latent.PRECOMPUTE = flag
            with torch.no_grad():
                outs[flag] = net(x.to(device), a.to(device), a.to(device),
                                 *[m.to(device) for m in me[:4]])
    finally:
        _latent.PRECOMPUTE = saved
        net.set_compute_dtype(torch.float32)
    for got in outs.values():
        assert rel(got[0], want[0]) < 5e-2
        assert abs(got[2].item() - want[2].item()) < 0.05 * want[2].item()
    b0 = outs[None][2].item()
    for flag in ("all", "tail"):
        assert abs(b0 - outs[flag][2].item()) < 0.02 * b0, flag


def test_rgb_forward_fp32_north_star_bar(device):
    """The north_star bar on real (non-zero) symbols: the seed-234 codec with Encoder.x4 x20
    (tests/golden/make_golden.py LATENT_GAIN), B=4 (alpha ones / half / blob / zero), fp32
    parity mode vs the oracle -- PSNR (trainRGB.py:305-306, from the model's masked MSE) and
    MS-SSIM of the clamped reconstruction (:308-311) within 1e-4, bpp within 2e-5 relative,
    and the integer symbols round(y - mu) of all slices identical except at near-ties."""
    import importlib.util
    import math
    import os
    spec = importlib.util.spec_from_file_location(
        "make_golden", os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                    "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    from oracle import ref_metrics
    from rgbac.metrics.ms_ssim_torch import ms_ssim
    net = mg.rgb_model(mg.LATENT_GAIN)
    sd = cpu_sd(net)
    x, a = _inputs(4, 192, 192, seed=7)            # MS-SSIM's 5 levels need > 160 px
    dev_net = net.to(device)
    worst = {"psnr": 0.0, "msssim": 0.0, "bpp": 0.0, "flips": 0, "flips_far": 0, "nsym": 0}
    for i in range(4):
        xi, ai = x[i:i + 1], a[i:i + 1]
        me = ref.supply_mask(ai)
        dbg = {}
        with torch.no_grad():
            want = ref.rgb_forward(sd, xi, ai, ai, *me[:4], dbg=dbg)
            gd = {}
            got = dev_net(xi.to(device), ai.to(device), ai.to(device),
                          *[m.to(device) for m in me[:4]], debug=gd)
        worst["bpp"] = max(worst["bpp"], abs(got[2].item() - want[2].item()) / want[2].item())
        if want[1].item() > 0:
            dp = abs(10 * math.log10(1 / got[1].item()) - 10 * math.log10(1 / want[1].item()))
            worst["psnr"] = max(worst["psnr"], dp)
        ms_g = ms_ssim(xi.to(device), got[0].clamp(0, 1), data_range=1.0).item()
        ms_r = ref_metrics.ms_ssim(xi, want[0].clamp(0, 1), data_range=1.0).item()
        worst["msssim"] = max(worst["msssim"], abs(ms_g - ms_r))
        y = gd["y"].t[..., :80].float().cpu()
        for s in range(10):
            mu_g = gd["musigma"][s].t[..., :8].float().cpu()
            sym_g = torch.round(y[..., 8 * s:8 * s + 8] - mu_g).permute(0, 3, 1, 2)
            d = dbg["y"][s] - dbg["mu"][s]
            sym_r = torch.round(d)
            near = (d - torch.floor(d) - 0.5).abs() < 1e-3
            worst["flips"] += int((sym_g != sym_r).sum())
            worst["flips_far"] += int(((sym_g != sym_r) & ~near).sum()) if s == 0 else 0
            worst["nsym"] += sym_r.numel()
    print("north-star bar (fp32):", worst)
    assert worst["flips_far"] == 0
    assert worst["flips"] <= 1e-4 * worst["nsym"] + 2
    assert worst["bpp"] < 2e-5
    assert worst["psnr"] < 1e-4
    assert worst["msssim"] < 1e-4
