"""CPU: analytic known-answer tests pinning the oracle (oracle/ref_model.py).

The reference ships no tests or vectors and cannot be imported here (SURVEY.md
§8c), so these KATs are derived from first principles for each restated op.
"""
import math
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import ref_model as ref


def _sd_prefix(module, prefix):
    return {f"{prefix}.{k}": v for k, v in module.state_dict().items()}


def test_window_partition_roundtrip():
    g = torch.Generator().manual_seed(0)
    for ws, H, W in ((8, 16, 24), (4, 8, 12)):
        x = torch.randn((2, H, W, 5), generator=g)
        w = ref.window_partition(x, ws)
        assert w.shape == (2 * (H // ws) * (W // ws), ws, ws, 5)
        # window (b, wy, wx) holds x[b, wy*ws:(wy+1)*ws, wx*ws:(wx+1)*ws]
        assert torch.equal(w[1], x[0, 0:ws, ws:2 * ws])
        assert torch.equal(ref.window_reverse(w, ws, H, W), x)


@pytest.mark.parametrize("ws", [4, 8])
def test_relative_position_index(ws):
    idx = ref.relative_position_index(ws)
    N = ws * ws
    assert idx.shape == (N, N) and idx.dtype == torch.int64
    assert idx.min() == 0 and idx.max() == (2 * ws - 1) ** 2 - 1
    center = (ws - 1) * (2 * ws - 1) + (ws - 1)
    assert torch.all(idx.diagonal() == center)
    assert torch.all(idx + idx.T == 2 * center)          # d(i,j) = -d(j,i)
    i, j = 1 * ws + 2, 3 * ws + 0                          # (1,2) vs (3,0): dy=-2, dx=+2
    assert idx[i, j] == (-2 + ws - 1) * (2 * ws - 1) + (2 + ws - 1)


def test_shift_region_ids():
    reg = ref._region_ids(1, 16, 16, 8, 4)[0, :, :, 0]
    # rows [0,8) -> 0, [8,12) -> 1, [12,16) -> 2; same for columns; id = 3*r + c
    assert reg[0, 0] == 0 and reg[0, 9] == 1 and reg[0, 13] == 2
    assert reg[9, 0] == 3 and reg[13, 13] == 8 and reg[10, 14] == 5
    assert torch.unique(reg).numel() == 9


def test_gdn_known_answer():
    """gamma <= bound -> gamma' = 2^-36 - 2^-36 = 0, so y = x / sqrt(beta^2 - 2^-36)."""
    C = 6
    beta = torch.linspace(0.5, 2.0, C)
    sd = {"g.beta": beta, "g.gamma": torch.zeros(C, C)}
    x = torch.randn((2, C, 3, 4), generator=torch.Generator().manual_seed(1))
    ped = (2.0 ** -18) ** 2
    b_eff = (torch.max(beta, torch.full_like(beta, (1e-6 + ped) ** 0.5)) ** 2 - ped)
    want = x / torch.sqrt(b_eff).view(1, C, 1, 1)
    assert torch.allclose(ref.gdn(x, sd, "g"), want, rtol=1e-6, atol=0)
    assert torch.allclose(ref.gdn(x, sd, "g", inverse=True),
                          x * torch.sqrt(b_eff).view(1, C, 1, 1), rtol=1e-6, atol=0)


@pytest.mark.parametrize("sigma", [0.05, 0.11, 0.5, 1.0, 3.0, 40.0])
def test_gaussian_likelihood_closed_form(sigma):
    """y == mu -> symbol 0, p = erf(0.5 / (s*sqrt2)) with s = max(sigma, 0.11)."""
    y = torch.full((1, 1, 2, 2), 0.25)
    _, lik = ref.gc_forward(y, torch.full_like(y, sigma), y.clone())
    s = max(sigma, float(np.float32(0.11)))
    want = max(math.erf(0.5 / (s * math.sqrt(2.0))), 1e-9)
    assert abs(lik[0, 0, 0, 0].item() - want) < 2e-6 * max(want, 1e-3)
    bits = ref._bits(lik) / 4
    assert abs(bits.item() - min(max(-math.log2(want + 1e-10), 0), 50)) < 1e-4


def test_quantiser_half_to_even():
    y = torch.tensor([0.5, 1.5, 2.5, -0.5, -1.5, 0.4999, 2.5001])
    mu = torch.zeros_like(y)
    out, _ = ref.gc_forward(y.view(1, 1, 1, -1), torch.ones(1, 1, 1, 7), mu.view(1, 1, 1, -1))
    assert out.flatten().tolist() == [0.0, 2.0, 2.0, -0.0, -2.0, 0.0, 3.0]
    assert torch.equal(ref.ste_round(y), torch.round(y))


def test_entropy_bottleneck_init_is_affine():
    """At compressai init (factors 0) the density model is affine: every layer is
    softplus(M) @ t + b with softplus(M) = 1/scale/f_out; re-derived in numpy."""
    import sys
    from rgbac.entropy import EntropyBottleneck
    torch.manual_seed(3)
    eb = EntropyBottleneck(4)
    sd = _sd_prefix(eb, "eb")
    x = torch.linspace(-3, 3, 7).repeat(4, 1, 1)                  # (C,1,L)
    got = ref.eb_logits_cumulative(sd, "eb", x).numpy()
    scale = 10.0 ** (1 / 5)
    f = (1, 3, 3, 3, 3, 1)
    t = x.numpy().astype(np.float64)
    for i in range(5):
        m = np.full((f[i + 1], f[i]), 1.0 / scale / f[i + 1])
        b = eb.state_dict()[f"_bias{i}"].numpy().astype(np.float64)    # (C, f_out, 1)
        t = np.einsum("oi,cil->col", m, t) + b
    np.testing.assert_allclose(got, t, rtol=1e-5, atol=1e-5)
    # medians are quantiles[:, :, 1] = 0 at init
    assert torch.all(ref.eb_medians(sd, "eb") == 0)


def test_masked_attention_special_alphas():
    from rgbac.layers.masked_win_attention import WinBasedAttention
    torch.manual_seed(5)
    m = WinBasedAttention(dim=16, num_heads=8, window_size=4, shift_size=2)
    sd = _sd_prefix(m, "blk")
    x = torch.randn((2, 16, 8, 12))
    zero = torch.zeros((2, 1, 8, 12))
    # all-transparent alpha: every window dropped -> block is the identity (x + 0)
    assert torch.equal(ref.win_based_attention(x, zero, sd, "blk", 4, 2), x)
    # all-opaque alpha == the unmasked variant (win_attention.py)
    ones = torch.ones_like(zero)
    a = ref.win_based_attention(x, ones, sd, "blk", 4, 2)
    b = ref.win_based_attention(x, None, sd, "blk", 4, 2, masked=False)
    assert torch.allclose(a, b, rtol=0, atol=1e-6)


def test_reconstruct_error_cases():
    g = torch.Generator().manual_seed(2)
    x, y = torch.rand((2, 3, 8, 8), generator=g), torch.rand((2, 3, 8, 8), generator=g)
    ones = torch.ones((2, 1, 8, 8))
    assert torch.allclose(ref.reconstruct_error(x, y, ones), F.mse_loss(x, y), rtol=1e-6)
    assert ref.reconstruct_error(x, y, torch.zeros_like(ones)).item() == 0.0
    half = ones.clone()
    half[..., :4] = 0
    want = ((x - y)[..., 4:] ** 2).sum(dim=(1, 2, 3)) / (3 * 8 * 4)
    assert torch.allclose(ref.reconstruct_error(x, y, half), want.mean(), rtol=1e-6)


def test_supply_mask_pyramid():
    a = torch.zeros((1, 1, 256, 256))
    a[..., 100:110, 40:41] = 0.2
    lv = ref.supply_mask(a)
    assert [t.shape[-1] for t in lv] == [128, 64, 32, 16, 8, 4]
    # with alpha >= 0 the non-zero pattern equals a 3x3/s2/p1 OR-pool chain
    nz = (a > 0).float()
    for t in lv:
        nz = (F.max_pool2d(nz, 3, stride=2, padding=1) > 0).float()
        assert torch.equal((t > 0).float(), nz)
    assert abs(lv[0].max().item() - 0.2 * 3 / 9) < 1e-7


def test_constraint_rgb():
    t = torch.ones((1, 1, 5, 5))
    t[0, 0, 2, 2] = 0                  # isolated zero -> 1
    u = torch.zeros((1, 1, 5, 5))
    u[0, 0, 1, 1] = 0.5                # isolated non-zero -> 0
    assert torch.equal(ref.constraint_rgb(t), torch.ones_like(t))
    assert torch.equal(ref.constraint_rgb(u), torch.zeros_like(u))


@pytest.mark.slow
def test_models_run_small():
    from rgbac.models.AutoEncoderMask_Journal import AutoEncoder as MaskAE
    from rgbac.models.AutoEncoderRGB_Journal import AutoEncoder
    torch.manual_seed(234)
    net = AutoEncoder().eval()
    x = torch.rand((1, 3, 64, 64))
    a = torch.ones((1, 1, 64, 64))
    me = ref.supply_mask(a)
    with torch.no_grad():
        out = ref.rgb_forward(net.state_dict(), x, a, a, *me[:4])
    assert out[0].shape == x.shape and torch.isfinite(out[0]).all()
    assert out[2] > 0 and abs(out[2] - out[3] - out[4]) < 1e-6
    m = MaskAE().eval()
    with torch.no_grad():
        o2 = ref.mask_forward(m.state_dict(), a)
    assert o2[0].shape == a.shape and torch.isfinite(o2[0]).all()


def test_ms_ssim_oracle_known_answers():
    """ssim(X, X) = ms_ssim(X, X) = 1; constant images a, b: cs = C2/C2 = 1 and
    ssim = (2ab + C1) / (a^2 + b^2 + C1) (ms_ssim_torch.py:70-71)."""
    from oracle import ref_metrics as rm
    g = torch.Generator().manual_seed(5)
    X = torch.rand((2, 3, 176, 176), generator=g)
    assert abs(rm.ms_ssim(X, X, data_range=1.0).item() - 1.0) < 1e-5
    assert abs(rm.ssim(X, X, data_range=1.0).item() - 1.0) < 1e-5
    a, b = 0.25, 0.75
    A, Bc = torch.full((1, 1, 32, 32), a), torch.full((1, 1, 32, 32), b)
    c1 = 0.01 ** 2
    want = (2 * a * b + c1) / (a * a + b * b + c1)
    s, cs = rm.ssim_level(A, Bc, rm.fspecial_gauss_1d(11, 1.5).repeat(1, 1, 1, 1), 1.0)
    # fp32 E[X^2] - mu^2 cancels to ~1e-7 against C2 = 9e-4: 1e-3 covers that noise
    assert abs(s.item() - want) < 1e-3 and abs(cs.item() - 1.0) < 1e-3


def test_masked_ms_ssim_oracle_known_answers():
    """masked_ms_ssim_torch.py: an all-ones mask keeps every valid pixel, so a level's masked
    per-channel mean is the plain map mean (:115-116); X = Y scores 1 under any mask that keeps
    pixels at every level; an all-zero mask scores 0 (0 / (0 + 1e-10), relu, 0 ** w)."""
    from oracle import ref_metrics as rm
    g = torch.Generator().manual_seed(6)
    X = torch.rand((2, 1, 48, 56), generator=g)
    Y = torch.clamp(X + 0.1 * torch.randn(X.shape, generator=g), 0, 1)
    win = rm.fspecial_gauss_1d(11, 1.5).repeat(1, 1, 1, 1)
    s0, c0 = rm.ssim_level(X, Y, win, 1.0)
    s1, c1 = rm.masked_ssim_level(X, Y, torch.ones_like(X), win, 1.0)
    assert (s1[:, 0] - s0).abs().max() < 1e-5 and (c1[:, 0] - c0).abs().max() < 1e-5
    X = torch.rand((2, 3, 176, 192), generator=g)
    m = torch.ones((2, 1, 176, 192))
    m[:, :, 120:, 150:] = 0         # the coarsest level's 1x2 valid map still samples a kept pixel
    assert abs(rm.masked_ms_ssim(X, X, m, data_range=1.0).item() - 1.0) < 1e-5
    assert rm.masked_ms_ssim(X, X * 0.5, torch.zeros_like(m), data_range=1.0).item() == 0.0


@pytest.mark.parametrize("hw", [(161, 177), (80, 96), (40, 45), (20, 23), (10, 12), (5, 6)])
@pytest.mark.parametrize("ws", [7, 11])
def test_masked_nearest_index_matches_interpolate(hw, ws):
    """csrc/msssim.hip masked_ssim_tile_kernel samples the level mask at
    min(floor(float32(o) * float32(in / out)), in - 1); that must be the source pixel
    F.interpolate(mode='nearest') (torchvision's NEAREST resize, :104) picks."""
    H, W = hw
    if H < ws or W < ws:
        pytest.skip("smaller than the window")
    Ho, Wo = H - ws + 1, W - ws + 1
    idx = torch.arange(H * W, dtype=torch.float32).reshape(1, 1, H, W)
    got = F.interpolate(idx, size=(Ho, Wo), mode="nearest")[0, 0].long()
    sh, sw = np.float32(H) / np.float32(Ho), np.float32(W) / np.float32(Wo)
    ys = np.minimum(np.floor(np.arange(Ho, dtype=np.float32) * sh).astype(np.int64), H - 1)
    xs = np.minimum(np.floor(np.arange(Wo, dtype=np.float32) * sw).astype(np.int64), W - 1)
    want = torch.from_numpy(ys[:, None] * W + xs[None, :])
    assert torch.equal(got, want)


def test_teacher_forcing_with_own_latents_is_identity():
    """oracle/parity.py: forcing the oracle's OWN z_hat / y_hat reproduces its free-running
    forward exactly, and the accounting of a forward against itself finds no flip."""
    import importlib.util
    from oracle import parity
    spec = importlib.util.spec_from_file_location(
        "make_golden", os.path.join(os.path.dirname(__file__), "golden", "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    sd = mg.rgb_model(mg.LATENT_GAIN).state_dict()
    x, a = mg.rgb_inputs(2, 64, 64, seed=3)
    me = ref.supply_mask(a)
    dbg = {}
    with torch.no_grad():
        free = ref.rgb_forward(sd, x, a, a, *me[:4], dbg=dbg)
    tf, dbg2 = parity.teacher_forced(sd, "rgb", x, dbg["y_hat"], dbg["z_hat"], a, a)
    for u, v in zip(free, tf):
        assert torch.equal(u, v)
    rep = parity.symbol_accounting(dbg["y"], dbg["mu"], dbg2["y"], dbg2["mu"], dbg["z"],
                                   dbg2["z"], dbg2["z_med"], dbg["lik"], dbg2["lik"])
    assert rep["flips"] == 0 and rep["z_flips"] == 0 and rep["noise_floor"] == 0.0
    assert rep["nonzero_symbols"] > rep["symbols"] // 4
    assert rep["bits_unflipped_rel"] == 0.0
    # a planted flip far from any tie is classified "far"
    y_bad = [t.clone() for t in dbg["y"]]
    y_bad[3][0, 0, 0, 0] += 1.0
    rep = parity.symbol_accounting(y_bad, dbg["mu"], dbg2["y"], dbg2["mu"])
    assert rep["flips"] == 1 and rep["far_flips"] == 1
