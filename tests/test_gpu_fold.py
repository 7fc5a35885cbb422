"""GPU: the folded slice-chain convs (csrc/fold.hip) against a plain PyTorch fp32 reference.

rgbac_conv_fold recomputes a narrow 3x3 128 -> 8 conv per workgroup and feeds its 8 values as
the last input channels of a wide 3x3 conv (+ bias + GELU):
  GAUSS: value = round(y - mu) + mu            (cc_mean_transforms[i][4] into lrp_transforms[i][0],
                                                models/AutoEncoderRGB_Journal.py:255-262)
  TANH:  value = pre + 0.5 * tanh(conv + b)    (lrp_transforms[i][4] into the next cc1, :263-264)
The reference computes the narrow conv, the value (rounded to bf16, as the kernel stores it) and
the wide conv in fp32 on the same bf16 inputs and bf16-rounded weights.  Tolerances: the wide
output is bf16 (relative 2e-2 of its range); mu is fp32 (1e-3 absolute: only the summation
order differs); y is drawn so that y - mu stays >= 0.1 from a rounding tie, so the quantised
values are exact.  rgbac_gauss_bits: the fp32 likelihood / bits of the same formula as
rgbac_gaussian_slice, per 64-pixel tile (relative 1e-3: the kernel's Phi is the
branch-free erfc of conv_common.h)."""
import math

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _mods(c_in, seed):
    g = torch.Generator().manual_seed(seed)
    wide = nn.Conv2d(c_in, 224, 3, padding=1)
    narrow = nn.Conv2d(128, 8, 3, padding=1)
    with torch.no_grad():
        for m in (wide, narrow):
            m.weight.copy_(torch.randn(m.weight.shape, generator=g) / math.sqrt(9 * m.in_channels))
            m.bias.copy_(0.1 * torch.randn(m.bias.shape, generator=g))
    return wide, narrow


def _bfw(m):
    return m.weight.detach().bfloat16().float(), m.bias.detach().float()


def _nchw(f):
    from rgbac import runtime as rt
    return rt.to_nchw(f)


@pytest.mark.parametrize("mode", ["gauss", "tanh"])
@pytest.mark.parametrize("n,bn,ng", [(0, 64, 1), (16, 128, 2), (40, 128, 3), (8, 64, 2)])
def test_conv_fold(device, mode, n, bn, ng):
    from rgbac import _lib
    from rgbac import runtime as rt
    from rgbac.models import _latent
    B, h, w, Cm, cs = 2, 8, 32, 80, 8
    dt = torch.bfloat16
    g = torch.Generator().manual_seed(7 + n + ng)
    means = rt.to_nhwc(torch.randn((B, Cm, h, w), generator=g).to(device), dt)
    YH = rt.to_nhwc(torch.randn((B, 80, h, w), generator=g).to(device), dt)
    pins = [rt.to_nhwc(torch.randn((B, 128, h, w), generator=g).to(device), dt) for _ in range(ng)]
    mods = [_mods(Cm + n + cs, 100 + i) for i in range(ng)]
    mods = [(wd.to(device), nr.to(device)) for wd, nr in mods]
    # reference narrow conv (fp32 on the bf16 values)
    mu_ref = []
    for i in range(ng):
        wn, bnn = _bfw(mods[i][1])
        mu_ref.append(F.conv2d(_nchw(pins[i]), wn, bnn, padding=1))
    if mode == "gauss":
        # y = mu + integer + offset in [-0.4, 0.4]: no quantisation tie within bf16 noise
        yc = torch.zeros((B, 80, h, w), device=device)
        for i in range(ng):
            off = (torch.randint(-3, 4, (B, cs, h, w), generator=g) +
                   0.8 * (torch.rand((B, cs, h, w), generator=g) - 0.5)).to(device)
            yc[:, i * cs:(i + 1) * cs] = mu_ref[i] + off
        y = rt.to_nhwc(yc, dt)
        auxes = [(y, i * cs) for i in range(ng)]
        a_ref = [_nchw(y)[:, i * cs:(i + 1) * cs] for i in range(ng)]
    else:
        pres = [rt.to_nhwc(torch.randn((B, cs, h, w), generator=g).to(device), dt)
                for _ in range(ng)]
        auxes = [(p, 0) for p in pres]
        a_ref = [_nchw(p) for p in pres]
    outs = [rt.new_feat(B, h, w, 224, dt, device) for _ in range(ng)]
    put = rt.new_feat(B, h, w, 80, dt, device)
    put.t.fill_(7.0)
    MU = torch.full((B, h, w, 80), 9.0, device=device)
    dummy = rt.new_feat(B, h, w, cs, dt, device)
    groups = []
    for i in range(ng):
        writer = mode == "gauss" or i == 0
        groups.append(_latent._fold_group(
            mods[i][0], [means.src(), YH.src(0, n), dummy.src()], Cm + n, outs[i], pins[i],
            mods[i][1], auxes[i], put=(put, i * cs) if writer else None,
            mu=(MU, i * cs) if mode == "gauss" else None))
    _latent._fold_launch(groups, _lib.FOLD_GAUSS if mode == "gauss" else _lib.FOLD_TANH, bn,
                         B, h, w, device, "conv_fold_kernel")
    torch.cuda.synchronize()
    put_c = _nchw(put)
    for i in range(ng):
        mu = mu_ref[i]
        val = (torch.round(a_ref[i] - mu) + mu) if mode == "gauss" else \
            a_ref[i] + 0.5 * torch.tanh(mu)
        val = val.bfloat16().float()
        inp = torch.cat([_nchw(means), _nchw(YH)[:, :n], val], 1)
        ww, wb = _bfw(mods[i][0])
        ref = F.gelu(F.conv2d(inp, ww, wb, padding=1))
        got = _nchw(outs[i])
        err = ((got - ref).abs().max() / ref.abs().max()).item()
        assert err < 2e-2, (i, err)
        writer = mode == "gauss" or i == 0
        sl = put_c[:, i * cs:(i + 1) * cs]
        if writer:
            assert (sl - val).abs().max().item() <= 1e-2 * max(val.abs().max().item(), 1.0)
            if mode == "gauss":
                mu_got = MU[..., i * cs:(i + 1) * cs].permute(0, 3, 1, 2)
                assert (mu_got - mu).abs().max().item() < 1e-3
        else:
            assert (sl == 7.0).all(), "a non-writer group wrote its folded values"
    if mode == "tanh":
        assert (MU == 9.0).all()


def test_gauss_bits(device):
    from rgbac import _lib
    from rgbac import runtime as rt
    from rgbac.models import _latent
    B, h, w, cs, ns = 2, 8, 32, 8, 3
    dt = torch.bfloat16
    g = torch.Generator().manual_seed(3)
    pins = [rt.to_nhwc(torch.randn((B, 128, h, w), generator=g).to(device), dt) for _ in range(ns)]
    convs = [_mods(88, 200 + i)[1].to(device) for i in range(ns)]
    y = rt.to_nhwc((3 * torch.randn((B, 80, h, w), generator=g)).to(device), dt)
    MU = (2 * torch.randn((B, h, w, 80), generator=g)).to(device)
    ypart = torch.zeros((ns, B * h * w // 32), dtype=torch.float64, device=device)
    import ctypes
    groups = []
    for i in range(ns):
        gg = _lib.BitsGroup()
        gg.pin, gg.pin_ldc = pins[i].ptr(), pins[i].ldc
        pw, pb = _latent._narrow_pack(convs[i], dt)
        gg.pweight, gg.pbias = pw.data_ptr(), pb.data_ptr()
        gg.y, gg.y_ldc = y.ptr(i * cs), y.ldc
        gg.mu, gg.mu_ldc = MU.data_ptr() + 4 * i * cs, 80
        gg.partial = ypart[i].data_ptr()
        groups.append(gg)
    arr = (_lib.BitsGroup * ns)(*groups)
    _lib.call("rgbac_gauss_bits", ctypes.cast(arr, ctypes.c_void_p), ns, B, h, w,
              _lib.stream_ptr(device))
    torch.cuda.synchronize()
    yc = _nchw(y)
    for i in range(ns):
        wn, bnn = _bfw(convs[i])
        sigma = F.conv2d(_nchw(pins[i]), wn, bnn, padding=1)
        mu = MU[..., i * cs:(i + 1) * cs].permute(0, 3, 1, 2)
        hat = torch.round(yc[:, i * cs:(i + 1) * cs] - mu) + mu
        d = (hat - mu).abs()
        sc = sigma.clamp_min(0.11)

        def phi(t):
            return 0.5 * torch.erfc(-t / math.sqrt(2.0))
        lik = (phi((0.5 - d) / sc) - phi((-0.5 - d) / sc)).clamp_min(1e-9)
        bits = (-torch.log(lik + 1e-10) / math.log(2.0)).clamp(0.0, 50.0).double()
        # per 4 x 16 tile, tiles in (batch, row, column) order
        tiles = bits.sum(1).reshape(B, h // 4, 4, w // 16, 16).sum((2, 4)).reshape(-1)
        got = ypart[i, :tiles.numel()]
        assert ((got - tiles).abs() <= 1e-3 * tiles.abs().clamp_min(1.0)).all(), i
        assert (ypart[i, tiles.numel():] == 0).all()


def test_fold_rejects_bad_shapes(device):
    from rgbac import _lib
    import ctypes
    arr = (_lib.FoldGroup * 1)()
    with pytest.raises(RuntimeError, match="multiple of 4"):
        _lib.call("rgbac_conv_fold", ctypes.cast(arr, ctypes.c_void_p), 1, 1, 6, 16,
                  _lib.FOLD_GAUSS, 64, _lib.stream_ptr(device))
    with pytest.raises(RuntimeError, match="source channels"):
        _lib.call("rgbac_conv_fold", ctypes.cast(arr, ctypes.c_void_p), 1, 1, 8, 16,
                  _lib.FOLD_GAUSS, 64, _lib.stream_ptr(device))
