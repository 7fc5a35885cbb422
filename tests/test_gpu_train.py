"""GPU parity of the training path (backward kernels) against autograd of the
CPU references: plain torch fp32 for single convs, the oracle
(oracle/ref_model.py, with the reference's LowerBound gradient rule) for GDN,
attention, entropy models and the whole RGB codec.

Tolerances (relative to the reference gradient's max magnitude unless stated):
fp32 single ops 1e-4 (exact-f32 MFMA, different summation order); bf16 single
convs 4e-2; whole-model parameter gradients 1e-4 norm-wise (||g - g_ref|| /
||g_ref||; measured max 5e-6 over every parameter of the RGB codec, median 3e-7).
"""
import zlib

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from oracle import ref_model as ref

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


def nrel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _gen(seed):
    return torch.Generator().manual_seed(seed)


def _rt():
    from rgbac import runtime as rt
    return rt


def _leaf(x, dtype):
    """fp32 NCHW CPU tensor -> NHWC Feat on the GPU whose tensor is an autograd leaf."""
    rt = _rt()
    f = rt.to_nhwc(x.cuda(), dtype)
    f.t.requires_grad_(True)
    return f


def _nchw_grad(f):
    rt = _rt()
    return rt.to_nchw(rt.Feat(f.t.grad, f.C)).cpu()


ACTS = [("none", 0.0), ("gelu", 0.0), ("relu", 0.0), ("lrelu", 0.01), ("tanh_half", 0.0),
        ("gate", 0.0), ("masksel", 0.0)]


def _ref_act(act, slope, v, r0, r1, r2, sel):
    if r0 is not None:
        v = v + r0
    if act == "gelu":
        v = F.gelu(v)
    elif act == "relu":
        v = F.relu(v)
    elif act == "lrelu":
        v = F.leaky_relu(v, slope)
    elif act == "tanh_half":
        v = r1 + 0.5 * torch.tanh(v)
    elif act == "gate":
        v = r1 * torch.sigmoid(v)
    elif act == "masksel":
        v = torch.where(sel[:, None].bool(), r1 + v, r1)
    if r2 is not None:
        v = v + r2
    return v


LAYERS = ["conv3_2src", "conv3_wide", "conv5s2", "conv3s2", "conv1", "convt5", "convt5_c3", "convt1",
          "subpel", "linear"]


def _make(name, g):
    if name == "conv3_2src":
        return nn.Conv2d(40, 24, 3, padding=1), [16, 24], 1
    if name == "conv3_wide":                  # K = 864 >= 512: the 64x128 wgrad tile
        return nn.Conv2d(96, 40, 3, padding=1), [96], 1
    if name == "conv5s2":
        return nn.Conv2d(3, 16, 5, stride=2, padding=2), [3], 2
    if name == "conv3s2":
        return nn.Conv2d(24, 16, 3, stride=2, padding=1), [24], 2
    if name == "conv1":
        return nn.Conv2d(20, 12, 1), [20], 1
    if name == "convt5":
        return nn.ConvTranspose2d(16, 8, 5, stride=2, padding=2, output_padding=1), [16], 0.5
    if name == "convt5_c3":
        return nn.ConvTranspose2d(16, 3, 5, stride=2, padding=2, output_padding=1), [16], 0.5
    if name == "convt1":
        return nn.ConvTranspose2d(8, 16, 1), [8], 1
    if name == "subpel":
        return nn.Sequential(nn.Conv2d(8, 16, 3, padding=1), nn.PixelShuffle(2)), [8], 0.5
    if name == "linear":
        return nn.Linear(24, 40), [24], 1


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("act,slope", ACTS)
@pytest.mark.parametrize("name", LAYERS)
def test_conv_fn_grads(name, act, slope, dtype):
    if name in ("subpel",) and act not in ("none", "gelu"):
        pytest.skip("subpel epilogue supports NONE/GELU")
    rt = _rt()
    from rgbac import autograd as ag
    g = _gen(zlib.crc32(f"{name}/{act}".encode()) % 100000)
    m, segs, scale = _make(name, g)
    # bf16 mode: the reference sees the same bf16-representable inputs and weights the
    # kernels see (fp32 math on them), so ReLU kinks are decided on equal pre-activations
    rnd = (lambda t: t.to(torch.bfloat16).float()) if dtype == torch.bfloat16 else (lambda t: t)
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(rnd(torch.randn(p.shape, generator=g) * 0.2))
    B, H, W = 2, 8, 12
    xs = [rnd(torch.randn((B, c, H, W), generator=g)).requires_grad_(True) for c in segs]
    x = torch.cat(xs, 1)
    if name == "linear":
        v = F.linear(x.permute(0, 2, 3, 1), m.weight, m.bias).permute(0, 3, 1, 2)
    else:
        v = m(x)
    Cout, Ho, Wo = v.shape[1], v.shape[2], v.shape[3]
    use0 = act in ("none", "gelu", "relu", "lrelu")
    use1 = act in ("tanh_half", "gate", "masksel")
    use2 = act in ("none", "gate")
    if name == "subpel":
        use0 = use1 = use2 = False
    def leaf(on):
        return rnd(torch.randn((B, Cout, Ho, Wo), generator=g)).requires_grad_(True) if on else None
    r0, r1, r2 = leaf(use0), leaf(use1), leaf(use2)
    sel = (torch.rand((B, Ho, Wo), generator=g) > 0.4).to(torch.uint8) if act == "masksel" else None
    want = _ref_act(act, slope, v, r0, r1, r2, sel)
    gy = torch.randn(want.shape, generator=g)
    want.backward(gy)

    mg = _make(name, g)[0].cuda()
    mg.load_state_dict(m.state_dict())
    fx = [_leaf(t.detach(), dtype) for t in xs]
    fr = [None if r is None else _leaf(r.detach(), dtype) for r in (r0, r1, r2)]
    kw = dict(act=act, act_param=slope, res0=fr[0], res1=fr[1], res2=fr[2],
              sel=None if sel is None else sel.cuda())
    if name == "subpel":
        out = ag.conv_t(mg[0], fx, kind="subpel", **kw)
    else:
        out = ag.conv_t(mg, fx, **kw)
    got = rt.to_nchw(rt.Feat(out.t.detach(), out.C)).cpu()
    # fp32: max-abs relative; bf16: norm-wise (a ReLU/LeakyReLU kink flips where the
    # bf16 pre-activation and the fp32 reference straddle 0 -- O(1) per flipped element)
    tol, err = (1e-4, rel) if dtype == torch.float32 else (3e-2, nrel)
    assert got.shape == want.shape
    assert err(got, want) < tol
    out.t.backward(rt.to_nhwc(gy.cuda(), dtype).t)
    for f, t in zip(fx, xs):
        assert err(_nchw_grad(f), t.grad) < tol
    for f, r in zip(fr, (r0, r1, r2)):
        if r is not None:
            assert err(_nchw_grad(f), r.grad) < tol
    pg = dict(mg.named_parameters())
    for k, p in m.named_parameters():
        assert err(pg[k].grad, p.grad) < tol, k


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("inverse", [False, True])
def test_gdn_grads(inverse, dtype):
    from rgbac.layers.GDN import GDN
    from rgbac.train_forward import gdn_t
    g = _gen(21 + inverse)
    m = GDN(32, inverse=inverse)
    with torch.no_grad():
        m.gamma.add_(0.05 * torch.rand(m.gamma.shape, generator=g))
        m.beta.add_(0.1 * torch.rand(m.beta.shape, generator=g))
        m.beta[:3] = 1e-4                  # below beta_bound: LowerBound gradient rule
    x = torch.randn((2, 32, 8, 8), generator=g, requires_grad=True)
    sd = {"m." + k: v.detach().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    want = ref.gdn(x, sd, "m", inverse)
    gy = torch.randn(want.shape, generator=g)
    want.backward(gy)
    mg = GDN(32, inverse=inverse).cuda()
    mg.load_state_dict(m.state_dict())
    fx = _leaf(x.detach(), dtype)
    out = gdn_t(mg, fx)
    rt = _rt()
    tol = 1e-4 if dtype == torch.float32 else 4e-2
    assert rel(rt.to_nchw(rt.Feat(out.t.detach(), 32)).cpu(), want) < tol
    out.t.backward(rt.to_nhwc(gy.cuda(), dtype).t)
    assert rel(_nchw_grad(fx), x.grad) < tol
    assert rel(mg.beta.grad, sd["m.beta"].grad) < tol
    assert rel(mg.gamma.grad, sd["m.gamma"].grad) < tol


def _alpha(kind, B, H, W, g):
    a = torch.ones((B, 1, H, W))
    if kind == "zero":
        a.zero_()
    elif kind == "half":
        a[..., :, : W // 2] = 0
    elif kind == "rand":
        a = (torch.rand((B, 1, H, W), generator=g) > 0.97).float()
    return a


@pytest.mark.parametrize("dim,ws,H", [(192, 8, 16), (80, 4, 16)])
@pytest.mark.parametrize("kind", ["ones", "half", "rand", "zero"])
def test_attention_block_grads(dim, ws, H, kind):
    """Win_noShift_Attention (Masked_Attention.py:182-189) incl. the masked window
    attention core backward and the relative-position-bias table gradient."""
    from rgbac.layers.Masked_Attention import Win_noShift_Attention
    from rgbac.train_forward import attention_block_t
    g = _gen(dim + ws + len(kind))
    m = Win_noShift_Attention(dim=dim, num_heads=8, window_size=ws, shift_size=ws // 2)
    with torch.no_grad():
        m.attn.attn.relative_position_bias_table.normal_(0, 0.5, generator=g)
    W = H + 2 * ws
    x = torch.randn((2, dim, H, W), generator=g, requires_grad=True)
    a = _alpha(kind, 2, H, W, g)
    sd = {"blk." + k: v.detach().clone().requires_grad_(v.is_floating_point())
          for k, v in m.state_dict().items()}
    want = ref.win_noshift_attention(x, a, sd, "blk", ws, ws // 2)
    gy = torch.randn(want.shape, generator=g)
    want.backward(gy)
    mg = Win_noShift_Attention(dim=dim, num_heads=8, window_size=ws, shift_size=ws // 2).cuda()
    mg.load_state_dict(m.state_dict())
    fx = _leaf(x.detach(), torch.float32)
    out = attention_block_t(mg, fx, a.cuda())
    rt = _rt()
    assert rel(rt.to_nchw(rt.Feat(out.t.detach(), dim)).cpu(), want) < 2e-4
    out.t.backward(rt.to_nhwc(gy.cuda(), torch.float32).t)
    assert rel(_nchw_grad(fx), x.grad) < 5e-4
    pg = dict(mg.named_parameters())
    for k, p in pg.items():
        r = sd["blk." + k].grad
        if r is None or r.abs().max() == 0:
            assert p.grad is None or p.grad.abs().max() < 1e-6, k
            continue
        assert nrel(p.grad, r) < 1e-3, k


def _attn_core_bwd(dt, qkv, dense, dout, alpha, C, ws, shift, nblk, amask=None):
    from rgbac import _lib
    B, H, W, _ = qkv.shape
    heads = dense.shape[0]
    q = qkv.to(dt).contiguous()
    go = dout.to(dt).contiguous()
    dq = torch.full_like(q, float("nan"))         # every q/k/v channel must be written
    part = torch.full((nblk * heads * ws ** 4,), float("nan"), device=q.device)
    _lib.call("rgbac_winattn_core_bwd_ex", _lib.dtype_code(dt), B, H, W, C, heads, ws, shift,
              0 if alpha is None else 1, (C // heads) ** -0.5, q.data_ptr(), 3 * C,
              _lib.ptr(alpha), dense.data_ptr(), go.data_ptr(), C, dq.data_ptr(), 3 * C, nblk,
              part.data_ptr(), _lib.ptr(amask), 0 if amask is None else amask.shape[0],
              _lib.stream_ptr(q.device))
    torch.cuda.synchronize()
    return dq.float(), part.view(nblk, heads, ws * ws, ws * ws).sum(0)


@pytest.mark.parametrize("ws,C,shift,kind,nblk", [
    (8, 192, 0, "ones", 64), (8, 192, 4, "rand", 5), (8, 192, 4, "half", 64),
    (4, 80, 2, "half", 64), (4, 80, 0, "ones", 3), (4, 80, 2, "rand", 64),
    (8, 96, 4, "half", 64), (4, 64, 2, "rand", 64)])
def test_winattn_core_bwd_bf16_vs_f32(ws, C, shift, kind, nblk):
    """bf16 attention-core backward (MFMA for head dims 24 / 10: P and dS enter dQ/dK/dV
    rounded to bf16; VALU otherwise) against the f32 one on the same bf16-valued inputs,
    with fewer blocks than window groups (grid-stride) for nblk < 64; the dense-bias
    partials of every block and every q/k/v gradient channel are written (NaN-filled
    before the call: the autograd Function allocates dqkv uninitialised)."""
    g = _gen(ws * C + shift + len(kind))
    B, H, W, heads = 2, 16, 24, 8
    N = ws * ws
    qkv = torch.randn((B, H, W, 3 * C), generator=g).bfloat16().float().cuda()
    dout = torch.randn((B, H, W, C), generator=g).bfloat16().float().cuda()
    dense = (torch.randn((heads, N, N), generator=g) * 0.5).cuda()
    al = None if kind == "ones" else _alpha(kind, B, H, W, g).cuda().contiguous()
    groups = -(-(B * (H // ws) * (W // ws)) // (64 // N))
    nblk = min(nblk, groups)
    d32, p32 = _attn_core_bwd(torch.float32, qkv, dense, dout, al, C, ws, shift, nblk)
    d16, p16 = _attn_core_bwd(torch.bfloat16, qkv, dense, dout, al, C, ws, shift, nblk)
    assert torch.isfinite(p32).all() and torch.isfinite(p16).all()
    assert torch.isfinite(d32).all() and torch.isfinite(d16).all()
    for k in range(3):
        sl = slice(k * C, (k + 1) * C)
        assert nrel(d16[..., sl], d32[..., sl]) < 1.5e-2, k
    assert nrel(p16, p32) < 1.5e-2


def test_winattn_core_bwd_explicit_mask():
    """The explicit (nW, N, N) additive mask of WindowAttention.forward(x, mask) in the
    attention-core backward (both kernels' shapes): f32 vs a torch autograd restatement."""
    from rgbac import _lib  # noqa: F401  (the library must load)
    g = _gen(77)
    for ws, C in ((8, 192), (4, 80)):
        B, H, W, heads = 1, 16, 16, 8
        N, nW, d = ws * ws, 3, C // heads
        qkv = torch.randn((B, H, W, 3 * C), generator=g)
        dout = torch.randn((B, H, W, C), generator=g)
        dense = torch.randn((heads, N, N), generator=g) * 0.5
        am = torch.zeros((nW, N, N))
        am[torch.rand((nW, N, N), generator=g) < 0.3] = -100.0
        groups = -(-(B * (H // ws) * (W // ws)) // (64 // N))
        dq, part = _attn_core_bwd(torch.float32, qkv.cuda(), dense.cuda(), dout.cuda(), None, C,
                                  ws, 0, min(groups, 64), am.cuda())
        # torch restatement: windows in raster order, window b adds am[b % nW]
        x = qkv.clone().requires_grad_(True)
        bias = dense.clone().requires_grad_(True)
        win = x.view(B, H // ws, ws, W // ws, ws, 3, heads, d).permute(5, 0, 1, 3, 6, 2, 4, 7)
        win = win.reshape(3, -1, heads, N, d)
        s = (win[0] * d ** -0.5) @ win[1].transpose(-1, -2) + bias
        s = s + am.repeat(win.shape[1] // nW + 1, 1, 1)[: win.shape[1]].unsqueeze(1)
        o = s.softmax(-1) @ win[2]
        o = o.view(B, H // ws, W // ws, heads, ws, ws, d).permute(0, 1, 4, 2, 5, 3, 6)
        o.reshape(B, H, W, C).backward(dout)
        assert nrel(dq.cpu(), x.grad) < 1e-5, ws
        assert nrel(part.cpu(), bias.grad) < 1e-5, ws


@pytest.mark.parametrize("ws,C", [(8, 192), (4, 80)])
@pytest.mark.parametrize("kind", ["half", "rand"])
def test_winattn_core_bwd_shift_alpha_vs_torch(ws, C, kind):
    """The MFMA attention-core backward with the Swin shift (region mask of -100,
    masked_win_attention.py:194-216) AND alpha window dropping (windows judged on the rolled
    alpha, dropped windows contribute 0: :178-190,235-236), f32, against a torch autograd
    restatement built from the oracle's window helpers -- so a shared region-id or
    mask-indexing bug of the kernel pair cannot pass."""
    g = _gen(91 + ws + len(kind))
    B, H, W, heads = 2, 16, 24, 8
    shift, N, d = ws // 2, ws * ws, C // heads
    qkv = torch.randn((B, H, W, 3 * C), generator=g)
    dout = torch.randn((B, H, W, C), generator=g)
    dense = torch.randn((heads, N, N), generator=g) * 0.5
    al = _alpha(kind, B, H, W, g)[:, 0].contiguous()
    groups = -(-(B * (H // ws) * (W // ws)) // (64 // N))
    dq, part = _attn_core_bwd(torch.float32, qkv.cuda(), dense.cuda(), dout.cuda(), al.cuda(),
                              C, ws, shift, min(groups, 64))
    x = qkv.clone().requires_grad_(True)
    bias = dense.clone().requires_grad_(True)
    xs = torch.roll(x, shifts=(-shift, -shift), dims=(1, 2))
    a_s = torch.roll(al, shifts=(-shift, -shift), dims=(1, 2)).unsqueeze(-1)
    win = ref.window_partition(xs, ws).reshape(-1, N, 3, heads, d).permute(2, 0, 3, 1, 4)
    keep = ref.window_partition(a_s, ws).sum(dim=(1, 2, 3)) != 0
    assert 0 < int(keep.sum()) < keep.numel()             # both kinds of window present
    reg = ref.window_partition(ref._region_ids(B, H, W, ws, shift), ws).reshape(-1, N)
    diff = reg.unsqueeze(1) - reg.unsqueeze(2)
    rmask = torch.where(diff != 0, -100.0, 0.0)
    s = (win[0] * d ** -0.5) @ win[1].transpose(-1, -2) + bias + rmask.unsqueeze(1)
    o = s.softmax(-1) @ win[2]                            # (nWin, heads, N, d)
    o = o * keep.view(-1, 1, 1, 1)
    o = o.transpose(1, 2).reshape(-1, ws, ws, C)
    y = torch.roll(ref.window_reverse(o, ws, H, W), shifts=(shift, shift), dims=(1, 2))
    y.backward(dout)
    assert nrel(dq.cpu(), x.grad) < 1e-5
    assert nrel(part.cpu(), bias.grad) < 1e-5


def test_gaussian_slice_grads():
    from rgbac import autograd as ag
    rt = _rt()
    g = _gen(31)
    B, H, W, M, cs = 2, 8, 8, 16, 8
    y = torch.randn((B, M, H, W), generator=g, requires_grad=True)
    mu = (torch.randn((B, cs, H, W), generator=g) * 0.5).requires_grad_(True)
    sc = (torch.rand((B, cs, H, W), generator=g) * 2).requires_grad_(True)   # some < 0.11
    noise = torch.rand((B, cs, H, W), generator=g) - 0.5
    a = torch.randn((B, cs, H, W), generator=g)
    ysl = y[:, cs:2 * cs]
    _, lik = ref.gc_forward(ysl, sc, mu, True, noise)
    hat = ref.ste_round(ysl - mu) + mu
    loss = ref._bits(lik) * 0.01 + (hat * a).sum()
    loss.backward()
    fy = _leaf(y.detach(), torch.float32)
    fmu, fsc = _leaf(mu.detach(), torch.float32), _leaf(sc.detach(), torch.float32)
    nz = noise.permute(0, 2, 3, 1).contiguous().cuda()
    h, bits = ag.gauss_t(fy, cs, fmu, fsc, nz)
    assert abs(bits.item() - ref._bits(lik).item()) < 1e-4 * ref._bits(lik).item()
    ga = rt.to_nhwc(a.cuda(), torch.float32)
    l2 = bits * 0.01 + (h.t * ga.t).sum()
    l2.backward()
    assert rel(_nchw_grad(fy), y.grad) < 1e-4
    assert rel(_nchw_grad(fmu), mu.grad) < 1e-4
    assert rel(_nchw_grad(fsc), sc.grad) < 1e-4


def test_entropy_bottleneck_grads():
    from rgbac import autograd as ag
    from rgbac.entropy import EntropyBottleneck
    from rgbac.train_forward import eb_params_t
    rt = _rt()
    g = _gen(41)
    C = 16
    eb = EntropyBottleneck(C)
    with torch.no_grad():
        for n, p in eb.named_parameters():
            if n.startswith("_factor"):
                p.copy_(torch.randn(p.shape, generator=g) * 0.3)
            elif n.startswith("_matrix"):
                p.add_(torch.randn(p.shape, generator=g) * 0.3)
    z = (torch.randn((2, C, 4, 4), generator=g) * 3).requires_grad_(True)
    noise = torch.rand((2, C, 4, 4), generator=g) - 0.5
    a = torch.randn((2, C, 4, 4), generator=g)
    sd = {"eb." + k: v.detach().clone().requires_grad_(v.is_floating_point())
          for k, v in eb.state_dict().items()}
    _, lik = ref.eb_forward(z, sd, "eb", True, noise)
    med = ref.eb_medians(sd, "eb")
    zh = ref.ste_round(z - med.reshape(1, C, 1, 1)) + med.reshape(1, C, 1, 1)
    loss = ref._bits(lik) * 0.01 + (zh * a).sum()
    loss.backward()
    ebg = EntropyBottleneck(C).cuda()
    ebg.load_state_dict(eb.state_dict())
    fz = _leaf(z.detach(), torch.float32)
    nz = noise.permute(0, 2, 3, 1).contiguous().cuda()
    zh_t, bits = ag.EBFn.apply(fz.t, C, eb_params_t(ebg), nz)
    assert abs(bits.item() - ref._bits(lik).item()) < 1e-4 * ref._bits(lik).item()
    ga = rt.to_nhwc(a.cuda(), torch.float32)
    (bits * 0.01 + (zh_t * ga.t).sum()).backward()
    assert rel(_nchw_grad(fz), z.grad) < 1e-4
    for n, p in ebg.named_parameters():
        r = sd["eb." + n].grad
        if n == "quantiles":
            assert p.grad is None or p.grad.abs().max() < 1e-6
            continue
        assert rel(p.grad, r) < 2e-4, n


def test_adam_clamp_matches_torch():
    from rgbac.optim import AdamClamp
    g = _gen(51)
    ps = [torch.randn(s, generator=g).cuda().requires_grad_(True) for s in ((7, 5), (13,), (3, 3, 2))]
    qs = [p.detach().clone().requires_grad_(True) for p in ps]
    opt = AdamClamp(ps, lr=1e-3, clip=0.5)
    topt = torch.optim.Adam(qs, lr=1e-3)
    for step in range(3):
        grads = [torch.randn(p.shape, generator=g).cuda() * 2 for p in ps]
        opt.zero_grad()
        topt.zero_grad()
        for p, q, gr in zip(ps, qs, grads):
            (p * gr).sum().backward()
            (q * gr).sum().backward()
            q.grad.clamp_(-0.5, 0.5)
        opt.step()
        topt.step()
    for p, q in zip(ps, qs):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-6, atol=1e-7)


def test_adam_clamp_device_step_matches_host_step():
    """rgbac_adam_clamp_dstep (step count in device memory, graph-replayable) reproduces the
    host-step entry bit for bit over several steps, and keeps the count in sync."""
    from rgbac.optim import AdamClamp
    g = _gen(52)
    ps = [torch.randn(s, generator=g).cuda().requires_grad_(True) for s in ((9, 4), (31,))]
    qs = [p.detach().clone().requires_grad_(True) for p in ps]
    oa = AdamClamp(ps, lr=1e-3, clip=0.5)
    ob = AdamClamp(qs, lr=1e-3, clip=0.5).use_device_step()
    for step in range(4):
        grads = [torch.randn(p.shape, generator=g).cuda() * 2 for p in ps]
        oa.zero_grad()
        ob.zero_grad()
        for p, q, gr in zip(ps, qs, grads):
            (p * gr).sum().backward()
            (q * gr).sum().backward()
        oa.step()
        ob.step()
    for p, q in zip(ps, qs):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-6, atol=1e-7)
    assert ob.state_dict()["step"] == 4


def test_rgb_train_step_graph_replay_matches_eager():
    """The training step captured in a HIP graph (bench.py's config-3 loop) and replayed gives
    the same parameters as the same steps run eagerly (bf16, B=2, 64x64, fixed noise)."""
    from rgbac.models.AutoEncoderRGB_Journal import AutoEncoder
    from rgbac.optim import AdamClamp
    torch.manual_seed(234)
    base = AutoEncoder().train()
    g = _gen(62)
    B, H, W = 2, 64, 64
    x = (torch.randint(0, 256, (B, 3, H, W), generator=g).float() / 255).cuda()
    a = torch.ones((B, 1, H, W)).cuda()
    me = [t.cuda() for t in ref.supply_mask(a.cpu())]
    nz = (torch.rand((B, 1, 1, 192), generator=g) - 0.5).cuda()
    ny = (torch.rand((B, 8, 8, 80), generator=g) - 0.5).cuda()
    nets, opts = [], []
    for _ in range(2):
        n = AutoEncoder().cuda().train().set_compute_dtype(torch.bfloat16)
        n.load_state_dict(base.state_dict())
        nets.append(n)
        opts.append(AdamClamp(n.parameters(), lr=1e-4, clip=5.0).use_device_step())

    def step(n, o):
        out = n(x, a, a, *me[:4], noise_z=nz, noise_y=ny)
        o.zero_grad()
        (4096.0 * out[1] + out[2]).backward()
        o.step()
        return out

    for _ in range(5):
        step(nets[0], opts[0])
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):                 # capture records without running: 2 + 3 replays
            step(nets[1], opts[1])
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    import warnings
    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter("always")
        with torch.cuda.graph(graph):
            step(nets[1], opts[1])
    # no autograd node of an earlier (eager) step may survive into the capture: an
    # AccumulateGrad bound to another stream "may break CUDA graph capture"
    bad = [str(w.message) for w in caught if "stream" in str(w.message).lower()]
    assert not bad, bad
    for _ in range(3):
        graph.replay()
    torch.cuda.synchronize()
    assert opts[1].state_dict()["step"] == 5
    # same update direction and size as the eager steps (bitwise equality is not required:
    # Adam's normalised update amplifies last-bit differences of near-zero gradients)
    p0 = torch.cat([p.detach().reshape(-1) for p in base.parameters()]).cuda()
    d0 = torch.cat([p.detach().reshape(-1) for p in nets[0].parameters()]) - p0
    d1 = torch.cat([p.detach().reshape(-1) for p in nets[1].parameters()]) - p0
    cos = (d0 @ d1 / (d0.norm() * d1.norm())).item()
    assert cos > 0.99, cos
    assert abs(d1.norm().item() / d0.norm().item() - 1) < 0.05


@pytest.mark.parametrize("dtype", [torch.float32])
def test_rgb_train_step_grads(dtype):
    """rd_loss = 4096*mse + bpp (trainRGB.py:178-186) backward: every parameter gradient
    of the HIP path against the oracle's autograd, same noise, B=2, 64x64, fp32."""
    from rgbac.models.AutoEncoderRGB_Journal import AutoEncoder
    torch.manual_seed(234)
    net = AutoEncoder().train()
    g = _gen(61)
    B, H, W = 2, 64, 64
    x = (torch.randint(0, 256, (B, 3, H, W), generator=g).float() / 255)
    a = torch.ones((B, 1, H, W))
    a[1, :, :, : W // 2] = 0
    me = ref.supply_mask(a)
    nz = torch.rand((B, 192, 1, 1), generator=g) - 0.5
    ny = torch.rand((B, 80, 8, 8), generator=g) - 0.5
    sd = {k: v.detach().clone().requires_grad_(v.is_floating_point())
          for k, v in net.state_dict().items()}
    out = ref.rgb_forward(sd, x * (a > 0), a, a, *me[:4], training=True, noise_z=nz, noise_y=ny)
    (4096 * out[1] + out[2]).backward()
    netg = AutoEncoder().cuda().train()
    netg.load_state_dict(net.state_dict())
    xg = (x * (a > 0)).cuda()
    ag_ = a.cuda()
    meg = [t.cuda() for t in me]
    o = netg(xg, ag_, ag_, *meg[:4], noise_z=nz.permute(0, 2, 3, 1).cuda(),
             noise_y=ny.permute(0, 2, 3, 1).cuda())
    assert abs(o[1].item() - out[1].item()) < 1e-3 * out[1].item()
    assert abs(o[2].item() - out[2].item()) < 1e-3 * out[2].item()
    (4096 * o[1] + o[2]).backward()
    bad, errs = [], []
    for n, p in netg.named_parameters():
        r = sd[n].grad
        if r is None or r.abs().max() == 0:
            continue
        e = nrel(p.grad, r)
        errs.append((e, n))
        if e > 1e-4:
            bad.append((n, e))
    errs.sort()
    print("rgb codec grads: median rel", errs[len(errs) // 2], "max", errs[-3:])
    assert not bad, bad[:10]


def test_weight_gather_multi_matches_single_gathers():
    """rgbac_weight_gather_multi (one launch over many packs, blocks found by binary search)
    equals one rgbac_weight_gather per pack, for bf16 and fp32 destinations, -1 pad slots and
    sizes that are not multiples of the 2048-element block."""
    from rgbac import _lib
    g = _gen(71)
    dev = torch.device("cuda")
    src = torch.randn(10000, generator=g).to(dev)
    tasks, want, got, blk0 = [], [], [], [0]
    for n, dt in ((5000, torch.bfloat16), (1, torch.float32), (2048, torch.bfloat16),
                  (7000, torch.float32), (4097, torch.bfloat16)):
        idx = torch.randint(-1, 10000, (n,), generator=g, dtype=torch.int32).to(dev)
        w = torch.empty(n, dtype=dt, device=dev)
        _lib.call("rgbac_weight_gather", _lib.dtype_code(dt), n, src.data_ptr(), idx.data_ptr(),
                  w.data_ptr(), _lib.stream_ptr(dev))
        o = torch.full((n,), 7.0, dtype=dt, device=dev)
        tasks.append([src.data_ptr(), idx.data_ptr(), o.data_ptr(), n, _lib.dtype_code(dt)])
        blk0.append(blk0[-1] + -(-n // 2048))
        want.append((w, idx))
        got.append(o)
    t = torch.tensor(tasks, dtype=torch.int64, device=dev)
    b = torch.tensor(blk0, dtype=torch.int64, device=dev)
    _lib.call("rgbac_weight_gather_multi", len(tasks), t.data_ptr(), b.data_ptr(), blk0[-1],
              _lib.stream_ptr(dev))
    torch.cuda.synchronize()
    for (w, idx), o in zip(want, got):
        assert torch.equal(w, o)


def test_direct_weight_grad_accumulation_matches_autograd():
    """Weight/bias gradients added straight into attached fp32 .grad buffers (AdamClamp's
    flat views; rgbac.autograd.DIRECT_GRAD) equal autograd's own accumulation, including
    a second backward accumulating on top of the first."""
    from rgbac import autograd as ag
    from rgbac.models.AutoEncoderRGB_Journal import AutoEncoder
    from rgbac.optim import AdamClamp
    torch.manual_seed(234)
    base = AutoEncoder().train()
    g = _gen(63)
    B, H, W = 2, 64, 64
    x = (torch.randint(0, 256, (B, 3, H, W), generator=g).float() / 255).cuda()
    a = torch.ones((B, 1, H, W)).cuda()
    me = [t.cuda() for t in ref.supply_mask(a.cpu())]
    nz = (torch.rand((B, 1, 1, 192), generator=g) - 0.5).cuda()
    ny = (torch.rand((B, 8, 8, 80), generator=g) - 0.5).cuda()
    grads = []
    for direct in (False, True):
        n = AutoEncoder().cuda().train()
        n.load_state_dict(base.state_dict())
        opt = AdamClamp(n.parameters(), lr=1e-4)
        ag.DIRECT_GRAD[0] = direct
        try:
            opt.zero_grad()
            for _ in range(2):
                out = n(x, a, a, *me[:4], noise_z=nz, noise_y=ny)
                (4096.0 * out[1] + out[2]).backward()
        finally:
            ag.DIRECT_GRAD[0] = True
        torch.cuda.synchronize()
        grads.append(opt.flat_grad.clone())
    assert rel(grads[1], grads[0]) < 1e-5


def test_fpatch_tile_never_reaches_a_training_pack():
    """A fragment-streamed tile (42..47, 50) cached or forced for a conv shape is valid for a
    forward PackedConv only: a training pack (TPack, re-gathered in the plain layout every
    step) of the same shape must fall back to a plain-layout tile and give the same output
    (a stale fragment-major copy would otherwise be used from step 2 on)."""
    from rgbac import runtime as rt
    from rgbac.autograd import TPack
    g = _gen(81)
    dev = torch.device("cuda")
    w = torch.randn((128, 128, 3, 3), generator=g).to(dev) * 0.05
    b = torch.randn(128, generator=g).to(dev)
    x = rt.to_nhwc(torch.randn((2, 128, 32, 32), generator=g).to(dev), torch.bfloat16)
    pk = rt.PackedConv(w, b, rt.CONV, [(128, 128)], torch.bfloat16)
    tp = TPack(pk, torch.zeros(pk.w.shape, dtype=torch.long, device=dev), torch.bfloat16)
    tp.w.copy_(pk.w)
    tp.bias.copy_(pk.bias)
    want = rt.launch([rt.prepare(pk, [x.src()])], force=(1, 1))[0]
    got = rt.launch([rt.prepare(tp, [x.src()])], force=(44, 1))[0]
    assert rt.LAST_CHOICE[0][0] not in rt.FRAG_TILES
    assert getattr(tp, "frag", None) is None
    torch.cuda.synchronize()
    assert torch.equal(got.t, want.t) or (got.t.float() - want.t.float()).abs().max() < 2e-2
    # the forward pack itself does take the fragment tile
    rt.launch([rt.prepare(pk, [x.src()])], force=(44, 1))
    assert rt.LAST_CHOICE[0][0] == 44


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_channel_copy_multi(dtype):
    """rgbac_channel_copy_multi (CatFn forward / backward in one launch) == torch channel
    slicing: vector (16-byte aligned) and scalar tasks, 1 and 17 tasks (two launches)."""
    from rgbac import autograd as ag
    from rgbac.runtime import Feat
    g = _gen(5)
    B, H, W = 2, 16, 12
    for Cs in ([8, 16, 24], [3, 5, 8, 13], [32], [8] * 17):
        parts = [Feat(torch.randn((B, H, W, c + (c % 8 and 8 - c % 8)), generator=g).to(dtype).cuda(), c)
                 for c in Cs]
        cat = ag.cat_t(parts)
        want = torch.cat([p.t[..., : p.C] for p in parts], -1)
        assert torch.equal(cat.t[..., : cat.C], want)
        gy = torch.randn(cat.t.shape, generator=g).to(dtype).cuda()
        leaves = [p.t.requires_grad_(True) for p in parts]
        out = ag.CatFn.apply((Cs, None, (None,) * len(Cs)), *leaves)
        out.backward(gy)
        off = 0
        for p, c in zip(leaves, Cs):
            assert torch.equal(p.grad[..., :c], gy[..., off:off + c])
            assert not p.grad[..., c:].any()
            off += c
    # accumulate mode (rgbac_channel_copy_multi_ex: a concatenation's backward split adding
    # into gradient sinks): dst += src, one rounding to the element type, copies beside it
    dst = [Feat(torch.randn((B, H, W, c), generator=g).to(dtype).cuda(), c) for c in (16, 8, 24)]
    src = Feat(torch.randn((B, H, W, 48), generator=g).to(dtype).cuda(), 48)
    want = [d.t.float() + src.t[..., o:o + d.C].float() for d, o in zip(dst, (0, 16, 24))]
    want[1] = src.t[..., 16:24].float()
    ag._copy_multi([(d, 0, src, o, d.C) for d, o in zip(dst, (0, 16, 24))], B * H * W,
                   [True, False, True])
    torch.cuda.synchronize()
    for d, w in zip(dst, want):
        assert torch.equal(d.t, w.to(dtype))


def test_reference_loop_torch_adam_clip_matches_adam_clamp():
    """The reference's own, unchanged optimizer loop (trainRGB.py:187-198: optimizer.zero_grad();
    rd_loss.backward(); clip_gradient(optimizer, 5) -- param.grad.data.clamp_ per element;
    torch.optim.Adam(lr 1e-4).step()) over the HIP codec, against rgbac.optim.AdamClamp (the
    fused drop-in of INTEGRATION.md §2), 2 steps, fp32, fixed noise: the clamped gradients are
    bit-identical in both steps (the optimizer does not touch the backward: the training packs
    are re-gathered from the parameters every step, torch.optim.Adam's in-place updates
    included) and the parameters agree to fp32 rounding of the Adam arithmetic."""
    from rgbac.models.AutoEncoderRGB_Journal import AutoEncoder
    from rgbac.optim import AdamClamp
    torch.manual_seed(234)
    base = AutoEncoder().train()
    g = _gen(64)
    B, H, W = 2, 64, 64
    x = (torch.randint(0, 256, (B, 3, H, W), generator=g).float() / 255).cuda()
    a = torch.ones((B, 1, H, W)).cuda()
    a[1, :, :, : W // 2] = 0
    x = torch.where(a > 0, x, a)
    me = [t.cuda() for t in ref.supply_mask(a.cpu())]
    nz = (torch.rand((B, 1, 1, 192), generator=g) - 0.5).cuda()
    ny = (torch.rand((B, 8, 8, 80), generator=g) - 0.5).cuda()

    def clip_gradient(optimizer, grad_clip):                 # trainRGB.py:190-194
        for group in optimizer.param_groups:
            for param in group["params"]:
                if param.grad is not None:
                    param.grad.data.clamp_(-grad_clip, grad_clip)

    nets = []
    for _ in range(2):
        n = AutoEncoder().cuda().train()
        n.load_state_dict(base.state_dict())
        nets.append(n)
    opt_t = torch.optim.Adam(nets[0].parameters(), lr=1e-4)
    opt_c = AdamClamp(nets[1].parameters(), lr=1e-4, clip=5.0)
    grads_t, grads_c = [], []
    for _ in range(2):
        out = nets[0](x, a, a, *me[:4], noise_z=nz, noise_y=ny)
        rd_loss = 4096.0 * out[1] + out[2]
        opt_t.zero_grad()
        rd_loss.backward()
        clip_gradient(opt_t, 5)
        grads_t.append(torch.cat([p.grad.reshape(-1) if p.grad is not None else
                                  torch.zeros(p.numel(), device=p.device)
                                  for p in nets[0].parameters()]).clone())
        opt_t.step()
        out = nets[1](x, a, a, *me[:4], noise_z=nz, noise_y=ny)
        opt_c.zero_grad()
        (4096.0 * out[1] + out[2]).backward()
        opt_c.step()                                         # clamps flat_grad in place
        grads_c.append(opt_c.flat_grad.clone())
    torch.cuda.synchronize()
    for s in range(2):
        assert torch.equal(grads_t[s], grads_c[s]), (s, rel(grads_t[s], grads_c[s]))
    pt = torch.cat([p.detach().reshape(-1) for p in nets[0].parameters()])
    pc = torch.cat([p.detach().reshape(-1) for p in nets[1].parameters()])
    p0 = torch.cat([p.detach().reshape(-1) for p in base.parameters()]).cuda()
    step = (pt - p0).abs().max().item()
    err = (pt - pc).abs().max().item()
    print(f"torch.optim.Adam vs AdamClamp after 2 steps: max |dp| {err:.3e}, max step {step:.3e}")
    assert step > 1e-5                                       # the parameters did move
    assert err <= 1e-3 * step, (err, step)


@pytest.mark.parametrize("cin,cout,k,stride,hw,nsrc", [
    (224, 128, 3, 1, 16, 2),      # slice-stack conv, two sources: the 128 x 256 tile
    (96, 192, 3, 1, 16, 1),       # n_pad 192: a half-filled second N tile
    (192, 192, 5, 2, 32, 1),      # Analysis 5x5/s2 (stride-2 S pieces)
    (120, 224, 3, 1, 8, 3),       # three sources, ragged K tile (k_pad 1088)
    (96, 96, 3, 1, 16, 1),        # 96 output channels: n_pad 128, partly empty N tile
])
def test_wgrad_wide_tiles_vs_torch(cin, cout, k, stride, hw, nsrc):
    """rgbac.autograd.wgrad on the shapes the 512-thread 128 x 256 weight-gradient tile takes
    (bf16, n_pad >= 128, k_pad >= 512; csrc/train.hip wgrad_ring_kernel<4, 4, 3, 2, 4>) and
    their bias sums, against torch.nn.grad.conv2d_weight in fp32 on the same bf16-valued
    operands (only the fp32 summation order differs: 1e-4 norm-wise)."""
    from rgbac import autograd as ag
    rt = _rt()
    g = _gen(cin + cout + k + hw + nsrc)
    B = 4
    ho = hw // stride
    x = torch.randn((B, cin, hw, hw), generator=g).bfloat16().float()
    gy = torch.randn((B, cout, ho, ho), generator=g).bfloat16().float()
    dev = torch.device("cuda")
    if nsrc == 1:
        cuts = [(0, cin)]
    elif nsrc == 2:
        cuts = [(0, 80), (80, cin)]
    else:
        cuts = [(0, 80), (80, 112), (112, cin)]
    S = [rt.to_nhwc(x[:, a:b].to(dev), torch.bfloat16) for a, b in cuts]
    G = rt.to_nhwc(gy.to(dev), torch.bfloat16)
    n_pad = rt.round_up(G.ldc, 64)
    cin_pad = sum(f.ldc for f in S)
    k_pad = rt.round_up(k * k * cin_pad, 64)
    tiles, target = ag.wgrad_tile(torch.bfloat16, n_pad, k_pad, False)
    assert target == 256, "the shape must take the wide tile"
    # slab slot (n, tap, channel of the concatenated padded sources) -> dense (n, c, ky, kx)
    fmap = torch.full((n_pad, k_pad), -1, dtype=torch.int32)
    pos, off = [], 0
    for f, (a, b) in zip(S, cuts):
        pos.extend(range(off, off + (b - a)))
        off += f.ldc
    for n in range(cout):
        for tap in range(k * k):
            for c, pc in enumerate(pos):
                fmap[n, tap * cin_pad + pc] = ((n * cin + c) * k + tap // k) * k + tap % k
    numel = cout * cin * k * k
    dw, db = ag.wgrad(G, S, k, stride, k // 2, False, k_pad, fmap.to(dev), numel, nbias=cout)
    torch.cuda.synchronize()
    want = torch.nn.grad.conv2d_weight(x, (cout, cin, k, k), gy, stride=stride, padding=k // 2)
    assert nrel(dw.view(cout, cin, k, k), want) < 1e-4
    assert nrel(db, gy.sum(dim=(0, 2, 3))) < 1e-4


@pytest.mark.parametrize("cin,cout,h,w,B", [
    (64, 192, 8, 32, 2),      # Analysis x2 / x3 shape class: 3 output blocks, 2 source blocks
    (32, 96, 4, 64, 3),       # ragged output block (96 = 64 + 32), one patch row per image
    (96, 64, 12, 32, 1),      # three source blocks, three patch rows
])
def test_wgrad_s2_vs_torch(cin, cout, h, w, B):
    """The polyphase weight-gradient kernel of the 5x5 stride-2 convs (csrc/train.hip
    wgrad_halo_kernel<2>: 4 stride phases of the source staged as halos, tap (ky, kx) = phase
    (ky & 1, kx & 1) at shift (ky >> 1, kx >> 1)) and its bias sums against
    torch.nn.grad.conv2d_weight in fp32 on the same bf16-valued operands, borders included
    (1e-4 norm-wise)."""
    from rgbac import autograd as ag
    rt = _rt()
    g = _gen(cin + cout + h + w + 5)
    x = torch.randn((B, cin, 2 * h, 2 * w), generator=g).bfloat16().float()
    gy = torch.randn((B, cout, h, w), generator=g).bfloat16().float()
    dev = torch.device("cuda")
    S = [rt.to_nhwc(x.to(dev), torch.bfloat16)]
    G = rt.to_nhwc(gy.to(dev), torch.bfloat16)
    assert ag.wgrad_halo_ok(torch.bfloat16, G.ldc, S, 5, 2, 2, False, h, w) == 2
    n_pad = rt.round_up(G.ldc, 64)
    cin_pad = S[0].ldc
    k_pad = rt.round_up(25 * cin_pad, 64)
    n_i = torch.arange(cout).view(-1, 1, 1)
    tap = torch.arange(25).view(1, -1, 1)
    c_i = torch.arange(cin).view(1, 1, -1)
    fmap = torch.full((n_pad, k_pad), -1, dtype=torch.int32)
    fmap[:cout].view(-1)[(n_i * k_pad + tap * cin_pad + c_i).reshape(-1)] = \
        (((n_i * cin + c_i) * 5 + tap // 5) * 5 + tap % 5).reshape(-1).int()
    numel = cout * cin * 25
    dw, db = ag.wgrad(G, S, 5, 2, 2, False, k_pad, fmap.to(dev), numel, nbias=cout)
    torch.cuda.synchronize()
    want = torch.nn.grad.conv2d_weight(x, (cout, cin, 5, 5), gy, stride=2, padding=2)
    assert nrel(dw.view(cout, cin, 5, 5), want) < 1e-4
    assert nrel(db, gy.sum(dim=(0, 2, 3))) < 1e-4


@pytest.mark.parametrize("cuts,cout,h,w,B", [
    ((96, 128), 128, 32, 32, 2),     # slice-stack conv over two concatenated sources (224 -> 128)
    ((40,), 40, 32, 32, 2),          # 40 -> 40: partial source block, partial output block
    ((80, 32, 8), 224, 8, 64, 1),    # three sources (a block straddles them), 4 output blocks
    ((96,), 96, 4, 32, 3),           # one patch per image, n blocks 64 + 32
])
def test_wgrad_halo_s1_vs_torch(cuts, cout, h, w, B):
    """The stride-1 halo weight-gradient kernel (csrc/train.hip wgrad_halo_kernel<1>: the
    3x3 convs with more than 32 outputs; taps as shifted halo rows, up to three concatenated
    sources, ragged channel blocks) and its bias sums against torch.nn.grad.conv2d_weight in
    fp32 on the same bf16-valued operands (1e-4 norm-wise)."""
    from rgbac import autograd as ag
    rt = _rt()
    cin = sum(cuts)
    g = _gen(cin + cout + h + w + 7)
    x = torch.randn((B, cin, h, w), generator=g).bfloat16().float()
    gy = torch.randn((B, cout, h, w), generator=g).bfloat16().float()
    dev = torch.device("cuda")
    S, off = [], 0
    for cc in cuts:
        S.append(rt.to_nhwc(x[:, off:off + cc].to(dev), torch.bfloat16))
        off += cc
    G = rt.to_nhwc(gy.to(dev), torch.bfloat16)
    assert ag.wgrad_halo_ok(torch.bfloat16, G.ldc, S, 3, 1, 1, False, h, w) == 1
    n_pad = rt.round_up(G.ldc, 64)
    cin_pad = sum(f.ldc for f in S)
    k_pad = rt.round_up(9 * cin_pad, 64)
    pos, o = [], 0
    for f, cc in zip(S, cuts):
        pos.extend(range(o, o + cc))
        o += f.ldc
    fmap = torch.full((n_pad, k_pad), -1, dtype=torch.int32)
    for n in range(cout):
        for tap in range(9):
            for c, pc in enumerate(pos):
                fmap[n, tap * cin_pad + pc] = ((n * cin + c) * 3 + tap // 3) * 3 + tap % 3
    numel = cout * cin * 9
    dw, db = ag.wgrad(G, S, 3, 1, 1, False, k_pad, fmap.to(dev), numel, nbias=cout)
    torch.cuda.synchronize()
    want = torch.nn.grad.conv2d_weight(x, (cout, cin, 3, 3), gy, stride=1, padding=1)
    assert nrel(dw.view(cout, cin, 3, 3), want) < 1e-4
    assert nrel(db, gy.sum(dim=(0, 2, 3))) < 1e-4


@pytest.mark.parametrize("cin,cout,h,w,B", [
    (32, 32, 32, 64, 2),      # the DSE 32 -> 32 conv shape (two 16-channel n tiles)
    (128, 8, 32, 32, 3),      # slice-stack tail 128 -> 8: one n tile, 4 channel blocks
    (64, 16, 16, 32, 2),      # 16 outputs, patch-high grid (2 patches per image)
    (32, 24, 8, 96, 1),       # ragged n tile (24), one patch row, three patches wide
])
def test_wgrad_patch_vs_torch(cin, cout, h, w, B):
    """The patch weight-gradient kernel (csrc/train.hip wgrad_patch_kernel: 8 x 32 output
    patches with their 10 x 34 source halo staged once, taps as shifted halo rows) and its bias
    sums against torch.nn.grad.conv2d_weight in fp32 on the same bf16-valued operands,
    including the zero-padded image borders of every patch (1e-4 norm-wise)."""
    from rgbac import autograd as ag
    rt = _rt()
    g = _gen(cin + cout + h + w)
    x = torch.randn((B, cin, h, w), generator=g).bfloat16().float()
    gy = torch.randn((B, cout, h, w), generator=g).bfloat16().float()
    dev = torch.device("cuda")
    S = [rt.to_nhwc(x.to(dev), torch.bfloat16)]
    G = rt.to_nhwc(gy.to(dev), torch.bfloat16)
    assert ag.wgrad_patch_ok(torch.bfloat16, G.ldc, S, 3, 1, 1, False, h, w)
    n_pad = rt.round_up(G.ldc, 64)
    cin_pad = S[0].ldc
    k_pad = rt.round_up(9 * cin_pad, 64)
    fmap = torch.full((n_pad, k_pad), -1, dtype=torch.int32)
    for n in range(cout):
        for tap in range(9):
            for c in range(cin):
                fmap[n, tap * cin_pad + c] = ((n * cin + c) * 3 + tap // 3) * 3 + tap % 3
    numel = cout * cin * 9
    dw, db = ag.wgrad(G, S, 3, 1, 1, False, k_pad, fmap.to(dev), numel, nbias=cout)
    torch.cuda.synchronize()
    want = torch.nn.grad.conv2d_weight(x, (cout, cin, 3, 3), gy, stride=1, padding=1)
    assert nrel(dw.view(cout, cin, 3, 3), want) < 1e-4
    assert nrel(db, gy.sum(dim=(0, 2, 3))) < 1e-4


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("act,slope", [("gelu", 0.0), ("relu", 0.0), ("lrelu", 0.2)])
@pytest.mark.parametrize("defer", [True, False])
def test_deferred_act_chain_and_shared_sink(act, slope, defer, dtype):
    """Training graph pieces the model relies on, against torch fp32 autograd:
    * a two-conv chain whose first activation is deferred (its backward folded into the
      second conv's input-gradient epilogue, ACT_DGELU / ACT_DLRELU; LeakyReLU with a nonzero
      slope) or not (RGBAC_DEFER_ACT=0 path);
    * a multiply-consumed activation y (gradient sink): one conv reads y TWICE as its two
      sources (built first, so its backward runs after the other consumer's deposit: the
      in-place accumulation path, only one group of the launch may take it) and another conv
      reads it once."""
    rt = _rt()
    from rgbac import autograd as ag
    g = _gen(zlib.crc32(f"chain/{act}/{defer}".encode()) % 100000)
    rnd = (lambda t: t.to(torch.bfloat16).float()) if dtype == torch.bfloat16 else (lambda t: t)
    m1, m2 = nn.Conv2d(16, 24, 3, padding=1), nn.Conv2d(24, 16, 3, padding=1)
    m3, m4 = nn.Conv2d(48, 8, 3, padding=1), nn.Conv2d(24, 8, 1)
    for m in (m1, m2, m3, m4):
        with torch.no_grad():
            for p in m.parameters():
                p.copy_(rnd(torch.randn(p.shape, generator=g) * 0.2))
    B, H, W = 2, 8, 12
    x = rnd(torch.randn((B, 16, H, W), generator=g)).requires_grad_(True)
    f = {"gelu": F.gelu, "relu": F.relu, "lrelu": lambda t: F.leaky_relu(t, slope)}[act]
    # torch reference
    h = f(m1(x))
    c = m2(h)                                   # chain: act(m1 x) -> m2
    y = F.gelu(m1(x))                           # shared activation (not deferred)
    z2 = m3(torch.cat([y, y], 1))
    z1 = m4(y)
    gs = [torch.randn(t.shape, generator=g) for t in (c, z2, z1)]
    (c * gs[0]).sum().backward(retain_graph=True)
    ((z2 * gs[1]).sum() + (z1 * gs[2]).sum()).backward()
    want_x = x.grad.clone()
    want_p = {f"m{i + 1}.{k}": p.grad.clone() for i, m in enumerate((m1, m2, m3, m4))
              for k, p in m.named_parameters()}

    ms = [m.cuda() for m in (nn.Conv2d(16, 24, 3, padding=1), nn.Conv2d(24, 16, 3, padding=1),
                             nn.Conv2d(48, 8, 3, padding=1), nn.Conv2d(24, 8, 1))]
    for mg, m in zip(ms, (m1, m2, m3, m4)):
        mg.load_state_dict(m.state_dict())
    prev = ag.DEFER_ACT
    ag.DEFER_ACT = defer
    try:
        fx = _leaf(x.detach(), dtype)
        hf = ag.conv_t(ms[0], [fx], act=act, act_param=slope, defer=True)
        cf = ag.conv_t(ms[1], [hf])
        yf = ag.conv_t(ms[0], [fx], act="gelu")   # a ConvFn output: it carries a sink
        z2f = ag.conv_t(ms[2], [yf, yf])        # built first: backward after z1's deposit
        z1f = ag.conv_t(ms[3], [yf])
        loss = sum((t.t * rt.to_nhwc(gg.cuda(), dtype).t).float().sum()
                   for t, gg in ((cf, gs[0]), (z2f, gs[1]), (z1f, gs[2])))
        loss.backward()
    finally:
        ag.DEFER_ACT = prev
    tol, err = (1e-4, rel) if dtype == torch.float32 else (3e-2, nrel)
    assert err(_nchw_grad(fx), want_x) < tol
    pg = {f"m{i + 1}.{k}": p.grad for i, m in enumerate(ms) for k, p in m.named_parameters()}
    for k, w in want_p.items():
        assert err(pg[k], w) < tol, k


def test_reduce_batch_matches_immediate_reductions():
    """RGBAC_REDUCE_BATCH (weight-gradient slab reductions queued and issued eight per launch,
    flushed at the end of backward): the AdamClamp flat gradient equals the one-launch-per-
    reduction path bit for bit (same fixed summation order), bf16 B=2 64^2 training step.
    Outside a backward pass the reduction goes out immediately (no engine callback)."""
    from rgbac import autograd as ag
    from rgbac.models.AutoEncoderRGB_Journal import AutoEncoder
    from rgbac.optim import AdamClamp
    g = _gen(71)
    B, H, W = 2, 64, 64
    x = (torch.randint(0, 256, (B, 3, H, W), generator=g).float() / 255).cuda()
    a = torch.ones((B, 1, H, W)).cuda()
    me = [t.cuda() for t in ref.supply_mask(a.cpu())]
    nz = (torch.rand((B, 1, 1, 192), generator=g) - 0.5).cuda()
    ny = (torch.rand((B, 8, 8, 80), generator=g) - 0.5).cuda()
    torch.manual_seed(234)
    net = AutoEncoder().cuda().train().set_compute_dtype(torch.bfloat16)
    opt = AdamClamp(net.parameters(), lr=1e-4, clip=5.0)
    grads = {}
    prev = ag.REDUCE_BATCH
    try:
        for mode in (False, True, False):
            ag.REDUCE_BATCH = mode
            opt.zero_grad()
            o = net(x, a, a, *me[:4], noise_z=nz, noise_y=ny)
            (4096 * o[1] + o[2]).backward()
            torch.cuda.synchronize()
            assert not ag._PENDING, "queued reductions left after backward"
            grads.setdefault(mode, []).append(opt.flat_grad.clone())
    finally:
        ag.REDUCE_BATCH = prev
    assert torch.equal(grads[False][0], grads[False][1])      # the step is deterministic
    assert torch.equal(grads[True][0], grads[False][0])


@pytest.mark.parametrize("chunks", [True, False])
def test_prefetch_frag_packs_equal_element_gather(chunks, monkeypatch):
    """prefetch_packs -- the strided-chunk repack (one launch writing every bf16 plain pack and
    its fragment-major copy, rgbac_weight_repack_multi) or, with RGBAC_REPACK_CHUNKS=0, the
    element gather + 16-byte chunk copy pair -- gives every training pack (plain and
    fragment-major) the same bits as a direct element gather through its own index map
    (TPack.idx / TPack.fidx), after a parameter update too."""
    from rgbac import _lib
    from rgbac import autograd as ag
    from rgbac.models.AutoEncoderRGB_Journal import AutoEncoder
    monkeypatch.setattr(ag, "REPACK_CHUNKS", chunks)
    monkeypatch.setattr(ag, "_TASKS", {})
    g = _gen(72)
    B, H, W = 2, 64, 64
    x = (torch.randint(0, 256, (B, 3, H, W), generator=g).float() / 255).cuda()
    a = torch.ones((B, 1, H, W)).cuda()
    me = [t.cuda() for t in ref.supply_mask(a.cpu())]
    torch.manual_seed(234)
    net = AutoEncoder().cuda().train().set_compute_dtype(torch.bfloat16)
    for step in range(3):
        o = net(x, a, a, *me[:4])
        (4096 * o[1] + o[2]).backward()
        with torch.no_grad():
            for p in net.parameters():
                p.add_(torch.randn_like(p) * 1e-3)     # parameters move between steps
    # scribble over every pack first: the checked bits must come from this prefetch
    # (the packs prefetch_packs owns: those of the model's own parameters -- GDN's
    # reparametrised weights are re-gathered by their layer in the forward)
    pset = {p.data_ptr() for p in net.parameters()}
    packs = [tp for m in net.modules() for tc in m.__dict__.get("_rgbac_train", {}).values()
             for tp in list(tc._fw.values()) + list(tc._bw.values())
             if tp.src is not None and tp.src[0] in pset and (tp.src[1] is None or tp.src[1] in pset)]
    for tp in packs:
        tp.w.fill_(7.0)
        if tp.frag is not None:
            tp.frag.view(-1).view(torch.int16).copy_(
                torch.where(tp.fidx.view(-1) >= 0, 7, 0).to(torch.int16))
    ag.prefetch_packs(net)
    torch.cuda.synchronize()
    n = nf = nc = 0
    for tp in packs:
        nc += int(tp._chunks not in (False, None))
        want = torch.empty_like(tp.w)
        _lib.call("rgbac_weight_gather", _lib.dtype_code(want.dtype), want.numel(),
                  tp.src[0], tp.idx.data_ptr(), want.data_ptr(), _lib.stream_ptr())
        torch.cuda.synchronize()
        assert torch.equal(want.view(torch.int16), tp.w.view(torch.int16))
        n += 1
        if tp.frag is None:
            continue
        want = torch.empty_like(tp.frag)
        _lib.call("rgbac_weight_gather", _lib.dtype_code(want.dtype), want.numel(),
                  tp.src[0], tp.fidx.data_ptr(), want.data_ptr(), _lib.stream_ptr())
        torch.cuda.synchronize()
        assert torch.equal(want.view(torch.int16), tp.frag.view(torch.int16))
        nf += 1
    assert n > 40 and nf > 10
    assert (nc == n) if chunks else (nc == 0)


def test_gdn_reparam_fn_bit_identical_to_torch_lowerbound():
    """rgbac.autograd.GdnReparamFn (one HIP launch each way) against the reference's torch
    graph LowerBound(p, bound) ** 2 - pedestal (layers/GDN.py:9-23, 71-78): forward values and
    parameter gradients bit-identical, with parameters below their bounds and gradients of
    both signs (LowerBound's pass-through rule), stored and added into an attached .grad."""
    from rgbac.autograd import GdnReparamFn
    from rgbac.layers.GDN import GDN, LowerBound
    torch.manual_seed(5)
    g = GDN(96).cuda()
    with torch.no_grad():
        g.beta.copy_(torch.rand(96) * 2e-3)                    # some below beta_bound (~1e-3)
        g.gamma.copy_(torch.randn(96, 96).abs() * 1e-3 - 2e-4)  # some below gamma_bound
    db_out = torch.randn(96, device="cuda")
    dg_out = torch.randn(96, 96, device="cuda")

    def torch_path(beta, gamma):
        b = LowerBound.apply(beta, g.beta_bound) ** 2 - g.pedestal
        gm = LowerBound.apply(gamma, g.gamma_bound) ** 2 - g.pedestal
        return b, gm

    for direct in (False, True):
        res = {}
        for name, fn in (("torch", torch_path),
                         ("hip", lambda b, gm: GdnReparamFn.apply(b, gm, g.beta_bound,
                                                                  g.gamma_bound, g.pedestal))):
            beta = g.beta.detach().clone().requires_grad_(True)
            gamma = g.gamma.detach().clone().requires_grad_(True)
            if direct:
                beta.grad = torch.full_like(beta, 0.25)
                gamma.grad = torch.full_like(gamma, -0.5)
            b, gm = fn(beta, gamma)
            torch.autograd.backward([b, gm], [db_out, dg_out])
            res[name] = (b.detach(), gm.detach(), beta.grad.clone(), gamma.grad.clone())
        for t, h in zip(res["torch"], res["hip"]):
            assert torch.equal(t, h), (direct, (t - h).abs().max().item())


def test_eb_params_fn_matches_torch_chain():
    """rgbac.autograd.EbParamsFn (one HIP launch each way) against the torch chain it replaces
    (softplus / tanh / cat / pad of the EntropyBottleneck parameters, compressai filters
    (3, 3, 3, 3)): the [C][64] block bit-identical; the 15 parameter gradients within fp32
    rounding of torch's (softplus / tanh backward), stored and added into an attached .grad."""
    import torch.nn.functional as Fn
    from rgbac.autograd import EbParamsFn
    from rgbac.entropy import EntropyBottleneck
    torch.manual_seed(6)
    eb = EntropyBottleneck(192).cuda()
    with torch.no_grad():
        for p in eb.parameters():
            p.add_(torch.randn_like(p) * 0.5)
    names = ([f"_matrix{i}" for i in range(5)] + [f"_bias{i}" for i in range(5)] +
             [f"_factor{i}" for i in range(4)] + ["quantiles"])
    dout = torch.randn(192, 64, device="cuda")

    def torch_chain(ps):
        C = 192
        parts = [Fn.softplus(ps[i]).reshape(C, -1) for i in range(5)]
        parts += [ps[5 + i].reshape(C, -1) for i in range(5)]
        parts += [torch.tanh(ps[10 + i]).reshape(C, -1) for i in range(4)]
        parts.append(ps[14][:, :, 1:2].reshape(C, 1))
        return Fn.pad(torch.cat(parts, dim=1), (0, 64 - 59)).contiguous()

    for direct in (False, True):
        res = {}
        for name, fn in (("torch", torch_chain), ("hip", lambda ps: EbParamsFn.apply(192, *ps))):
            ps = [getattr(eb, n).detach().clone().requires_grad_(True) for n in names]
            if direct:
                for p in ps:
                    p.grad = torch.full_like(p, 0.125)
            out = fn(ps)
            out.backward(dout)
            res[name] = (out.detach(), [p.grad.clone() for p in ps])
        assert torch.equal(res["torch"][0], res["hip"][0])
        for gt, gh in zip(res["torch"][1], res["hip"][1]):
            assert torch.allclose(gt, gh, rtol=2e-6, atol=1e-7), (direct, (gt - gh).abs().max().item())
