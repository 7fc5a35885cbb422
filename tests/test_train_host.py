"""CPU: the training path's packing maps, checked by emulating the kernels' GEMMs.

For every layer kind the backward uses (conv s1 multi-source, conv s2 k5 / k3,
1x1 / Linear, ConvTranspose k5 s2 and k1, subpel conv, GDN's x^2 pool):
  * the gathered forward pack equals runtime.PackedConv of the weight;
  * the input-gradient pack, run through the conv GEMM emulation, equals
    torch autograd's grad_input;
  * D[n][k] = sum_m G[m][n] Col(S)[m][k] (the wgrad kernel's GEMM) scattered
    through the inverse map equals torch autograd's grad_weight (and the
    column sums its grad_bias).
No GPU: the emulation runs the same index arithmetic in plain torch.
"""
import pytest
import torch
import torch.nn.functional as F

from test_host import _emulate


def _gather(w, idx):
    flat = w.reshape(-1)
    return torch.where(idx >= 0, flat[idx.clamp(min=0).long()], torch.zeros((), dtype=w.dtype))


class _Pk:
    def __init__(self, tp_meta, w):
        pk, idx = tp_meta
        self.mode, self.ksize, self.stride = pk.mode, pk.ksize, pk.stride
        self.cin, self.cin_pad, self.cout, self.cout_pad = pk.cin, pk.cin_pad, pk.cout, pk.cout_pad
        self.k_pad = pk.k_pad
        self.w = _gather(w, idx)
        self.bias = torch.zeros(pk.cout_pad)


def _col(S, k, stride, pad, Hg, Wg):
    """(B, ntaps*Cpad, Hg*Wg) im2col in the kernel's k = tap*cin_pad + ci order."""
    sp = F.pad(S, (pad, pad, pad, pad))
    cols = [sp[:, :, ty:ty + stride * (Hg - 1) + 1:stride, tx:tx + stride * (Wg - 1) + 1:stride]
            for ty in range(k) for tx in range(k)]
    X = torch.stack(cols, 1)                                # B, taps, C, Hg, Wg
    B = X.shape[0]
    return X.reshape(B, -1, Hg * Wg)


def _pad_c(t):
    c = t.shape[1]
    return F.pad(t, (0, 0, 0, 0, 0, (-c) % 8))


def _wgrad_emulate(tc, G, S, k, stride, pad):
    """G (B, n, Hg, Wg), S (B, Cpad, Hs, Ws) already channel padded."""
    B, n, Hg, Wg = G.shape
    X = _col(S, k, stride, pad, Hg, Wg)
    D = torch.einsum("bnm,bkm->nk", G.reshape(B, n, -1).double(), X.double())
    Dp = torch.zeros((max(n, 1), tc.wg_kpad), dtype=torch.float64)
    Dp[:, :D.shape[1]] = D
    flat = Dp.reshape(-1)
    inv = tc.wg_map.long()
    assert (inv >= 0).all()
    return flat[inv].float()


CONV_CASES = [
    # name, cin segments, cout, k, stride
    ("k3s1_2src", [40, 80], 24, 3, 1),
    ("k5s2", [3], 16, 5, 2),
    ("k3s2", [24], 16, 3, 2),
    ("k1", [20], 12, 1, 1),
]


@pytest.mark.parametrize("name,segs,cout,k,s", CONV_CASES)
def test_conv_maps(name, segs, cout, k, s):
    from rgbac import autograd as ag
    g = torch.Generator().manual_seed(len(name) + cout)
    cin = sum(segs)
    conv = torch.nn.Conv2d(cin, cout, k, stride=s, padding=k // 2)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g))
    H, W = 8, 12
    xs = [torch.randn((2, c, H, W), generator=g, requires_grad=True) for c in segs]
    y = conv(torch.cat(xs, 1))
    gy = torch.randn(y.shape, generator=g)
    y.backward(gy)
    tc = ag.TrainConv("conv", tuple(conv.weight.shape), s, [(c, -(-c // 8) * 8) for c in segs],
                      torch.device("cpu"))
    # forward pack == PackedConv
    from rgbac import runtime as rt
    ref = rt.PackedConv(conv.weight, None, rt.CONV, tc.segs, torch.float32, stride=s)
    assert torch.equal(_gather(conv.weight.detach(), tc.fwd[1]), ref.w)
    # input gradients, one source at a time
    Ho, Wo = y.shape[2], y.shape[3]
    for i, x in enumerate(xs):
        pk = _Pk(tc.bwd[i], conv.weight.detach())
        got = _emulate(pk, [gy], Ho, Wo)
        assert got.shape[2:] == x.shape[2:]
        torch.testing.assert_close(got[:, :x.shape[1]], x.grad, rtol=1e-5, atol=1e-4)
    # weight gradient through the inverse map
    S = torch.cat([_pad_c(x.detach()) for x in xs], 1)
    dw = _wgrad_emulate(tc, _pad_c(gy), S, k, s, k // 2)
    torch.testing.assert_close(dw.view_as(conv.weight), conv.weight.grad, rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(gy.sum((0, 2, 3)), conv.bias.grad, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("cin,cout,k", [(16, 8, 5), (16, 3, 5), (8, 16, 1)])
def test_convtranspose_maps(cin, cout, k):
    from rgbac import autograd as ag
    from rgbac import runtime as rt
    g = torch.Generator().manual_seed(cin * cout + k)
    if k == 5:
        m = torch.nn.ConvTranspose2d(cin, cout, 5, stride=2, padding=2, output_padding=1)
    else:
        m = torch.nn.ConvTranspose2d(cin, cout, 1)
    H, W = 6, 10
    x = torch.randn((2, cin, H, W), generator=g, requires_grad=True)
    y = m(x)
    gy = torch.randn(y.shape, generator=g)
    y.backward(gy)
    tc = ag.TrainConv("convt", tuple(m.weight.shape), m.stride[0], [(cin, -(-cin // 8) * 8)],
                      torch.device("cpu"))
    if k == 5:
        ref = rt.PackedConv(m.weight, None, rt.CONVT_S2, tc.segs, torch.float32, stride=2)
    else:
        ref = rt.PackedConv(m.weight, None, rt.CONV, tc.segs, torch.float32, transposed=True)
    assert torch.equal(_gather(m.weight.detach(), tc.fwd[1]), ref.w)
    pk = _Pk(tc.bwd[0], m.weight.detach())
    got = _emulate(pk, [gy], y.shape[2], y.shape[3])
    torch.testing.assert_close(got[:, :cin], x.grad, rtol=1e-5, atol=1e-4)
    # wgrad: G = x (convT input grid), S = dY sampled k5 s2 p2 (or k1)
    dw = _wgrad_emulate(tc, _pad_c(x.detach()), _pad_c(gy), k, 2 if k == 5 else 1, k // 2)
    torch.testing.assert_close(dw.view_as(m.weight), m.weight.grad, rtol=1e-5, atol=1e-3)


def test_subpel_maps():
    """compressai subpel_conv3x3: conv3x3(C, 4C') + PixelShuffle(2); the backward works on
    the un-shuffled gradient (rgbac_pixel_shuffle dir 1)."""
    from rgbac import autograd as ag
    g = torch.Generator().manual_seed(9)
    conv = torch.nn.Conv2d(8, 16, 3, padding=1)
    x = torch.randn((2, 8, 5, 7), generator=g, requires_grad=True)
    y = F.pixel_shuffle(conv(x), 2)
    gy = torch.randn(y.shape, generator=g)
    y.backward(gy)
    tc = ag.TrainConv("subpel", tuple(conv.weight.shape), 1, [(8, 8)], torch.device("cpu"))
    gz = F.pixel_unshuffle(gy, 2)
    pk = _Pk(tc.bwd[0], conv.weight.detach())
    got = _emulate(pk, [gz], 5, 7)
    torch.testing.assert_close(got[:, :8], x.grad, rtol=1e-5, atol=1e-4)
    dw = _wgrad_emulate(tc, _pad_c(gz), _pad_c(x.detach()), 3, 1, 1)
    torch.testing.assert_close(dw.view_as(conv.weight), conv.weight.grad, rtol=1e-5, atol=1e-3)


def test_gdn_pool_maps():
    """GDN's pool conv(x^2, gamma'): d(x^2) through the transposed 1x1 pack, d gamma' =
    sum_m dnorm[m][i] x[m][j]^2 (wgrad with square_input)."""
    from rgbac import autograd as ag
    g = torch.Generator().manual_seed(10)
    C = 16
    gamma = torch.rand((C, C), generator=g, requires_grad=True)
    x = torch.randn((2, C, 4, 6), generator=g)
    x2 = (x ** 2).requires_grad_(True)
    norm = F.conv2d(x2, gamma.view(C, C, 1, 1))
    gn = torch.randn(norm.shape, generator=g)
    norm.backward(gn)
    tc = ag.TrainConv("gdn", (C, C, 1, 1), 1, [(C, C)], torch.device("cpu"))
    pk = _Pk(tc.bwd[0], gamma.detach().view(C, C, 1, 1))
    got = _emulate(pk, [gn], 4, 6)
    torch.testing.assert_close(got[:, :C], x2.grad, rtol=1e-5, atol=1e-4)
    dw = _wgrad_emulate(tc, gn, x ** 2, 1, 1, 0)
    torch.testing.assert_close(dw.view(C, C), gamma.grad, rtol=1e-5, atol=1e-3)


def test_oracle_lower_bound_gradient_rule():
    """GDN.py:16-23: the gradient passes where x >= bound OR the incoming gradient is < 0."""
    from oracle import ref_model as ref
    x = torch.tensor([0.05, 0.2, 0.05, 0.2], requires_grad=True)
    y = ref._lower_bound(x, 0.11)
    assert torch.equal(y.detach(), torch.tensor([0.11, 0.2, 0.11, 0.2]))
    y.backward(torch.tensor([1.0, 1.0, -1.0, -1.0]))
    assert torch.equal(x.grad, torch.tensor([0.0, 1.0, -1.0, -1.0]))


# (kind, wshape, stride, segs): the RGB model's pack kinds, incl. the slice stacks' multi-source
# 3x3 convs and unpadded / padded channel segments
REPACK_CASES = [
    ("conv", (24, 120, 3, 3), 1, [(80, 80), (8, 8), (8, 8), (8, 8), (8, 8), (8, 8)]),
    ("conv", (16, 3, 5, 5), 2, [(3, 8)]),
    ("conv", (16, 24, 3, 3), 2, [(24, 24)]),
    ("conv", (12, 20, 1, 1), 1, [(20, 24)]),
    ("convt", (16, 8, 5, 5), 2, [(16, 16)]),
    ("convt", (8, 16, 1, 1), 1, [(8, 8)]),
    ("subpel", (32, 8, 3, 3), 1, [(8, 8)]),
    ("gdn", (24, 24, 1, 1), 1, [(24, 24)]),
]


@pytest.mark.parametrize("kind,wshape,stride,segs", REPACK_CASES)
def test_repack_chunk_form_rebuilds_the_gathered_packs(kind, wshape, stride, segs):
    """rgbac_weight_repack_multi's chunk maps (TPack.chunk_form), emulated: every plain pack
    and fragment-major copy it writes equals the element gather + chunk copy it replaces."""
    from rgbac import autograd as ag
    tc = ag.TrainConv(kind, wshape, stride, segs, torch.device("cpu"))
    numel = tc.numel
    src = torch.randn(numel, generator=torch.Generator().manual_seed(numel))
    metas = [tc.fwd] + list(tc.bwd)
    for pk, idx in metas:
        tp = ag.TPack(pk, idx, torch.bfloat16)
        if ag._frag_eligible(tp):
            tp.enable_frag()
        cf = tp.chunk_form()
        assert cf is not None, "every pack kind of the model has the strided-chunk form"
        cmap, stride_, fmap = cf
        want = _gather(src, idx.reshape(-1)).to(torch.bfloat16)
        # the kernel's arithmetic: base | (nv - 1) << 28, element j < nv = src[base + j*stride]
        m = cmap.to(torch.int64)
        base, nv = m & 0x0FFFFFFF, ((m >> 28) & 7) + 1
        j = torch.arange(8)
        pos = base[:, None] + j[None, :] * stride_
        ok = (m[:, None] >= 0) & (j[None, :] < nv[:, None])
        got = torch.where(ok, src[pos.clamp(0, numel - 1)], torch.zeros(())).to(torch.bfloat16)
        assert torch.equal(got.reshape(-1), want)
        if tp.frag is not None:
            assert fmap is not None
            frag_want = torch.zeros(tp.frag.numel() // 8, 8, dtype=torch.bfloat16)
            sel = tp.fcmap >= 0
            frag_want[sel] = want.reshape(-1, 8)[tp.fcmap[sel].long()]
            frag_got = torch.zeros_like(frag_want)
            fs = fmap >= 0
            frag_got[fmap[fs].long()] = got[fs]
            assert torch.equal(frag_got, frag_want)
        else:
            assert fmap is None
