"""SSIM / MS-SSIM on the HIP path (rgbac.metrics.ms_ssim_torch) vs the CPU oracle restatement of
metrics/ms_ssim_torch.py.  Tolerance 1e-5 absolute on values in [0, 1] (the north-star bar for
MS-SSIM is 1e-4): the kernels differ from the oracle only in fp32 summation order."""
import pytest
import torch

from oracle import ref_metrics as rm

pytestmark = pytest.mark.gpu


def _pair(B, C, H, W, seed, noise=0.05):
    g = torch.Generator().manual_seed(seed)
    X = torch.round(torch.rand((B, C, H, W), generator=g) * 255) / 255
    X = torch.nn.functional.avg_pool2d(X, 3, 1, 1)          # some spatial structure
    Y = torch.clamp(X + noise * torch.randn((B, C, H, W), generator=g), 0, 1)
    return X, Y


@pytest.mark.parametrize("shape", [(2, 3, 256, 256), (3, 3, 200, 184), (1, 1, 161, 177)])
@pytest.mark.parametrize("size_average", [True, False])
def test_ms_ssim(device, shape, size_average):
    from rgbac.metrics.ms_ssim_torch import ms_ssim
    X, Y = _pair(*shape, seed=sum(shape))
    want = rm.ms_ssim(X, Y, data_range=1.0, size_average=size_average)
    got = ms_ssim(X.to(device), Y.to(device), data_range=1.0, size_average=size_average)
    assert got.shape == want.shape
    assert (got.cpu() - want).abs().max().item() < 1e-5


def test_ms_ssim_255_and_identity(device):
    from rgbac.metrics.ms_ssim_torch import MS_SSIM, ms_ssim
    X, Y = _pair(2, 3, 192, 192, seed=9, noise=0.2)
    X, Y = X * 255, Y * 255
    want = rm.ms_ssim(X, Y)                      # data_range default 255
    assert abs(ms_ssim(X.to(device), Y.to(device)).item() - want.item()) < 1e-5
    m = MS_SSIM(data_range=255.0, channel=3)
    assert abs(m(X.to(device), Y.to(device)).item() - want.item()) < 1e-5
    assert abs(ms_ssim(X.to(device), X.to(device)).item() - 1.0) < 1e-5


@pytest.mark.parametrize("win_size", [7, 11, 15])
def test_ssim(device, win_size):
    from rgbac.metrics.ms_ssim_torch import ssim
    X, Y = _pair(2, 3, 64, 80, seed=win_size, noise=0.1)
    want = rm.ssim(X, Y, win_size=win_size, data_range=1.0, size_average=False)
    got = ssim(X.to(device), Y.to(device), win_size=win_size, data_range=1.0,
               size_average=False)
    assert (got.cpu() - want).abs().max().item() < 1e-5


# ---- masked variant (rgbac.metrics.masked_ms_ssim_torch) vs oracle.ref_metrics.masked_*;
# same 1e-5 absolute bar: the kernels sum the kept pixels in double, the oracle in fp32.

def _alpha(B, Cm, H, W, seed):
    """An alpha-like mask: an off-centre disc of full opacity, a soft rim, a few holes."""
    g = torch.Generator().manual_seed(seed)
    yy, xx = torch.meshgrid(torch.arange(H, dtype=torch.float32),
                            torch.arange(W, dtype=torch.float32), indexing="ij")
    m = torch.empty((B, Cm, H, W))
    for b in range(B):
        cy, cx = H * (0.4 + 0.2 * b / max(B, 1)), W * 0.55
        r = torch.sqrt((yy - cy) ** 2 + (xx - cx) ** 2) / (0.45 * min(H, W))
        m[b] = torch.clamp(1.5 - r, 0, 1)
    holes = torch.rand((B, Cm, H, W), generator=g) < 0.02
    m[holes] = 0
    return m


@pytest.mark.parametrize("shape,cm", [((2, 3, 256, 256), 1), ((3, 3, 200, 184), 3),
                                      ((1, 1, 161, 177), 1)])
@pytest.mark.parametrize("size_average", [True, False])
def test_masked_ms_ssim(device, shape, cm, size_average):
    from rgbac.metrics.masked_ms_ssim_torch import ms_ssim
    X, Y = _pair(*shape, seed=sum(shape) + 1)
    M = _alpha(shape[0], cm, shape[2], shape[3], seed=shape[2])
    want = rm.masked_ms_ssim(X, Y, M, data_range=1.0, size_average=size_average)
    got = ms_ssim(X.to(device), Y.to(device), M.to(device), data_range=1.0,
                  size_average=size_average)
    assert got.shape == want.shape
    assert (got.cpu() - want).abs().max().item() < 1e-5


def test_masked_ms_ssim_modules_and_edges(device):
    from rgbac.metrics.masked_ms_ssim_torch import MS_SSIM, SSIM, ms_ssim, ssim
    X, Y = _pair(2, 3, 192, 208, seed=11, noise=0.2)
    X, Y = X * 255, Y * 255
    M = _alpha(2, 1, 192, 208, seed=3)
    Xd, Yd, Md = X.to(device), Y.to(device), M.to(device)
    want = rm.masked_ms_ssim(X, Y, M)                  # data_range default 255
    assert abs(ms_ssim(Xd, Yd, Md).item() - want.item()) < 1e-5
    assert abs(MS_SSIM(channel=3)(Xd, Yd, Md).item() - want.item()) < 1e-5
    # an all-transparent mask keeps nothing: 0 / (0 + 1e-10) -> 0 at every level -> 0
    z = torch.zeros_like(Md)
    assert ms_ssim(Xd, Yd, z).item() == 0.0 and rm.masked_ms_ssim(X, Y, M * 0).item() == 0.0
    # single-scale masked ssim (the reference's :171 call with the mask it omits)
    for ws in (7, 11, 15):
        w = rm.masked_ssim(X, Y, M, win_size=ws, size_average=False)
        g = ssim(Xd, Yd, Md, win_size=ws, size_average=False)
        assert (g.cpu() - w).abs().max().item() < 1e-5
    w = rm.masked_ssim(X, Y, M, nonnegative_ssim=True)
    assert abs(SSIM(channel=3, nonnegative_ssim=True)(Xd, Yd, Md).item() - w.item()) < 1e-5
    with pytest.raises(ValueError):
        ms_ssim(Xd, Yd, Md[:, :, :100])
