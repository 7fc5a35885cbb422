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
