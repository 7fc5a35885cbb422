"""SSIM / MS-SSIM (reference: metrics/ms_ssim_torch.py:5-259) on the HIP path.

Same functions and arguments as the reference: ``ssim(X, Y, win_size=11, win_sigma=1.5,
win=None, data_range=255, size_average=True, full=False)``, ``ms_ssim(..., weights=None)`` and
the ``SSIM`` / ``MS_SSIM`` modules.  Per scale one tile launch computes the valid ssim/cs maps
and their per-image means (csrc/msssim.hip); the 2x2 average pool and the final weighted
product are kernels too, so the metric never leaves the GPU (trainRGB.py:308-311 evaluates it
on the CPU).  Inputs must be CUDA tensors; they are computed in fp32.
"""
import torch

from .. import _lib
from .. import runtime as rt

_TILE = 16


def _fspecial_gauss_1d(size, sigma):
    """:5-18 (host constant, built exactly as the reference builds it)."""
    coords = torch.arange(size).to(dtype=torch.float)
    coords -= size // 2
    g = torch.exp(-(coords ** 2) / (2 * sigma ** 2))
    g /= g.sum()
    return g.unsqueeze(0).unsqueeze(0)


def _check(X, Y, win_size):
    if len(X.shape) != 4:
        raise ValueError('Input images must 4-d tensor.')
    if not X.type() == Y.type():
        raise ValueError('Input images must have the same dtype.')
    if not X.shape == Y.shape:
        raise ValueError('Input images must have the same dimensions.')
    if not (win_size % 2 == 1):
        raise ValueError('Window size must be odd.')
    rt.check_gpu(X, Y)


def _win_1d(win, win_size, win_sigma, device):
    if win is None:
        w = _fspecial_gauss_1d(win_size, win_sigma)
    else:
        w = win[0] if win.dim() == 4 else win
    return w.reshape(-1).to(device=device, dtype=torch.float32).contiguous()


def _ssim_level(X, Y, w1d, data_range, K=(0.01, 0.03)):
    """One scale of _ssim (:36-83) with size_average=False -> (ssim[B], cs[B])."""
    B, C, H, W = X.shape
    ws = w1d.numel()
    nt = (-(-(H - ws + 1) // _TILE)) * (-(-(W - ws + 1) // _TILE))
    part = torch.empty((B * C * nt * 2,), dtype=torch.float32, device=X.device)
    s = torch.empty((B,), dtype=torch.float32, device=X.device)
    cs = torch.empty((B,), dtype=torch.float32, device=X.device)
    c1 = (K[0] * data_range) ** 2
    c2 = (K[1] * data_range) ** 2
    _lib.call("rgbac_ssim_level", B, C, H, W, ws, X.data_ptr(), Y.data_ptr(), w1d.data_ptr(),
              c1, c2, part.data_ptr(), s.data_ptr(), cs.data_ptr(), _lib.stream_ptr(X.device))
    return s, cs


def _pool(X):
    B, C, H, W = X.shape
    ph, pw = H % 2, W % 2
    out = torch.empty((B, C, (H + 2 * ph - 2) // 2 + 1, (W + 2 * pw - 2) // 2 + 1),
                      dtype=torch.float32, device=X.device)
    _lib.call("rgbac_avgpool2", B * C, H, W, X.data_ptr(), out.data_ptr(),
              _lib.stream_ptr(X.device))
    return out


def ssim(X, Y, win_size=11, win_sigma=1.5, win=None, data_range=255, size_average=True,
         full=False):
    """:86-132"""
    if win is not None:
        win_size = win.shape[-1]
    _check(X, Y, win_size)
    w1d = _win_1d(win, win_size, win_sigma, X.device)
    ssim_val, cs = _ssim_level(X.contiguous().float(), Y.contiguous().float(), w1d, data_range)
    if size_average:
        ssim_val = ssim_val.mean()
        cs = cs.mean()
    if full:
        return ssim_val, cs
    return ssim_val


def ms_ssim(X, Y, win_size=11, win_sigma=1.5, win=None, data_range=255, size_average=True,
            full=False, weights=None):
    """:135-194 (including the broadcast of ssim_val ** w[-1] into every level's factor)."""
    if win is not None:
        win_size = win.shape[-1]
    _check(X, Y, win_size)
    if weights is None:
        weights = torch.tensor([0.0448, 0.2856, 0.3001, 0.2363, 0.1333], dtype=torch.float32)
    wts = weights.to(device=X.device, dtype=torch.float32).contiguous()
    w1d = _win_1d(win, win_size, win_sigma, X.device)
    levels = wts.shape[0]
    X, Y = X.contiguous().float(), Y.contiguous().float()
    B = X.shape[0]
    mcs = torch.empty((levels, B), dtype=torch.float32, device=X.device)
    ssim_val = None
    for i in range(levels):
        ssim_val, cs = _ssim_level(X, Y, w1d, data_range)
        mcs[i].copy_(cs)
        if i + 1 < levels:     # the reference's last pool feeds nothing
            X, Y = _pool(X), _pool(Y)
    per_image = torch.empty((B,), dtype=torch.float32, device=X.device)
    mean = torch.empty((), dtype=torch.float32, device=X.device)
    _lib.call("rgbac_msssim_combine", levels, B, mcs.data_ptr(), ssim_val.data_ptr(),
              wts.data_ptr(), per_image.data_ptr(), mean.data_ptr(), _lib.stream_ptr(X.device))
    return mean if size_average else per_image


class SSIM(torch.nn.Module):
    """:197-217"""

    def __init__(self, win_size=11, win_sigma=1.5, data_range=None, size_average=True,
                 channel=3):
        super().__init__()
        self.win = _fspecial_gauss_1d(win_size, win_sigma).repeat(channel, 1, 1, 1)
        self.size_average = size_average
        self.data_range = data_range

    def forward(self, X, Y):
        return ssim(X, Y, win=self.win, data_range=self.data_range,
                    size_average=self.size_average)


class MS_SSIM(torch.nn.Module):
    """:219-259"""

    def __init__(self, win_size=11, win_sigma=1.5, data_range=None, size_average=True,
                 channel=3, weights=None):
        super().__init__()
        self.win = _fspecial_gauss_1d(win_size, win_sigma).repeat(channel, 1, 1, 1)
        self.size_average = size_average
        self.data_range = data_range
        self.weights = weights

    def forward(self, X, Y):
        return ms_ssim(X, Y, win=self.win, size_average=self.size_average,
                       data_range=self.data_range, weights=self.weights)
