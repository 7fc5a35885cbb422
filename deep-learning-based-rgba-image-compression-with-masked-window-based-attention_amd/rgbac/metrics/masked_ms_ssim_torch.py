"""Masked SSIM / MS-SSIM (reference: metrics/masked_ms_ssim_torch.py:10-351) on the HIP path.

The reference's masked variant scores only the pixels an alpha mask keeps.  Per level
(:245-256): the mask is binarised, X and Y are multiplied by it, the VALID ssim / cs maps are
averaged per (image, channel) over the pixels where the mask, NEAREST-resized to the valid map
size, is nonzero; X, Y and the mask are then 2x2 average-pooled.  The last level's relu(ssim)
and the earlier levels' relu(cs) combine as prod(v ** w) per (image, channel) (:258-265).
Every step is a kernel of csrc/msssim.hip (rgbac_masked_apply / _masked_ssim_level /
rgbac_avgpool2 / _masked_msssim_combine); inputs must be CUDA tensors, computed in fp32.

Where the reference cannot run as written, the evident intent is built and the difference is
stated: its ``ssim()`` calls ``_ssim`` without the mask (:171) and its ``SSIM`` / ``MS_SSIM``
modules call ``ssim`` / ``ms_ssim`` without one (:300, :343) -- all TypeErrors.  Here ``ssim``
passes the mask through, and the modules take it as a third ``forward`` argument.  5-D
(video) inputs and images smaller than the window (the reference warns and skips the blur,
:49-51) raise instead.
"""
import torch

from .. import _lib
from .. import runtime as rt
from .ms_ssim_torch import _TILE, _pool

_WEIGHTS = [0.0448, 0.2856, 0.3001, 0.2363, 0.1333]


def _fspecial_gauss_1d(size, sigma):
    """:10-24 (host constant, built exactly as the reference builds it)."""
    coords = torch.arange(size, dtype=torch.float)
    coords -= size // 2
    g = torch.exp(-(coords ** 2) / (2 * sigma ** 2))
    g /= g.sum()
    return g.unsqueeze(0).unsqueeze(0)


def _prepare(X, Y, mask, win_size):
    """The reference's argument checks (:148-165 / :207-228), then fp32 contiguous planes."""
    if not X.shape == Y.shape:
        raise ValueError(f"Input images should have the same dimensions, but got {X.shape} and "
                         f"{Y.shape}.")
    for d in range(len(X.shape) - 1, 1, -1):
        X = X.squeeze(dim=d)
        Y = Y.squeeze(dim=d)
    if len(X.shape) != 4:
        raise ValueError(f"Input images should be 4-d tensors, but got {X.shape}")
    if not (win_size % 2 == 1):
        raise ValueError("Window size should be odd.")
    B, C, H, W = X.shape
    if mask.dim() != 4 or mask.shape[0] != B or mask.shape[2:] != X.shape[2:] or \
            mask.shape[1] not in (1, C):
        raise ValueError(f"mask must be (B, 1 or C, H, W) = ({B}, 1|{C}, {H}, {W}), got "
                         f"{tuple(mask.shape)}")
    rt.check_gpu(X, Y, mask)
    return X.contiguous().float(), Y.contiguous().float(), mask.contiguous().float()


def _win_1d(win, win_size, win_sigma, device):
    w = _fspecial_gauss_1d(win_size, win_sigma) if win is None else win.reshape(-1, win.shape[-1])[0]
    return w.reshape(-1).to(device=device, dtype=torch.float32).contiguous()


def _masked_level(X, Y, M, w1d, data_range, K):
    """_ssim (:56-118) with size_average=False on already-masked planes -> (ssim, cs), (B, C)."""
    B, C, H, W = X.shape
    ws = w1d.numel()
    if H < ws or W < ws:
        raise ValueError(f"image {H}x{W} smaller than the {ws}-tap window")
    nt = (-(-(H - ws + 1) // _TILE)) * (-(-(W - ws + 1) // _TILE))
    part = torch.empty((B * C * nt * 3,), dtype=torch.float32, device=X.device)
    s = torch.empty((B, C), dtype=torch.float32, device=X.device)
    cs = torch.empty((B, C), dtype=torch.float32, device=X.device)
    c1 = (K[0] * data_range) ** 2
    c2 = (K[1] * data_range) ** 2
    _lib.call("rgbac_masked_ssim_level", B, C, M.shape[1], H, W, ws, X.data_ptr(), Y.data_ptr(),
              M.data_ptr(), w1d.data_ptr(), c1, c2, part.data_ptr(), s.data_ptr(), cs.data_ptr(),
              _lib.stream_ptr(X.device))
    return s, cs


def _apply(X, Y, M):
    """:246-248 -> (X * bin(M), Y * bin(M), bin(M))."""
    B, C, H, W = X.shape
    xo, yo, mo = torch.empty_like(X), torch.empty_like(Y), torch.empty_like(M)
    _lib.call("rgbac_masked_apply", B, C, M.shape[1], H, W, X.data_ptr(), Y.data_ptr(),
              M.data_ptr(), xo.data_ptr(), yo.data_ptr(), mo.data_ptr(),
              _lib.stream_ptr(X.device))
    return xo, yo, mo


def ssim(X, Y, mask, data_range=255, size_average=True, win_size=11, win_sigma=1.5, win=None,
         K=(0.01, 0.03), nonnegative_ssim=False):
    """:121-178 (with the mask passed to _ssim, which the reference omits at :171).  Like the
    reference, X and Y are NOT multiplied by the mask here; only the averaging is masked."""
    if win is not None:
        win_size = win.shape[-1]
    X, Y, mask = _prepare(X, Y, mask, win_size)
    w1d = _win_1d(win, win_size, win_sigma, X.device)
    s, _ = _masked_level(X, Y, (mask > 0).float(), w1d, data_range, K)
    if nonnegative_ssim:
        s = torch.relu(s)
    return s.mean() if size_average else s.mean(1)


def ms_ssim(X, Y, mask, data_range=255, size_average=True, win_size=11, win_sigma=1.5, win=None,
            weights=None, K=(0.01, 0.03)):
    """:181-265"""
    if win is not None:
        win_size = win.shape[-1]
    X, Y, mask = _prepare(X, Y, mask, win_size)
    smaller_side = min(X.shape[-2:])
    assert smaller_side > (win_size - 1) * (2 ** 4), \
        "Image size should be larger than %d due to the 4 downsamplings in ms-ssim" % (
            (win_size - 1) * (2 ** 4))
    wts = torch.as_tensor(weights if weights is not None else _WEIGHTS, dtype=torch.float32)
    wts = wts.to(X.device).contiguous()
    w1d = _win_1d(win, win_size, win_sigma, X.device)
    levels = wts.shape[0]
    B, C = X.shape[:2]
    mcs = torch.empty((max(levels - 1, 1), B, C), dtype=torch.float32, device=X.device)
    s = None
    for i in range(levels):
        X, Y, mask = _apply(X, Y, mask)
        s, cs = _masked_level(X, Y, mask, w1d, data_range, K)
        if i < levels - 1:
            mcs[i].copy_(cs)
            X, Y, mask = _pool(X), _pool(Y), _pool(mask)
    per_image = torch.empty((B,), dtype=torch.float32, device=X.device)
    mean = torch.empty((), dtype=torch.float32, device=X.device)
    _lib.call("rgbac_masked_msssim_combine", levels, B, C, mcs.data_ptr(), s.data_ptr(),
              wts.data_ptr(), per_image.data_ptr(), mean.data_ptr(), _lib.stream_ptr(X.device))
    return mean if size_average else per_image


class SSIM(torch.nn.Module):
    """:268-308 (forward takes the mask the reference's forward never passes)."""

    def __init__(self, data_range=255, size_average=True, win_size=11, win_sigma=1.5, channel=3,
                 spatial_dims=2, K=(0.01, 0.03), nonnegative_ssim=False):
        super().__init__()
        self.win_size = win_size
        self.win = _fspecial_gauss_1d(win_size, win_sigma).repeat([channel, 1] + [1] * spatial_dims)
        self.size_average = size_average
        self.data_range = data_range
        self.K = K
        self.nonnegative_ssim = nonnegative_ssim

    def forward(self, X, Y, mask):
        return ssim(X, Y, mask, data_range=self.data_range, size_average=self.size_average,
                    win=self.win, K=self.K, nonnegative_ssim=self.nonnegative_ssim)


class MS_SSIM(torch.nn.Module):
    """:311-351 (forward takes the mask the reference's forward never passes)."""

    def __init__(self, data_range=255, size_average=True, win_size=11, win_sigma=1.5, channel=3,
                 spatial_dims=2, weights=None, K=(0.01, 0.03)):
        super().__init__()
        self.win_size = win_size
        self.win = _fspecial_gauss_1d(win_size, win_sigma).repeat([channel, 1] + [1] * spatial_dims)
        self.size_average = size_average
        self.data_range = data_range
        self.weights = weights
        self.K = K

    def forward(self, X, Y, mask):
        return ms_ssim(X, Y, mask, data_range=self.data_range, size_average=self.size_average,
                       win=self.win, weights=self.weights, K=self.K)
