"""CPU oracle (TEST INFRASTRUCTURE ONLY -- never imported by the product path) for the
SSIM / MS-SSIM metric: an op-for-op fp32 PyTorch restatement of the reference's
metrics/ms_ssim_torch.py.  Parity unpinned: the reference ships no metric outputs; the
known answers pinned in tests/test_oracle.py are ssim(X, X) = ms_ssim(X, X) = 1 and the
closed form of a constant-image pair."""
import torch
import torch.nn.functional as F


def fspecial_gauss_1d(size, sigma):
    """ms_ssim_torch.py:5-18"""
    coords = torch.arange(size).to(dtype=torch.float)
    coords -= size // 2
    g = torch.exp(-(coords ** 2) / (2 * sigma ** 2))
    g /= g.sum()
    return g.unsqueeze(0).unsqueeze(0)


def gaussian_filter(x, win):
    """:21-33: depthwise valid conv along W, then along H."""
    C = x.shape[1]
    out = F.conv2d(x, win, stride=1, padding=0, groups=C)
    return F.conv2d(out, win.transpose(2, 3), stride=1, padding=0, groups=C)


def ssim_level(X, Y, win, data_range):
    """:36-83 with size_average=False, full=True -> (ssim[B], cs[B])."""
    C1 = (0.01 * data_range) ** 2
    C2 = (0.03 * data_range) ** 2
    mu1 = gaussian_filter(X, win)
    mu2 = gaussian_filter(Y, win)
    mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    s11 = gaussian_filter(X * X, win) - mu1_sq
    s22 = gaussian_filter(Y * Y, win) - mu2_sq
    s12 = gaussian_filter(X * Y, win) - mu1_mu2
    cs_map = (2 * s12 + C2) / (s11 + s22 + C2)
    ssim_map = ((2 * mu1_mu2 + C1) / (mu1_sq + mu2_sq + C1)) * cs_map
    return ssim_map.mean(-1).mean(-1).mean(-1), cs_map.mean(-1).mean(-1).mean(-1)


def ssim(X, Y, win_size=11, win_sigma=1.5, data_range=255, size_average=True):
    """:86-132"""
    win = fspecial_gauss_1d(win_size, win_sigma).repeat(X.shape[1], 1, 1, 1)
    s, cs = ssim_level(X, Y, win, data_range)
    return s.mean() if size_average else s


def ms_ssim(X, Y, win_size=11, win_sigma=1.5, data_range=255, size_average=True, weights=None):
    """:135-194"""
    if weights is None:
        weights = torch.FloatTensor([0.0448, 0.2856, 0.3001, 0.2363, 0.1333])
    win = fspecial_gauss_1d(win_size, win_sigma).repeat(X.shape[1], 1, 1, 1)
    mcs = []
    for _ in range(weights.shape[0]):
        ssim_val, cs = ssim_level(X, Y, win, data_range)
        mcs.append(cs)
        padding = (X.shape[2] % 2, X.shape[3] % 2)
        X = F.avg_pool2d(X, kernel_size=2, padding=padding)
        Y = F.avg_pool2d(Y, kernel_size=2, padding=padding)
    mcs = torch.stack(mcs, dim=0)
    val = torch.prod((mcs[:-1] ** weights[:-1].unsqueeze(1)) * (ssim_val ** weights[-1]), dim=0)
    return val.mean() if size_average else val


# ---- masked variant: op-for-op restatement of metrics/masked_ms_ssim_torch.py (parity
# unpinned as above: the reference imports torchvision, absent here, and holds no outputs; its
# torchvision NEAREST resize of a tensor is F.interpolate(mode="nearest"), used directly).

def masked_ssim_level(X, Y, mask, win, data_range, K=(0.01, 0.03)):
    """masked_ms_ssim_torch.py:56-118 -> (ssim_per_channel, cs), each (B, C)."""
    C1 = (K[0] * data_range) ** 2
    C2 = (K[1] * data_range) ** 2
    mu1 = gaussian_filter(X, win)
    mu2 = gaussian_filter(Y, win)
    mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    s11 = gaussian_filter(X * X, win) - mu1_sq
    s22 = gaussian_filter(Y * Y, win) - mu2_sq
    s12 = gaussian_filter(X * Y, win) - mu1_mu2
    cs_map = (2 * s12 + C2) / (s11 + s22 + C2)
    ssim_map = ((2 * mu1_mu2 + C1) / (mu1_sq + mu2_sq + C1)) * cs_map
    one_win = win.shape[3] - 1
    m = F.interpolate(mask, size=(mask.shape[2] - one_win, mask.shape[3] - one_win),
                      mode="nearest")
    m = (m > 0.0).float()
    fs, fc, fm = torch.flatten(ssim_map, 2), torch.flatten(cs_map, 2), torch.flatten(m, 2)
    nz = fm != 0
    eps = 1e-10
    return (fs * nz).sum(-1) / (nz.sum(-1) + eps), (fc * nz).sum(-1) / (nz.sum(-1) + eps)


def masked_ssim(X, Y, mask, data_range=255, size_average=True, win_size=11, win_sigma=1.5,
                nonnegative_ssim=False):
    """:121-178 with the mask passed to _ssim (the reference omits it at :171)."""
    win = fspecial_gauss_1d(win_size, win_sigma).repeat(X.shape[1], 1, 1, 1)
    s, _ = masked_ssim_level(X, Y, mask, win, data_range)
    if nonnegative_ssim:
        s = torch.relu(s)
    return s.mean() if size_average else s.mean(1)


def masked_ms_ssim(X, Y, mask, data_range=255, size_average=True, win_size=11, win_sigma=1.5,
                   weights=None):
    """:181-265"""
    if weights is None:
        weights = [0.0448, 0.2856, 0.3001, 0.2363, 0.1333]
    wt = X.new_tensor(weights)
    win = fspecial_gauss_1d(win_size, win_sigma).repeat(X.shape[1], 1, 1, 1)
    mcs = []
    for i in range(wt.shape[0]):
        mask = (mask > 0.0).float()
        X = X * mask
        Y = Y * mask
        s, cs = masked_ssim_level(X, Y, mask, win, data_range)
        if i < wt.shape[0] - 1:
            mcs.append(torch.relu(cs))
            padding = [d % 2 for d in X.shape[2:]]
            X = F.avg_pool2d(X, kernel_size=2, padding=padding)
            Y = F.avg_pool2d(Y, kernel_size=2, padding=padding)
            mask = F.avg_pool2d(mask, kernel_size=2, padding=padding)
    s = torch.relu(s)
    val = torch.prod(torch.stack(mcs + [s], dim=0) ** wt.view(-1, 1, 1), dim=0)
    return val.mean() if size_average else val.mean(1)
