"""CPU: the host side of the GPU data pipeline (rgbac/data.py) -- random parameter draws in the
reference's order (MYdataset.py:86-111: RandomResizedCrop.get_params on the torch RNG, two
python random.random() flips, RandomApply's torch.rand(1) for the fill) and their invariants."""
import math
import random

import pytest
import torch

from rgbac import data


def test_params_in_bounds_and_ratio():
    torch.manual_seed(0)
    random.seed(0)
    for H, W in [(480, 640), (100, 1000), (1000, 100), (7, 9), (256, 256)]:
        for _ in range(200):
            i, j, h, w, fh, fv, fill = data.draw_params(H, W)
            assert 0 <= i and 0 <= j and 0 < h and 0 < w and i + h <= H and j + w <= W
            assert isinstance(fh, bool) and isinstance(fv, bool) and isinstance(fill, bool)


def test_param_rng_order():
    """The draws consume exactly: torch RNG for the crop, 2 python randoms, 1 torch.rand."""
    torch.manual_seed(3)
    random.seed(3)
    p = data.draw_params(480, 640, 0.25)
    t_after, r_after = torch.rand(1).item(), random.random()
    torch.manual_seed(3)
    random.seed(3)
    i, j, h, w = data.random_resized_crop_params(480, 640)
    fh, fv = random.random() < 0.5, random.random() < 0.5
    fill = not (0.25 < torch.rand(1))
    assert p == (i, j, h, w, fh, fv, bool(fill))
    assert torch.rand(1).item() == t_after and random.random() == r_after


def test_fill_and_flip_rates():
    torch.manual_seed(1)
    random.seed(1)
    n = 4000
    ps = [data.draw_params(300, 300, 0.25) for _ in range(n)]
    for k, want in ((4, 0.5), (5, 0.5), (6, 0.25)):
        rate = sum(p[k] for p in ps) / n
        assert abs(rate - want) < 0.03, (k, rate)
    areas = [p[2] * p[3] / 90000 for p in ps]
    assert min(areas) >= 0.07 and max(areas) <= 1.0
    ratios = [math.log(p[3] / p[2]) for p in ps]
    assert max(abs(r) for r in ratios) <= math.log(4 / 3) + 0.05


def test_fallback_center_crop():
    """Extreme aspect ratios fail the 10 attempts often: the fallback centre crop is clamped
    to the ratio range (torchvision get_params)."""
    torch.manual_seed(0)
    hits = 0
    for _ in range(300):
        i, j, h, w = data.random_resized_crop_params(10, 1000)
        assert 0 < h <= 10 and 0 < w <= 1000 and j + w <= 1000
        if h == 10 and w == round(10 * 4 / 3):
            assert j == (1000 - w) // 2 and i == 0
            hits += 1
    assert hits > 0
