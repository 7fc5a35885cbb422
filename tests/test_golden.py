"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py).

CPU: the oracle still reproduces its committed outputs (regression pin).
GPU: the HIP path (fp32 parity mode) matches the same fixtures without
running the oracle on the GPU box."""
import os

import numpy as np
import pytest
import torch

from oracle import ref_model as ref

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    with np.load(os.path.join(HERE, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def _models():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(HERE, "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    return mg


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-12))


@pytest.mark.slow
def test_oracle_reproduces_golden_rgb():
    mg = _models()
    g = _load("rgb_64x64_b2.npz")
    net = mg.rgb_model()
    x, a = torch.from_numpy(g["x"]), torch.from_numpy(g["alpha"])
    me = ref.supply_mask(a)
    with torch.no_grad():
        out = ref.rgb_forward(net.state_dict(), x, a, a, *me[:4])
    assert _rel(out[0].numpy(), g["x_hat"]) < 1e-4
    np.testing.assert_allclose([t.item() for t in out[1:]], g["scalars"], rtol=1e-4)


@pytest.mark.slow
def test_oracle_reproduces_golden_mask():
    mg = _models()
    g = _load("mask_64x64_b2.npz")
    net = mg.mask_model()
    with torch.no_grad():
        out = ref.mask_forward(net.state_dict(), torch.from_numpy(g["alpha"]))
    assert _rel(out[0].numpy(), g["x_hat"]) < 1e-4
    np.testing.assert_allclose([t.item() for t in out[1:]], g["scalars"], rtol=1e-4)


@pytest.mark.gpu
def test_hip_matches_golden_rgb(device):
    mg = _models()
    g = _load("rgb_64x64_b2.npz")
    net = mg.rgb_model().to(device)
    x, a = torch.from_numpy(g["x"]).to(device), torch.from_numpy(g["alpha"]).to(device)
    from rgbac.layers.SupplyMask import mask_pyramid
    _, me = mask_pyramid(a, 4)
    dbg = {}
    out = net(x, a, a, *me, debug=dbg)
    from rgbac import runtime as rt
    assert _rel(rt.to_nchw(dbg["y"]).cpu().numpy(), g["y"]) < 1e-4
    assert _rel(out[0].cpu().numpy(), g["x_hat"]) < 1e-3
    np.testing.assert_allclose([t.item() for t in out[1:]], g["scalars"], rtol=1e-4)


@pytest.mark.gpu
def test_hip_matches_golden_mask(device):
    mg = _models()
    g = _load("mask_64x64_b2.npz")
    net = mg.mask_model().to(device)
    with torch.no_grad():
        out = net(torch.from_numpy(g["alpha"]).to(device))
    assert _rel(out[0].cpu().numpy(), g["x_hat"]) < 1e-3
    np.testing.assert_allclose([t.item() for t in out[1:]], g["scalars"], rtol=1e-4)
