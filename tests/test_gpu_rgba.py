"""RGBA evaluation pipeline (trainRGB.py:98-111, :282-306) on the HIP path vs the CPU oracle:
constraint / alpha reconstruction bit-exact, the device-side all-ones flag, and the whole
alpha -> RGB chain in fp32 parity mode."""
import pytest
import torch

from oracle import ref_model as ref

pytestmark = pytest.mark.gpu


def _grid_alpha(B, H, W, seed, p_one=0.5):
    """k/255 alpha with planted isolated zeros / non-zeros (incl. at the borders)."""
    g = torch.Generator().manual_seed(seed)
    a = (torch.rand((B, 1, H, W), generator=g) < p_one).float()
    a[:, :, : H // 2, : W // 2] = 1.0            # solid block: planted holes
    a[:, :, H // 2:, W // 2:] = 0.0              # empty block: planted specks
    for b in range(B):
        off = b % 2
        for y in range(1 + off, H // 2 - 1, 3):          # isolated holes in the solid block
            for x in range(1, W // 2 - 1, 3):
                a[b, 0, y, x] = 0.0
        for y in range(H // 2 + 1, H - 2, 3):            # isolated specks in the empty block
            for x in range(W // 2 + 1 + off, W - 2, 3):
                a[b, 0, y, x] = float(torch.randint(1, 256, (1,), generator=g)) / 255
        a[b, 0, H - 1, W - 1] = 0.5                # border speck (cleared)
        a[b, 0, 0, 0] = 0.0                        # border hole (never filled: padding)
    return a


@pytest.mark.parametrize("shape", [(1, 8, 8), (2, 64, 64), (3, 37, 53)])
def test_constraint_exact(device, shape):
    from rgbac.rgba import constraint
    B, H, W = shape
    a = _grid_alpha(B, H, W, seed=H * W)
    want = ref.constraint_rgb(a)
    t = a.to(device)
    got = constraint(t)
    assert got is t
    assert torch.equal(got.cpu(), want)
    assert not torch.equal(want, a)          # the planted pixels did change


def test_recon_alpha_exact(device):
    from rgbac.rgba import recon_alpha
    g = torch.Generator().manual_seed(3)
    x = torch.rand((2, 1, 64, 96), generator=g) * 1.4 - 0.2
    x[:, :, 10:30, 10:30] = 1.3                 # clamps to 1 with planted holes
    x[:, :, 15, 15] = -0.01
    x[:, :, 40:60, 40:60] = -0.3                # clamps to 0 with planted specks
    x[:, :, 50, 50] = 0.7
    x[0, 0, 0, :8] = torch.tensor([0.5, 1.5, 2.5, 126.5, 127.5, 0.25, 254.5, 253.5]) / 255
    want = ref.recon_alpha(x)
    got = recon_alpha(x.to(device)).cpu()
    assert torch.equal(got, want)


@pytest.mark.parametrize("all_ones", [True, False])
def test_rgba_finish_flag(device, all_ones):
    from rgbac import _lib
    mask = torch.ones((2, 1, 16, 16), device=device)
    if not all_ones:
        mask[1, 0, 7, 9] = 254 / 255
    flag = torch.empty((1,), dtype=torch.int32, device=device)
    rm = torch.empty_like(mask)
    _lib.call("rgbac_alpha_recon", 2, 16, 16, 1, mask.data_ptr(), rm.data_ptr(),
              mask.data_ptr(), flag.data_ptr(), _lib.stream_ptr(device))
    x = torch.linspace(-0.5, 1.5, 2 * 3 * 16 * 16, device=device).view(2, 3, 16, 16)
    img = torch.empty_like(x)
    bpp = torch.tensor(0.25, device=device)
    bppm = torch.tensor(0.0625, device=device)
    mse = torch.tensor(0.01, device=device)
    bt = torch.empty((), device=device)
    ps = torch.empty((), device=device)
    _lib.call("rgbac_rgba_finish", x.numel(), x.data_ptr(), img.data_ptr(), bpp.data_ptr(),
              bppm.data_ptr(), flag.data_ptr(), mse.data_ptr(), bt.data_ptr(), ps.data_ptr(),
              _lib.stream_ptr(device))
    assert int(flag.item()) == (0 if all_ones else 1)
    assert bt.item() == (0.25 if all_ones else 0.3125)
    assert abs(ps.item() - 20.0) < 1e-4
    assert torch.equal(img, torch.clamp(x, 0, 1))


def test_rgba_forward_fp32(device):
    from rgbac.models.AutoEncoderMask_Journal import AutoEncoder as MaskNet
    from rgbac.models.AutoEncoderRGB_Journal import AutoEncoder as RGBNet
    from rgbac.rgba import rgba_forward
    torch.manual_seed(234)
    rgb, msk = RGBNet().eval(), MaskNet().eval()
    sdr = {k: v.detach().cpu() for k, v in rgb.state_dict().items()}
    sdm = {k: v.detach().cpu() for k, v in msk.state_dict().items()}
    g = torch.Generator().manual_seed(0)
    B, H, W = 2, 192, 192
    x = torch.round(torch.rand((B, 3, H, W), generator=g) * 255) / 255
    a = torch.ones((B, 1, H, W))
    a[0, :, :, : W // 2] = 0
    a[1, :, 60:120, 30:150] = 0
    xm = torch.where(a > 0, x, a)
    with torch.no_grad():
        want = ref.rgba_forward(sdm, sdr, xm, a, msssim=True)
    img, rm, mse, bpp, psnr, om, ms = rgba_forward(msk.to(device), rgb.to(device),
                                                    xm.to(device), a.to(device), msssim=True)
    assert abs(ms.item() - want[5].item()) < 1e-4
    # the recon mask is integer-valued work: identical unless the alpha net's fp32 output
    # sits within rounding noise of a .5/255 boundary
    diff = (rm.cpu() != want[1]).float().mean().item()
    assert diff < 1e-3
    assert (img.cpu() - want[0]).abs().max().item() < 1e-3
    assert float(img.min()) >= 0.0 and float(img.max()) <= 1.0
    assert abs(bpp.item() - want[3].item()) / want[3].item() < 1e-3
    assert abs(psnr.item() - want[4].item()) < 1e-3
    assert abs(mse.item() - want[2].item()) / want[2].item() < 1e-3
