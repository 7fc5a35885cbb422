"""CPU: the C-ABI library, its ctypes binding and the host-side packing logic.

No kernel is launched here.  The packed-weight layout and the kernel's index
conventions (tap order, ConvTranspose phases, PixelShuffle channel order,
multi-source channel concat) are checked by a pure-PyTorch emulation of the
implicit GEMM the kernel performs, against F.conv2d / F.conv_transpose2d."""
import ctypes
import os
import re
import subprocess
import sys

import pytest
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rgbac.h")


def header_functions():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(rgbac_\w+)\s*\(", txt, re.M)))


def test_library_exports_every_header_symbol():
    from rgbac import _lib
    lib = _lib.load()
    names = header_functions()
    assert len(names) >= 12
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(_lib.SIGNATURES), set(names) ^ set(_lib.SIGNATURES)
    assert lib.rgbac_abi_version() == 2
    from rgbac import runtime as rt
    assert lib.rgbac_conv_num_tiles() == len(rt.TILES)
    assert lib.rgbac_conv_max_groups() == 10


def test_argument_errors_are_reported_without_launching():
    from rgbac import _lib
    a = _lib.ConvArgs()                 # all zero: rejected by the shape checks
    with pytest.raises(RuntimeError, match="rgbac_conv2d failed"):
        _lib.call("rgbac_conv2d", a, None)
    with pytest.raises(RuntimeError, match="window size"):
        _lib.call("rgbac_winattn_core", 0, 1, 8, 8, 16, 8, 3, 0, 0, 1.0, None, 48, None, None,
                  None, 16, None, None)


@pytest.mark.parametrize("pyname,cname", [("ConvArgs", "rgbac_conv_args"),
                                           ("WgradArgs", "rgbac_wgrad_args")])
def test_args_struct_layout_matches_c(tmp_path, pyname, cname):
    """Compile a probe against include/rgbac.h with gcc and compare offsets with ctypes."""
    from rgbac import _lib
    cls = getattr(_lib, pyname)
    fields = [f for f, _ in cls._fields_]
    src = tmp_path / "probe.c"
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"',
             'int main(void){', f'printf("%zu\\n", sizeof({cname}));']
    lines += [f'printf("%zu\\n", offsetof({cname}, {f}));' for f in fields]
    lines += ['printf("%zu\\n", sizeof(rgbac_src)); return 0;}']
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-O0", str(src), "-o", str(exe)], check=True)
    vals = [int(v) for v in subprocess.run([str(exe)], check=True, capture_output=True,
                                           text=True).stdout.split()]
    assert vals[0] == ctypes.sizeof(cls)
    for f, off in zip(fields, vals[1:-1]):
        assert getattr(cls, f).offset == off, f
    assert vals[-1] == ctypes.sizeof(_lib.Src)


# ---------------------------------------------------------------- packing emulation
def _emulate(pk, xs, H, W):
    """The kernel's GEMM D[n][m] = sum_k Wp[n][k] X[m][k] in plain torch (fp32)."""
    from rgbac import runtime as rt
    x = torch.cat([F.pad(t, (0, 0, 0, 0, 0, rt.round_up(t.shape[1], 8) - t.shape[1]))
                   for t in xs], 1)
    assert x.shape[1] == pk.cin_pad
    B = x.shape[0]
    out = None
    if pk.mode == rt.CONVT_S2:
        outs = torch.zeros((B, pk.cout, 2 * H, 2 * W))
        for ph in range(4):
            py, px = ph >> 1, ph & 1
            tw = 3 - px
            ntaps = (3 - py) * tw
            cols = []
            for tap in range(ntaps):
                ty, tx = divmod(tap, tw)
                dy, dx = 1 - ty, 1 - tx
                sh = F.pad(x, (1, 1, 1, 1))[:, :, 1 + dy:1 + dy + H, 1 + dx:1 + dx + W]
                cols.append(sh)
            X = torch.cat(cols, 1)                                   # B, ntaps*cin_pad, H, W
            Wp = pk.w[ph, :pk.cout, :ntaps * pk.cin_pad].float()
            D = torch.einsum("nk,bkhw->bnhw", Wp, X) + pk.bias[:pk.cout].view(1, -1, 1, 1)
            outs[:, :, py::2, px::2] = D
        return outs
    k, s, p = pk.ksize, pk.stride, pk.ksize // 2
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    xp = F.pad(x, (p, p, p, p))
    cols = [xp[:, :, ty:ty + s * (Ho - 1) + 1:s, tx:tx + s * (Wo - 1) + 1:s]
            for ty in range(k) for tx in range(k)]
    X = torch.cat(cols, 1)
    Wp = pk.w[0, :pk.cout, :k * k * pk.cin_pad].float()
    D = torch.einsum("nk,bkhw->bnhw", Wp, X) + pk.bias[:pk.cout].view(1, -1, 1, 1)
    if pk.mode == rt.SUBPEL2:
        D = F.pixel_shuffle(D, 2)
    return D


@pytest.mark.parametrize("cin,cout,k,s", [(3, 16, 5, 2), (40, 24, 3, 1), (16, 8, 1, 1)])
def test_packed_conv_matches_torch(cin, cout, k, s):
    from rgbac import runtime as rt
    g = torch.Generator().manual_seed(cin)
    m = torch.nn.Conv2d(cin, cout, k, stride=s, padding=k // 2)
    x = torch.randn((2, cin, 10, 12), generator=g)
    pk = rt.PackedConv(m.weight, m.bias, rt.CONV, [(cin, rt.round_up(cin, 8))], torch.float32,
                       stride=s)
    assert pk.cout_pad % 128 == 0 and pk.k_pad % 64 == 0
    assert torch.allclose(_emulate(pk, [x], 10, 12), m(x), atol=1e-5)


def test_packed_multisource_concat():
    from rgbac import runtime as rt
    g = torch.Generator().manual_seed(9)
    parts = [torch.randn((1, c, 6, 6), generator=g) for c in (80, 40, 8)]
    m = torch.nn.Conv2d(128, 8, 3, padding=1)
    pk = rt.PackedConv(m.weight, m.bias, rt.CONV, [(80, 80), (40, 40), (8, 8)], torch.float32)
    assert torch.allclose(_emulate(pk, parts, 6, 6), m(torch.cat(parts, 1)), atol=1e-5)


@pytest.mark.parametrize("cin,cout", [(16, 12), (3, 5)])
def test_packed_conv_transpose_phases(cin, cout):
    from rgbac import runtime as rt
    g = torch.Generator().manual_seed(cin + cout)
    m = torch.nn.ConvTranspose2d(cin, cout, 5, stride=2, padding=2, output_padding=1)
    x = torch.randn((2, cin, 5, 7), generator=g)
    pk = rt.PackedConv(m.weight, m.bias, rt.CONVT_S2, [(cin, rt.round_up(cin, 8))],
                       torch.float32, stride=2)
    assert torch.allclose(_emulate(pk, [x], 5, 7), m(x), atol=1e-5)


def test_packed_subpel_and_transposed_1x1():
    from rgbac import runtime as rt
    from rgbac.layers._blocks import subpel_conv3x3
    g = torch.Generator().manual_seed(4)
    sp = subpel_conv3x3(24, 10, 2)
    x = torch.randn((1, 24, 4, 5), generator=g)
    pk = rt.PackedConv(sp[0].weight, sp[0].bias, rt.SUBPEL2, [(24, 24)], torch.float32)
    assert torch.allclose(_emulate(pk, [x], 4, 5), sp(x), atol=1e-5)
    ct = torch.nn.ConvTranspose2d(16, 24, 1)
    pk = rt.PackedConv(ct.weight, ct.bias, rt.CONV, [(16, 16)], torch.float32, transposed=True)
    x = torch.randn((1, 16, 3, 3), generator=g)
    assert torch.allclose(_emulate(pk, [x], 3, 3), ct(x), atol=1e-5)


def test_tile_candidates():
    from rgbac import runtime as rt
    c = rt._candidates(8192, 8, 18)
    assert all(rt.TILES[t][1] <= 32 for t, _ in c)      # no 128-wide tiles for 8 channels
    assert (0, 1) in rt._candidates(32768, 192, 30)
    t, ks = rt._heuristic(128, 768, 27)
    assert ks > 1                                       # tiny grids split K


def test_pw3_admission_mirror():
    """rgbac.runtime._pw3_admits (the host mirror of csrc/pw3.hip pw3_ok, which names the
    pointwise kernel in the bench tables): GDN / IGDN with x as the epilogue operand and 192
    channels; the gate only with both operands and from 8,192 tiles on; never a pre-activation
    store, a res0 operand or a 96-channel input."""
    import types
    from rgbac import _lib
    from rgbac import runtime as rt

    def prep(act, cin=192, cout=192, square=True, res1="x", res2=False, res0=False, zout=False,
             mgrid=8 * 64 * 64):
        a = _lib.ConvArgs()
        a.mode, a.act, a.square_input = rt.CONV, rt.ACT[act], 1 if square else 0
        a.cin_pad, a.k_pad, a.cout, a.out_ldc, a.out_coff = cin, cin, cout, cout, 0
        a.src[0].ptr, a.src[0].ldc = 4096, cin
        a.res1 = 4096 if res1 == "x" else (8192 if res1 else None)
        a.res1_ldc = cin if res1 == "x" else cout
        a.res2, a.res2_ldc = (12288 if res2 else None), cout
        a.res0, a.zout = (16384 if res0 else None), (20480 if zout else None)
        return types.SimpleNamespace(a=a, mgrid=mgrid)

    assert rt._pw3_admits([prep("gdn")]) and rt._pw3_admits([prep("igdn")])
    assert rt._pw3_admits([prep("gdn"), prep("gdn")])
    assert not rt._pw3_admits([prep("gdn", zout=True)])
    assert not rt._pw3_admits([prep("gdn", res0=True)])
    assert not rt._pw3_admits([prep("gdn", cin=96)])
    assert not rt._pw3_admits([prep("gdn", cout=96)])
    assert not rt._pw3_admits([prep("gdn", res1="a")])          # x must be the epilogue operand
    gate = dict(square=False, res1="a", res2=True)
    assert not rt._pw3_admits([prep("gate", **gate)])           # 2,048 tiles: stays on pw2
    assert rt._pw3_admits([prep("gate", mgrid=8 * 128 * 128, **gate)])
    assert not rt._pw3_admits([prep("gate", mgrid=8 * 128 * 128, square=False, res1="a")])
    assert not rt._pw3_admits([prep("gelu", square=False, res1=None)])


def test_state_dict_layout_matches_reference_names():
    """Key names/shapes the reference's checkpoints use."""
    from rgbac.models.AutoEncoderRGB_Journal import AutoEncoder
    sd = AutoEncoder().state_dict()
    want = {
        "Encoder.x1.weight": (192, 3, 5, 5),
        "Encoder.gdn1.gamma": (192, 192),
        "Encoder.attention1.conv_a.0.conv.2.weight": (96, 96, 3, 3),
        "Encoder.attention1.attn.attn.relative_position_bias_table": (225, 8),
        "Encoder.attention1.attn.attn.relative_position_index": (64, 64),
        "Encoder.attention1.attn.attn.qkv.weight": (576, 192),
        "Encoder.attention2.attn.attn.relative_position_bias_table": (49, 8),
        "Encoder.attention1.conv_b.3.weight": (192, 192, 1, 1),
        "Decoder.x2.weight": (192, 192, 5, 5),
        "Decoder.dse.enh3.conv2.weight": (32, 32, 3, 3),
        "h_mean_s.0.0.weight": (768, 192, 3, 3),
        "h_a.8.weight": (192, 224, 3, 3),
        "cc_mean_transforms.9.0.weight": (224, 120, 3, 3),
        "lrp_transforms.0.0.weight": (224, 88, 3, 3),
        "entropy_bottleneck._matrix1": (192, 3, 3),
        "entropy_bottleneck.quantiles": (192, 1, 3),
        "gaussian_conditional.lower_bound_scale.bound": (1,),
    }
    for k, shape in want.items():
        assert tuple(sd[k].shape) == shape, k
    assert sd["Encoder.attention1.attn.attn.relative_position_index"].dtype == torch.int64
    assert sum(v.numel() for k, v in sd.items() if not k.endswith("index")
               and "gaussian_conditional" not in k and "bound" not in k
               and "target" not in k) == 34068518


def test_cpu_tensors_fail_loudly():
    from rgbac.layers.GDN import GDN
    with pytest.raises(RuntimeError, match="GPU"):
        GDN(8)(torch.randn(1, 8, 4, 4))


@pytest.mark.parametrize("cout", [1, 3, 4])
def test_convtranspose_small_cout_as_subpel(cout):
    """ConvTranspose2d(5, s2, p2, op1) repacked as conv3x3(4*Cout) + PixelShuffle(2)."""
    from rgbac import runtime as rt
    g = torch.Generator().manual_seed(cout)
    m = torch.nn.ConvTranspose2d(16, cout, 5, stride=2, padding=2, output_padding=1)
    x = torch.randn((2, 16, 5, 6), generator=g)
    pk = rt.PackedConv(m.weight, m.bias, rt.SUBPEL2, [(16, 16)], torch.float32, stride=2,
                       transposed=True)
    assert pk.mode == rt.SUBPEL2 and pk.ksize == 3 and pk.stride == 1 and pk.cout == 4 * cout
    assert torch.allclose(_emulate(pk, [x], 5, 6), m(x), atol=1e-5)


def test_geometry_matches_reference_behaviour():
    """The whole-codec forward needs H, W multiples of 64: the oracle (an op-for-op
    restatement of AutoEncoderRGB_Journal.forward) fails at 96x96 exactly like the reference
    (torch.cat of the 16x16 hyper-synthesis output with the 12x12 latent slice, :242), and
    the HIP model refuses such sizes up front with a RuntimeError of its own."""
    import torch
    from oracle import ref_model as ref
    from rgbac.models.AutoEncoderRGB_Journal import AutoEncoder, GeometryError, check_geometry
    torch.manual_seed(234)
    sd = {k: v.detach() for k, v in AutoEncoder().eval().state_dict().items()}
    x = torch.rand((1, 3, 96, 96))
    a = torch.ones((1, 1, 96, 96))
    me = ref.supply_mask(a)
    with pytest.raises(RuntimeError, match="Sizes of tensors must match"):
        with torch.no_grad():
            ref.rgb_forward(sd, x, a, a, *me[:4])
    for hw in ((96, 96), (160, 224), (64, 96), (0, 64)):
        with pytest.raises(GeometryError):
            check_geometry(*hw)
    assert issubclass(GeometryError, RuntimeError) and issubclass(GeometryError, ValueError)
    check_geometry(64, 192)


def test_bench_gpus_flag_spawns_ranks(monkeypatch):
    """`bench.py --gpus N` without a launcher spawns N ranks itself (before any GPU call);
    under a launcher a mismatching --gpus is rejected."""
    import bench
    calls = []
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench, "spawn_ranks", lambda n: calls.append(n) or 0)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "1"])
    assert bench.main() == 0 and calls == [4]
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4"])
    with pytest.raises(SystemExit):
        bench.main()


def test_masked_ms_ssim_argument_checks():
    """rgbac.metrics.masked_ms_ssim_torch: the reference's shape / window errors
    (masked_ms_ssim_torch.py:148-165, :207-228) and the mask's shape are checked before any
    launch, and CPU tensors fail loudly (no CPU fallback)."""
    from rgbac.metrics.masked_ms_ssim_torch import ms_ssim, ssim
    X = torch.rand((1, 3, 192, 192))
    M = torch.ones((1, 1, 192, 192))
    with pytest.raises(ValueError, match="same dimensions"):
        ms_ssim(X, X[:, :, :100], M)
    with pytest.raises(ValueError, match="odd"):
        ssim(X, X, M, win_size=10)
    with pytest.raises(ValueError, match="mask"):
        ms_ssim(X, X, torch.ones((1, 2, 192, 192)))
    with pytest.raises(ValueError, match="4-d"):
        ms_ssim(X[0], X[0], M)
    with pytest.raises(RuntimeError, match="GPU"):
        ms_ssim(X, X, M)
