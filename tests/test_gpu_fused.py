"""GPU: the fused block kernels against the unfused launch sequence they replace and the
fp32 oracle (tests/../oracle/ref_model.py).

DSE (rgbac_dse_block, reference layers/TransformRGB.py:16-49 and
models/AutoEncoderMask_Journal.py:39-48): three launches instead of eight.  The fused path
keeps every bf16 rounding point of the unfused one (block outputs, the ReLU map, x_first,
block3 + x_first); only in_conv's 3-term sum is formed on the VALU instead of the MFMA, so
an x_first value can differ by one bf16 ulp.  Bar: the fused output is as close to the fp32
oracle as the unfused bf16 path (within 1.5x of its max error, or 1e-2 relative), and the
two bf16 paths agree to 2 bf16 ulps of the output range at 99.9 % of the elements."""
import pytest
import torch

from oracle import ref_model as ref

pytestmark = pytest.mark.gpu


def _dse(kind, seed):
    torch.manual_seed(seed)
    if kind == "rgb":
        from rgbac.layers.TransformRGB import DSE
        m = DSE(32)
    else:
        from rgbac.models.AutoEncoderMask_Journal import DSE
        m = DSE(1, 32)
    with torch.no_grad():                  # larger than default init: the blocks matter
        for e in (m.enh1, m.enh2, m.enh3):
            e.conv1.weight.mul_(2.0)
            e.conv2.weight.mul_(2.0)
    return m.cuda().eval()


@pytest.mark.parametrize("kind,B,H,W", [("rgb", 2, 64, 96), ("rgb", 1, 40, 50),
                                        ("mask", 2, 48, 64), ("rgb", 2, 256, 256),
                                        ("mask", 1, 17, 33)])
def test_dse_fused_matches_unfused_and_oracle(device, kind, B, H, W):
    from rgbac import runtime as rt
    from rgbac.layers.TransformRGB import dse_fused, dse_fused_ok
    m = _dse(kind, 3)
    C = 3 if kind == "rgb" else 1
    x = torch.rand((B, C, H, W), generator=torch.Generator().manual_seed(4)).cuda()
    with torch.no_grad():
        f = rt.to_nhwc(x, torch.bfloat16)
        assert dse_fused_ok(m, f)
        got = rt.to_nchw(dse_fused(m, f)).float().cpu()
        old = rt.DSE_FUSED
        rt.DSE_FUSED = False
        try:
            base = rt.to_nchw(m.nhwc(f)).float().cpu()
        finally:
            rt.DSE_FUSED = old
    sd = {f"m.{k}": v.detach().cpu() for k, v in m.state_dict().items()}
    want = ref.dse(x.cpu(), sd, "m", leaky=(kind == "mask")).detach()
    scale = want.abs().max().item()
    e_got = (got - want).abs().max().item() / scale
    e_base = (base - want).abs().max().item() / scale
    ulp = scale * 2.0 ** -7
    frac = ((got - base).abs() > 2 * ulp).float().mean().item()
    print(f"DSE {kind} {B}x{H}x{W}: fused err {e_got:.2e}, unfused err {e_base:.2e}, "
          f"elements > 2 ulp apart {frac:.1e}")
    assert e_got <= max(1.5 * e_base, 1e-2), (e_got, e_base)
    assert frac <= 1e-3, frac


def test_dse_module_forward_uses_fused_path(device):
    """DSE.forward under no_grad at bf16 goes through rgbac_dse_block (3 launches)."""
    from rgbac import runtime as rt
    m = _dse("rgb", 5)
    f = rt.to_nhwc(torch.rand((1, 3, 64, 64), device="cuda"), torch.bfloat16)
    prof = rt.LaunchProfiler()
    old = rt.PROFILER
    rt.PROFILER = prof
    try:
        with torch.no_grad():
            m.nhwc(f)
    finally:
        rt.PROFILER = old
    names = [r[0] for r in prof.records]
    assert names == ["dse_block_kernel"] * 3, names


# ---------------------------------------------------------------------------------------
# Masked shifted-window attention block (rgbac_winattn_block; reference
# layers/masked_win_attention.py:96-131, 169-251): one launch instead of qkv GEMM + core +
# MASKSEL proj GEMM.  The fused path skips the bf16 round trip of the qkv tensor (q is scaled
# before its single rounding), so it is compared with the fp32 oracle at the unfused bf16
# path's own error (within 1.5x, or 2e-2 of the output range), and with the unfused path at
# 3 bf16 ulps of the output range on 99.5 % of the elements.
@pytest.mark.parametrize("C,ws,B,H,W,shift,masked", [
    (192, 8, 2, 64, 64, 4, True), (192, 8, 1, 32, 48, 0, False), (192, 8, 1, 24, 40, 4, True),
    (192, 8, 2, 16, 16, 0, True), (192, 8, 1, 8, 24, 0, True),
    # ws 4 / C 80 (rgbac_winattn_block_ws4): heads of 10 channels straddle the 16-row tiles
    (80, 4, 2, 32, 32, 2, True), (80, 4, 1, 16, 24, 0, False), (80, 4, 1, 12, 20, 2, True),
    (80, 4, 2, 8, 8, 0, True), (80, 4, 3, 4, 12, 0, True)])
def test_winattn_block_fused_matches_unfused_and_oracle(device, C, ws, B, H, W, shift, masked):
    from rgbac import runtime as rt
    from rgbac.layers.masked_win_attention import WinBasedAttention
    torch.manual_seed(11)
    m = WinBasedAttention(C, 8, ws, shift).cuda().eval()
    with torch.no_grad():
        m.attn.relative_position_bias_table.normal_(0, 0.5)   # make the bias matter
    m.masked = masked
    g = torch.Generator().manual_seed(12)
    x = torch.randn((B, C, H, W), generator=g)
    alpha = torch.ones((B, 1, H, W))
    if masked:
        alpha[:, :, : H // 2, : W // 2] = 0                  # some all-transparent windows
        alpha[0, 0, 3, 5] = 1.0                              # ... and one nearly transparent
    xg, ag = x.cuda(), alpha.cuda()
    with torch.no_grad():
        f = rt.to_nhwc(xg, torch.bfloat16)
        assert m.attn.block_fused_ok(f, True, None)
        got = rt.to_nchw(m.nhwc(f, ag)).float().cpu()
        old = (rt.WINBLOCK_FUSED, rt.WINBLOCK4_FUSED)
        rt.WINBLOCK_FUSED = rt.WINBLOCK4_FUSED = False
        try:
            base = rt.to_nchw(m.nhwc(f, ag)).float().cpu()
        finally:
            rt.WINBLOCK_FUSED, rt.WINBLOCK4_FUSED = old
    sd = {f"m.{k}": v.detach().cpu() for k, v in m.state_dict().items()}
    want = ref.win_based_attention(x, alpha, sd, "m", ws, shift, heads=8,
                                   masked=masked).detach()
    scale = want.abs().max().item()
    e_got = (got - want).abs().max().item() / scale
    e_base = (base - want).abs().max().item() / scale
    ulp = scale * 2.0 ** -7
    frac = ((got - base).abs() > 3 * ulp).float().mean().item()
    print(f"winblock {B}x{H}x{W} shift {shift} masked {masked}: fused err {e_got:.2e}, "
          f"unfused err {e_base:.2e}, elements > 3 ulp apart {frac:.1e}")
    assert e_got <= max(1.5 * e_base, 2e-2), (e_got, e_base)
    assert frac <= 5e-3, frac
    if masked and shift == 0 and H >= 4 * ws:                # transparent windows: exactly x
        xb = rt.to_nchw(f).float().cpu()
        assert torch.equal(got[:, :, ws:H // 2, ws:W // 2], xb[:, :, ws:H // 2, ws:W // 2])


# The head-pair ws-8 block (round 6, rgbac_winattn_block's form for >= 2,048 windows): per-window
# flags (winflag_kernel), device-side compaction and one head pair per persistent workgroup
# (winblock_kernel), the proj over the compacted list (winproj_kernel).  It keeps every product
# and rounding point of the round-3 kernel (winblock_v2_kernel, the form below 2,048 windows),
# so the two forms (RGBAC_WINBLOCK_FORM=3 / 2) are compared bit for bit, over repeated calls on
# one workspace.  B 3 at 512^2 (12,288 windows) spans two launches of at most 8,192 windows.
@pytest.mark.parametrize("B,H,W,shift,alpha_kind", [
    (8, 64, 64, 0, "bench"), (2, 64, 64, 4, "quarter"), (1, 32, 48, 0, "ones"),
    (1, 24, 40, 4, "quarter"), (2, 16, 16, 0, "zeros"), (1, 8, 8, 0, "one_pixel"),
    (3, 8, 24, 0, "unmasked"), (3, 512, 512, 0, "quarter"), (4, 256, 256, 4, "bench")])
def test_winblock_head_pair_kernel_bit_identical(device, B, H, W, shift, alpha_kind):
    import os
    from rgbac import runtime as rt
    from rgbac.layers.masked_win_attention import WinBasedAttention
    torch.manual_seed(21)
    m = WinBasedAttention(192, 8, 8, shift).cuda().eval()
    with torch.no_grad():
        m.attn.relative_position_bias_table.normal_(0, 0.5)
        m.attn.qkv.bias.normal_(0, 0.2)
        m.attn.proj.bias.normal_(0, 0.2)
    m.masked = alpha_kind != "unmasked"
    g = torch.Generator().manual_seed(22)
    x = torch.randn((B, 192, H, W), generator=g)
    alpha = torch.ones((B, 1, H, W))
    if alpha_kind == "quarter":
        alpha[:, :, : H // 2, : W // 2] = 0
    elif alpha_kind == "zeros":
        alpha.zero_()
    elif alpha_kind == "one_pixel":
        alpha.zero_()
        alpha[0, 0, 5, 2] = 0.25
    elif alpha_kind == "bench":                       # ones / half / ellipse / all-zero cycle
        yy, xx = torch.meshgrid(torch.linspace(-1, 1, H), torch.linspace(-1, 1, W), indexing="ij")
        for b in range(B):
            k = b % 4
            alpha[b, 0] = (1.0 if k == 0 else 0.5 if k == 1 else
                           ((xx / 0.8) ** 2 + (yy / 0.6) ** 2 <= 1).float() if k == 2 else 0.0)
    xg, ag = x.cuda(), alpha.cuda()
    with torch.no_grad():
        f = rt.to_nhwc(xg, torch.bfloat16)
        outs = []
        try:
            os.environ["RGBAC_WINBLOCK_FORM"] = "3"
            for _ in range(3):                        # repeated calls on one workspace
                outs.append(rt.to_nchw(m.attn.run_block(f, ag, shift, m.masked)).float())
            os.environ["RGBAC_WINBLOCK_FORM"] = "2"
            ref_out = rt.to_nchw(m.attn.run_block(f, ag, shift, m.masked)).float()
        finally:
            os.environ.pop("RGBAC_WINBLOCK_FORM", None)
    for o in outs:
        assert torch.equal(o, ref_out), (o - ref_out).abs().max().item()
    if alpha_kind == "zeros":
        assert torch.equal(outs[0], rt.to_nchw(f).float())


# ---------------------------------------------------------------------------------------
# Fused bottleneck residual blocks (rgbac_residual_unit_ex): the ResidualUnit at C = 192 / 80
# (Masked_Attention.py:150-169; C = 192 with W % 16 == 0 runs the weight-streaming kernel,
# 16 x 24 the chunk-ring one) and the alpha codec's
# ResBlock at C = 192 / 80 (AutoEncoderMask_Journal.py:96-110).  Same bf16 rounding points
# as the three-launch path (both intermediates are rounded to bf16 in LDS exactly where the
# unfused path stores them), so the two agree to 2 bf16 ulps on 99.9 % of the elements and
# the fused result is as close to the fp32 oracle as the unfused one.
@pytest.mark.parametrize("kind,C,B,H,W,groups", [("ru", 80, 2, 32, 32, 2), ("ru", 80, 1, 16, 24, 1),
                                                 ("rb", 192, 1, 32, 48, 2), ("rb", 80, 2, 32, 32, 2),
                                                 ("rb", 80, 1, 8, 16, 1), ("ru", 192, 2, 64, 64, 2),
                                                 ("ru", 192, 1, 24, 32, 1), ("rb", 192, 2, 16, 16, 1),
                                                 ("ru", 192, 1, 16, 24, 2)])
def test_bottleneck_fused_matches_unfused_and_oracle(device, kind, C, B, H, W, groups):
    from rgbac import runtime as rt
    from rgbac.layers import Masked_Attention as MA
    from rgbac.models import AutoEncoderMask_Journal as AM
    torch.manual_seed(21)
    if kind == "ru":
        mods = [MA.ResidualUnit(C).cuda() for _ in range(groups)]
    else:
        mods = [AM.ResBlock(C).cuda() for _ in range(groups)]
    g = torch.Generator().manual_seed(22)
    xs = [torch.randn((B, C, H, W), generator=g) for _ in range(groups)]
    with torch.no_grad():
        fs = [rt.to_nhwc(x.cuda(), torch.bfloat16) for x in xs]
        run = MA.run_residual_units if kind == "ru" else AM.run_resblocks
        pairs = list(zip(mods, fs))
        assert MA._fused_ok(pairs)
        got = [rt.to_nchw(o).float().cpu() for o in run(pairs)]
        old = MA.FUSED
        MA.FUSED = False
        try:
            base = [rt.to_nchw(o).float().cpu() for o in run(pairs)]
        finally:
            MA.FUSED = old
    for m, x, gt, bs in zip(mods, xs, got, base):
        sd = {f"m.{k}": v.detach().cpu() for k, v in m.state_dict().items()}
        want = (ref.residual_unit(x, sd, "m") if kind == "ru" else ref.resblock(x, sd, "m")).detach()
        scale = want.abs().max().item()
        e_got = (gt - want).abs().max().item() / scale
        e_base = (bs - want).abs().max().item() / scale
        frac = ((gt - bs).abs() > 2 * scale * 2.0 ** -7).float().mean().item()
        print(f"{kind} C{C} {B}x{H}x{W} g{groups}: fused err {e_got:.2e}, unfused {e_base:.2e}, "
              f"> 2 ulp apart {frac:.1e}")
        assert e_got <= max(1.5 * e_base, 1e-2), (e_got, e_base)
        assert frac <= 1e-3, frac


@pytest.mark.parametrize("kind", [0, 1])
def test_stream_unit_matches_chunk_ring_kernel(device, kind):
    """ru_stream_kernel (fragment-major packs) against ru_fused_kernel (chunk-ring packs) on
    the same C = 192 units: identical GEMM order per output and the same bf16 rounding
    points, so they agree to 1 bf16 ulp of the output range at 99.9 % of the elements."""
    from rgbac import runtime as rt
    from rgbac.layers import Masked_Attention as MA
    from rgbac.models import AutoEncoderMask_Journal as AM
    torch.manual_seed(31 + kind)
    mods = [(MA.ResidualUnit(192) if kind == 0 else AM.ResBlock(192)).cuda() for _ in range(2)]
    units = [((m.conv[0], m.conv[2], m.conv[4]) if kind == 0 else (m.conv1, m.conv2, m.conv3))
             for m in mods]
    xs = [rt.to_nhwc(torch.randn((2, 192, 32, 64), device="cuda"), torch.bfloat16) for _ in mods]
    with torch.no_grad():
        got = [rt.to_nchw(o).float() for o in MA.run_bottlenecks_fused(list(zip(units, xs)), kind)]
        old = MA.STREAM
        MA.STREAM = False
        try:
            base = [rt.to_nchw(o).float() for o in MA.run_bottlenecks_fused(list(zip(units, xs)), kind)]
        finally:
            MA.STREAM = old
    for a, b in zip(got, base):
        scale = b.abs().max().item()
        frac = ((a - b).abs() > scale * 2.0 ** -8).float().mean().item()
        print(f"kind {kind}: max diff {(a - b).abs().max().item() / scale:.2e}, > 1 ulp {frac:.1e}")
        assert frac <= 1e-3, frac


@pytest.mark.parametrize("kind,B,H,W", [("ru", 1, 72, 136), ("rb", 1, 72, 136), ("ru", 4, 128, 128)])
def test_small_unit_two_tile_matches_one_tile(device, monkeypatch, kind, B, H, W):
    """ru_small_kernel<RB, 2> (multi-round C = 80 launches: two 4-wave halves per workgroup, each
    on its own tile over the shared LDS weights) against the one-tile form
    (RGBAC_RU_SMALL_DUAL=0) on two grouped units: identical per-tile arithmetic, so bit-identical;
    9 x 17 = 153 tiles leave the last workgroup's second half without a tile."""
    from rgbac import runtime as rt
    from rgbac.layers import Masked_Attention as MA
    from rgbac.models import AutoEncoderMask_Journal as AM
    torch.manual_seed(51)
    mods = [(MA.ResidualUnit(80) if kind == "ru" else AM.ResBlock(80)).cuda() for _ in range(2)]
    g = torch.Generator().manual_seed(52)
    xs = [rt.to_nhwc(torch.randn((B, 80, H, W), generator=g).cuda(), torch.bfloat16) for _ in mods]
    run = MA.run_residual_units if kind == "ru" else AM.run_resblocks
    outs = {}
    with torch.no_grad():
        for mode in ("0", "1"):
            monkeypatch.setenv("RGBAC_RU_SMALL_DUAL", mode)
            outs[mode] = [o.t.clone() for o in run(list(zip(mods, xs)))]
        torch.cuda.synchronize()
    for a, b in zip(outs["1"], outs["0"]):
        assert torch.equal(a.view(torch.int16), b.view(torch.int16))




# ---------------------------------------------------------------------------------------
# The last unit pair + gate of a C = 192 Win_noShift_Attention block in one launch
# (rgbac_residual_unit_gate, Masked_Attention.py:177-189) against the pair launch + the gate
# conv launch it replaces.  The b3 tile is rounded to bf16 in LDS exactly where the unfused
# path stores it, the gate GEMM runs the same MFMA k-step order and the epilogue the same
# arithmetic as conv_pw2_kernel's gate, so the block outputs agree bit for bit (bar: at most
# 1e-3 of the elements 1 bf16 ulp apart).  Shapes: config 2's encoder block (one round of
# workgroups), a multi-round grid (group-1 workgroups waiting on group-0 ones dispatched rounds
# earlier), a small odd grid; the hand-off words are left zero and the timeout word unset.
@pytest.mark.parametrize("B,H,W,masked", [(8, 64, 64, True), (4, 128, 128, True), (1, 24, 48, False),
                                          (2, 32, 32, True)])
def test_gated_last_unit_pair_matches_unfused(device, B, H, W, masked):
    from rgbac import runtime as rt
    from rgbac.layers import Masked_Attention as MA
    torch.manual_seed(31)
    m = MA.Win_noShift_Attention(192, num_heads=8, window_size=8, shift_size=4).cuda().eval()
    g = torch.Generator().manual_seed(32)
    x = torch.randn((B, 192, H, W), generator=g).cuda()
    mask = torch.ones((B, 1, H, W))
    if masked:
        mask[:, :, : H // 3, :] = 0.0
    mask = mask.cuda()
    with torch.no_grad():
        f = rt.to_nhwc(x, torch.bfloat16)
        assert MA.gated_ok(m, f, f, f)
        old = MA.GATE_FUSED
        try:
            MA.GATE_FUSED = False
            want = rt.to_nchw(m.nhwc(f, mask)).float()
            MA.GATE_FUSED = True
            gots = [rt.to_nchw(m.nhwc(f, mask)).float() for _ in range(2)]
        finally:
            MA.GATE_FUSED = old
    torch.cuda.synchronize()
    flags = MA.gate_flags(f.t.device, 1)
    assert int(flags.abs().sum().item()) == 0, "hand-off words left set (or a wait timed out)"
    for got in gots:
        diff = (got - want).abs()
        ulp = want.abs().clamp(min=2.0 ** -126) * 2.0 ** -7
        frac = (diff > 0).float().mean().item()
        print(f"gated {B}x{H}x{W}: differing fraction {frac:.2e}, max |d| {diff.max().item():.3e}")
        assert (diff <= ulp).all()
        assert frac <= 1e-3
