import os, sys, torch
sys.path[:0] = ["/root/repo", "/root/repo/deep-learning-based-rgba-image-compression-with-masked-window-based-attention_amd"]
from rgbac import runtime as rt
from rgbac.layers.masked_win_attention import WinBasedAttention
for (B,H,W,shift,kind) in [(2,64,64,4,"quarter"),(2,64,64,0,"quarter"),(1,32,48,0,"ones"),(2,64,64,0,"ones")]:
    torch.manual_seed(21)
    m = WinBasedAttention(192, 8, 8, shift).cuda().eval()
    with torch.no_grad():
        m.attn.relative_position_bias_table.normal_(0, 0.5)
    x = torch.randn((B,192,H,W), device="cuda")
    al = torch.ones((B,1,H,W), device="cuda")
    if kind == "quarter": al[:, :, :H//2, :W//2] = 0
    with torch.no_grad():
        f = rt.to_nhwc(x, torch.bfloat16)
        o3 = rt.to_nchw(m.attn.run_block(f, al, shift, True)).float()
        os.environ["RGBAC_WINBLOCK_V2"] = "1"
        o2 = rt.to_nchw(m.attn.run_block(f, al, shift, True)).float()
        os.environ.pop("RGBAC_WINBLOCK_V2")
    d = (o3 - o2).abs() > 0
    pix = d.any(1)  # B,H,W
    print(B,H,W,shift,kind, "diff frac", d.float().mean().item(), "pixels", pix.float().mean().item())
    if pix.any():
        # shifted-frame window index of each differing pixel
        bs, ys, xs = torch.nonzero(pix, as_tuple=True)
        ws = set()
        for b_, y_, x_ in zip(bs.tolist(), ys.tolist(), xs.tolist()):
            ry, rx = (y_ - shift) % H, (x_ - shift) % W
            ws.add((b_, ry // 8, rx // 8))
        print("  windows", sorted(ws)[:40], len(ws))
        print("  channel frac among diff pixels", d.permute(0,2,3,1)[pix].float().mean().item())
