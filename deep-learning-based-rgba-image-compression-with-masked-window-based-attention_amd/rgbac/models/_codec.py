"""AutoEncoder.compress / decompress on the HIP path
(reference: models/AutoEncoderRGB_Journal.py:312-416).

Same dataflow as the reference, restructured like the forward's latent path (_latent.py):
  * the hyperprior and every slice stack run on the conv engine; concatenations are read
    in place (multi-source convs), y_hat slices land in one NHWC buffer YH;
  * the last cc_mean / cc_scale convs of a slice form one block-diagonal (mu | sigma) conv
    (act none), then ``rgbac_gauss_code`` does quantize("symbols") + build_indexes + y_q + mu
    (compress), or build_indexes, then dequantize after the host decoder ran (decompress);
  * slices >= max_support_slices see the same support, so they run as one wave; their
    symbols are contiguous in the stream in slice order, so decompress decodes the whole
    wave with one rANS call (one device->host index copy + one host->device symbol copy per
    wave instead of one per slice);
  * all conv tiles come from the fixed shape rule (rt.fixed_tiles): mu / sigma are then
    bit-identical between compress and decompress in any process, which the decoder needs
    (a CDF index computed from a scale that differs in the last bit desynchronises rANS).
The strings are compressai's: strings[0] = [one y string for the batch, slices in order,
NCHW within a slice] (:354-355,:367-369), strings[1] = one z string per image (:319).
"""
import torch

from .. import _lib
from .. import runtime as rt
from ..ans import BufferedRansEncoder, RansDecoder
from ..layers.SupplyMask import mask_pyramid
from ..layers.TransformRGB import prep_conv
from ._latent import _hyper_a, _hyper_s_pair, _musigma_pack


def _eb_code(eb, mode, f, sym, zhat):
    med = eb._get_medians().detach().reshape(-1).float().contiguous()
    _lib.call("rgbac_eb_code", _lib.dtype_code(zhat.t.dtype), mode, zhat.B, zhat.H, zhat.W,
              zhat.C, f.ptr() if f is not None else None, f.ldc if f is not None else 0,
              med.data_ptr(), sym.data_ptr(), zhat.ptr(), zhat.ldc,
              _lib.stream_ptr(zhat.t.device))
    return med


def _gauss_code(gc, mode, y, ycoff, ms, cs, sym, idx, pre):
    st = gc.scale_table.float().contiguous()
    bound = float(gc.lower_bound_scale.bound.item())
    _lib.call("rgbac_gauss_code", _lib.dtype_code(ms.t.dtype), mode, ms.B, ms.H, ms.W, cs,
              y.ptr(ycoff) if y is not None else None, y.ldc if y is not None else 0,
              ms.ptr(), ms.ldc, st.data_ptr(), st.numel(), bound, _lib.ptr(sym), _lib.ptr(idx),
              pre.ptr() if pre is not None else None, pre.ldc if pre is not None else 0,
              _lib.stream_ptr(ms.t.device))
    return st


def latent_code(model, y=None, z_sym=None, z_shape=None, y_decoder=None):
    """compress (y given): -> (YH, z_sym, y_sym, y_idx); decompress (z_sym + y_decoder
    given): -> (YH, z_sym, y_sym, y_idx) with y_sym decoded.  z_sym int32 (B, C, h, w) NCHW,
    y_sym / y_idx int32 (num_slices, B*cs*H*W) in the reference's stream order."""
    eb, gc = model.entropy_bottleneck, model.gaussian_conditional
    encode = y is not None
    ns, msup, M = model.num_slices, model.max_support_slices, model.M
    cs = M // ns
    with rt.fixed_tiles():
        if encode:
            dev, dt = y.t.device, y.t.dtype
            z = _hyper_a(model.h_a, y)
            B, zh, zw, C = z.B, z.H, z.W, z.C
            z_hat = rt.new_feat(B, zh, zw, C, dt, dev)
            z_sym = torch.empty((B, C, zh, zw), dtype=torch.int32, device=dev)
            _eb_code(eb, 0, z, z_sym, z_hat)
        else:
            dev, dt = z_sym.device, model.compute_dtype
            B, C, zh, zw = z_sym.shape
            z_hat = rt.new_feat(B, zh, zw, C, dt, dev)
            _eb_code(eb, 1, None, z_sym.contiguous(), z_hat)
        scales, means = _hyper_s_pair((model.h_scale_s, model.h_mean_s), z_hat)
        h, w = zh * 8, zw * 8                                   # :378
        if encode:
            assert (y.H, y.W) == (h, w)
        YH = rt.new_feat(B, h, w, M, dt, dev)
        n = B * cs * h * w
        y_sym = torch.empty((ns, n), dtype=torch.int32, device=dev)
        y_idx = torch.empty((ns, n), dtype=torch.int32, device=dev)
        waves = [[i] for i in range(min(msup, ns))]
        if ns > msup:
            waves.append(list(range(msup, ns)))
        tables = None if encode else gc.tables()
        for wave in waves:
            sup = [cs * min(i, msup) for i in wave]
            k = len(wave)
            t1 = rt.launch(
                [prep_conv(model.cc_mean_transforms[i][0], [means.src(), YH.src(0, s)], act="gelu")
                 for i, s in zip(wave, sup)] +
                [prep_conv(model.cc_scale_transforms[i][0], [scales.src(), YH.src(0, s)],
                           act="gelu") for i, s in zip(wave, sup)])
            t2 = rt.launch(
                [prep_conv(model.cc_mean_transforms[i][2], [t1[j].src()], act="gelu")
                 for j, i in enumerate(wave)] +
                [prep_conv(model.cc_scale_transforms[i][2], [t1[k + j].src()], act="gelu")
                 for j, i in enumerate(wave)])
            mss = rt.launch([rt.prepare(_musigma_pack(model.cc_mean_transforms[i][4],
                                                      model.cc_scale_transforms[i][4], dt,
                                                      t2[j].ldc),
                                        [t2[j].src(), t2[k + j].src()],
                                        out=rt.new_feat(B, h, w, 2 * cs, dt, dev))
                             for j, i in enumerate(wave)])
            pres = [rt.new_feat(B, h, w, cs, dt, dev) for _ in wave]
            if encode:
                for j, i in enumerate(wave):
                    _gauss_code(gc, 0, y, i * cs, mss[j], cs, y_sym[i], y_idx[i], pres[j])
            else:
                for j, i in enumerate(wave):
                    _gauss_code(gc, 1, None, 0, mss[j], cs, None, y_idx[i], None)
                lo, hi = wave[0], wave[-1] + 1
                idx_host = y_idx[lo:hi].cpu()                   # one sync per wave
                sym = y_decoder.decode_stream_np(idx_host.reshape(-1).numpy(), tables)
                y_sym[lo:hi].copy_(torch.from_numpy(sym).view(hi - lo, n))
                for j, i in enumerate(wave):
                    _gauss_code(gc, 2, None, 0, mss[j], cs, y_sym[i], None, pres[j])
            # lrp stacks: y_hat_i = (y_q + mu) + 0.5 * tanh(lrp([means, y_hat_<i, y_q + mu]))
            l1 = rt.launch([prep_conv(model.lrp_transforms[i][0],
                                      [means.src(), YH.src(0, s), pres[j].src()], act="gelu")
                            for j, (i, s) in enumerate(zip(wave, sup))])
            l2 = rt.launch([prep_conv(model.lrp_transforms[i][2], [l1[j].src()], act="gelu")
                            for j, i in enumerate(wave)])
            rt.launch([prep_conv(model.lrp_transforms[i][4], [l2[j].src()], out=YH,
                                 out_coff=i * cs, act="tanh_half", res1=pres[j])
                       for j, i in enumerate(wave)])
    return YH, z_sym, y_sym, y_idx


def _check(model, *ts):
    rt.check_gpu(*ts)
    model.gaussian_conditional._check_cdf()
    model.entropy_bottleneck._check_cdf()


def compress(model, input, mask):
    """:312-371 -> {"strings": [[y_string], z_strings], "shape": z spatial size}."""
    _check(model, input, mask)
    B, _, H, W = input.shape
    from .AutoEncoderRGB_Journal import check_geometry
    check_geometry(H, W)
    with torch.no_grad():
        xf = rt.to_nhwc(input.contiguous().float(), model.compute_dtype)
        _, me = mask_pyramid(mask, 4)                            # EncMakeMask(mask) (:314)
        y = model.Encoder.nhwc(xf, me[1], me[2])                 # :315
        _, z_sym, y_sym, y_idx = latent_code(model, y=y)
        z_host, ys_host, yi_host = z_sym.cpu(), y_sym.cpu(), y_idx.cpu()   # one sync
    eb = model.entropy_bottleneck
    C, zh, zw = z_host.shape[1:]
    z_idx = torch.arange(C, dtype=torch.int32).view(C, 1).expand(C, zh * zw).reshape(-1)
    z_tab = eb.tables()
    z_strings = []
    for b in range(B):                                           # EntropyBottleneck.compress
        enc = BufferedRansEncoder()
        enc.encode_with_indexes(z_host[b].reshape(-1), z_idx, z_tab)
        z_strings.append(enc.flush())
    enc = BufferedRansEncoder()                                  # :334,:367-368
    enc.encode_with_indexes(ys_host.reshape(-1), yi_host.reshape(-1),
                            model.gaussian_conditional.tables())
    return {"strings": [[enc.flush()], z_strings], "shape": torch.Size((zh, zw))}


def decompress(model, strings, shape, mask):
    """:373-416 -> {"x_hat": (B,3,H,W) clamped to [0, 1]}; B = len(strings[1])."""
    _check(model, mask)
    eb = model.entropy_bottleneck
    zh, zw = int(shape[0]), int(shape[1])
    B = len(strings[1])
    C = eb.channels
    z_idx = torch.arange(C, dtype=torch.int32).view(C, 1).expand(C, zh * zw).reshape(-1)
    z_tab = eb.tables()
    z_sym = torch.empty((B, C, zh, zw), dtype=torch.int32)
    for b, s in enumerate(strings[1]):                           # EntropyBottleneck.decompress
        dec = RansDecoder()
        dec.set_stream(s)
        z_sym[b] = torch.from_numpy(dec.decode_stream_np(z_idx, z_tab)).view(C, zh, zw)
    dec = RansDecoder()
    dec.set_stream(strings[0][0])                                # :387-388
    dev = mask.device
    with torch.no_grad():
        YH, _, _, _ = latent_code(model, z_sym=z_sym.to(dev), y_decoder=dec)
        _, md = mask_pyramid(mask, 4)                            # DecMakeMask(mask) (:412)
        xh = model.Decoder.nhwc(YH, md[1], md[2])                # :414
        x_hat = rt.to_nchw(xh).clamp_(0, 1)
    return {"x_hat": x_hat}
