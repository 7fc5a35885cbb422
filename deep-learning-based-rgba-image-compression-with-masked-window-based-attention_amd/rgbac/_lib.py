"""ctypes binding of librgbac_hip.so (the C ABI declared in include/rgbac.h).

The product path has no CPU or eager-PyTorch fallback: if the shared object is
missing or fails to load, every op raises.  Build it with
``python -c "import __graft_entry__ as g; g.build()"`` (or ``make -C csrc``).
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# RGBAC_LIB_PATH: an alternative build of the same library (A/B experiments)
LIB_PATH = os.environ.get("RGBAC_LIB_PATH") or os.path.join(_HERE, "librgbac_hip.so")

F32, BF16 = 0, 1
ACT = dict(none=0, gelu=1, relu=2, lrelu=3, tanh_half=4, gate=5, gdn=6, igdn=7, masksel=8,
           gauss=9, sqbwd=10, dgelu=11, dlrelu=12)
CONV, CONVT_S2, SUBPEL2 = 0, 1, 2


class Src(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("ldc", ctypes.c_int64),
                ("channels", ctypes.c_int32), ("_pad", ctypes.c_int32)]


class ConvArgs(ctypes.Structure):
    _fields_ = [
        ("dtype", ctypes.c_int32), ("mode", ctypes.c_int32),
        ("batch", ctypes.c_int32), ("in_h", ctypes.c_int32), ("in_w", ctypes.c_int32),
        ("ksize", ctypes.c_int32), ("stride", ctypes.c_int32),
        ("nsrc", ctypes.c_int32), ("src", Src * 3),
        ("cin_pad", ctypes.c_int32), ("k_pad", ctypes.c_int32),
        ("weight", ctypes.c_void_p), ("bias", ctypes.c_void_p),
        ("cout", ctypes.c_int32), ("cout_pad", ctypes.c_int32),
        ("out_h", ctypes.c_int32), ("out_w", ctypes.c_int32),
        ("out", ctypes.c_void_p), ("out_ldc", ctypes.c_int64),
        ("out_coff", ctypes.c_int32), ("act", ctypes.c_int32),
        ("act_param", ctypes.c_float), ("square_input", ctypes.c_int32),
        ("res0", ctypes.c_void_p), ("res0_ldc", ctypes.c_int64),
        ("res1", ctypes.c_void_p), ("res1_ldc", ctypes.c_int64),
        ("res2", ctypes.c_void_p), ("res2_ldc", ctypes.c_int64),
        ("sel", ctypes.c_void_p),
        ("tile", ctypes.c_int32), ("ksplit", ctypes.c_int32),
        ("workspace", ctypes.c_void_p),
        ("aux0", ctypes.c_void_p), ("aux1", ctypes.c_void_p), ("partial", ctypes.c_void_p),
        ("zout", ctypes.c_void_p), ("zout_ldc", ctypes.c_int64),
        ("tile_counters", ctypes.c_void_p),
    ]


class WgradArgs(ctypes.Structure):
    _fields_ = [
        ("dtype", ctypes.c_int32),
        ("batch", ctypes.c_int32), ("grid_h", ctypes.c_int32), ("grid_w", ctypes.c_int32),
        ("g", ctypes.c_void_p), ("g_ldc", ctypes.c_int64), ("g_channels", ctypes.c_int32),
        ("in_h", ctypes.c_int32), ("in_w", ctypes.c_int32), ("ksize", ctypes.c_int32),
        ("stride", ctypes.c_int32), ("pad", ctypes.c_int32),
        ("nsrc", ctypes.c_int32), ("cin_pad", ctypes.c_int32),
        ("src", Src * 3),
        ("square_input", ctypes.c_int32),
        ("n_pad", ctypes.c_int32), ("k_pad", ctypes.c_int32),
        ("nsplit", ctypes.c_int32),
        ("partial", ctypes.c_void_p), ("bias_partial", ctypes.c_void_p),
    ]


class RuArgs(ctypes.Structure):
    _fields_ = [
        ("dtype", ctypes.c_int32), ("channels", ctypes.c_int32), ("batch", ctypes.c_int32),
        ("h", ctypes.c_int32), ("w", ctypes.c_int32), ("_pad0", ctypes.c_int32),
        ("x", ctypes.c_void_p), ("x_ldc", ctypes.c_int64),
        ("w1", ctypes.c_void_p), ("w2", ctypes.c_void_p), ("w3", ctypes.c_void_p),
        ("w1_kpad", ctypes.c_int32), ("w2_kpad", ctypes.c_int32), ("w3_kpad", ctypes.c_int32),
        ("_pad1", ctypes.c_int32),
        ("b1", ctypes.c_void_p), ("b2", ctypes.c_void_p), ("b3", ctypes.c_void_p),
        ("out", ctypes.c_void_p), ("out_ldc", ctypes.c_int64),
    ]


class RansDecoderState(ctypes.Structure):
    """rgbac_rans_decoder_t"""
    _fields_ = [("state", ctypes.c_uint64), ("data", ctypes.c_void_p), ("size", ctypes.c_int64),
                ("pos", ctypes.c_int64)]


_VP, _I32, _I64, _F = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float
_D = ctypes.c_double
# name -> argtypes (restype int unless noted); must match include/rgbac.h
SIGNATURES = {
    "rgbac_abi_version": [],
    "rgbac_last_error": [],
    "rgbac_conv2d": [ctypes.POINTER(ConvArgs), _VP],
    "rgbac_conv_num_tiles": [],
    "rgbac_conv_tile_weight_layout": [ctypes.c_int],
    "rgbac_conv2d_grouped": [ctypes.c_void_p, _I32, _VP],
    "rgbac_conv2d_grouped_part": [ctypes.c_void_p, _I32, _I32, _VP],
    "rgbac_conv_max_groups": [],
    "rgbac_timer_create": [ctypes.POINTER(ctypes.c_void_p)],
    "rgbac_timer_record": [_VP, _VP],
    "rgbac_timer_elapsed_ms": [_VP, _VP, ctypes.POINTER(ctypes.c_float)],
    "rgbac_timer_destroy": [_VP],
    "rgbac_winattn_core": [_I32, _I32, _I32, _I32, _I32, _I32, _I32, _I32, _I32, _F,
                           _VP, _I64, _VP, _VP, _VP, _I64, _VP, _VP],
    "rgbac_winattn_core_ex": [_I32, _I32, _I32, _I32, _I32, _I32, _I32, _I32, _I32, _F,
                              _VP, _I64, _VP, _VP, _VP, _I64, _VP, _VP, _I32, _I32, _VP],
    "rgbac_gaussian_slice": [_I32, _I64, _I32, _VP, _I64, _VP, _I64, _VP, _I64, _VP,
                             _VP, _I64, _VP, _VP, _VP],
    "rgbac_eb_forward": [_I32, _I64, _I32, _VP, _I64, _VP, _VP, _VP, _I64, _VP, _VP, _VP],
    "rgbac_reduce_blocks": [_I64],
    "rgbac_finalize": [_I32, _I32, _I32, _I32, _I32, _I32, _VP, _VP, _I64, _VP, _VP, _I32,
                       _VP, _I32, _VP, _VP, _VP],
    "rgbac_finalize_blocks": [_I32, _I32],
    "rgbac_finalize_ex": [_I32, _I32, _I32, _I32, _I32, _I32, _VP, _VP, _I64, _VP, _VP, _I32,
                          _VP, _I32, _VP, _VP, _VP, _VP],
    "rgbac_forward_prologue": [_I32, _I32, _I32, _I32, _I32, _VP, _VP, _I64, _VP, _I32, _VP,
                               _I32, _VP, _VP, _I64, _VP],
    "rgbac_mask_pyramid": [_I32, _I32, _I32, _VP, _I32, _VP, _I32, _VP, _VP],
    "rgbac_nchw_to_nhwc": [_I32, _I32, _I32, _I32, _I32, _VP, _VP, _I64, _VP],
    "rgbac_nhwc_to_nchw": [_I32, _I32, _I32, _I32, _I32, _VP, _I64, _VP, _VP],
    "rgbac_residual_unit": [_VP, _I32, _VP],
    "rgbac_residual_unit_ex": [_VP, _I32, _I32, _VP],
    "rgbac_residual_unit_gate": [_VP, _VP, _VP, _VP, _I64, _VP, _I64, _VP],
    "rgbac_stem_gdn": [_I32, _I32, _I32, _VP, _I64, _VP, _I32, _VP, _VP, _I32, _VP, _I32, _VP,
                       _I64, _VP],
    "rgbac_winattn_block": [_I32, _I32, _I32, _I32, _I32, _F, _VP, _I64, _VP, _VP, _VP, _VP, _VP,
                            _VP, _I64, _VP, _I64, _VP],
    "rgbac_winattn_block_workspace": [_I32, _I32, _I32],
    "rgbac_gdn_reparam": [_I32, _I32, _VP, _VP, _F, _F, _F, _VP, _VP, _VP],
    "rgbac_gdn_reparam_bwd": [_I32, _I32, _VP, _VP, _F, _F, _VP, _VP, _VP, _VP, _I32, _VP],
    "rgbac_eb_params": [_I32, _VP, _VP, _VP],
    "rgbac_eb_params_bwd": [_I32, _VP, _VP, _VP, _I32, _VP],
    "rgbac_winattn_block_ws4": [_I32, _I32, _I32, _I32, _I32, _F, _VP, _I64, _VP, _VP, _VP, _VP,
                                _VP, _VP, _VP, _I64, _VP],
    "rgbac_rgba_augment": [_I32, _VP, _I32, _I32, _I32, _VP, _VP, _VP, _VP, _VP],
    "rgbac_dse_block": [_I32, _I32, _I32, _I32, _I32, _F, _VP, _I64, _VP, _I64, _VP, _I32, _VP, _VP,
                        _I32, _VP, _VP, _I32, _VP, _VP, _I32, _VP, _VP, _I64, _VP],
    # training step
    "rgbac_act_bwd": [_I32, _I32, _F, _I64, _I32, _VP, _I64, _VP, _I64, _VP, _I64, _VP, _VP,
                      _I64, _VP, _I64, _VP],
    "rgbac_conv_wgrad": [ctypes.POINTER(WgradArgs), _VP],
    "rgbac_wgrad_reduce": [_I64, _VP, _VP, _I32, _I64, _VP, _I32, _VP, _I32, _VP, _I32, _VP],
    "rgbac_wgrad_reduce_multi": [_I32, _VP, _VP],
    "rgbac_winattn_core_bwd": [_I32, _I32, _I32, _I32, _I32, _I32, _I32, _I32, _I32, _F, _VP,
                               _I64, _VP, _VP, _VP, _I64, _VP, _I64, _I32, _VP, _VP],
    "rgbac_winattn_core_bwd_ex": [_I32, _I32, _I32, _I32, _I32, _I32, _I32, _I32, _I32, _F,
                                  _VP, _I64, _VP, _VP, _VP, _I64, _VP, _I64, _I32, _VP, _VP,
                                  _I32, _VP],
    "rgbac_relpos_bwd": [_I32, _I32, _I32, _VP, _VP, _VP, _VP, _VP, _VP],
    "rgbac_gaussian_bwd": [_I32, _I64, _I32, _VP, _I64, _VP, _I64, _VP, _I64, _VP, _VP, _VP,
                           _I64, _VP, _I64, _VP, _I64, _VP, _I64, _VP],
    "rgbac_eb_bwd": [_I32, _I64, _I32, _VP, _I64, _VP, _VP, _VP, _VP, _I64, _VP, _I64, _VP, _VP],
    "rgbac_mse_bwd": [_I32, _I32, _I32, _I32, _I32, _I32, _VP, _VP, _I64, _VP, _VP, _VP, _VP,
                      _I64, _VP],
    "rgbac_adam_clamp": [_I64, _VP, _VP, _VP, _VP, _D, _D, _D, _D, _I64, _F, _F, _VP],
    "rgbac_adam_clamp_dstep": [_I64, _VP, _VP, _VP, _VP, _D, _D, _D, _D, _VP, _F, _F, _VP],
    "rgbac_pixel_shuffle": [_I32, _I32, _I32, _I32, _I32, _I32, _VP, _I64, _VP, _I64, _VP],
    "rgbac_channel_copy": [_I32, _I64, _I32, _VP, _I64, _I32, _VP, _I64, _I32, _VP],
    "rgbac_channel_copy_multi": [_I32, _I64, _I32, _VP, _VP],
    "rgbac_channel_copy_multi_ex": [_I32, _I64, _I32, _VP, _VP],
    "rgbac_weight_gather": [_I32, _I64, _VP, _VP, _VP, _VP],
    "rgbac_weight_gather_multi": [_I32, _VP, _VP, _I64, _VP],
    "rgbac_weight_repack_multi": [_I32, _VP, _VP, _I64, _VP],
    "rgbac_colsum": [_I32, _I64, _I32, _VP, _I64, _I32, _VP, _VP],
    "rgbac_sum_partials": [_I32, _I32, _VP, _VP, _VP],
    # bitstream (GPU symbol/index work + host rANS coder)
    "rgbac_gauss_code": [_I32, _I32, _I32, _I32, _I32, _I32, _VP, _I64, _VP, _I64, _VP, _I32, _F,
                         _VP, _VP, _VP, _I64, _VP],
    "rgbac_eb_code": [_I32, _I32, _I32, _I32, _I32, _I32, _VP, _I64, _VP, _VP, _VP, _I64, _VP],
    # RGBA eval pipeline (alpha recon -> RGB codec)
    "rgbac_alpha_recon": [_I32, _I32, _I32, _I32, _VP, _VP, _VP, _VP, _VP],
    "rgbac_rgba_finish": [_I64, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP],
    # MS-SSIM metric
    "rgbac_ssim_level": [_I32, _I32, _I32, _I32, _I32, _VP, _VP, _VP, _F, _F, _VP, _VP, _VP, _VP],
    "rgbac_avgpool2": [_I32, _I32, _I32, _VP, _VP, _VP],
    "rgbac_msssim_combine": [_I32, _I32, _VP, _VP, _VP, _VP, _VP, _VP],
    "rgbac_masked_apply": [_I32, _I32, _I32, _I32, _I32, _VP, _VP, _VP, _VP, _VP, _VP, _VP],
    "rgbac_masked_ssim_level": [_I32, _I32, _I32, _I32, _I32, _I32, _VP, _VP, _VP, _VP, _F, _F,
                                _VP, _VP, _VP, _VP],
    "rgbac_masked_msssim_combine": [_I32, _I32, _I32, _VP, _VP, _VP, _VP, _VP, _VP],
    "rgbac_pmf_to_quantized_cdf": [_VP, _I32, _I32, _VP],
    "rgbac_rans_encoder_create": [ctypes.POINTER(ctypes.c_void_p)],
    "rgbac_rans_encoder_destroy": [_VP],
    "rgbac_rans_encoder_put": [_VP, _VP, _VP, _I64, _VP, _I32, _VP, _VP, _I32],
    "rgbac_comm_load": [ctypes.c_char_p],
    "rgbac_comm_unique_id": [_VP],
    "rgbac_comm_init": [_VP, _I32, _I32, _I32, ctypes.POINTER(ctypes.c_void_p)],
    "rgbac_comm_allreduce_sum": [_VP, _I32, _VP, _I64, _VP],
    "rgbac_comm_destroy": [_VP],
    "rgbac_comm_count": [_VP, ctypes.POINTER(ctypes.c_int)],
    "rgbac_comm_async_error": [_VP, ctypes.POINTER(ctypes.c_int)],
    "rgbac_comm_abort": [_VP],
    "rgbac_rans_encoder_bound": [_VP],
    "rgbac_rans_encoder_flush": [_VP, _VP, _I64, ctypes.POINTER(ctypes.c_int64)],
    "rgbac_rans_decoder_init": [ctypes.POINTER(RansDecoderState), _VP, _I64],
    "rgbac_rans_decode": [ctypes.POINTER(RansDecoderState), _VP, _I64, _VP, _I32, _VP, _VP, _I32,
                          _VP],
}
_RESTYPE = {"rgbac_last_error": ctypes.c_char_p, "rgbac_rans_encoder_bound": ctypes.c_int64,
            "rgbac_winattn_block_workspace": ctypes.c_int64}

_lib = None


def load(path=LIB_PATH):
    """Load (once) and return the library; raises if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(
            f"rgbac: HIP library not found at {path}; build it first "
            "(make -C <pkg>/csrc or __graft_entry__.build()). There is no fallback path.")
    lib = ctypes.CDLL(path)
    for name, args in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = _RESTYPE.get(name, ctypes.c_int)
    _lib = lib
    return lib


def call(name, *args):
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.rgbac_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed ({rc}): {msg}")
    return rc


def finalize_scratch_doubles(batch, h, w):
    """Doubles of the rgbac_finalize / rgbac_finalize_ex scratch (rgbac_finalize_blocks)."""
    return batch * load().rgbac_finalize_blocks(h, w) * 2


def stream_ptr(device=None):
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t):
    return None if t is None else t.data_ptr()


def dtype_code(dt):
    if dt == torch.float32:
        return F32
    if dt == torch.bfloat16:
        return BF16
    raise ValueError(f"rgbac supports float32 and bfloat16 activations, got {dt}")
