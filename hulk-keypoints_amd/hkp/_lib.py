"""ctypes binding of libhulkkp.so (the C ABI declared in include/hulkkp.h).

This is the only place the product touches native code.  There is no CPU or
PyTorch fallback: if the library is missing or a call fails, it raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# the product loads its own in-tree library; A/B tooling may point this process at
# another build of the same ABI with use_library() before the first call
LIB_PATH = os.path.join(_HERE, "libhulkkp.so")

HKP_LAYOUT_NHWC = 0
HKP_LAYOUT_NCHW = 1
HKP_LOSS_BCE = 0
HKP_LOSS_MSE = 1


class HkpError(RuntimeError):
    pass


class ConvDesc(ctypes.Structure):
    """hkp_conv_desc; `tile` (HKP_TILE_*, default 0 = the planner) is per call."""
    _fields_ = [(n, ctypes.c_int32) for n in
                ("n", "h", "w", "c", "k", "r", "s", "stride", "pad", "dilation", "in_layout", "tile")]


# hkp_conv_desc.tile policies (include/hulkkp.h)
(HKP_TILE_AUTO, HKP_TILE_NO_SK, HKP_TILE_SK, HKP_TILE_256, HKP_TILE_128_MF16, HKP_TILE_128_MF32, HKP_TILE_64_PAIR,
 HKP_TILE_RESERVED_7, HKP_TILE_RESERVED_8, HKP_TILE_256_TAIL, HKP_TILE_HALO, HKP_TILE_256_A3, HKP_TILE_AUTO_A3,
 HKP_TILE_DUO, HKP_TILE_RESERVED_14, HKP_TILE_192_A3, HKP_TILE_160_A3) = range(17)
# hkp_conv_kernel_name ops
HKP_KOP_FWD_X3, HKP_KOP_DGRAD_X3, HKP_KOP_FWD_F16, HKP_KOP_STEM_X3, HKP_KOP_WGRAD_X3, HKP_KOP_FWD_X3_W16, \
    HKP_KOP_FWD_X3_X16, HKP_KOP_STEM_X3_IMAGE, HKP_KOP_STEM_X3_IMAGE_U8 = range(9)
HKP_X3_W16, HKP_X3_ALL, HKP_X3_X16 = 2, 3, 4          # hkp_conv2d_fwd_x3_products product sets


class PackJob(ctypes.Structure):
    """hkp_pack_job (hkp_weight_pack_x3_batch)."""
    _fields_ = [("w", ctypes.c_void_p), ("out", ctypes.c_void_p), ("inv_scale", ctypes.c_void_p),
                ("kind", ctypes.c_int32), ("k", ctypes.c_int32), ("rs", ctypes.c_int32), ("c", ctypes.c_int32),
                ("r", ctypes.c_int32), ("s", ctypes.c_int32), ("pad", ctypes.c_int32), ("phase", ctypes.c_int32)]


class AdamTensor(ctypes.Structure):
    """hkp_adam_tensor (hkp_adam_step)."""
    _fields_ = [("param", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p),
                ("exp_avg_sq", ctypes.c_void_p), ("n", ctypes.c_int64)]


_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_F = ctypes.c_float
_CD = ctypes.POINTER(ConvDesc)

# name -> (restype, argtypes); must cover every function include/hulkkp.h declares
SIGNATURES = {
    "hkp_last_error": (ctypes.c_char_p, []),
    "hkp_version": (ctypes.c_char_p, []),
    "hkp_conv_out_hw": (ctypes.c_int, [_CD, ctypes.POINTER(_I32), ctypes.POINTER(_I32)]),
    "hkp_conv_stat_tiles": (_I64, [_CD]),
    "hkp_conv_x3_stat_tile_rows": (_I32, [_CD, _I32]),
    "hkp_conv2d_fwd": (ctypes.c_int, [_CD, _P, _P, _P, _P, _P]),
    "hkp_bn_finalize": (ctypes.c_int, [_I32, _I64, _I64, _I32, _P, _P, _P, _F, _F, _P, _P, _P, _P, _P, _P]),
    "hkp_bn_finalize_workspace_bytes": (_I64, [_I32, _I64]),
    "hkp_bn_finalize_ws": (ctypes.c_int, [_I32, _I64, _I64, _I32, _P, _P, _P, _F, _F, _P, _P, _P, _P, _P, _P, _I64,
                                          _P]),
    "hkp_bn_stats": (ctypes.c_int, [_I32, _I64, _I64, _I32, _P, _P, _P, _I64, _P]),
    "hkp_bn_finalize_ranks": (ctypes.c_int, [_I32, _I32, _P, _P, _P, _F, _F, _P, _P, _P, _P, _P, _P]),
    "hkp_bn_eval_params": (ctypes.c_int, [_I32, _P, _P, _P, _P, _F, _P, _P, _P]),
    "hkp_bn_apply": (ctypes.c_int, [_I64, _I32, _P, _P, _P, _P, _P, _I32, _P, _P, _I32, _P]),
    "hkp_bn_apply_f16": (ctypes.c_int, [_I64, _I32, _P, _P, _P, _P, _I32, _P, _P, _P]),
    "hkp_bn_relu_maxpool": (ctypes.c_int, [_I32, _I32, _I32, _I32, _P, _P, _P, _P, _I32, _P, _P]),
    "hkp_head_fc": (ctypes.c_int, [_I32, _I32, _I32, _I32, _P, _P, _P, _P, _P]),
    "hkp_bn_apply_head": (ctypes.c_int, [_I32, _I32, _I32, _I32, _I32, _P, _P, _P, _P, _I32, _P, _P, _P, _P]),
    "hkp_upsample_sigmoid": (ctypes.c_int, [_I32, _I32, _I32, _I32, _I32, _I32, _I32, _P, _P, _P, _P, _P]),
    "hkp_gauss_target": (ctypes.c_int, [_I32, _I32, _I32, _I32, _F, _P, _P, _P]),
    "hkp_weight_pack_x3": (ctypes.c_int, [_I32, _I32, _I32, _P, _P, _P, _P]),
    "hkp_conv2d_fwd_x3": (ctypes.c_int, [_CD, _P, _P, _P, _P, _P, _P, _I64, _P]),
    "hkp_conv2d_fwd_x3_products": (ctypes.c_int, [_CD, _P, _P, _P, _I32, _P, _P, _P, _I64, _P]),
    "hkp_conv2d_fwd_x3_bnin": (ctypes.c_int, [_CD, _P, _P, _P, _P, _P, _P, _P, _I64, _P]),
    "hkp_conv2d_fwd_f16_bnin": (ctypes.c_int, [_CD, _P, _P, _P, _P, _P, _P, _P, _I64, _P]),
    "hkp_conv_x3_sk_workspace_bytes": (_I64, []),
    "hkp_absmax": (ctypes.c_int, [_I64, _P, _P, _P]),
    "hkp_weight_pack_f16": (ctypes.c_int, [_I32, _I32, _P, _P, _P, _P]),
    "hkp_conv2d_fwd_f16": (ctypes.c_int, [_CD, _P, _P, _P, _P, _P, _P, _I64, _P]),
    "hkp_conv2d_fwd_f16_bn": (ctypes.c_int, [_CD, _P, _P, _P, _P, _P, _P, _I32, _P, _P, _I64, _P]),
    "hkp_gram_f16_workspace_bytes": (_I64, [_I64, _I32]),
    "hkp_gram_f16": (ctypes.c_int, [_I64, _I32, _P, _P, _P, _P, _I64, _P]),
    "hkp_bn_from_gram_workspace_bytes": (_I64, [_I32, _I32]),
    "hkp_bn_from_gram": (ctypes.c_int, [_I32, _I32, _I64, _P, _P, _P, _P, _P, _P, _F, _F, _P, _P, _P, _P, _P, _P,
                                        _I64, _P]),
    "hkp_conv_kernel_name": (_I32, [_CD, _I32, _I32, ctypes.c_char_p, _I32]),
    "hkp_upsample_argmax_ws_bytes": (_I64, [_I32, _I32, _I32, _I32]),
    "hkp_stem_pack_x3_elems": (_I64, [_CD]),
    "hkp_stem_pack_x3": (ctypes.c_int, [_CD, _P, _P, _P]),
    "hkp_stem_pack_x3_u8": (ctypes.c_int, [_CD, _P, _P, _P]),
    "hkp_images_u8_to_nchw": (ctypes.c_int, [_I32, _I32, _I32, _I32, _P, _P, _P]),
    "hkp_soft_argmax": (ctypes.c_int, [_I32, _I32, _I32, _I32, _F, _P, _P, _P]),
    "hkp_heat_overlay": (ctypes.c_int, [_I32, _I32, _I32, _I32, _P, _P, _P, _P, _P, _P]),
    "hkp_stem_weight_pack_x3": (ctypes.c_int, [_I32, _I32, _P, _P, _P, _P]),
    "hkp_conv2d_fwd_stem_x3": (ctypes.c_int, [_CD, _P, _P, _P, _P, _P, _P]),
    "hkp_stem_x3_image_ok": (_I32, [_CD]),
    "hkp_conv2d_fwd_stem_x3_image": (ctypes.c_int, [_CD, _P, _I32, _P, _P, _P, _P, _P]),
    "hkp_split_pack_x3": (ctypes.c_int, [_I64, _I32, _P, _P, _P, _P]),
    "hkp_weight_flip_pack_x3": (ctypes.c_int, [_CD, _P, _P, _P, _P]),
    "hkp_conv2d_bwd_data_x3": (ctypes.c_int, [_CD, _P, _P, _P, _P, _P, _P, _P, _I64, _P]),
    "hkp_phase_taps": (_I32, [_I32, _I32, _I32, _I32]),
    "hkp_conv2d_bwd_data_x3_strided": (ctypes.c_int, [_CD, _P, ctypes.POINTER(_P), ctypes.POINTER(_P), _P, _P, _P,
                                                       _P, _I64, _P]),
    "hkp_weight_pack_x3_batch_ws_bytes": (_I64, [_I32, ctypes.POINTER(PackJob)]),
    "hkp_weight_pack_x3_batch": (ctypes.c_int, [_I32, ctypes.POINTER(PackJob), _P, _I64, _P]),
    "hkp_conv_bwd_filter_x3_workspace": (_I64, [_CD]),
    "hkp_conv2d_bwd_filter_x3": (ctypes.c_int, [_CD, _P, _P, _P, _P, _P, _I64, _P]),
    "hkp_adam_step": (ctypes.c_int, [_I32, ctypes.POINTER(AdamTensor), _F, _F, _F, _F, _F, _F, _F, _P]),
    # backward
    "hkp_conv_weight_flip":(ctypes.c_int, [_CD, _P, _P, _P]),
    "hkp_conv2d_bwd_data": (ctypes.c_int, [_CD, _P, _P, _P, _P, _P]),
    "hkp_conv_bwd_filter_workspace": (_I64, [_CD]),
    "hkp_conv2d_bwd_filter": (ctypes.c_int, [_CD, _P, _P, _P, _I32, _P, _I64, _P]),
    "hkp_bn_bwd_tiles": (_I64, [_I64]),
    "hkp_bn_bwd_reduce": (ctypes.c_int, [_I64, _I32, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "hkp_bn_bwd_finalize": (ctypes.c_int, [_I32, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "hkp_bn_bwd_stats": (ctypes.c_int, [_I32, _I64, _P, _P, _P, _P, _P]),
    "hkp_bn_bwd_finalize_ranks": (ctypes.c_int, [_I32, _I32, _P, _P, _I32, _P, _P, _P, _P, _P, _P, _P]),
    "hkp_bn_bwd_apply": (ctypes.c_int, [_I64, _I32, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "hkp_maxpool_bwd": (ctypes.c_int, [_I32, _I32, _I32, _I32, _P, _P, _P, _P]),
    "hkp_heat_loss_workspace": (_I64, []),
    "hkp_heat_loss": (ctypes.c_int, [_I32, _I32, _I32, _I32, _I32, _P, _P, _P, _F, _P, _P, _P, _P]),
    "hkp_head_bwd_workspace": (_I64, [_I32, _I32, _I32, _I32]),
    "hkp_head_bwd": (ctypes.c_int, [_I32, _I32, _I32, _I32, _I32, _I32, _P, _P, _P, _P, _I64, _P]),
    "hkp_head_fc_bwd_workspace": (_I64, [_I32, _I32, _I32, _I32]),
    "hkp_head_fc_bwd": (ctypes.c_int, [_I32, _I32, _I32, _I32, _P, _P, _P, _P, _P, _P, _P, _I64, _P]),
    # hybrid JPEG decode, device half (the geometry struct: hkp.jpeg.Geom)
    "hkp_jpeg_planes_bytes": (_I64, [_P]),
    "hkp_jpeg_reconstruct": (ctypes.c_int, [_I32, _P, _P, _P, _P, _I64, _P, _P]),
}

# the A/B instruments of the tools-only build (include/hulkkp_ab.h, `make ab`);
# bound only when the loaded library exports them — the product library does not
AB_SIGNATURES = {
    "hkp_debug_x3_stamps": (None, [_P]),
    "hkp_debug_x3_stagger": (None, [_I32]),
    "hkp_debug_x3_split_tail": (None, [_I32]),
    "hkp_debug_stem_pair": (None, [_I32]),
    "hkp_debug_fin_regs": (None, [_I32]),
    "hkp_debug_x3_pair128": (None, [_I32]),
    "hkp_debug_x3_store": (None, [_I32]),
    "hkp_debug_duo_stagger": (None, [_I32]),
    "hkp_debug_x3_prio": (None, [_I32]),
    "hkp_debug_x3_a_wrap": (None, [_I32]),
}
AB_LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "tools", "ab_lib", "libhulkkp_ab.so")

_lib = None


def use_library(path):
    """Tools only (in-process A/B of two builds): load `path` instead of the in-tree
    library.  Must run before the first kernel call of the process."""
    global LIB_PATH
    if _lib is not None:
        raise HkpError("use_library: %s is already loaded" % LIB_PATH)
    LIB_PATH = path


def use_ab_library():
    """Tools only: load the A/B build (tools/ab_lib/libhulkkp_ab.so, `make -C
    hulk-keypoints_amd/csrc ab`), whose hkp_debug_* knobs the product library lacks."""
    if not os.path.exists(AB_LIB_PATH):
        raise HkpError("the A/B build is missing (%s): run `make -C hulk-keypoints_amd/csrc ab`" % AB_LIB_PATH)
    use_library(AB_LIB_PATH)


def lib():
    """Load libhulkkp.so once; raise HkpError (never fall back) if it is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise HkpError("libhulkkp.so is not built (%s); run `python -c 'import __graft_entry__ as g; g.build()'`"
                           % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        other = os.path.abspath(LIB_PATH) != os.path.join(_HERE, "libhulkkp.so")
        for name, (res, args) in SIGNATURES.items():
            if other and not hasattr(L, name):
                continue                # tools: an older build of the ABI (its missing calls raise if used)
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        for name, (res, args) in AB_SIGNATURES.items():
            if hasattr(L, name):
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
        _lib = L
    return _lib


def call(name, *args):
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        msg = lib().hkp_last_error().decode(errors="replace")
        raise HkpError("%s failed (rc=%d): %s" % (name, rc, msg))
    return rc


def version():
    return lib().hkp_version().decode()
