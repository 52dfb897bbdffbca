"""Tensor-level wrappers over the C ABI (one function per kernel family).

Every wrapper validates device/dtype/contiguity/shape on the host BEFORE the
launch (a mis-shaped launch can fault the GPU), launches on PyTorch's current
stream, and allocates outputs with the caching allocator.  No fallback path.
"""
import ctypes

import torch

from ._lib import (HKP_KOP_DGRAD_X3, HKP_KOP_FWD_F16, HKP_KOP_FWD_X3, HKP_KOP_FWD_X3_W16, HKP_KOP_FWD_X3_X16,
                   HKP_KOP_STEM_X3, HKP_KOP_STEM_X3_IMAGE, HKP_KOP_STEM_X3_IMAGE_U8, HKP_KOP_WGRAD_X3, HKP_X3_ALL,
                   HKP_LAYOUT_NCHW, HKP_LAYOUT_NHWC, HKP_TILE_160_A3, HKP_TILE_192_A3, ConvDesc, HkpError, call)

CONV_TILE_ROWS = 128  # BM of conv_fwd.hip (rows per BN statistic tile)

# Optional launch observer (bench.py's roofline timer): called as
# observer(kernel_symbol, algorithmic_flops, algorithmic_bytes, launch_fn).
_observer = None


def set_observer(fn):
    global _observer
    _observer = fn


def conv_kernel_symbol(layout, cout):
    bn = 128 if cout % 128 == 0 else 64
    return "conv_fwd_kernel<128, %d, %s>" % (bn, "true" if layout != "nhwc" else "false")


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


# Stream-K workspace of the x3 convs, one per (device, stream): zeroed once (its
# arrival counters must start at zero; every launch leaves them zero).  Launches
# sharing one stream never run concurrently, as the workspace requires.
_sk_ws = {}


def _sk_workspace(enable=True):
    from ._lib import lib
    if not enable:
        return ctypes.c_void_p(0), ctypes.c_int64(0)
    st = torch.cuda.current_stream()
    key = (st.device_index, st.cuda_stream)
    ws = _sk_ws.get(key)
    if ws is None:
        nb = lib().hkp_conv_x3_sk_workspace_bytes()
        ws = torch.zeros(nb, device=torch.device("cuda", st.device_index), dtype=torch.uint8)
        _sk_ws[key] = ws
    return ctypes.c_void_p(ws.data_ptr()), ctypes.c_int64(ws.numel())


def _ptr(t):
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def _need(t, dtype, name, ndim=None):
    if not isinstance(t, torch.Tensor):
        raise HkpError("%s: expected a tensor" % name)
    if t.device.type != "cuda":
        raise HkpError("%s: tensor must be on the GPU (got %s)" % (name, t.device))
    if t.dtype != dtype:
        raise HkpError("%s: expected %s, got %s" % (name, dtype, t.dtype))
    if not t.is_contiguous():
        raise HkpError("%s: tensor must be contiguous" % name)
    if ndim is not None and t.dim() != ndim:
        raise HkpError("%s: expected %d dims, got %s" % (name, ndim, tuple(t.shape)))


def conv_out_hw(h, w, r, s, stride, pad, dil):
    return ((h + 2 * pad - dil * (r - 1) - 1) // stride + 1, (w + 2 * pad - dil * (s - 1) - 1) // stride + 1)


def conv2d_fwd(x, w, stride=1, pad=0, dil=1, layout="nhwc", stats=True, out=None):
    """x NHWC [N,H,W,C] (or NCHW for the stem) fp32; w KRSC [K,R,S,C] (stem: OIHW).

    Returns (y NHWC [N,Ho,Wo,K], partials [tiles,K,2] or None)."""
    _need(x, torch.float32, "conv2d_fwd.x", 4)
    _need(w, torch.float32, "conv2d_fwd.w", 4)
    if layout == "nhwc":
        n, h, wd, c = x.shape
        k, r, s, cw = w.shape
        lay = HKP_LAYOUT_NHWC
    else:
        n, c, h, wd = x.shape
        k, cw, r, s = w.shape
        lay = HKP_LAYOUT_NCHW
    if cw != c:
        raise HkpError("conv2d_fwd: weight Cin %d != input C %d" % (cw, c))
    ho, wo = conv_out_hw(h, wd, r, s, stride, pad, dil)
    d = ConvDesc(n, h, wd, c, k, r, s, stride, pad, dil, lay)
    y = out if out is not None else torch.empty((n, ho, wo, k), device=x.device, dtype=torch.float32)
    _need(y, torch.float32, "conv2d_fwd.y", 4)
    if tuple(y.shape) != (n, ho, wo, k):
        raise HkpError("conv2d_fwd: out shape %s != %s" % (tuple(y.shape), (n, ho, wo, k)))
    part = None
    if stats:
        tiles = (n * ho * wo + CONV_TILE_ROWS - 1) // CONV_TILE_ROWS
        part = torch.empty((tiles, k, 2), device=x.device, dtype=torch.float32)
    def launch():
        call("hkp_conv2d_fwd", ctypes.byref(d), _ptr(x), _ptr(w), _ptr(y), _ptr(part), _stream())

    if _observer is None:
        launch()
    else:
        flops = 2.0 * n * ho * wo * k * r * s * c
        _observer(conv_kernel_symbol(layout, k), flops, 4.0 * (x.numel() + w.numel() + y.numel()), launch)
    return y, part


class PackedWeight(tuple):
    """(split, inv_scale): a weight in the packed split layout (fp16, each output
    channel scaled by a power of two) and the per-output-channel inverse scales."""

    def __new__(cls, split, inv_scale):
        return super().__new__(cls, (split, inv_scale))

    @property
    def split(self):
        return self[0]

    @property
    def inv_scale(self):
        return self[1]


def kernel_name(d, op, sk=True):
    """The kernel symbol a launch with ConvDesc d runs (hkp_conv_kernel_name: the
    launcher's own tile choice, so the name cannot drift from what runs)."""
    from ._lib import lib
    buf = ctypes.create_string_buffer(128)
    n = lib().hkp_conv_kernel_name(ctypes.byref(d), op, int(bool(sk)), buf, 128)
    if n < 0:
        raise HkpError("hkp_conv_kernel_name failed: %s" % lib().hkp_last_error().decode(errors="replace"))
    return buf.value.decode()


def weight_pack_x3(w):
    """fp32 KRSC weight → PackedWeight: [K, R, S, 2C] fp16 ([..][C/32][hi32|lo32]) + [K] scales."""
    _need(w, torch.float32, "weight_pack_x3.w", 4)
    k, r, s, c = w.shape
    ws = torch.empty((k, r, s, 2 * c), device=w.device, dtype=torch.float16)
    sc = torch.empty(k, device=w.device, dtype=torch.float32)
    call("hkp_weight_pack_x3", k, r * s * c, c, _ptr(w), _ptr(ws), _ptr(sc), _stream())
    return PackedWeight(ws, sc)


def split_of(x):
    """(split tensor, passes) of an activation: x itself when it IS a split-only
    activation (fp16), else the split a producer attached to fp32 x, else None."""
    if x.dtype == torch.float16:
        return x, x._hkp_split_passes
    return getattr(x, "_hkp_split", None)


def channels_of(x):
    """Channel count of an fp32 activation or of a split-only one."""
    if x.dtype == torch.float16 and x._hkp_split_passes == 3:
        return x.shape[-1] // 2
    return x.shape[-1]


def _stat_partials(n_rows, k, device, part_out, name, tile_rows=CONV_TILE_ROWS):
    """BN tile partials [tiles, k, 2] of an n_rows-pixel conv output, tile_rows rows
    per tile: part_out (a caller's slice of a larger buffer) or a new tensor.  A
    tile size other than CONV_TILE_ROWS rides on the tensor (_hkp_tile_rows) to
    bn_finalize / bn_stats."""
    tiles = (n_rows + tile_rows - 1) // tile_rows
    if part_out is None:
        part = torch.empty((tiles, k, 2), device=device, dtype=torch.float32)
    else:
        _need(part_out, torch.float32, name, 3)
        if tuple(part_out.shape) != (tiles, k, 2):
            raise HkpError("%s: shape %s != %s" % (name, tuple(part_out.shape), (tiles, k, 2)))
        part = part_out
    if tile_rows != CONV_TILE_ROWS:
        part._hkp_tile_rows = tile_rows
    return part


def stat_tile_rows(part):
    """Rows per BN statistic tile of conv partials (hkp_conv_x3_stat_tile_rows)."""
    return getattr(part, "_hkp_tile_rows", CONV_TILE_ROWS)


def conv2d_fwd_x3(xs, wp, stride=1, pad=0, dil=1, stats=True, out=None, part_out=None, sk=True, tile=0,
                  products=HKP_X3_ALL):
    """f16x3 NHWC conv on packed split operands: xs [N,H,W,2C] (from a producer with
    split=3), wp = weight_pack_x3(w) → fp32 y [N,Ho,Wo,K] (+ BN partials, into
    part_out when given).  sk=False: never stream-K (one tile per block);
    tile: HKP_TILE_* policy (0 = the planner); products: HKP_X3_ALL (f16x3), or
    HKP_X3_W16 / HKP_X3_X16 (two of the three products: the weights / the
    activation at fp16, hkp_conv2d_fwd_x3_products)."""
    ws, wsc = wp
    _need(xs, torch.float16, "conv2d_fwd_x3.x_split", 4)
    _need(ws, torch.float16, "conv2d_fwd_x3.w_split", 4)
    _need(wsc, torch.float32, "conv2d_fwd_x3.w_inv_scale", 1)
    n, h, wd, c2 = xs.shape
    k, r, s, cw2 = ws.shape
    if cw2 != c2:
        raise HkpError("conv2d_fwd_x3: weight Cin %d != input C %d" % (cw2 // 2, c2 // 2))
    c = c2 // 2
    ho, wo = conv_out_hw(h, wd, r, s, stride, pad, dil)
    d = ConvDesc(n, h, wd, c, k, r, s, stride, pad, dil, HKP_LAYOUT_NHWC, tile)
    y = out if out is not None else torch.empty((n, ho, wo, k), device=xs.device, dtype=torch.float32)
    kop = HKP_KOP_FWD_X3 if products == HKP_X3_ALL else HKP_KOP_FWD_X3_W16 if products == 2 else HKP_KOP_FWD_X3_X16
    part = None
    if stats:
        rows = CONV_TILE_ROWS
        if tile in (HKP_TILE_192_A3, HKP_TILE_160_A3):      # 96- / 80-row statistic tiles (the library says)
            from ._lib import lib
            rows = lib().hkp_conv_x3_stat_tile_rows(ctypes.byref(d), kop)
        part = _stat_partials(n * ho * wo, k, xs.device, part_out, "conv2d_fwd_x3.part_out", rows)

    if products == HKP_X3_ALL:
        def launch():
            call("hkp_conv2d_fwd_x3", ctypes.byref(d), _ptr(xs), _ptr(ws), _ptr(wsc), _ptr(y), _ptr(part),
                 *_sk_workspace(sk), _stream())
    else:
        def launch():
            call("hkp_conv2d_fwd_x3_products", ctypes.byref(d), _ptr(xs), _ptr(ws), _ptr(wsc), int(products),
                 _ptr(y), _ptr(part), *_sk_workspace(sk), _stream())

    if _observer is None:
        launch()
    else:
        _observer(kernel_name(d, kop, sk), 2.0 * n * ho * wo * k * r * s * c,
                  2.0 * (xs.numel() + ws.numel()) + 4.0 * y.numel(), launch)
    return y, part


def bnin_kernel(n, h, w, c, k, r, s, stride, pad, dil, f16=False, tile=0, sk=True):
    """The kernel a fused-input-BN conv (hkp_conv2d_fwd_x3_bnin / _f16_bnin) of this
    shape runs, or None where it has none: the fused conv runs where the unfused
    one runs the halo-tile body (conv_x3_halo_bnin_kernel<P>) — the same tiles
    and summation order, so the same bits."""
    cg = 64 if f16 else 32
    if c % cg or k % 64:
        return None
    try:
        ho, wo = conv_out_hw(h, w, r, s, stride, pad, dil)
    except HkpError:
        return None
    d = ConvDesc(n, h, w, c, k, r, s, stride, pad, dil, HKP_LAYOUT_NHWC, tile)
    name = kernel_name(d, HKP_KOP_FWD_F16 if f16 else HKP_KOP_FWD_X3, sk)
    if name.startswith("conv_x3_halo_kernel<"):
        return name.replace("_kernel<", "_bnin_kernel<")
    return None


def conv2d_fwd_bnin(y_in, in_ss, wp, stride=1, pad=1, dil=1, stats=True, sk=True, tile=0):
    """Inference conv whose input is the producer conv's raw output y_in with the
    producer's BN + ReLU applied inside the conv (hkp_conv2d_fwd_x3_bnin for fp32
    y_in with wp = weight_pack_x3(w); hkp_conv2d_fwd_f16_bnin for fp16 y_in with
    wp = weight_pack_f16(w)): the same y (and BN partials) as
    conv2d_fwd_x3(bn_apply(y_in, in_ss, relu, split=3)) / conv2d_fwd_f16(
    bn_apply_f16(y_in, in_ss, relu)) with the same sk / tile, bit for bit, without
    the apply pass (shapes: bnin_kernel)."""
    ws, wsc = wp
    f16 = y_in.dtype == torch.float16
    _need(y_in, torch.float16 if f16 else torch.float32, "conv2d_fwd_bnin.y_in", 4)
    _need(in_ss, torch.float32, "conv2d_fwd_bnin.in_scale_shift", 1)
    _need(ws, torch.float16, "conv2d_fwd_bnin.w", 4)
    n, h, wd, c = y_in.shape
    k, r, s, cw = ws.shape
    if cw != (c if f16 else 2 * c):
        raise HkpError("conv2d_fwd_bnin: weight Cin %d != input C %d" % (cw if f16 else cw // 2, c))
    if in_ss.numel() != 2 * c:
        raise HkpError("conv2d_fwd_bnin: in_scale_shift size %d != 2C" % in_ss.numel())
    ho, wo = conv_out_hw(h, wd, r, s, stride, pad, dil)
    d = ConvDesc(n, h, wd, c, k, r, s, stride, pad, dil, HKP_LAYOUT_NHWC, tile)
    y = torch.empty((n, ho, wo, k), device=y_in.device, dtype=torch.float16 if f16 else torch.float32)
    part = _stat_partials(n * ho * wo, k, y_in.device, None, "conv2d_fwd_bnin") if stats else None
    fn = "hkp_conv2d_fwd_f16_bnin" if f16 else "hkp_conv2d_fwd_x3_bnin"

    def launch():
        call(fn, ctypes.byref(d), _ptr(y_in), _ptr(in_ss), _ptr(ws), _ptr(wsc), _ptr(y), _ptr(part),
             *_sk_workspace(sk), _stream())

    if _observer is None:
        launch()
    else:
        name = kernel_name(d, HKP_KOP_FWD_F16 if f16 else HKP_KOP_FWD_X3, sk).replace("_kernel<", "_bnin_kernel<")
        _observer(name, 2.0 * n * ho * wo * k * r * s * c,
                  y_in.element_size() * y_in.numel() + 2.0 * ws.numel() + y.element_size() * y.numel(), launch)
    return y, part


def weight_pack_f16(w):
    """fp32 KRSC weight → PackedWeight: [K, R, S, C] fp16 (each output channel scaled
    by a power of two) + [K] inverse scales — the plain-fp16 conv's operand."""
    _need(w, torch.float32, "weight_pack_f16.w", 4)
    k, r, s, c = w.shape
    out = torch.empty((k, r, s, c), device=w.device, dtype=torch.float16)
    sc = torch.empty(k, device=w.device, dtype=torch.float32)
    call("hkp_weight_pack_f16", k, r * s * c, _ptr(w), _ptr(out), _ptr(sc), _stream())
    return PackedWeight(out, sc)


def conv2d_fwd_f16(x16, wp, stride=1, pad=0, dil=1, stats=True, sk=True, tile=0):
    """Plain-fp16 NHWC conv (BASELINE config C4): x16 fp16 [N,H,W,C] (a producer's
    split=1 output), wp = weight_pack_f16(w) → y fp16 [N,Ho,Wo,K] (autocast
    semantics) + BN partials from the fp32 accumulators."""
    ws, wsc = wp
    _need(x16, torch.float16, "conv2d_fwd_f16.x", 4)
    _need(ws, torch.float16, "conv2d_fwd_f16.w", 4)
    _need(wsc, torch.float32, "conv2d_fwd_f16.w_inv_scale", 1)
    n, h, wd, c = x16.shape
    k, r, s, cw = ws.shape
    if cw != c:
        raise HkpError("conv2d_fwd_f16: weight Cin %d != input C %d" % (cw, c))
    ho, wo = conv_out_hw(h, wd, r, s, stride, pad, dil)
    d = ConvDesc(n, h, wd, c, k, r, s, stride, pad, dil, HKP_LAYOUT_NHWC, tile)
    y = torch.empty((n, ho, wo, k), device=x16.device, dtype=torch.float16)
    part = _stat_partials(n * ho * wo, k, x16.device, None, "conv2d_fwd_f16") if stats else None

    def launch():
        call("hkp_conv2d_fwd_f16", ctypes.byref(d), _ptr(x16), _ptr(ws), _ptr(wsc), _ptr(y), _ptr(part),
             *_sk_workspace(sk), _stream())

    if _observer is None:
        launch()
    else:
        _observer(kernel_name(d, HKP_KOP_FWD_F16, sk), 2.0 * n * ho * wo * k * r * s * c,
                  2.0 * (x16.numel() + ws.numel() + y.numel()), launch)
    return y, part


def conv2d_fwd_f16_bn(x16, wp, ss, res=None, res_ss=None, relu=True, stride=1, pad=0, dil=1, sk=True, tile=0):
    """conv2d_fwd_f16 with the output's BN apply fused into the epilogue
    (hkp_conv2d_fwd_f16_bn): fp16 out = [relu](y*scale + shift [+ res | + res*rscale
    + rshift]) — what conv2d_fwd_f16 + bn_apply_f16 return with the same ss, y
    never written.  ss [2K] must be known before the conv (bn_from_gram, or
    eval-mode BN).  Returns the fp16 activation (a split=1 operand)."""
    ws, wsc = wp
    _need(x16, torch.float16, "conv2d_fwd_f16_bn.x", 4)
    _need(ws, torch.float16, "conv2d_fwd_f16_bn.w", 4)
    _need(wsc, torch.float32, "conv2d_fwd_f16_bn.w_inv_scale", 1)
    _need(ss, torch.float32, "conv2d_fwd_f16_bn.scale_shift", 1)
    n, h, wd, c = x16.shape
    k, r, s_, cw = ws.shape
    if cw != c:
        raise HkpError("conv2d_fwd_f16_bn: weight Cin %d != input C %d" % (cw, c))
    if ss.numel() != 2 * k:
        raise HkpError("conv2d_fwd_f16_bn: scale_shift size %d != 2K" % ss.numel())
    ho, wo = conv_out_hw(h, wd, r, s_, stride, pad, dil)
    if res is not None:
        _need(res, torch.float16, "conv2d_fwd_f16_bn.res", 4)
        if tuple(res.shape) != (n, ho, wo, k):
            raise HkpError("conv2d_fwd_f16_bn: residual %s != %s" % (tuple(res.shape), (n, ho, wo, k)))
    if res_ss is not None:
        _need(res_ss, torch.float32, "conv2d_fwd_f16_bn.res_scale_shift", 1)
        if res is None or res_ss.numel() != 2 * k:
            raise HkpError("conv2d_fwd_f16_bn: res_scale_shift needs a residual and 2K entries")
    d = ConvDesc(n, h, wd, c, k, r, s_, stride, pad, dil, HKP_LAYOUT_NHWC, tile)
    out = _split_out((n, ho, wo, k), x16.device, 1)

    def launch():
        call("hkp_conv2d_fwd_f16_bn", ctypes.byref(d), _ptr(x16), _ptr(ws), _ptr(wsc), _ptr(ss), _ptr(res),
             _ptr(res_ss), int(bool(relu)), _ptr(out), *_sk_workspace(sk), _stream())

    if _observer is None:
        launch()
    else:
        _observer(kernel_name(d, HKP_KOP_FWD_F16, sk), 2.0 * n * ho * wo * k * r * s_ * c,
                  2.0 * (x16.numel() + ws.numel() + out.numel() + (res.numel() if res is not None else 0)), launch)
    return out


def gram_f16(a16):
    """Mean and second moments of the channels of an fp16 activation [.., C] over
    all its pixels (hkp_gram_f16) → (mean fp64 [C], E = a^T a / M fp64 [C, C])."""
    from ._lib import lib
    _need(a16, torch.float16, "gram_f16.a")
    c = a16.shape[-1]
    m = a16.numel() // c
    nb = lib().hkp_gram_f16_workspace_bytes(m, c)
    if nb < 0:
        raise HkpError("gram_f16: unsupported shape (m=%d c=%d)" % (m, c))
    ws = torch.empty((nb + 7) // 8, device=a16.device, dtype=torch.float64)
    mean = torch.empty(c, device=a16.device, dtype=torch.float64)
    second = torch.empty((c, c), device=a16.device, dtype=torch.float64)
    call("hkp_gram_f16", m, c, _ptr(a16), _ptr(mean), _ptr(second), _ptr(ws), nb, _stream())
    return mean, second


def bn_from_gram(mean, second, wp, count, gamma, beta, running_mean=None, running_var=None,
                 num_batches_tracked=None, momentum=0.1, eps=1e-5):
    """Train-mode BN parameters of the output of a 1x1 conv with packed fp16 weight
    wp (weight_pack_f16 of [K,1,1,C]) from its input's mean / second moments
    (gram_f16) → (scale_shift [2K], mean_invstd [2K]); running stats updated as
    bn_finalize does."""
    ws, wsc = wp
    _need(mean, torch.float64, "bn_from_gram.mean", 1)
    _need(second, torch.float64, "bn_from_gram.second", 2)
    _need(ws, torch.float16, "bn_from_gram.w", 4)
    k, r, s_, c = ws.shape
    if (r, s_) != (1, 1) or mean.numel() != c or tuple(second.shape) != (c, c):
        raise HkpError("bn_from_gram: needs a 1x1 weight over the gram's %d channels (got %s)"
                       % (mean.numel(), tuple(ws.shape)))
    for t, nm in ((gamma, "gamma"), (beta, "beta"), (running_mean, "running_mean"), (running_var, "running_var")):
        if t is not None:
            _need(t, torch.float32, "bn_from_gram." + nm, 1)
            if t.numel() != k:
                raise HkpError("bn_from_gram.%s: %d != K=%d" % (nm, t.numel(), k))
    from ._lib import lib
    ss = torch.empty(2 * k, device=ws.device, dtype=torch.float32)
    mi = torch.empty(2 * k, device=ws.device, dtype=torch.float32)
    nb = lib().hkp_bn_from_gram_workspace_bytes(k, c)
    work = torch.empty((max(nb, 8) + 7) // 8, device=ws.device, dtype=torch.float64)
    call("hkp_bn_from_gram", k, c, int(count), _ptr(mean), _ptr(second), _ptr(ws), _ptr(wsc), _ptr(gamma), _ptr(beta),
         momentum, eps, _ptr(running_mean), _ptr(running_var), _ptr(num_batches_tracked), _ptr(ss), _ptr(mi),
         _ptr(work), work.numel() * 8, _stream())
    return ss, mi


def stem_x3_ok(x_shape, w_shape, stride, pad, dil):
    """Whether the stem conv (NCHW x, OIHW w) takes the f16x3 stem kernel."""
    def one(v):
        return int(v[0]) if isinstance(v, (tuple, list)) else int(v)
    k, c, r, s = w_shape
    return (r, s, one(stride), one(pad), one(dil)) == (7, 7, 2, 3, 1) and 1 <= c <= 4 and k % 64 == 0 \
        and x_shape[1] == c


def stem_weight_pack_x3(w):
    """OIHW [K,C<=4,7,7] fp32 stem weight → PackedWeight [K,7,64] fp16 + [K] scales."""
    _need(w, torch.float32, "stem_weight_pack_x3.w", 4)
    k, c = w.shape[:2]
    out = torch.empty((k, 7, 64), device=w.device, dtype=torch.float16)
    sc = torch.empty(k, device=w.device, dtype=torch.float32)
    call("hkp_stem_weight_pack_x3", k, c, _ptr(w), _ptr(out), _ptr(sc), _stream())
    return PackedWeight(out, sc)


# A/B (tools/infer_ab.py stem_img=0): the image-direct stem off by default in this process
STEM_IMAGE_DIRECT = True


def conv2d_fwd_stem_x3(x, wp, k, stats=True, part_out=None, tile=0, image_direct=None):
    """f16x3 stem conv (7x7/s2/p3) → NHWC fp32 y (+ BN partials).  x: the NCHW fp32
    image, or the uint8 NHWC (BGR) batch cv2.imread gives — ToTensor's /255 is then
    fused into the stem's operand split.  tile: 0 = the patch body
    where the output tiles into 8 x 32 patches, HKP_TILE_64_PAIR = the one-tile
    stem (the BN partials then group raster-order rows instead of patches).  On the
    patch body the image is split per tile in LDS (hkp_conv2d_fwd_stem_x3_image:
    no packed planes in HBM) unless image_direct=False (pack + planes, the same
    bits)."""
    from ._lib import lib
    ws, wsc = wp
    u8 = x.dtype == torch.uint8
    _need(x, torch.uint8 if u8 else torch.float32, "conv2d_fwd_stem_x3.x", 4)
    _need(ws, torch.float16, "conv2d_fwd_stem_x3.w_split", 3)
    if u8:
        n, h, wd, c = x.shape
    else:
        n, c, h, wd = x.shape
    d = ConvDesc(n, h, wd, c, k, 7, 7, 2, 3, 1, HKP_LAYOUT_NCHW, tile)
    ho, wo = conv_out_hw(h, wd, 7, 7, 2, 3, 1)
    y = torch.empty((n, ho, wo, k), device=x.device, dtype=torch.float32)
    part = _stat_partials(n * ho * wo, k, x.device, part_out, "conv2d_fwd_stem_x3.part_out") if stats else None
    if image_direct is None:
        image_direct = STEM_IMAGE_DIRECT
    if image_direct and lib().hkp_stem_x3_image_ok(ctypes.byref(d)):
        xin = x.contiguous()
        op = HKP_KOP_STEM_X3_IMAGE_U8 if u8 else HKP_KOP_STEM_X3_IMAGE

        def launch():
            call("hkp_conv2d_fwd_stem_x3_image", ctypes.byref(d), _ptr(xin), 1 if u8 else 0, _ptr(ws), _ptr(wsc),
                 _ptr(y), _ptr(part), _stream())
        nbytes = float(xin.numel() * xin.element_size()) + 2.0 * ws.numel() + 4.0 * y.numel()
    else:
        xs = torch.empty(lib().hkp_stem_pack_x3_elems(ctypes.byref(d)), device=x.device, dtype=torch.float16)
        call("hkp_stem_pack_x3_u8" if u8 else "hkp_stem_pack_x3", ctypes.byref(d), _ptr(x), _ptr(xs), _stream())
        op = HKP_KOP_STEM_X3

        def launch():
            call("hkp_conv2d_fwd_stem_x3", ctypes.byref(d), _ptr(xs), _ptr(ws), _ptr(wsc), _ptr(y), _ptr(part),
                 _stream())
        nbytes = 2.0 * (xs.numel() + ws.numel()) + 4.0 * y.numel()
    if _observer is None:
        launch()
    else:
        _observer(kernel_name(d, op), 2.0 * n * ho * wo * k * 49 * c, nbytes, launch)
    return y, part


def images_u8_to_nchw(img):
    """ToTensor on the device: uint8 [B,H,W,C] (BGR, cv2.imread) → fp32 [B,C,H,W] / 255."""
    _need(img, torch.uint8, "images_u8_to_nchw.img", 4)
    n, h, w, c = img.shape
    x = torch.empty((n, c, h, w), device=img.device, dtype=torch.float32)
    call("hkp_images_u8_to_nchw", n, h, w, c, _ptr(img), _ptr(x), _stream())
    return x


def heat_overlay(heat, img, yx):
    """Prediction.plot's picture on the GPU: heat [B,K,H,W] fp32,
    img uint8 [B,H,W,3] BGR, yx int32 [B,K,2] argmax → uint8 [B, H*K/2, 2W, 3]
    (K = 1: [B,H,W,3]) — the reference's two-column grid of JET overlays."""
    _need(heat, torch.float32, "heat_overlay.heat", 4)
    _need(img, torch.uint8, "heat_overlay.img", 4)
    _need(yx, torch.int32, "heat_overlay.yx", 3)
    n, k, h, w = heat.shape
    if tuple(img.shape) != (n, h, w, 3) or tuple(yx.shape) != (n, k, 2):
        raise HkpError("heat_overlay: img %s / yx %s do not match heat %s" % (tuple(img.shape), tuple(yx.shape),
                                                                            tuple(heat.shape)))
    if k != 1 and k % 2:
        raise HkpError("heat_overlay: K must be 1 or even (two equal columns)")
    out = torch.empty((n, h, w, 3) if k == 1 else (n, h * (k // 2), 2 * w, 3), device=heat.device,
                      dtype=torch.uint8)
    mm = torch.empty(n * k * 2, device=heat.device, dtype=torch.float32)
    call("hkp_heat_overlay", n, k, h, w, _ptr(heat), _ptr(img), _ptr(yx), _ptr(mm), _ptr(out), _stream())
    return out


def soft_argmax(heat, beta=1.0):
    """heat [N,K,H,W] fp32 → float32 [N,K,2] (x, y): softmax(beta*h)-weighted mean
    position per plane — Prediction.expectation (prediction.py:31-38) with its
    axis mix-up fixed."""
    _need(heat, torch.float32, "soft_argmax.heat", 4)
    n, k, h, w = heat.shape
    out = torch.empty((n, k, 2), device=heat.device, dtype=torch.float32)
    call("hkp_soft_argmax", n, k, h, w, float(beta), _ptr(heat), _ptr(out), _stream())
    return out


# two-level finalize (hkp_bn_finalize_ws) from this many partial tiles on: C4 +2.2 %
# (R50 C = 2048 convs, 4,800+ tiles); at 300-1,200 tiles (C2 layer2-4, the C3
# shard) the one-kernel merge already fills the chip and its single launch won
# (C2 neutral, C3 training -1.2 % with the two-level form everywhere)
FIN_TWO_LEVEL_TILES = 2048


def bn_finalize(part, count, gamma, beta, running_mean=None, running_var=None, num_batches_tracked=None,
                momentum=0.1, eps=1e-5, want_mean_invstd=True, two_level_tiles=FIN_TWO_LEVEL_TILES):
    """Train-mode BN statistics from conv partials → (scale_shift [2C], mean_invstd [2C]).
    Lists of >= two_level_tiles tiles take the two-level merge (hkp_bn_finalize_ws)."""
    _need(part, torch.float32, "bn_finalize.partials", 3)
    tiles, c, _ = part.shape
    ss = torch.empty(2 * c, device=part.device, dtype=torch.float32)
    mi = torch.empty(2 * c, device=part.device, dtype=torch.float32) if want_mean_invstd else None
    for t, nm in ((gamma, "gamma"), (beta, "beta"), (running_mean, "running_mean"), (running_var, "running_var")):
        if t is not None:
            _need(t, torch.float32, "bn_finalize." + nm, 1)
            if t.numel() != c:
                raise HkpError("bn_finalize.%s: %d != C=%d" % (nm, t.numel(), c))
    if num_batches_tracked is not None:
        _need(num_batches_tracked, torch.int64, "bn_finalize.num_batches_tracked")
    if tiles >= two_level_tiles:
        # two-level merge (chunks of 128 tiles over [C/64][chunks] blocks, then per channel)
        from ._lib import lib
        nb = lib().hkp_bn_finalize_workspace_bytes(c, tiles)
        ws = torch.empty((nb + 7) // 8, device=part.device, dtype=torch.float64)
        call("hkp_bn_finalize_ws", c, count, tiles, stat_tile_rows(part), _ptr(part), _ptr(gamma), _ptr(beta), momentum,
             eps, _ptr(running_mean), _ptr(running_var), _ptr(num_batches_tracked), _ptr(ss), _ptr(mi), _ptr(ws),
             nb, _stream())
        return ss, mi
    call("hkp_bn_finalize", c, count, tiles, stat_tile_rows(part), _ptr(part), _ptr(gamma), _ptr(beta), momentum, eps,
         _ptr(running_mean), _ptr(running_var), _ptr(num_batches_tracked), _ptr(ss), _ptr(mi), _stream())
    return ss, mi


def bn_stats(part, count, two_level_tiles=FIN_TWO_LEVEL_TILES):
    """SyncBN: this rank's per-channel BN statistics from its conv tile partials →
    fp64 [2C+1] = [mean | M2 | count] (hkp_bn_stats; gathered in rank order and
    merged by bn_finalize_ranks)."""
    _need(part, torch.float32, "bn_stats.partials", 3)
    tiles, c, _ = part.shape
    st = torch.empty(2 * c + 1, device=part.device, dtype=torch.float64)
    ws, nb = None, 0
    if tiles >= two_level_tiles:
        from ._lib import lib
        nb = lib().hkp_bn_finalize_workspace_bytes(c, tiles)
        ws = torch.empty((nb + 7) // 8, device=part.device, dtype=torch.float64)
    call("hkp_bn_stats", c, count, tiles, stat_tile_rows(part), _ptr(part), _ptr(st), _ptr(ws), nb, _stream())
    return st


def bn_finalize_ranks(stats, gamma, beta, running_mean=None, running_var=None, num_batches_tracked=None,
                      momentum=0.1, eps=1e-5):
    """SyncBN: the ranks' bn_stats blocks [R, 2C+1] (rank order) merged in fixed
    order → (scale_shift [2C], mean_invstd [2C]) of the global batch, as bn_finalize."""
    _need(stats, torch.float64, "bn_finalize_ranks.stats", 2)
    r, l = stats.shape
    if l % 2 != 1:
        raise HkpError("bn_finalize_ranks.stats: row length %d is not 2C+1" % l)
    c = (l - 1) // 2
    for t, nm in ((gamma, "gamma"), (beta, "beta"), (running_mean, "running_mean"), (running_var, "running_var")):
        if t is not None:
            _need(t, torch.float32, "bn_finalize_ranks." + nm, 1)
            if t.numel() != c:
                raise HkpError("bn_finalize_ranks.%s: %d != C=%d" % (nm, t.numel(), c))
    if num_batches_tracked is not None:
        _need(num_batches_tracked, torch.int64, "bn_finalize_ranks.num_batches_tracked")
    ss = torch.empty(2 * c, device=stats.device, dtype=torch.float32)
    mi = torch.empty(2 * c, device=stats.device, dtype=torch.float32)
    call("hkp_bn_finalize_ranks", c, r, _ptr(stats.contiguous()), _ptr(gamma), _ptr(beta), momentum, eps,
         _ptr(running_mean), _ptr(running_var), _ptr(num_batches_tracked), _ptr(ss), _ptr(mi), _stream())
    return ss, mi


def bn_eval_params(gamma, beta, running_mean, running_var, eps=1e-5):
    c = running_mean.numel()
    ss = torch.empty(2 * c, device=running_mean.device, dtype=torch.float32)
    mi = torch.empty(2 * c, device=running_mean.device, dtype=torch.float32)
    call("hkp_bn_eval_params", c, _ptr(gamma), _ptr(beta), _ptr(running_mean), _ptr(running_var), eps, _ptr(ss),
         _ptr(mi), _stream())
    return ss, mi


def _split_out(shape, device, split):
    """Split output of a producer: passes 1 → fp16 [.., C]; passes 3 → packed [.., 2C]."""
    shp = tuple(shape[:-1]) + (shape[-1] * (2 if split == 3 else 1),)
    t = torch.empty(shp, device=device, dtype=torch.float16)
    t._hkp_split_passes = split
    return t


def _check_split(split, c, who):
    if split not in (0, 1, 3):
        raise HkpError("%s: split must be 0, 1 or 3" % who)
    if split and c % 32:
        raise HkpError("%s: split output needs C %% 32 == 0 (C=%d)" % (who, c))


def bn_apply(y, ss, res=None, res_ss=None, relu=True, out=None, split=0, keep_fp32=True):
    """out = [relu](y*scale+shift [+ res | + res*rscale+rshift]).
    split = 1 or 3 also writes the next conv's operand (attached as out._hkp_split);
    keep_fp32=False (with split): the fp32 activation is not written and the split
    tensor itself is returned (an activation only a conv consumes).  res may be a
    split-only activation (packed, split=3): the residual is then read as hi + lo."""
    _need(y, torch.float32, "bn_apply.y")
    c = y.shape[-1]
    m = y.numel() // c
    _check_split(split, c, "bn_apply")
    if ss.numel() != 2 * c:
        raise HkpError("bn_apply: scale_shift size %d != 2C" % ss.numel())
    res_sp = None
    if res is not None and res.dtype == torch.float16:
        if res_ss is not None or getattr(res, "_hkp_split_passes", 0) != 3:
            raise HkpError("bn_apply: a split residual must be a packed (split=3) raw residual")
        _need(res, torch.float16, "bn_apply.res_split")
        if tuple(res.shape[:-1]) != tuple(y.shape[:-1]) or res.shape[-1] != 2 * c:
            raise HkpError("bn_apply: split residual shape %s vs %s" % (tuple(res.shape), tuple(y.shape)))
        res, res_sp = None, res
    elif res is not None:
        _need(res, torch.float32, "bn_apply.res")
        if res.shape != y.shape:
            raise HkpError("bn_apply: residual shape %s != %s" % (tuple(res.shape), tuple(y.shape)))
    if not keep_fp32 and not split:
        raise HkpError("bn_apply: keep_fp32=False needs a split output")
    o = None if not keep_fp32 else (out if out is not None else torch.empty_like(y))
    sp = _split_out(y.shape, y.device, split) if split else None
    call("hkp_bn_apply", m, c, _ptr(y), _ptr(ss), _ptr(res), _ptr(res_ss), _ptr(res_sp), int(bool(relu)), _ptr(o),
         _ptr(sp), int(split), _stream())
    if o is None:
        return sp
    if split:
        o._hkp_split = (sp, split)
    return o


def bn_apply_f16(y16, ss, res=None, res_ss=None, relu=True, keep_fp32=False):
    """Plain-fp16 path (config C4): fp16 out = [relu](y16*scale+shift [+ res | +
    res*rscale+rshift]), res an fp16 activation or (with res_ss) the downsample's
    fp16 y.  Returns the fp16 activation (a split=1 operand of the next conv), or
    with keep_fp32 the fp32 copy carrying it as its split (the head reads fp32)."""
    _need(y16, torch.float16, "bn_apply_f16.y")
    c = y16.shape[-1]
    m = y16.numel() // c
    if ss.numel() != 2 * c:
        raise HkpError("bn_apply_f16: scale_shift size %d != 2C" % ss.numel())
    if res is not None:
        _need(res, torch.float16, "bn_apply_f16.res")
        if res.shape != y16.shape:
            raise HkpError("bn_apply_f16: residual shape %s != %s" % (tuple(res.shape), tuple(y16.shape)))
    if res_ss is not None and (res is None or res_ss.numel() != 2 * c):
        raise HkpError("bn_apply_f16: res_scale_shift needs a residual and 2C entries")
    out = _split_out(y16.shape, y16.device, 1)
    o32 = torch.empty(y16.shape, device=y16.device, dtype=torch.float32) if keep_fp32 else None
    call("hkp_bn_apply_f16", m, c, _ptr(y16), _ptr(ss), _ptr(res), _ptr(res_ss), int(bool(relu)), _ptr(out),
         _ptr(o32), _stream())
    if o32 is None:
        return out
    o32._hkp_split = (out, 1)
    return o32


def bn_relu_maxpool(y, ss, split=0, route=False, keep_fp32=True):
    """maxpool3x3/s2/p1(relu(y*scale+shift)); route=True (training) also records
    each window's gradient tap as out._hkp_route (uint8, out's shape) for maxpool_bwd.
    keep_fp32=False (with split): only the split is written and returned."""
    _need(y, torch.float32, "bn_relu_maxpool.y", 4)
    n, h, w, c = y.shape
    _check_split(split, c, "bn_relu_maxpool")
    if not keep_fp32 and (not split or route):
        raise HkpError("bn_relu_maxpool: keep_fp32=False needs a split output and no route")
    shape = (n, (h - 1) // 2 + 1, (w - 1) // 2 + 1, c)
    out = torch.empty(shape, device=y.device, dtype=torch.float32) if keep_fp32 else None
    sp = _split_out(shape, y.device, split) if split else None
    rt = torch.empty(shape, device=y.device, dtype=torch.uint8) if route else None
    call("hkp_bn_relu_maxpool", n, h, w, c, _ptr(y), _ptr(ss), _ptr(out), _ptr(sp), int(split), _ptr(rt),
         _stream())
    if out is None:
        return sp
    if split:
        out._hkp_split = (sp, split)
    if route:
        out._hkp_route = rt
    return out


def head_fc(feat, w_kc, bias_k):
    """feat NHWC [N,h,w,C]; w [K,C]; bias [K] → lowres NCHW [N,K,h,w]."""
    _need(feat, torch.float32, "head_fc.feat", 4)
    _need(w_kc, torch.float32, "head_fc.w", 2)
    _need(bias_k, torch.float32, "head_fc.bias", 1)
    n, h, w, c = feat.shape
    k = w_kc.shape[0]
    if w_kc.shape[1] != c or bias_k.numel() != k:
        raise HkpError("head_fc: weight %s / bias %s do not match C=%d" % (tuple(w_kc.shape), bias_k.numel(), c))
    low = torch.empty((n, k, h, w), device=feat.device, dtype=torch.float32)
    call("hkp_head_fc", n, h * w, c, k, _ptr(feat), _ptr(w_kc), _ptr(bias_k), _ptr(low), _stream())
    return low


def head_fusable(c, k):
    """hkp_bn_apply_head covers this (channels, keypoints) pair."""
    return c % 512 == 0 and c <= 2048 and 0 < k <= 16


def bn_apply_head(y, ss, res, res_ss, w_kc, bias_k):
    """Inference tail: lowres [N,K,h,w] = head_fc(relu(y*scale+shift + residual))
    without writing the feature map.  y fp32 or fp16 NHWC; res: None, a raw
    residual of y's dtype, a packed split-only activation (fp32 y), or (with
    res_ss) the downsample's y."""
    n, h, w, c = y.shape
    k = w_kc.shape[0]
    if y.dtype not in (torch.float32, torch.float16):
        raise HkpError("bn_apply_head: y must be fp32 or fp16")
    _need(y, y.dtype, "bn_apply_head.y", 4)
    _need(w_kc, torch.float32, "bn_apply_head.w", 2)
    _need(bias_k, torch.float32, "bn_apply_head.bias", 1)
    if not head_fusable(c, k) or w_kc.shape[1] != c or bias_k.numel() != k or ss.numel() != 2 * c:
        raise HkpError("bn_apply_head: C=%d K=%d weight %s bias %d ss %d" % (c, k, tuple(w_kc.shape), bias_k.numel(),
                                                                         ss.numel()))
    kind = 0
    if res is not None:
        if res.dtype == torch.float16 and y.dtype == torch.float32:
            if res_ss is not None or getattr(res, "_hkp_split_passes", 0) != 3 or res.shape[-1] != 2 * c:
                raise HkpError("bn_apply_head: a split residual must be a packed (split=3) raw residual")
            kind = 3
        else:
            if res.dtype != y.dtype or res.shape != y.shape:
                raise HkpError("bn_apply_head: residual %s %s vs y %s %s" % (res.dtype, tuple(res.shape), y.dtype,
                                                                           tuple(y.shape)))
            kind = 2 if res_ss is not None else 1
        _need(res, res.dtype, "bn_apply_head.res")
        if tuple(res.shape[:-1]) != tuple(y.shape[:-1]):
            raise HkpError("bn_apply_head: residual pixels %s vs %s" % (tuple(res.shape), tuple(y.shape)))
    if res_ss is not None and (res is None or res_ss.numel() != 2 * c):
        raise HkpError("bn_apply_head: res_scale_shift needs a residual and 2C entries")
    low = torch.empty((n, k, h, w), device=y.device, dtype=torch.float32)
    call("hkp_bn_apply_head", n, h * w, c, k, int(y.dtype == torch.float16), _ptr(y), _ptr(ss), _ptr(res),
         _ptr(res_ss), kind, _ptr(w_kc), _ptr(bias_k), _ptr(low), _stream())
    return low


def upsample_sigmoid(low, H, W, heat=True, argmax=True, sigmoid=True, out=None):
    """lowres [N,K,h,w] → (heat [N,K,H,W] (into out when given) or None, argmax
    int32 [N,K,2] (y,x) or None)."""
    _need(low, torch.float32, "upsample_sigmoid.lowres", 4)
    n, k, h, w = low.shape
    hm = None
    if heat:
        hm = out if out is not None else torch.empty((n, k, H, W), device=low.device, dtype=torch.float32)
        _need(hm, torch.float32, "upsample_sigmoid.out", 4)
        if tuple(hm.shape) != (n, k, H, W):
            raise HkpError("upsample_sigmoid: out shape %s != %s" % (tuple(hm.shape), (n, k, H, W)))
    ws = yx = None
    if argmax:
        from ._lib import lib
        ws = torch.empty(lib().hkp_upsample_argmax_ws_bytes(n, k, H, W) // 8, device=low.device, dtype=torch.int64)
        yx = torch.empty((n, k, 2), device=low.device, dtype=torch.int32)
    call("hkp_upsample_sigmoid", n, k, h, w, H, W, int(bool(sigmoid)), _ptr(low), _ptr(hm), _ptr(ws), _ptr(yx), _stream())
    return hm, yx


def gauss_target(uv, H, W, sigma):
    """uv float32 [N,K,2] (u=x, v=y) → float64 [N,K,H,W]."""
    _need(uv, torch.float32, "gauss_target.uv", 3)
    n, k, _ = uv.shape
    out = torch.empty((n, k, H, W), device=uv.device, dtype=torch.float64)
    call("hkp_gauss_target", n, k, H, W, float(sigma), _ptr(uv), _ptr(out), _stream())
    return out


# ------------------------------------------------------------------ backward


def _fwd_desc(x_shape, w_shape, stride, pad, dil, layout):
    if layout == "nhwc":
        n, h, wd, c = x_shape
        k, r, s, _ = w_shape
        lay = HKP_LAYOUT_NHWC
    else:
        n, c, h, wd = x_shape
        k, _, r, s = w_shape
        lay = HKP_LAYOUT_NCHW
    return ConvDesc(n, h, wd, c, k, r, s, stride, pad, dil, lay)


def conv_weight_flip(w):
    """KRSC [K,R,S,C] → flipped CRSK [C,R,S,K] (the dgrad weight)."""
    _need(w, torch.float32, "conv_weight_flip.w", 4)
    k, r, s, c = w.shape
    d = ConvDesc(1, 1, 1, c, k, r, s, 1, 0, 1, HKP_LAYOUT_NHWC)
    wf = torch.empty((c, r, s, k), device=w.device, dtype=torch.float32)
    call("hkp_conv_weight_flip", ctypes.byref(d), _ptr(w), _ptr(wf), _stream())
    return wf


def conv2d_bwd_data(dy, w_flip, x_shape, stride=1, pad=0, dil=1, add=None):
    """dL/dx (NHWC) of conv2d_fwd; ``add`` (same shape as x, nullable) is summed in."""
    _need(dy, torch.float32, "conv2d_bwd_data.dy", 4)
    _need(w_flip, torch.float32, "conv2d_bwd_data.w_flip", 4)
    c, r, s, k = w_flip.shape
    d = _fwd_desc(x_shape, (k, r, s, c), stride, pad, dil, "nhwc")
    ho, wo = conv_out_hw(x_shape[1], x_shape[2], r, s, stride, pad, dil)
    if tuple(dy.shape) != (x_shape[0], ho, wo, k):
        raise HkpError("conv2d_bwd_data: dy shape %s != %s" % (tuple(dy.shape), (x_shape[0], ho, wo, k)))
    if add is not None:
        _need(add, torch.float32, "conv2d_bwd_data.add", 4)
        if tuple(add.shape) != tuple(x_shape):
            raise HkpError("conv2d_bwd_data: add shape mismatch")
    dx = torch.empty(tuple(x_shape), device=dy.device, dtype=torch.float32)
    call("hkp_conv2d_bwd_data", ctypes.byref(d), _ptr(dy), _ptr(w_flip), _ptr(add), _ptr(dx), _stream())
    return dx


def absmax(x):
    """max |x| as a device uint32 (IEEE bits) — feeds the split kernels' power-of-two scaling."""
    _need(x, torch.float32, "absmax.x")
    out = torch.empty(1, device=x.device, dtype=torch.int32)
    call("hkp_absmax", x.numel(), _ptr(x), _ptr(out), _stream())
    return out


def split_pack_x3(x, amax=None):
    """fp32 NHWC x (scaled by the power of two of amax, if given) → packed split [.., 2C]."""
    _need(x, torch.float32, "split_pack_x3.x")
    c = x.shape[-1]
    out = torch.empty(tuple(x.shape[:-1]) + (2 * c,), device=x.device, dtype=torch.float16)
    call("hkp_split_pack_x3", x.numel(), c, _ptr(x), _ptr(amax), _ptr(out), _stream())
    out._hkp_split_passes = 3
    return out


def weight_flip_pack_x3(w):
    """KRSC [K,R,S,C] fp32 → packed flipped [C,R,S,2K] fp16 for conv2d_bwd_data_x3."""
    _need(w, torch.float32, "weight_flip_pack_x3.w", 4)
    k, r, s, c = w.shape
    d = ConvDesc(1, 1, 1, c, k, r, s, 1, 0, 1, HKP_LAYOUT_NHWC)
    out = torch.empty((c, r, s, 2 * k), device=w.device, dtype=torch.float16)
    sc = torch.empty(c, device=w.device, dtype=torch.float32)
    call("hkp_weight_flip_pack_x3", ctypes.byref(d), _ptr(w), _ptr(out), _ptr(sc), _stream())
    return PackedWeight(out, sc)


def phase_taps(r, pad, phase, stride=2):
    """Taps of output phase `phase` along a filter axis of r taps (hkp_phase_taps)."""
    from ._lib import lib
    return lib().hkp_phase_taps(r, pad, stride, phase)


def weight_pack_x3_batch(items, outs=None, keep_launch=None):
    """Many weight packs in one launch pair (hkp_weight_pack_x3_batch): items =
    [(kind, w)] with kind "x3" (= weight_pack_x3(w)) or "flip_x3"
    (= weight_flip_pack_x3(w)), or ("phase_x3", w, (phase, pad)) — output phase
    phase = py*2+px of a stride-2 conv's dgrad operand (conv2d_bwd_data_x3_strided);
    returns the PackedWeights in order.  outs (optional, same order; None entries
    allowed) are PackedWeights to overwrite.  keep_launch (a dict, optional)
    receives a `relaunch()` that repeats this exact launch (same pointers) — for
    callers that repack the same weights in place every step."""
    from ._lib import PackJob, lib
    jobs = (PackJob * max(1, len(items)))()
    res = []
    for i, item in enumerate(items):
        kind, w = item[0], item[1]
        _need(w, torch.float32, "weight_pack_x3_batch.w", 4)
        k, r, s, c = w.shape
        if kind == "x3":
            code, shape, n_sc = 0, (k, r, s, 2 * c), k
        elif kind == "flip_x3":
            code, shape, n_sc = 1, (c, r, s, 2 * k), c
        elif kind == "phase_x3":
            ph, pad = item[2]
            r2, s2 = phase_taps(r, pad, ph >> 1), phase_taps(s, pad, ph & 1)
            if r2 <= 0 or s2 <= 0:
                raise HkpError("weight_pack_x3_batch: phase %d has no taps" % ph)
            code, shape, n_sc = 2, (c, r2, s2, 2 * k), c
            jobs[i].r, jobs[i].s, jobs[i].pad, jobs[i].phase = r, s, pad, ph
        else:
            raise HkpError("weight_pack_x3_batch: unknown kind %r" % (kind,))
        o = outs[i] if outs is not None else None
        if o is None or tuple(o.split.shape) != shape or o.split.device != w.device:
            o = PackedWeight(torch.empty(shape, device=w.device, dtype=torch.float16),
                             torch.empty(n_sc, device=w.device, dtype=torch.float32))
        res.append(o)
        jobs[i].w, jobs[i].out, jobs[i].inv_scale = _ptr(w), _ptr(o.split), _ptr(o.inv_scale)
        jobs[i].kind, jobs[i].k, jobs[i].rs, jobs[i].c = code, k, r * s, c
    if not items:
        return res
    nb = lib().hkp_weight_pack_x3_batch_ws_bytes(len(items), jobs)
    ws = torch.empty(max(4, nb), device=items[0][1].device, dtype=torch.uint8)
    n = len(items)

    def relaunch():
        call("hkp_weight_pack_x3_batch", n, jobs, _ptr(ws), nb, _stream())

    relaunch()
    if keep_launch is not None:
        keep_launch["relaunch"] = relaunch
    return res


def weight_phase_pack_x3(w, pad):
    """The four output-phase dgrad operands of a stride-2 KRSC conv weight (None for a
    phase no tap reaches), for conv2d_bwd_data_x3_strided."""
    k, r, s, c = w.shape
    phases = [ph for ph in range(4) if phase_taps(r, pad, ph >> 1) > 0 and phase_taps(s, pad, ph & 1) > 0]
    packs = weight_pack_x3_batch([("phase_x3", w, (ph, pad)) for ph in phases])
    out = [None] * 4
    for ph, pk in zip(phases, packs):
        out[ph] = pk
    return out


def conv2d_bwd_data_x3_strided(dys, phase_packs, x_shape, w_shape, pad=0, add=None, amax=None, sk=True, tile=0):
    """f16x3 dL/dx of a stride-2 (dilation-1) NHWC conv with KRSC weight shape
    w_shape, one stride-1 conv per output phase: dys = split_pack_x3(dy, amax),
    phase_packs = weight_phase_pack_x3(w, pad).  sk=False: no stream-K (one tile
    per block, e.g. while another stream's kernel shares the CUs)."""
    _need(dys, torch.float16, "conv2d_bwd_data_x3_strided.dy_split", 4)
    k, r, s, c = w_shape
    if len(phase_packs) != 4:
        raise HkpError("conv2d_bwd_data_x3_strided: need 4 phase packs (None for empty phases)")
    for ph, p in enumerate(phase_packs):
        taps = (phase_taps(r, pad, ph >> 1), phase_taps(s, pad, ph & 1))
        want = None if min(taps) <= 0 else (c,) + taps + (2 * k,)
        if (p is None) != (want is None) or (p is not None and tuple(p.split.shape) != want):
            raise HkpError("conv2d_bwd_data_x3_strided: phase %d pack %s, expected %s" % (
                ph, None if p is None else tuple(p.split.shape), want))
    d = _fwd_desc(x_shape, (k, r, s, c), 2, pad, 1, "nhwc")
    d.tile = tile
    ho, wo = conv_out_hw(x_shape[1], x_shape[2], r, s, 2, pad, 1)
    if tuple(dys.shape) != (x_shape[0], ho, wo, 2 * k):
        raise HkpError("conv2d_bwd_data_x3_strided: dy split shape %s != %s" % (tuple(dys.shape),
                                                                               (x_shape[0], ho, wo, 2 * k)))
    if add is not None:
        _need(add, torch.float32, "conv2d_bwd_data_x3_strided.add", 4)
        if tuple(add.shape) != tuple(x_shape):
            raise HkpError("conv2d_bwd_data_x3_strided: add shape mismatch")
    dx = torch.empty(tuple(x_shape), device=dys.device, dtype=torch.float32)
    sp = (ctypes.c_void_p * 4)(*[None if p is None else p.split.data_ptr() for p in phase_packs])
    sc = (ctypes.c_void_p * 4)(*[None if p is None else p.inv_scale.data_ptr() for p in phase_packs])
    call("hkp_conv2d_bwd_data_x3_strided", ctypes.byref(d), _ptr(dys), sp, sc, _ptr(amax), _ptr(add), _ptr(dx),
         *_sk_workspace(sk), _stream())
    return dx


def conv2d_bwd_data_x3(dys, wfp, x_shape, pad=0, dil=1, add=None, amax=None, sk=True, tile=0):
    """f16x3 dL/dx of a stride-1 NHWC conv from packed dy (split_pack_x3 with `amax`)
    and wfp = weight_flip_pack_x3(w).  sk=False: no stream-K; tile: HKP_TILE_*."""
    wfs, wfsc = wfp
    _need(dys, torch.float16, "conv2d_bwd_data_x3.dy_split", 4)
    _need(wfs, torch.float16, "conv2d_bwd_data_x3.wf_split", 4)
    c, r, s, k2 = wfs.shape
    k = k2 // 2
    d = _fwd_desc(x_shape, (k, r, s, c), 1, pad, dil, "nhwc")
    d.tile = tile
    ho, wo = conv_out_hw(x_shape[1], x_shape[2], r, s, 1, pad, dil)
    if tuple(dys.shape) != (x_shape[0], ho, wo, 2 * k):
        raise HkpError("conv2d_bwd_data_x3: dy split shape %s != %s" % (tuple(dys.shape), (x_shape[0], ho, wo, 2 * k)))
    if add is not None:
        _need(add, torch.float32, "conv2d_bwd_data_x3.add", 4)
        if tuple(add.shape) != tuple(x_shape):
            raise HkpError("conv2d_bwd_data_x3: add shape mismatch")
    dx = torch.empty(tuple(x_shape), device=dys.device, dtype=torch.float32)

    def launch():
        call("hkp_conv2d_bwd_data_x3", ctypes.byref(d), _ptr(dys), _ptr(wfs), _ptr(wfsc), _ptr(amax), _ptr(add),
             _ptr(dx), *_sk_workspace(sk), _stream())

    if _observer is None:
        launch()
    else:
        _observer(kernel_name(d, HKP_KOP_DGRAD_X3, sk),
                  2.0 * x_shape[0] * x_shape[1] * x_shape[2] * c * r * s * k,
                  2.0 * (dys.numel() + wfs.numel()) + 4.0 * dx.numel(), launch)
    return dx


# The wgrad's split-K slabs, one buffer per (device, launching stream), grown to the
# largest request: the launches on a stream run in order, each reading its slabs back
# (the reduce) before the next writes them.  A per-call allocation instead left each
# side-stream workspace pending on its stream's progress when freed: the caching
# allocator levelled off at 38 GB of blocks after ~25 C3 training steps, 28 GB with
# this buffer (5.6 GB without the overlap; step time unchanged; tools/alloc_probe.py).
_wg_ws = {}


def _wgrad_workspace(device, nbytes, alloc_stream=None):
    st = torch.cuda.current_stream(device)
    key = (st.device_index, st.cuda_stream)
    ws = _wg_ws.get(key)
    if ws is None or ws.numel() * 4 < nbytes:
        if ws is not None:
            ws.record_stream(st)                     # the last launches on st may still read it
        n = max(nbytes, 4) // 4
        if alloc_stream is None:
            ws = torch.empty(n, device=device, dtype=torch.float32)
        else:
            with torch.cuda.stream(alloc_stream):
                ws = torch.empty(n, device=device, dtype=torch.float32)
            ws.record_stream(st)
        _wg_ws[key] = ws
    return ws


def conv2d_bwd_filter_x3(xs, dys, w_shape, stride=1, pad=0, dil=1, amax=None, alloc_stream=None, cus=0):
    """f16x3 dL/dw (KRSC) from packed x (forward operand) and packed dy (split_pack_x3 with `amax`).
    cus: the CUs the grid should occupy (pixel-range splits = max(1, cus / tiles);
    0: the planner's count, filling whole rounds of every CU; -1: the planner's
    count on the tiled body — the halo body of 3x3 stride-1 convs off).
    alloc_stream: take dw (and a new workspace buffer) from that stream's memory pool (marked
    as used by the launching stream) — a side-stream wgrad then shares the main
    stream's cached blocks instead of growing a second pool (C5 at 245 GB: the
    second pool forced allocator flushes every step, 5x slower)."""
    from ._lib import lib
    _need(xs, torch.float16, "conv2d_bwd_filter_x3.x_split", 4)
    _need(dys, torch.float16, "conv2d_bwd_filter_x3.dy_split", 4)
    n, h, wd, c2 = xs.shape
    d = _fwd_desc((n, h, wd, c2 // 2), tuple(w_shape), stride, pad, dil, "nhwc")
    d.tile = int(cus)
    ho, wo = conv_out_hw(h, wd, d.r, d.s, stride, pad, dil)
    if tuple(dys.shape) != (n, ho, wo, 2 * d.k):
        raise HkpError("conv2d_bwd_filter_x3: dy split shape %s != %s" % (tuple(dys.shape), (n, ho, wo, 2 * d.k)))
    nbytes = lib().hkp_conv_bwd_filter_x3_workspace(ctypes.byref(d))
    ws = _wgrad_workspace(xs.device, nbytes, alloc_stream)
    if alloc_stream is None:
        dw = torch.empty(tuple(w_shape), device=xs.device, dtype=torch.float32)
    else:
        launching = torch.cuda.current_stream(xs.device)
        with torch.cuda.stream(alloc_stream):
            dw = torch.empty(tuple(w_shape), device=xs.device, dtype=torch.float32)
        dw.record_stream(launching)

    def launch():
        call("hkp_conv2d_bwd_filter_x3", ctypes.byref(d), _ptr(xs), _ptr(dys), _ptr(amax), _ptr(dw), _ptr(ws),
             nbytes, _stream())

    if _observer is None:
        launch()
    else:
        _observer(kernel_name(d, HKP_KOP_WGRAD_X3),
                  2.0 * n * ho * wo * d.k * d.r * d.s * d.c, 2.0 * (xs.numel() + dys.numel()) + 4.0 * dw.numel(),
                  launch)
    return dw


def conv2d_bwd_filter(x, dy, w_shape, stride=1, pad=0, dil=1, layout="nhwc", out=None, accumulate=False):
    """dL/dw in the weight's own layout (KRSC, or OIHW for the NCHW stem)."""
    _need(x, torch.float32, "conv2d_bwd_filter.x", 4)
    _need(dy, torch.float32, "conv2d_bwd_filter.dy", 4)
    d = _fwd_desc(tuple(x.shape), tuple(w_shape), stride, pad, dil, layout)
    ho, wo = conv_out_hw(d.h, d.w, d.r, d.s, stride, pad, dil)
    if tuple(dy.shape) != (d.n, ho, wo, d.k):
        raise HkpError("conv2d_bwd_filter: dy shape %s != %s" % (tuple(dy.shape), (d.n, ho, wo, d.k)))
    from ._lib import lib
    nbytes = lib().hkp_conv_bwd_filter_workspace(ctypes.byref(d))
    ws = torch.empty(max(nbytes, 4) // 4, device=x.device, dtype=torch.float32)
    dw = out if out is not None else torch.empty(tuple(w_shape), device=x.device, dtype=torch.float32)
    _need(dw, torch.float32, "conv2d_bwd_filter.dw")
    call("hkp_conv2d_bwd_filter", ctypes.byref(d), _ptr(x), _ptr(dy), _ptr(dw), int(bool(accumulate)), _ptr(ws),
         nbytes, _stream())
    return dw


def bn_bwd_begin(g, out_mask, y, mean_invstd, gamma, want_dz=False, want_amax=False, split_only=False,
                 relu_ss=None):
    """First half of bn_bwd: validates and launches the reduce pass (per-tile
    channel sums; dz = g*mask when want_dz).  Returns the state bn_bwd_end /
    bn_bwd_local_stats take; state["dz"] is dz (written once the pass runs)."""
    _need(g, torch.float32, "bn_bwd.g")
    _need(y, torch.float32, "bn_bwd.y")
    if g.shape != y.shape or (out_mask is not None and out_mask.shape != y.shape):
        raise HkpError("bn_bwd: shape mismatch")
    c = y.shape[-1]
    if relu_ss is not None:
        if out_mask is not None:
            raise HkpError("bn_bwd: out_mask and relu_ss are exclusive")
        _need(relu_ss, torch.float32, "bn_bwd.relu_ss", 1)
        if relu_ss.numel() != 2 * c:
            raise HkpError("bn_bwd: relu_ss must be [2C]")
    m = y.numel() // c
    if split_only and c % 32:
        raise HkpError("bn_bwd: split_only needs C % 32 == 0")
    from ._lib import lib
    tiles = lib().hkp_bn_bwd_tiles(m)
    part = torch.empty((tiles, c, 2), device=y.device, dtype=torch.float32)
    maxima = torch.empty((tiles, c, 2), device=y.device, dtype=torch.float32) if split_only else None
    amax = torch.empty(1, device=y.device, dtype=torch.int32) if (want_amax or split_only) else None
    dz = torch.empty_like(y) if want_dz else None
    call("hkp_bn_bwd_reduce", m, c, _ptr(g), _ptr(out_mask), _ptr(relu_ss), _ptr(y), _ptr(mean_invstd), _ptr(dz),
         _ptr(part), _ptr(maxima), _ptr(amax if split_only else None), _stream())
    return dict(g=g, out_mask=out_mask, y=y, mi=mean_invstd, gamma=gamma, relu_ss=relu_ss, m=m, c=c, part=part,
                maxima=maxima, amax=amax, dz=dz, split_only=split_only, want_amax=want_amax)


def bn_bwd_local_stats(st):
    """SyncBN: this rank's [Σdz | Σdz·(y−mean) | max|dz| | max|y−mean| | m] fp64
    block (hkp_bn_bwd_stats) of a begun BN backward, to be all-gathered."""
    own = torch.empty(4 * st["c"] + 1, device=st["y"].device, dtype=torch.float64)
    call("hkp_bn_bwd_stats", st["c"], st["m"], _ptr(st["part"]), _ptr(st["maxima"]), _ptr(st["mi"]), _ptr(own),
         _stream())
    return own


def bn_bwd_end(st, ranks=None, own=None):
    """Second half of bn_bwd: coefficients (from this rank's sums, or — SyncBN —
    from `ranks` [R, 4C+1], every rank's bn_bwd_local_stats block in rank order,
    with `own` this rank's) and the apply pass → (dy, dgamma, dbeta, dz)."""
    y, c, m = st["y"], st["c"], st["m"]
    dgamma = torch.empty(c, device=y.device, dtype=torch.float32)
    dbeta = torch.empty(c, device=y.device, dtype=torch.float32)
    coef = torch.empty(3 * c, device=y.device, dtype=torch.float32)
    if ranks is None:
        call("hkp_bn_bwd_finalize", c, m, _ptr(st["part"]), _ptr(st["maxima"]), _ptr(st["mi"]), _ptr(st["gamma"]),
             _ptr(dgamma), _ptr(dbeta), _ptr(coef), _ptr(st["amax"]), _stream())
    else:
        _need(ranks, torch.float64, "bn_bwd_end.ranks")
        if ranks.dim() != 2 or ranks.shape[1] != 4 * c + 1 or own is None or own.numel() != 4 * c + 1:
            raise HkpError("bn_bwd_end: rank statistics must be [R, 4C+1] with this rank's block")
        call("hkp_bn_bwd_finalize_ranks", c, ranks.shape[0], _ptr(ranks.contiguous()), _ptr(own),
             1 if st["maxima"] is not None else 0, _ptr(st["mi"]), _ptr(st["gamma"]), _ptr(dgamma), _ptr(dbeta),
             _ptr(coef), _ptr(st["amax"]), _stream())
    if st["split_only"]:
        dy = _split_out(y.shape, y.device, 3)
        call("hkp_bn_bwd_apply", m, c, _ptr(st["g"]), _ptr(st["out_mask"]), _ptr(st["relu_ss"]), _ptr(y),
             _ptr(st["mi"]), _ptr(coef), None, _ptr(st["amax"]), _ptr(dy), _stream())
    else:
        dy = torch.empty_like(y)
        call("hkp_bn_bwd_apply", m, c, _ptr(st["g"]), _ptr(st["out_mask"]), _ptr(st["relu_ss"]), _ptr(y),
             _ptr(st["mi"]), _ptr(coef), _ptr(dy), _ptr(st["amax"]), None, _stream())
    if st["want_amax"] or st["split_only"]:
        dy._hkp_amax = st["amax"]
    return dy, dgamma, dbeta, st["dz"]


def bn_bwd(g, out_mask, y, mean_invstd, gamma, want_dz=False, want_amax=False, split_only=False, relu_ss=None,
           sync_group=None):
    """Train-mode BN(+ReLU mask) backward → (dy, dgamma, dbeta, dz or None).
    The ReLU mask is out_mask > 0, or (relu_ss = the forward's scale_shift) is
    recomputed from y bit-identically — no read of the fp32 activation.
    want_amax: max|dy| (uint32 IEEE bits, as absmax) is computed in the same pass
    and attached as dy._hkp_amax.  split_only: dy is returned as the packed f16x3
    split of dy * 2^e (the x3 backward convs' operand, _hkp_split_passes = 3) with
    2^e from an upper bound of max|dy| (attached as _hkp_amax, the scale's source);
    no fp32 dy is written.  sync_group = (group,): SyncBN — the dx coefficients
    from the channel sums of every rank of group (hkp.parallel.active_sync_group)."""
    st = bn_bwd_begin(g, out_mask, y, mean_invstd, gamma, want_dz, want_amax, split_only, relu_ss)
    if sync_group is None:
        return bn_bwd_end(st)
    from . import parallel
    own = bn_bwd_local_stats(st)
    return bn_bwd_end(st, parallel.gather_bn_stats(own, sync_group[0]), own)


def maxpool_bwd(dpool, route, in_shape):
    """Stem: dL/d(BN output) [in_shape] from dL/d(maxpool output) and the forward's
    route (bn_relu_maxpool(..., route=True)._hkp_route; ReLU mask included)."""
    _need(dpool, torch.float32, "maxpool_bwd.dpool", 4)
    _need(route, torch.uint8, "maxpool_bwd.route", 4)
    n, h, w, c = in_shape
    if tuple(dpool.shape) != (n, (h - 1) // 2 + 1, (w - 1) // 2 + 1, c) or route.shape != dpool.shape:
        raise HkpError("maxpool_bwd: dpool / route shape mismatch")
    dz = torch.empty(tuple(in_shape), device=dpool.device, dtype=torch.float32)
    call("hkp_maxpool_bwd", n, h, w, c, _ptr(dpool), _ptr(route), _ptr(dz), _stream())
    return dz


def heat_loss(heat, target=None, uv=None, sigma=8.0, kind="bce", want_grad=True):
    """fp64 BCE/MSE over [N,K,H,W] heatmaps → (loss 0-dim f64 tensor, dheat f32 or None)."""
    from ._lib import HKP_LOSS_BCE, HKP_LOSS_MSE, lib
    _need(heat, torch.float32, "heat_loss.heat", 4)
    n, k, H, W = heat.shape
    if target is not None:
        _need(target, torch.float64, "heat_loss.target", 4)
        if target.shape != heat.shape:
            raise HkpError("heat_loss: target shape %s != %s" % (tuple(target.shape), tuple(heat.shape)))
    else:
        _need(uv, torch.float32, "heat_loss.uv", 3)
        if tuple(uv.shape) != (n, k, 2):
            raise HkpError("heat_loss: uv must be [N,K,2]")
    ws = torch.empty(lib().hkp_heat_loss_workspace() // 8, device=heat.device, dtype=torch.float64)
    loss = torch.empty((), device=heat.device, dtype=torch.float64)
    dheat = torch.empty_like(heat) if want_grad else None
    call("hkp_heat_loss", n, k, H, W, HKP_LOSS_BCE if kind == "bce" else HKP_LOSS_MSE, _ptr(heat), _ptr(target),
         _ptr(uv), float(sigma), _ptr(loss), _ptr(dheat), _ptr(ws), _stream())
    return loss, dheat


def head_bwd(dheat, heat, h, w):
    """dlow [N,K,h,w] = upsample-adjoint(dheat * (1-heat) * heat)."""
    _need(dheat, torch.float32, "head_bwd.dheat", 4)
    n, k, H, W = dheat.shape
    if heat is not None and heat.shape != dheat.shape:
        raise HkpError("head_bwd: heat shape mismatch")
    from ._lib import lib
    dlow = torch.empty((n, k, h, w), device=dheat.device, dtype=torch.float32)
    nb = lib().hkp_head_bwd_workspace(n, k, w, H)
    ws = torch.empty(nb // 4, device=dheat.device, dtype=torch.float32)
    call("hkp_head_bwd", n, k, h, w, H, W, _ptr(dheat), _ptr(heat), _ptr(dlow), _ptr(ws), nb, _stream())
    return dlow


def head_fc_bwd(dlow, feat, w_kc):
    """→ (dfeat NHWC, dW [K,C], db [K])."""
    from ._lib import lib
    _need(dlow, torch.float32, "head_fc_bwd.dlow", 4)
    _need(feat, torch.float32, "head_fc_bwd.feat", 4)
    _need(w_kc, torch.float32, "head_fc_bwd.w", 2)
    n, h, w, c = feat.shape
    k = dlow.shape[1]
    if tuple(dlow.shape) != (n, k, h, w) or tuple(w_kc.shape) != (k, c):
        raise HkpError("head_fc_bwd: shape mismatch")
    nbytes = lib().hkp_head_fc_bwd_workspace(n, h * w, c, k)
    ws = torch.empty(nbytes // 4, device=feat.device, dtype=torch.float32)
    dfeat = torch.empty_like(feat)
    dw = torch.empty((k, c), device=feat.device, dtype=torch.float32)
    db = torch.empty(k, device=feat.device, dtype=torch.float32)
    call("hkp_head_fc_bwd", n, h * w, c, k, _ptr(dlow), _ptr(feat), _ptr(w_kc), _ptr(dfeat), _ptr(dw), _ptr(db),
         _ptr(ws), nbytes, _stream())
    return dfeat, dw, db
