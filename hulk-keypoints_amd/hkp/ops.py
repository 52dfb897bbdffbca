"""Tensor-level wrappers over the C ABI (one function per kernel family).

Every wrapper validates device/dtype/contiguity/shape on the host BEFORE the
launch (a mis-shaped launch can fault the GPU), launches on PyTorch's current
stream, and allocates outputs with the caching allocator.  No fallback path.
"""
import ctypes

import torch

from ._lib import ConvDesc, HKP_LAYOUT_NCHW, HKP_LAYOUT_NHWC, HkpError, call

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


def bn_finalize(part, count, gamma, beta, running_mean=None, running_var=None, num_batches_tracked=None,
                momentum=0.1, eps=1e-5, want_mean_invstd=True):
    """Train-mode BN statistics from conv partials → (scale_shift [2C], mean_invstd [2C])."""
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
    call("hkp_bn_finalize", c, count, tiles, CONV_TILE_ROWS, _ptr(part), _ptr(gamma), _ptr(beta), momentum, eps,
         _ptr(running_mean), _ptr(running_var), _ptr(num_batches_tracked), _ptr(ss), _ptr(mi), _stream())
    return ss, mi


def bn_eval_params(gamma, beta, running_mean, running_var, eps=1e-5):
    c = running_mean.numel()
    ss = torch.empty(2 * c, device=running_mean.device, dtype=torch.float32)
    mi = torch.empty(2 * c, device=running_mean.device, dtype=torch.float32)
    call("hkp_bn_eval_params", c, _ptr(gamma), _ptr(beta), _ptr(running_mean), _ptr(running_var), eps, _ptr(ss),
         _ptr(mi), _stream())
    return ss, mi


def bn_apply(y, ss, res=None, res_ss=None, relu=True, out=None):
    _need(y, torch.float32, "bn_apply.y")
    c = y.shape[-1]
    m = y.numel() // c
    if ss.numel() != 2 * c:
        raise HkpError("bn_apply: scale_shift size %d != 2C" % ss.numel())
    if res is not None:
        _need(res, torch.float32, "bn_apply.res")
        if res.shape != y.shape:
            raise HkpError("bn_apply: residual shape %s != %s" % (tuple(res.shape), tuple(y.shape)))
    o = out if out is not None else torch.empty_like(y)
    call("hkp_bn_apply", m, c, _ptr(y), _ptr(ss), _ptr(res), _ptr(res_ss), int(bool(relu)), _ptr(o), _stream())
    return o


def bn_relu_maxpool(y, ss):
    _need(y, torch.float32, "bn_relu_maxpool.y", 4)
    n, h, w, c = y.shape
    out = torch.empty((n, (h - 1) // 2 + 1, (w - 1) // 2 + 1, c), device=y.device, dtype=torch.float32)
    call("hkp_bn_relu_maxpool", n, h, w, c, _ptr(y), _ptr(ss), _ptr(out), _stream())
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


def upsample_sigmoid(low, H, W, heat=True, argmax=True, sigmoid=True):
    """lowres [N,K,h,w] → (heat [N,K,H,W] or None, argmax int32 [N,K,2] (y,x) or None)."""
    _need(low, torch.float32, "upsample_sigmoid.lowres", 4)
    n, k, h, w = low.shape
    hm = torch.empty((n, k, H, W), device=low.device, dtype=torch.float32) if heat else None
    ws = yx = None
    if argmax:
        ws = torch.empty(n * k, device=low.device, dtype=torch.int64)
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
