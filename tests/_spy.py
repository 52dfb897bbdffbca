"""Call spies over hkp.net's per-layer entry points (test infrastructure).

spy_calls(...) replaces, for the duration of a `with` block, the functions the
network walk runs each conv forward, conv backward, BN backward and the stem
wgrad through, calling the given observer after each real call with that call's
inputs and outputs:

    on_conv_fwd(conv, bn, x, layout, y, part)
    on_conv_bwd(conv, x, dy, add, dx, dw)
    on_bn_bwd(bn, g, out_mask, relu_ss, y, mi, dy, dgamma, dbeta)
    on_stem_wgrad(x, dy, w_shape, stride, pad, dil, layout, dw)
"""
import contextlib


@contextlib.contextmanager
def spy_calls(on_conv_fwd=None, on_conv_bwd=None, on_bn_bwd=None, on_stem_wgrad=None):
    from hkp import net, ops
    orig = dict(fwd=net._conv_fwd, bwd=net._conv_backward, fin=net._bn_bwd_finish, wst=ops.conv2d_bwd_filter)

    def fwd_spy(conv, bn, x, pol, layout="nhwc", sk=True):
        y, part = orig["fwd"](conv, bn, x, pol, layout, sk)
        if on_conv_fwd is not None:
            on_conv_fwd(conv, bn, x, layout, y, part)
        return y, part

    def bwd_spy(conv, x, dy, grads, pol, need_dx=True, add=None):
        dx = orig["bwd"](conv, x, dy, grads, pol, need_dx, add)
        if on_conv_bwd is not None:
            on_conv_bwd(conv, x, dy, add, dx, grads[conv.weight])
        return dx

    def fin_spy(states, items, grads, pol):
        out = orig["fin"](states, items, grads, pol)
        if on_bn_bwd is not None:
            for it, (dy, _) in zip(items, out):
                on_bn_bwd(it["bn"], it["g"], it.get("out_mask"), it.get("relu_ss"), it["y"], it["mi"], dy,
                          grads[it["bn"].weight], grads[it["bn"].bias])
        return out

    def wst_spy(x, dy, w_shape, stride=1, pad=0, dil=1, layout="nhwc", out=None, accumulate=False):
        dw = orig["wst"](x, dy, w_shape, stride, pad, dil, layout, out, accumulate)
        if on_stem_wgrad is not None:
            on_stem_wgrad(x, dy, w_shape, stride, pad, dil, layout, dw)
        return dw

    net._conv_fwd, net._conv_backward, net._bn_bwd_finish, ops.conv2d_bwd_filter = fwd_spy, bwd_spy, fin_spy, wst_spy
    try:
        yield
    finally:
        net._conv_fwd, net._conv_backward, net._bn_bwd_finish, ops.conv2d_bwd_filter = \
            orig["fwd"], orig["bwd"], orig["fin"], orig["wst"]
