"""Two-lane inference forward: the keypoint net of net.keypoints_forward
(src/resnet.py:198-213, src/resnet_dilated.py:16-27, src/model.py:19-22) with the
batch split into two halves on two HIP streams.

Train-mode BatchNorm needs the whole batch's statistics, so the lanes meet once
per BN layer: both halves' convs write their BN tile partials into one buffer
(lane A's tiles first), one finalize on the main stream gives the full-batch
scale/shift — bit-identical to the one-lane forward because the halves' 128-row
tiles are exactly the full batch's (checked by lanes_ok) — and then lane A
applies BN, and lane B applies it only after A's apply has finished: B's apply
(HBM-bound) runs beside A's next conv (MFMA-bound) instead of both applies
splitting the memory bandwidth at the same moment.  Every kernel is the one-lane
forward's, on half the images, with stream-K off (a half batch's grid would pick
it where the full batch's does not, and it reorders the fp32 K sum): outputs are
bit-identical to the one-lane forward whenever that one takes no stream-K either
(C2: none of its grids does; tested).

Lane A is the caller's current stream, lane B a second stream.  Tensors that
cross streams are marked with record_stream so the caching allocator never hands
their memory out while the other lane may still use it.
"""
import os

import torch

from . import net, ops

# Off by default (HKP_LANES=2 turns it on): measured on C2, two lanes ran 6.5 %
# SLOWER than one (1345 vs 1438 img/s, same box, interleaved runs).  The x3 conv
# blocks hold all 512 registers per SIMD lane and all 160 KiB of LDS of their CU,
# so a BN apply cannot share a CU with them: the "overlap" only partitions the
# CUs between apply and conv, while the half-batch grids add a second tail round
# and twice the launches.
ENABLED = os.environ.get("HKP_LANES", "1") == "2"
_side = {}


def _stream_b(dev):
    s = _side.get(dev)
    if s is None:
        s = _side[dev] = torch.cuda.Stream(dev)
    return s


def _shapes_ok(resnet, n_half, H, W):
    """Every conv of the net on the x3 path and every conv output's half-batch
    pixel count a multiple of the BN tile (128 rows)."""
    if net.conv_precision() != "f16x3":
        return False
    rows = ops.CONV_TILE_ROWS
    c1 = resnet.conv1
    if not ops.stem_x3_ok((n_half, 3, H, W), tuple(c1.weight.shape), net._i(c1.stride), net._i(c1.padding),
                          net._i(c1.dilation)):
        return False
    h, w = ops.conv_out_hw(H, W, 7, 7, net._i(c1.stride), net._i(c1.padding), net._i(c1.dilation))
    if (n_half * h * w) % rows:
        return False
    h, w = (h - 1) // 2 + 1, (w - 1) // 2 + 1          # maxpool 3x3 / 2, pad 1

    def out(hw, conv):
        k, r, s, c = conv.weight.shape
        if k % 64 or c % 32:
            return None
        o = ops.conv_out_hw(hw[0], hw[1], r, s, net._i(conv.stride), net._i(conv.padding), net._i(conv.dilation))
        return o if (n_half * o[0] * o[1]) % rows == 0 else None

    hw = (h, w)
    for layer in (resnet.layer1, resnet.layer2, resnet.layer3, resnet.layer4):
        for block in layer:
            o = hw
            for conv in [block.conv1, block.conv2] + ([block.conv3] if block.kind == "bottleneck" else []):
                o = out(o, conv)
                if o is None:
                    return False
            if block.downsample is not None and out(hw, block.downsample[0]) is None:
                return False
            hw = o
    return True


def lanes_ok(resnet, x):
    if not ENABLED or x.dim() != 4 or x.shape[0] < 2 or x.shape[0] % 2 or not x.is_cuda:
        return False
    H, W = net.image_nchw_shape(x)[2:]
    return _shapes_ok(resnet, x.shape[0] // 2, H, W)


class _Lanes:
    def __init__(self, dev):
        self.a = torch.cuda.current_stream(dev)
        self.b = _stream_b(dev)

    def on_b(self, *ts):
        for t in ts:
            if t is not None:
                t.record_stream(self.b)

    def each(self, fn, xs):
        """fn(i, x_i) on lane i's stream, no ordering between the lanes."""
        out0 = fn(0, xs[0])
        with torch.cuda.stream(self.b):
            out1 = fn(1, xs[1])
        return [out0, out1]

    def conv_bn(self, conv, bn, xs, layout="nhwc"):
        """Both lanes' conv, partials into one buffer, one finalize on lane A."""
        part = None
        if bn.training:
            k = conv.weight.shape[0]
            if layout == "nchw":
                H, W = net.image_nchw_shape(xs[0])[2:]
                ho, wo = ops.conv_out_hw(H, W, 7, 7, net._i(conv.stride), net._i(conv.padding),
                                         net._i(conv.dilation))
            else:
                _, r, s, _ = conv.weight.shape
                ho, wo = ops.conv_out_hw(xs[0].shape[1], xs[0].shape[2], r, s, net._i(conv.stride),
                                         net._i(conv.padding), net._i(conv.dilation))
            t = xs[0].shape[0] * ho * wo // ops.CONV_TILE_ROWS
            part = torch.empty((2 * t, k, 2), device=xs[0].device, dtype=torch.float32)
            # lane B writes memory lane A's stream just handed out: B waits for A's
            # queue so far (A's previous apply, which B waits for anyway)
            self.b.wait_stream(self.a)
            self.on_b(part)
        ya, _ = net._conv_fwd(conv, bn, xs[0], layout, part_out=part[:t] if part is not None else None, sk=False)
        with torch.cuda.stream(self.b):
            yb, _ = net._conv_fwd(conv, bn, xs[1], layout, part_out=part[t:] if part is not None else None,
                                  sk=False)
        self.a.wait_stream(self.b)
        count = 2 * ya.numel() // ya.shape[-1]
        ss, mi = net._bn_params(bn, part, count)
        self.on_b(ss, mi)
        return [ya, yb], ss, mi

    def apply(self, fn):
        """fn(i) on lane A, then on lane B once A's is done (staggered)."""
        out0 = fn(0)
        self.b.wait_stream(self.a)
        with torch.cuda.stream(self.b):
            out1 = fn(1)
        return [out0, out1]

    def block(self, block, xs, final):
        def act(ys, s):
            sp = net._split_for(ys[0].shape[-1])
            return self.apply(lambda i: ops.bn_apply(ys[i], s, relu=True, split=sp, keep_fp32=not sp))

        y1, s1, _ = self.conv_bn(block.conv1, block.bn1, xs)
        a = act(y1, s1)
        y2, s2, _ = self.conv_bn(block.conv2, block.bn2, a)
        last_y, last_s = y2, s2
        if block.kind == "bottleneck":
            a = act(y2, s2)
            last_y, last_s, _ = self.conv_bn(block.conv3, block.bn3, a)
        pl = net._split_for(last_y[0].shape[-1])
        keep_out = final or pl != 3
        if block.downsample is not None:
            yd, sd, _ = self.conv_bn(block.downsample[0], block.downsample[1], xs)
            return self.apply(lambda i: ops.bn_apply(last_y[i], last_s, res=yd[i], res_ss=sd, relu=True, split=pl,
                                                     keep_fp32=keep_out))
        return self.apply(lambda i: ops.bn_apply(last_y[i], last_s, res=xs[i], relu=True, split=pl,
                                                 keep_fp32=keep_out))


def keypoints_forward_lanes(resnet, x, k, heat=True, argmax=False):
    """net.keypoints_forward (inference, no trace) over two lanes; same outputs."""
    L = _Lanes(x.device)
    n = x.shape[0]
    h = n // 2
    net.prepack_x3(resnet, flip=False)            # on lane A, before lane B forks
    L.b.wait_stream(L.a)
    L.on_b(x)
    xs = [x[:h], x[h:]]
    ins = L.each(lambda i, xi: net._image_input(resnet, xi, None), xs)
    y, ss, _ = L.conv_bn(resnet.conv1, resnet.bn1, ins, layout="nchw")
    sp = net._split_for(y[0].shape[-1])
    feats = L.apply(lambda i: ops.bn_relu_maxpool(y[i], ss, split=sp, route=False, keep_fp32=sp != 3))
    blocks = [b for layer in (resnet.layer1, resnet.layer2, resnet.layer3, resnet.layer4) for b in layer]
    for i, block in enumerate(blocks):
        feats = L.block(block, feats, final=i == len(blocks) - 1)
    w, b = net.fc_rows(resnet, k)
    H, W = net.image_nchw_shape(x)[2:]
    hm = torch.empty((n, k, H, W), device=x.device, dtype=torch.float32) if heat else None
    L.on_b(hm)
    lows = L.each(lambda i, f: ops.head_fc(f, w, b), feats)
    res = L.each(lambda i, lo: ops.upsample_sigmoid(lo, H, W, heat=heat, argmax=argmax,
                                                    out=hm[i * h:(i + 1) * h] if heat else None), lows)
    L.a.wait_stream(L.b)
    for t in (lows[1], res[1][1]):
        if t is not None:
            t.record_stream(L.a)
    yx = torch.cat([res[0][1], res[1][1]]) if argmax else None
    return hm, yx, torch.cat(lows)
