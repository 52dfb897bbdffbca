"""The train-mode BN finalize folded into the producing conv (hkp_bn_fold,
conv_x3.hip x3_fold_tile): on every conv body that writes BN partials, the
conv's own blocks give the separate two-level finalize's bits
(hkp_bn_finalize_ws: scale/shift, mean/invstd, running statistics,
num_batches_tracked), the conv's output and partials are unchanged, and the
arrival counters are left zero (back-to-back calls agree).  Reference: the BN
forward of src/resnet.py:46,49,57,61,78,85,87,139,187 in train mode."""
import pytest
import torch

pytestmark = pytest.mark.gpu

# (precision, n, h, w, cin, cout, k, stride, pad, dil, tile): each body that writes
# partials — over chunks of 64 m-tiles (>= 3 chunks where M allows), ragged M
FOLD_CASES = [
    ("x3", 8, 60, 80, 256, 256, 3, 1, 2, 2, 11),      # A3 + split-K tail, 3 chunks (64, 64, 22 m-tiles)
    ("x3", 8, 60, 80, 256, 256, 3, 1, 2, 2, 0),       # the planner (B=8 shard layer3: stream-K 256x128)
    ("x3", 8, 60, 80, 512, 512, 3, 1, 4, 4, 0),       # the planner (B=8 layer4: A3, two column tiles)
    ("x3", 9, 60, 80, 256, 512, 3, 1, 4, 4, 3),       # 256x256 2-stage body, ragged M
    ("x3", 9, 60, 80, 256, 512, 3, 1, 4, 4, 9),       # 256x256 + tail launch
    ("x3", 5, 37, 41, 128, 256, 3, 1, 1, 1, 2),       # stream-K wherever it splits
    ("x3", 5, 37, 41, 128, 256, 3, 1, 1, 1, 4),       # 256x128 16x16x32
    ("x3", 5, 37, 41, 128, 256, 3, 1, 1, 1, 5),       # 256x128 32x32x16
    ("x3", 5, 37, 41, 128, 128, 3, 1, 1, 1, 6),       # 256x64 pairs
    ("x3", 4, 120, 160, 64, 64, 3, 1, 1, 1, 0),       # halo body (layer1), 150 patches
    ("x3", 2, 31, 41, 64, 128, 1, 2, 0, 1, 0),        # 1x1 stride-2 downsample, one chunk
    ("f16", 8, 60, 80, 512, 256, 1, 1, 0, 1, 0),      # plain fp16 A3
    ("f16", 8, 60, 80, 256, 1024, 1, 1, 0, 1, 0),     # plain fp16, 4 column tiles
    ("f16", 4, 60, 80, 256, 512, 1, 1, 0, 1, 13),     # DUO (two 4-wave blocks per CU)
    ("f16", 2, 120, 160, 64, 64, 3, 1, 1, 1, 0),      # plain fp16 halo body
]


def _bn_params(k, d, seed):
    g = torch.Generator(device=d).manual_seed(seed)
    return (torch.rand(k, device=d, generator=g) + 0.5, torch.rand(k, device=d, generator=g) - 0.5,
            torch.randn(k, device=d, generator=g), torch.rand(k, device=d, generator=g) + 0.5)


def _check(conv, k, rows, d, seed):
    """conv(fold, alt) → (y, part) on input `alt` (0 / 1: two different inputs, so a
    merge that read another call's partials at the same address would show);
    compare with the unfolded conv + hkp_bn_finalize_ws."""
    from hkp import ops
    gamma, beta, rm0, rv0 = _bn_params(k, d, seed)
    for rep, alt in enumerate((0, 1, 0, 1)):      # the counters are left zero: repeated calls agree
        y0, p0 = conv(None, alt)
        rm, rv = rm0.clone(), rv0.clone()
        nbt = torch.zeros(1, device=d, dtype=torch.int64)
        ss, mi = ops.bn_finalize(p0, rows, gamma, beta, rm, rv, nbt, momentum=0.1, eps=1e-5, two_level_tiles=1)
        del p0
        frm, frv = rm0.clone(), rv0.clone()
        fnbt = torch.zeros(1, device=d, dtype=torch.int64)
        fold = ops.FoldBN(gamma, beta, frm, frv, fnbt, momentum=0.1, eps=1e-5)
        y1, p1 = conv(fold, alt)
        torch.cuda.synchronize()
        assert fold.done
        assert torch.equal(y1, y0), rep
        assert torch.equal(fold.scale_shift, ss), (rep, (fold.scale_shift - ss).abs().max().item())
        assert torch.equal(fold.mean_invstd, mi), rep
        assert torch.equal(frm, rm) and torch.equal(frv, rv) and fnbt.item() == 1, rep


@pytest.mark.parametrize("case", FOLD_CASES)
def test_fold_equals_two_level_finalize(cuda_device, case):
    from hkp import ops
    prec, n, h, w, cin, cout, k, st, pad, dil, tile = case
    d = cuda_device
    g = torch.Generator(device=d).manual_seed(n * 131 + cin + cout)
    xa = [torch.relu(torch.randn(n, h, w, cin, device=d, generator=g)) * s for s in (1.0, 1.7)]
    wt = torch.randn(cout, k, k, cin, device=d, generator=g) * (2.0 / (k * k * cout)) ** 0.5
    ho, wo = ops.conv_out_hw(h, w, k, k, st, pad, dil)
    if prec == "x3":
        ss_id = torch.cat([torch.ones(cin, device=d), torch.zeros(cin, device=d)])
        xs = [ops.bn_apply(x, ss_id, relu=False, split=3, keep_fp32=False) for x in xa]
        wp = ops.weight_pack_x3(wt)

        def conv(fold, alt):
            return ops.conv2d_fwd_x3(xs[alt], wp, st, pad, dil, tile=tile, fold=fold)
    else:
        x16, wp = [x.half() for x in xa], ops.weight_pack_f16(wt)

        def conv(fold, alt):
            return ops.conv2d_fwd_f16(x16[alt], wp, st, pad, dil, tile=tile, fold=fold)
    _check(conv, cout, n * ho * wo, d, cin + cout)


@pytest.mark.parametrize("prec", ["x3", "f16"])
def test_fold_fused_input_bn(cuda_device, prec):
    """The halo body with its input's BN applied inside (conv2d_fwd_bnin) folds its
    own finalize too."""
    from hkp import ops
    d = cuda_device
    n, h, w, c = 3, 120, 160, 64
    g = torch.Generator(device=d).manual_seed(77)
    y_in = [torch.randn(n, h, w, c, device=d, generator=g) for _ in range(2)]
    in_ss = torch.cat([torch.rand(c, device=d, generator=g) + 0.5, torch.rand(c, device=d, generator=g) - 0.5])
    wt = torch.randn(64, 3, 3, c, device=d, generator=g) * 0.05
    if prec == "f16":
        y_in = [y.half() for y in y_in]
        wp = ops.weight_pack_f16(wt)
    else:
        wp = ops.weight_pack_x3(wt)

    def conv(fold, alt):
        return ops.conv2d_fwd_bnin(y_in[alt], in_ss, wp, 1, 1, 1, fold=fold)
    _check(conv, 64, n * h * w, d, 5)


@pytest.mark.parametrize("shape,tile", [((4, 3, 480, 640), 0), ((2, 3, 96, 128), 6), ((3, 3, 50, 70), 0)])
def test_fold_stem(cuda_device, shape, tile):
    """The stem: the image-direct patch body (19,200 patches at 480x640 x 4: 300
    chunks), the one-tile stem (HKP_TILE_64_PAIR), the packed-plane stem of a shape
    the patch body does not take."""
    from hkp import ops
    d = cuda_device
    x = [torch.rand(*shape, generator=torch.Generator().manual_seed(s)).to(d) for s in (9, 11)]
    wt = (torch.randn(64, 3, 7, 7, generator=torch.Generator().manual_seed(10)) * 0.05).to(d)
    wp = ops.stem_weight_pack_x3(wt)
    ho, wo = ops.conv_out_hw(shape[2], shape[3], 7, 7, 2, 3, 1)

    def conv(fold, alt):
        return ops.conv2d_fwd_stem_x3(x[alt], wp, 64, tile=tile, fold=fold)
    _check(conv, 64, shape[0] * ho * wo, d, 3)


def test_fold_rejected_where_not_taken(cuda_device):
    """bn_fold on an entry point that does not take it (the fused-epilogue fp16
    conv, the fp32 conv) is an argument error, not ignored; without partials the
    fold does nothing (stats=False)."""
    import ctypes
    from hkp import ops
    from hkp._lib import BnFold, ConvDesc, call
    d = cuda_device
    x = torch.ones(1, 8, 8, 64, device=d)
    w = torch.ones(64, 1, 1, 64, device=d)
    f = BnFold()
    desc = ConvDesc(1, 8, 8, 64, 64, 1, 1, 1, 0, 1, 0, 0)
    desc.bn_fold = ctypes.addressof(f)
    y = torch.empty(1, 8, 8, 64, device=d)
    with pytest.raises(ops.HkpError, match="bn_fold"):
        call("hkp_conv2d_fwd", ctypes.byref(desc), ops._ptr(x), ops._ptr(w), ops._ptr(y), None, ops._stream())
    fold = ops.FoldBN(None, None)
    y2, p2 = ops.conv2d_fwd_f16(x.half(), ops.weight_pack_f16(w), stats=False, fold=fold)
    assert p2 is None and not fold.done


@pytest.mark.parametrize("bb,prec,b,hw", [("resnet34", "f16x3", 2, (96, 128)), ("resnet50", "f16", 2, (96, 128)),
                                          ("resnet34", "f16x3", 8, (480, 640))])
def test_fold_network_equals_two_level(cuda_device, bb, prec, b, hw):
    """A whole forward with every finalize folded (Policy.fold_bn, the default)
    gives the bits of the same forward with every finalize as the separate
    two-level kernels (fold_bn=False, fin_two_level_tiles=1): heatmaps, argmax,
    running statistics."""
    from oracle import recipe
    from src.model import KeypointsGauss
    d = cuda_device
    H, W = hw
    x = recipe.to_tensor_nchw(recipe.seeded_images_u8(b, H, W, 3)).to(d)
    outs = []
    for pol in ({}, dict(fold_bn=False, fin_two_level_tiles=1)):
        m = KeypointsGauss(4, H, W, backbone=bb, pretrained=False, precision=prec)
        m.load_state_dict(recipe.seeded_state_dict(bb, 2))
        m = m.to(d)
        with torch.no_grad():
            hm, yx = m.heatmaps_and_keypoints(x, policy=m.policy.with_(**pol))
        outs.append((hm, yx, [t.clone() for n, t in m.state_dict().items() if "running" in n]))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    for a, c in zip(outs[0][2], outs[1][2]):
        assert torch.equal(a, c)
