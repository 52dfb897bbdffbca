"""BN statistics from the input's second moments and the fused BN-apply epilogue
(config C4's Bottleneck tail: conv3 -> bn3 -> + residual -> ReLU in one launch).

* hkp_gram_f16: mean and covariance of an fp16 activation vs fp64 torch, every
  tile width (C = 64 .. 512), ragged row counts, multi-split reductions;
* hkp_bn_from_gram: the scale/shift, mean/invstd and running statistics of a 1x1
  conv's output vs hkp_bn_finalize over that output's own tile partials, and vs
  fp64 statistics of the fp64 conv of the same fp16 operands;
* hkp_conv2d_fwd_f16_bn == hkp_conv2d_fwd_f16 + hkp_bn_apply_f16 with the same
  scale/shift, bit for bit (raw and scaled residual, no residual, every tile body);
* the R50 network in plain fp16 with the fused tail (the default policy) vs the
  unfused one: same argmax, heatmaps within fp16 noise.
"""
import numpy as np
import pytest
import torch

from oracle import recipe

pytestmark = pytest.mark.gpu


def _relu_f16(shape, seed, dev):
    g = torch.Generator(device=dev).manual_seed(seed)
    return torch.relu(torch.randn(*shape, device=dev, generator=g) * 0.7 + 0.2).half()


@pytest.mark.parametrize("m,c", [(1000, 64), (4096 + 17, 128), (30000, 256), (61440 + 5, 512), (257, 64)])
def test_gram_f16_matches_fp64(cuda_device, m, c):
    from hkp import ops
    a = _relu_f16((m, c), m + c, cuda_device)
    a._hkp_split_passes = 1
    mean, e2 = ops.gram_f16(a)
    a64 = a.double()
    mu = a64.mean(0)
    ref = a64.T @ a64 / m
    assert torch.allclose(mean, mu, rtol=1e-6, atol=1e-9)
    err = (e2 - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-6, err
    cov = e2 - torch.outer(mean, mean)                 # the centred form the statistics use
    cref = (a64 - mu).T @ (a64 - mu) / m
    assert (cov - cref).abs().max().item() < 2e-6 * ref.abs().max().item()
    assert torch.equal(e2, e2.T)                       # written symmetric
    mean2, e22 = ops.gram_f16(a)                       # deterministic
    assert torch.equal(mean, mean2) and torch.equal(e2, e22)


def _bn_params(k, seed, dev):
    g = torch.Generator(device=dev).manual_seed(seed)
    gamma = torch.rand(k, device=dev, generator=g) + 0.5
    beta = torch.rand(k, device=dev, generator=g) - 0.5
    return gamma, beta


@pytest.mark.parametrize("n,h,w,c,k", [(2, 30, 40, 64, 256), (3, 17, 23, 128, 512), (1, 60, 80, 256, 1024),
                                       (2, 15, 20, 512, 2048)])
def test_bn_from_gram_matches_output_statistics(cuda_device, n, h, w, c, k):
    from hkp import ops
    d = cuda_device
    x = _relu_f16((n, h, w, c), 7 + c, d)
    x._hkp_split_passes = 1
    wt = torch.randn(k, 1, 1, c, device=d, generator=torch.Generator(device=d).manual_seed(3)) * (2.0 / c) ** 0.5
    wp = ops.weight_pack_f16(wt)
    gamma, beta = _bn_params(k, 5, d)
    m = n * h * w
    # reference 1: the unfused path's statistics (conv tile partials -> bn_finalize)
    y, part = ops.conv2d_fwd_f16(x, wp)
    rm1, rv1 = torch.zeros(k, device=d), torch.ones(k, device=d)
    nb1 = torch.zeros(1, device=d, dtype=torch.int64)
    ss1, mi1 = ops.bn_finalize(part, m, gamma, beta, rm1, rv1, nb1)
    # reference 2: fp64 statistics of the fp64 conv of the same fp16 operands
    wd = wp.split.double().reshape(k, c) * wp.inv_scale.double()[:, None]
    y64 = x.double().reshape(m, c) @ wd.T
    mean64, var64 = y64.mean(0), y64.var(0, unbiased=False)
    mean, e2 = ops.gram_f16(x)
    rm2, rv2 = torch.zeros(k, device=d), torch.ones(k, device=d)
    nb2 = torch.zeros(1, device=d, dtype=torch.int64)
    ss2, mi2 = ops.bn_from_gram(mean, e2, wp, m, gamma, beta, rm2, rv2, nb2)
    sd = var64.sqrt()
    assert ((mi2[:k].double() - mean64).abs() <= 1e-5 * sd + 1e-7).all()
    assert torch.allclose(mi2[k:].double(), 1 / torch.sqrt(var64 + 1e-5), rtol=2e-5)
    # the partial-based statistics agree as closely (both from fp32 sums)
    assert torch.allclose(mi2[k:], mi1[k:], rtol=3e-5)
    assert torch.allclose(ss2, ss1, rtol=3e-5, atol=3e-5)
    assert torch.allclose(rm2, rm1, rtol=1e-4, atol=1e-6) and torch.allclose(rv2, rv1, rtol=1e-4, atol=1e-6)
    assert nb2.item() == 1


@pytest.mark.parametrize("res_kind", ["none", "raw", "scaled"])
@pytest.mark.parametrize("tile", [0, 3, 4, 5, 6, 11, 13])
def test_fused_epilogue_equals_conv_plus_apply(cuda_device, res_kind, tile):
    from hkp import ops
    d = cuda_device
    n, h, w, c, k = 2, 31, 41, 128, 256 if tile != 6 else 128
    x = _relu_f16((n, h, w, c), 11, d)
    x._hkp_split_passes = 1
    wt = torch.randn(k, 1, 1, c, device=d, generator=torch.Generator(device=d).manual_seed(12)) * 0.1
    wp = ops.weight_pack_f16(wt)
    g = torch.Generator(device=d).manual_seed(13)
    ss = torch.cat([torch.rand(k, device=d, generator=g) + 0.5, torch.rand(k, device=d, generator=g) - 0.5])
    res = rss = None
    if res_kind != "none":
        res = torch.randn(n, h, w, k, device=d, generator=g).half()
    if res_kind == "scaled":
        rss = torch.cat([torch.rand(k, device=d, generator=g) + 0.5, torch.rand(k, device=d, generator=g) - 0.5])
    y, _ = ops.conv2d_fwd_f16(x, wp, stats=False, tile=tile)
    ref = ops.bn_apply_f16(y, ss, res=res, res_ss=rss, relu=True)
    got = ops.conv2d_fwd_f16_bn(x, wp, ss, res=res, res_ss=rss, relu=True, tile=tile)
    assert got.dtype == torch.float16 and got.shape == ref.shape
    assert torch.equal(got, ref)


@pytest.mark.parametrize("case", ["fwd_r50_k8_96x128", "fwd_r50_k8_480x640_b2"])
def test_r50_f16_fused_tail_vs_unfused(cuda_device, golden, case):
    """The plain-fp16 R50 forward with the Gram-statistics fused tail (default) vs
    the unfused conv3 + partial-statistics + apply path: argmax equal, heatmaps
    within fp16 noise, BN running statistics within fp32 rounding."""
    import hashlib
    from hkp.policy import DEFAULT
    from src.model import KeypointsGauss
    g = golden(case)
    K = int(g["k"])
    if "images_u8" in g:
        imgs = g["images_u8"]
    else:
        imgs = recipe.seeded_images_u8(int(g["batch"]), int(g["height"]), int(g["width"]), int(g["iseed"]))
        assert hashlib.sha256(imgs.tobytes()).hexdigest() == str(g["images_sha256"])
    x = recipe.to_tensor_nchw(imgs).to(cuda_device)
    out = {}
    for fused in (True, False):
        m = KeypointsGauss(K, backbone="resnet50", pretrained=False,
                           policy=DEFAULT.with_(precision="f16", gram_bn=fused))
        m.load_state_dict(recipe.seeded_state_dict("resnet50", int(g["wseed"])))
        m = m.to(cuda_device)
        with torch.no_grad():
            hm, yx = m.heatmaps_and_keypoints(x)
        out[fused] = (hm, yx, {kk: v.clone() for kk, v in m.state_dict().items() if "running" in kk})
    (h1, y1, s1), (h0, y0, s0) = out[True], out[False]
    d = (h1 - h0).abs().max().item()
    agree = (y1 == y0).all(-1).float().mean().item()
    ref_err = np.abs(h1.cpu().numpy()[..., ::int(g["step"]), ::int(g["step"])] - g["heat_sub"]).max() \
        if "heat_sub" in g else np.abs(h1.cpu().numpy() - g["heat"]).max()
    print("%s: fused vs unfused heat max diff %.3g, argmax agreement %.3f, fused vs reference %.3g"
          % (case, d, agree, ref_err))
    assert d < 0.1 and agree >= 0.75 and ref_err < 0.08
    # running statistics: the fp16 noise of the two paths propagates through the
    # later train-mode BN layers (measured 0.4 % of a tensor's largest entry)
    worst = max((s1[kk] - s0[kk]).abs().max().item() / (s0[kk].abs().max().item() + 1e-6) for kk in s0)
    assert worst < 2e-2, worst
