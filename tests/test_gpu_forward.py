"""GPU parity of the forward hot path, through the C ABI, against the oracle
(oracle/cpu_ref.py, pinned to the reference's own outputs) and the golden
fixtures.  Tolerances (north_star): heatmaps within 1e-3 abs fp32, argmax (y,x)
bit-exact; per-kernel checks are much tighter."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import cpu_ref, recipe

pytestmark = pytest.mark.gpu


def rand(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g) * scale


CONV_CASES = [
    # n, h, w, cin, cout, k, stride, pad, dil
    (2, 17, 23, 64, 64, 3, 1, 1, 1),
    (2, 30, 40, 64, 128, 3, 2, 1, 1),     # layer2.0.conv1 (stride 2)
    (2, 30, 40, 64, 128, 1, 2, 0, 1),     # layer2 downsample 1x1/s2
    (1, 15, 20, 128, 256, 3, 1, 2, 2),    # layer3 (dilation 2)
    (1, 15, 20, 256, 512, 3, 1, 4, 4),    # layer4 (dilation 4)
    (3, 9, 11, 96, 192, 3, 1, 1, 1),      # odd sizes, M not a multiple of 128, Cout%128!=0
    (1, 12, 16, 256, 1024, 1, 1, 0, 1),   # bottleneck 1x1 expand
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_matches_oracle(cuda_device, case):
    from hkp import ops
    n, h, w, cin, cout, k, st, pad, dil = case
    x = rand(n, cin, h, w, seed=1)
    wt = rand(cout, cin, k, k, seed=2, scale=(2.0 / (k * k * cout)) ** 0.5)
    ref = F.conv2d(x, wt, None, st, pad, dil)
    y, part = ops.conv2d_fwd(x.permute(0, 2, 3, 1).contiguous().to(cuda_device),
                             wt.permute(0, 2, 3, 1).contiguous().to(cuda_device), st, pad, dil)
    got = y.cpu().permute(0, 3, 1, 2)
    scale = ref.abs().max().item()
    assert (got - ref).abs().max().item() < 2e-5 * max(1.0, scale)
    # BN partials: tile sums and M2 reproduce the per-channel batch statistics
    p = part.cpu().double()
    cnt = n * ref.shape[2] * ref.shape[3]
    mean = p[:, :, 0].sum(0) / cnt
    tiles = p.shape[0]
    nt = torch.tensor([min(128, cnt - t * 128) for t in range(tiles)], dtype=torch.float64)[:, None]
    m2 = (p[:, :, 1] + nt * (p[:, :, 0] / nt - mean) ** 2).sum(0)
    r64 = ref.double()
    np.testing.assert_allclose(mean.numpy(), r64.mean((0, 2, 3)).numpy(), rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose((m2 / cnt).numpy(), r64.var((0, 2, 3), unbiased=False).numpy(), rtol=1e-4, atol=1e-8)


def test_stem_conv_matches_oracle(cuda_device):
    from hkp import ops
    x = torch.rand(2, 3, 50, 70, generator=torch.Generator().manual_seed(3))
    wt = rand(64, 3, 7, 7, seed=4, scale=(2.0 / (49 * 64)) ** 0.5)
    ref = F.conv2d(x, wt, None, 2, 3)
    y, _ = ops.conv2d_fwd(x.to(cuda_device), wt.to(cuda_device), 2, 3, 1, layout="nchw")
    assert (y.cpu().permute(0, 3, 1, 2) - ref).abs().max().item() < 1e-5


def test_bn_train_stats_and_apply(cuda_device):
    from hkp import ops
    n, h, w, c = 2, 19, 21, 128
    x = rand(n, c, h, w, seed=5) * 3 + 1.5
    wt = rand(c, c, 1, 1, seed=6, scale=0.1)
    y_ref = F.conv2d(x, wt)
    gamma, beta = rand(c, seed=7) * 0.2 + 1, rand(c, seed=8) * 0.1
    rm, rv = rand(c, seed=9) * 0.1, torch.rand(c) + 0.5
    rm_ref, rv_ref = rm.clone(), rv.clone()
    out_ref = F.relu(F.batch_norm(y_ref, rm_ref, rv_ref, gamma, beta, True, 0.1, 1e-5))
    d = cuda_device
    y, part = ops.conv2d_fwd(x.permute(0, 2, 3, 1).contiguous().to(d), wt.permute(0, 2, 3, 1).contiguous().to(d))
    rm_g, rv_g, nbt = rm.to(d), rv.to(d), torch.zeros((), dtype=torch.int64, device=d)
    ss, mi = ops.bn_finalize(part, n * h * w, gamma.to(d), beta.to(d), rm_g, rv_g, nbt)
    out = ops.bn_apply(y, ss, relu=True)
    np.testing.assert_allclose(out.cpu().permute(0, 3, 1, 2).numpy(), out_ref.numpy(), atol=2e-5)
    np.testing.assert_allclose(rm_g.cpu().numpy(), rm_ref.numpy(), atol=1e-6)
    np.testing.assert_allclose(rv_g.cpu().numpy(), rv_ref.numpy(), rtol=1e-5)
    assert nbt.item() == 1
    # residual forms
    res = rand(n, h, w, c, seed=10).to(d)
    rss = torch.cat([rand(c, seed=11), rand(c, seed=12)]).to(d)
    o1 = ops.bn_apply(y, ss, res=res, relu=True).cpu()
    o2 = ops.bn_apply(y, ss, res=res, res_ss=rss, relu=True).cpu()
    base = y.cpu() * ss[:c].cpu() + ss[c:].cpu()
    assert (o1 - F.relu(base + res.cpu())).abs().max() < 1e-5
    r2 = res.cpu() * rss[:c].cpu() + rss[c:].cpu()
    assert (o2 - F.relu(base + r2)).abs().max() < 1e-5


def test_bn_relu_maxpool(cuda_device):
    from hkp import ops
    y = rand(2, 25, 31, 64, seed=13)
    ss = torch.cat([rand(64, seed=14), rand(64, seed=15)])
    ref = F.max_pool2d(F.relu(y.permute(0, 3, 1, 2) * ss[:64, None, None] + ss[64:, None, None]), 3, 2, 1)
    out = ops.bn_relu_maxpool(y.to(cuda_device), ss.to(cuda_device))
    assert (out.cpu().permute(0, 3, 1, 2) - ref).abs().max() < 1e-6


def upsample_emulated(low, H, W):
    """The exact fp32 arithmetic of ATen's CPU bilinear align_corners=True kernel
    as measured on the fixture-generating host (torch 2.10, contracted form
    t = fma(x0, l0, x1*l1)); host-ISA independent, so it pins the GPU bitwise."""
    f = np.float32
    x = low.numpy().astype(f)
    h, w = x.shape[2:]

    def idx(inn, out):
        scale = f(inn - 1) / f(out - 1)
        src = (scale * np.arange(out, dtype=f)).astype(f)
        i0 = np.minimum(np.floor(src).astype(np.int64), inn - 1)
        l1 = np.clip((src - i0.astype(f)).astype(f), f(0), f(1))
        return i0, i0 + (i0 < inn - 1), (f(1) - l1).astype(f), l1

    def fma(a, b, c):
        return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(f)

    h0, h1, lh0, lh1 = idx(h, H)
    w0, w1, lw0, lw1 = idx(w, W)

    def row(hi):
        return fma(x[:, :, hi][..., w0], lw0, (x[:, :, hi][..., w1] * lw1).astype(f))
    return torch.from_numpy(fma(row(h0), lh0[:, None], (row(h1) * lh1[:, None]).astype(f)))


@pytest.mark.parametrize("shape", [(2, 4, 12, 16, 96, 128), (1, 4, 60, 80, 480, 640), (2, 3, 10, 13, 75, 100)])
def test_upsample_sigmoid_bitwise_and_argmax(cuda_device, shape):
    from hkp import ops
    n, k, h, w, H, W = shape
    low = rand(n, k, h, w, seed=16)
    up = F.interpolate(low, size=(H, W), mode="bilinear", align_corners=True)
    raw, _ = ops.upsample_sigmoid(low.to(cuda_device), H, W, heat=True, argmax=False, sigmoid=False)
    assert torch.equal(raw.cpu(), upsample_emulated(low, H, W)), "upsample not bit-identical to the ATen formula"
    assert (raw.cpu() - up).abs().max() < 1e-6   # this host's ATen build (ISA-dependent contraction)
    hm, yx = ops.upsample_sigmoid(low.to(cuda_device), H, W, heat=True, argmax=True)
    ref = torch.sigmoid(up)
    assert (hm.cpu() - ref).abs().max() < 2e-7
    assert np.array_equal(yx.cpu().numpy(), cpu_ref.argmax_yx(hm.cpu()))
    _, yx2 = ops.upsample_sigmoid(low.to(cuda_device), H, W, heat=False, argmax=True)
    assert torch.equal(yx2, yx)


def test_argmax_ties_first_index(cuda_device):
    from hkp import ops
    low = torch.full((1, 2, 4, 5), 30.0)   # sigmoid saturates to exactly 1.0 everywhere → all ties
    low[0, 1, 2:, :] = 40.0
    _, yx = ops.upsample_sigmoid(low.to(cuda_device), 16, 20, heat=False, argmax=True)
    assert yx.cpu().tolist() == [[[0, 0], [0, 0]]]


def test_head_fc(cuda_device):
    from hkp import ops
    feat = rand(2, 6, 7, 512, seed=17)
    w = rand(1000, 512, seed=18, scale=0.01)
    b = rand(1000, seed=19, scale=0.01)
    ref = F.conv2d(feat.permute(0, 3, 1, 2), w[:, :, None, None], b)[:, :8]
    low = ops.head_fc(feat.to(cuda_device), w[:8].contiguous().to(cuda_device), b[:8].contiguous().to(cuda_device))
    assert (low.cpu() - ref).abs().max() < 1e-5


HEAD_CASES = [
    # n, h, w, C, K, y dtype, residual kind (0 none, 1 raw, 2 affine, 3 packed split)
    (2, 7, 9, 512, 4, "f32", 3),      # C2's last BasicBlock (split-only residual stream)
    (1, 5, 13, 512, 4, "f32", 1),     # fp32 residual (fp32 precision mode)
    (1, 6, 6, 512, 16, "f32", 2),     # downsample residual, K = 16
    (1, 3, 5, 1024, 8, "f32", 0),     # two waves per pixel, ragged M (15 pixels)
    (2, 5, 7, 2048, 8, "f16", 1),     # C4's last Bottleneck (fp16 residual stream)
    (1, 4, 9, 2048, 3, "f16", 2),     # K = 3 < KP
    (1, 3, 11, 512, 8, "f16", 0),     # fp16, no residual, ragged 16-pixel group
    (16, 60, 80, 512, 8, "f16", 1),   # fp16, more 16-pixel groups than the grid's waves
]


@pytest.mark.parametrize("case", HEAD_CASES)
def test_bn_apply_head_fused(cuda_device, case):
    """hkp_bn_apply_head = the final block's BN apply (+ residual, ReLU) followed by
    the K-row head, against the same two steps in float64 (and the activation it
    fuses is exactly hkp_bn_apply's / hkp_bn_apply_f16's).  fp16 y (config C4,
    K <= 8): the activation and the head rows enter the head as fp16, as under
    autocast (MFMA head, fp32 accumulation) — the float64 reference rounds both
    the same way."""
    from hkp import ops
    n, h, w, c, k, yt, kind = case
    dt = torch.float16 if yt == "f16" else torch.float32
    y = rand(n, h, w, c, seed=11).to(dt)
    ss = torch.cat([rand(c, seed=12) * 0.5 + 1.0, rand(c, seed=13) * 0.3])
    res = rss = None
    res_dev = None
    if kind in (1, 2):
        res = rand(n, h, w, c, seed=14).to(dt)
        res_dev = res.to(cuda_device)
    if kind == 2:
        rss = torch.cat([rand(c, seed=15) * 0.5 + 1.0, rand(c, seed=16) * 0.3])
    if kind == 3:
        res = rand(n, h, w, c, seed=14)
        res_dev = ops.split_pack_x3(res.to(cuda_device))
        hi = res.half().float()
        res = hi + (res - hi).half().float()           # what the packed pair holds
    wk = rand(k, c, seed=17) * 0.05
    bk = rand(k, seed=18)
    low = ops.bn_apply_head(y.to(cuda_device), ss.to(cuda_device), res_dev,
                            None if rss is None else rss.to(cuda_device), wk.to(cuda_device), bk.to(cuda_device))
    o = y.double() * ss[:c].double() + ss[c:].double()
    if res is not None:
        r = res.double()
        o = o + (r * rss[:c].double() + rss[c:].double() if rss is not None else r)
    o = o.clamp_min(0)
    wr = wk.double()
    if yt == "f16" and k <= 8:
        # the kernel's fp32 apply (two roundings per op), then fp16: computed the
        # same way here so no fp16 rounding tie breaks differently
        o32 = y.float() * ss[:c] + ss[c:]
        if res is not None:
            o32 = o32 + (res.float() * rss[:c] + rss[c:] if rss is not None else res.float())
        o, wr = o32.clamp_min(0).half().double(), wk.half().double()
    ref = torch.einsum("nhwc,kc->nkhw", o, wr) + bk.double()[None, :, None, None]
    got = low.cpu().double()
    assert got.shape == ref.shape
    assert (got - ref).abs().max().item() < 2e-5 * max(1.0, ref.abs().max().item())


def test_gauss_target_matches_reference(cuda_device, golden):
    from hkp import ops
    g = golden("gauss")
    for i in range(3):
        w, h, s = (int(v) for v in g["case%d_whs" % i])
        uv = np.stack([g["case%d_U" % i], g["case%d_V" % i]], -1).astype(np.float32)[None]
        out = ops.gauss_target(torch.from_numpy(uv).to(cuda_device), h, w, s).cpu().numpy()[0]
        ref = g["case%d_G" % i]
        # expf on the GPU vs Sleef on the CPU: at most 1 ulp of fp32
        np.testing.assert_allclose(out, ref, rtol=2.4e-7, atol=1e-30)
        assert (out == ref).mean() > 0.9


FWD_CASES = ["fwd_r18_k2_96x128", "fwd_r34_k4_96x128", "fwd_r34_k4_75x100", "fwd_r50_k8_96x128"]


def _model(bb, k, wseed, dev):
    from src.model import KeypointsGauss
    m = KeypointsGauss(k, backbone=bb, pretrained=False)
    m.load_state_dict(recipe.seeded_state_dict(bb, wseed))
    return m.to(dev)


@pytest.mark.parametrize("case", FWD_CASES)
def test_forward_matches_golden(cuda_device, golden, case):
    g = golden(case)
    bb, k = str(g["backbone"]), int(g["k"])
    m = _model(bb, k, int(g["wseed"]), cuda_device)
    x = recipe.to_tensor_nchw(g["images_u8"]).to(cuda_device)
    with torch.no_grad():
        hm, yx = m.heatmaps_and_keypoints(x)
    err = (hm.cpu().numpy() - g["heat"]).__abs__().max()
    assert err < 1e-3, err
    assert np.array_equal(yx.cpu().numpy(), g["argmax_yx"])
    # BN running statistics updated like nn.BatchNorm2d in train mode
    sd = m.state_dict()
    np.testing.assert_allclose(sd["resnet.%s_8s.bn1.running_var" % bb].cpu().numpy(), g["bn1_running_var"],
                               rtol=1e-4)
    assert int(sd["resnet.%s_8s.bn1.num_batches_tracked" % bb]) == 1


def test_forward_full_size_r34(cuda_device, golden):
    g = golden("fwd_r34_k4_480x640")
    m = _model("resnet34", 4, int(g["wseed"]), cuda_device)
    x = recipe.to_tensor_nchw(g["images_u8"]).to(cuda_device)
    with torch.no_grad():
        hm, yx = m.heatmaps_and_keypoints(x)
    assert np.array_equal(yx.cpu().numpy(), g["argmax_yx"])
    np.testing.assert_allclose(hm.double().sum(3).cpu().numpy(), g["heat_row_sum"], rtol=1e-4)


def test_eval_mode_bn(cuda_device, golden):
    g = golden("fwd_r34_k4_96x128")
    m = _model("resnet34", 4, int(g["wseed"]), cuda_device).eval()
    x = recipe.to_tensor_nchw(g["images_u8"]).to(cuda_device)
    with torch.no_grad():
        hm = m(x)
    assert (hm.cpu().numpy() - g["heat_eval"]).__abs__().max() < 1e-3


def test_forward_deterministic(cuda_device):
    m = _model("resnet18", 2, 0, cuda_device)
    x = torch.rand(2, 3, 64, 96, generator=torch.Generator().manual_seed(0)).to(cuda_device)
    with torch.no_grad():
        a = m(x)
        b = m(x)
    assert torch.equal(a, b)
