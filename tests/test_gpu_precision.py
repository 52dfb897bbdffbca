"""Split-precision fp16 MFMA conv ("f16x3", fp32-accurate) and plain fp16 ("f16",
BASELINE config C4): accuracy vs an fp64 oracle, and full-network parity."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import cpu_ref, recipe

pytestmark = pytest.mark.gpu

CASES = [
    (2, 17, 23, 64, 64, 3, 1, 1, 1),
    (2, 30, 40, 64, 128, 3, 2, 1, 1),
    (1, 15, 20, 128, 256, 3, 1, 2, 2),
    (1, 15, 20, 512, 512, 3, 1, 4, 4),     # layer4 shape: K = 4608
    (3, 9, 11, 96, 192, 3, 1, 1, 1),
    (1, 12, 16, 256, 1024, 1, 1, 0, 1),
]


def rand(*shape, seed=0, scale=1.0):
    return torch.randn(*shape, generator=torch.Generator().manual_seed(seed)) * scale


@pytest.mark.parametrize("case", CASES)
def test_f16x3_is_fp32_accurate(cuda_device, case):
    from hkp import ops
    n, h, w, cin, cout, k, st, pad, dil = case
    x = F.relu(rand(n, cin, h, w, seed=1))            # post-ReLU activations, like the network's
    wt = rand(cout, cin, k, k, seed=2, scale=(2.0 / (k * k * cout)) ** 0.5)
    ref = F.conv2d(x.double(), wt.double(), None, st, pad, dil)
    xd = x.permute(0, 2, 3, 1).contiguous().to(cuda_device)
    wd = wt.permute(0, 2, 3, 1).contiguous().to(cuda_device)
    y32, p32 = ops.conv2d_fwd(xd, wd, st, pad, dil)
    hi, lo = ops.weight_split(wd, 3)
    y3, p3 = ops.conv2d_fwd_split(xd, hi, lo, 3, st, pad, dil)
    scale = ref.abs().max().item()
    e32 = (y32.cpu().double().permute(0, 3, 1, 2) - ref).abs().max().item() / scale
    e3 = (y3.cpu().double().permute(0, 3, 1, 2) - ref).abs().max().item() / scale
    assert e3 < 2e-6, (e3, e32)             # fp32-class error (fp32 MFMA itself: e32)
    assert e3 < 10 * max(e32, 1e-7)
    # BN partials identical in form to the fp32 kernel's
    assert torch.allclose(p3, p32, rtol=1e-4, atol=1e-3)
    hi1, _ = ops.weight_split(wd, 1)
    y1, _ = ops.conv2d_fwd_split(xd, hi1, None, 1, st, pad, dil)
    e1 = (y1.cpu().double().permute(0, 3, 1, 2) - ref).abs().max().item() / scale
    assert 1e-5 < e1 < 5e-3, e1             # genuinely fp16 operands


@pytest.mark.parametrize("case", [c for c in CASES if c[6] == 1 and c[3] % 64 == 0])
@pytest.mark.parametrize("gscale", [1.0, 1e-9])
def test_f16x3_dgrad_scaled(cuda_device, case, gscale):
    """Backward-data on the split kernel: fp32-class accuracy even for gradients
    far below fp16's normal range (power-of-two scaling from max|dy|)."""
    from hkp import ops
    n, h, w, cin, cout, k, st, pad, dil = case
    wt = rand(cout, cin, k, k, seed=5, scale=(2.0 / (k * k * cout)) ** 0.5)
    ho = (h + 2 * pad - dil * (k - 1) - 1) + 1
    wo = (w + 2 * pad - dil * (k - 1) - 1) + 1
    gy = rand(n, cout, ho, wo, seed=6) * gscale
    add = rand(n, cin, h, w, seed=7) * gscale
    ref = torch.nn.grad.conv2d_input((n, cin, h, w), wt.double(), gy.double(), 1, pad, dil) + add.double()
    d = cuda_device
    gy_d = gy.permute(0, 2, 3, 1).contiguous().to(d)
    hi, lo = ops.conv_weight_flip_split(wt.permute(0, 2, 3, 1).contiguous().to(d))
    dx = ops.conv2d_bwd_data_split(gy_d, hi, lo, (n, h, w, cin), pad, dil,
                                   add=add.permute(0, 2, 3, 1).contiguous().to(d), amax=ops.absmax(gy_d))
    err = (dx.cpu().double().permute(0, 3, 1, 2) - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-6, err


@pytest.mark.parametrize("case", [c for c in CASES if c[3] % 64 == 0 and c[4] % 64 == 0]
                         + [(2, 31, 41, 64, 128, 1, 2, 0, 1)])
@pytest.mark.parametrize("gscale", [1.0, 1e-9])
def test_f16x3_wgrad_scaled(cuda_device, case, gscale):
    from hkp import ops
    n, h, w, cin, cout, k, st, pad, dil = case
    x = F.relu(rand(n, cin, h, w, seed=8))
    ho = (h + 2 * pad - dil * (k - 1) - 1) // st + 1
    wo = (w + 2 * pad - dil * (k - 1) - 1) // st + 1
    gy = rand(n, cout, ho, wo, seed=9) * gscale
    ref = torch.nn.grad.conv2d_weight(x.double(), (cout, cin, k, k), gy.double(), st, pad, dil)
    d = cuda_device
    gy_d = gy.permute(0, 2, 3, 1).contiguous().to(d)
    dw = ops.conv2d_bwd_filter_split(x.permute(0, 2, 3, 1).contiguous().to(d), gy_d, (cout, k, k, cin), st, pad,
                                     dil, amax=ops.absmax(gy_d))
    err = (dw.cpu().double().permute(0, 3, 1, 2) - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-6, err


def _model(bb, k, wseed, dev):
    from src.model import KeypointsGauss
    m = KeypointsGauss(k, backbone=bb, pretrained=False)
    m.load_state_dict(recipe.seeded_state_dict(bb, wseed))
    return m.to(dev)


@pytest.fixture
def precision():
    from hkp import net
    old = net.conv_precision()
    yield net.set_conv_precision
    net.set_conv_precision(old)


@pytest.mark.parametrize("case", ["fwd_r18_k2_96x128", "fwd_r34_k4_96x128", "fwd_r34_k4_75x100",
                                  "fwd_r50_k8_96x128", "fwd_r34_k4_480x640"])
def test_f16x3_forward_matches_golden(cuda_device, golden, precision, case):
    precision("f16x3")
    g = golden(case)
    bb, k = str(g["backbone"]), int(g["k"])
    m = _model(bb, k, int(g["wseed"]), cuda_device)
    x = recipe.to_tensor_nchw(g["images_u8"]).to(cuda_device)
    with torch.no_grad():
        hm, yx = m.heatmaps_and_keypoints(x)
    assert np.array_equal(yx.cpu().numpy(), g["argmax_yx"])
    if "heat" in g:
        assert np.abs(hm.cpu().numpy() - g["heat"]).max() < 1e-3
    else:
        np.testing.assert_allclose(hm.double().sum(3).cpu().numpy(), g["heat_row_sum"], rtol=1e-4)


def test_f16_forward_close_to_reference(cuda_device, golden, precision):
    """Plain fp16 operands (config C4): heatmaps close, argmax reported not promised."""
    precision("f16")
    g = golden("fwd_r50_k8_96x128")
    m = _model("resnet50", 8, int(g["wseed"]), cuda_device)
    x = recipe.to_tensor_nchw(g["images_u8"]).to(cuda_device)
    with torch.no_grad():
        hm, yx = m.heatmaps_and_keypoints(x)
    err = np.abs(hm.cpu().numpy() - g["heat"]).max()
    agree = (yx.cpu().numpy() == g["argmax_yx"]).all(-1).mean()
    print("fp16 R50: max heat err %.3g, argmax agreement %.2f" % (err, agree))
    assert err < 1e-1 and agree >= 0.5   # fp16 operands through 53 train-mode-BN layers
