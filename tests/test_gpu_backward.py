"""GPU parity of the backward / training path through the C ABI, against torch
CPU autograd on the oracle's functional restatement and the reference-generated
train-step goldens."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import REPO
from oracle import cpu_ref, recipe

pytestmark = pytest.mark.gpu


def rand(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g) * scale


def nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def nchw(t):
    return t.permute(0, 3, 1, 2)


CASES = [
    # n, h, w, cin, cout, k, stride, pad, dil
    (2, 17, 23, 64, 64, 3, 1, 1, 1),
    (2, 30, 40, 64, 128, 3, 2, 1, 1),     # strided 3x3 → transposed dgrad loader
    (2, 31, 41, 64, 128, 1, 2, 0, 1),     # strided 1x1 downsample, odd input
    (1, 15, 20, 128, 256, 3, 1, 2, 2),    # dilation 2
    (1, 15, 20, 256, 512, 3, 1, 4, 4),    # dilation 4
    (2, 9, 11, 128, 192, 3, 1, 1, 1),     # Cout % 128 != 0, M not a multiple of 128
    (1, 12, 16, 256, 1024, 1, 1, 0, 1),   # bottleneck expand
]


@pytest.mark.parametrize("case", CASES)
def test_conv_backward(cuda_device, case):
    from hkp import ops
    n, h, w, cin, cout, k, st, pad, dil = case
    x = rand(n, cin, h, w, seed=1).requires_grad_(True)
    wt = (rand(cout, cin, k, k, seed=2) * (2.0 / (k * k * cout)) ** 0.5).requires_grad_(True)
    y = F.conv2d(x, wt, None, st, pad, dil)
    gy = rand(*y.shape, seed=3)
    y.backward(gy)
    d = cuda_device
    wk = nhwc(wt.detach()).to(d)
    add = rand(n, h, w, cin, seed=4).to(d)
    dx = ops.conv2d_bwd_data(nhwc(gy).to(d), ops.conv_weight_flip(wk), (n, h, w, cin), st, pad, dil, add=add)
    ref_dx = x.grad + nchw(add.cpu())
    assert (nchw(dx.cpu()) - ref_dx).abs().max() < 2e-5 * max(1, ref_dx.abs().max().item())
    dw = ops.conv2d_bwd_filter(nhwc(x.detach()).to(d), nhwc(gy).to(d), tuple(wk.shape), st, pad, dil)
    ref_dw = wt.grad
    err = (nchw(dw.cpu()) - ref_dw).abs().max().item()
    assert err < 2e-5 * max(1, ref_dw.abs().max().item()), err


def test_stem_wgrad(cuda_device):
    from hkp import ops
    x = torch.rand(2, 3, 50, 70, generator=torch.Generator().manual_seed(3))
    wt = (rand(64, 3, 7, 7, seed=4) * 0.05).requires_grad_(True)
    y = F.conv2d(x, wt, None, 2, 3)
    gy = rand(*y.shape, seed=5)
    y.backward(gy)
    dw = ops.conv2d_bwd_filter(x.to(cuda_device), nhwc(gy).to(cuda_device), (64, 3, 7, 7), 2, 3, 1, layout="nchw")
    assert (dw.cpu() - wt.grad).abs().max() < 2e-5 * wt.grad.abs().max()


@pytest.mark.parametrize("mask", [True, False])
@pytest.mark.parametrize("c", [64, 256, 2048])
def test_bn_backward(cuda_device, mask, c):
    from hkp import ops
    n, h, w = 2, 7, 9
    y = (rand(n, c, h, w, seed=6) * 2 + 0.3).requires_grad_(True)
    gamma = (rand(c, seed=7) * 0.2 + 1).requires_grad_(True)
    beta = (rand(c, seed=8) * 0.1).requires_grad_(True)
    z = F.batch_norm(y, None, None, gamma, beta, True, 0.1, 1e-5)
    out = F.relu(z) if mask else z
    g = rand(*out.shape, seed=9)
    out.backward(g)
    d = cuda_device
    y_d = nhwc(y.detach()).to(d)
    # forward stats from our own finalize (mean/invstd as the forward produced them)
    part = torch.zeros(1, c, 2)
    part[0, :, 0] = y.detach().sum((0, 2, 3))
    part[0, :, 1] = ((y.detach() - y.detach().mean((0, 2, 3), keepdim=True)) ** 2).sum((0, 2, 3))
    # bn_finalize expects tiles of 128 rows; here one tile holds all m rows, so tile_rows=m via ops-level call
    from hkp._lib import call
    import ctypes
    m = n * h * w
    ss = torch.empty(2 * c, device=d)
    mi = torch.empty(2 * c, device=d)
    part_d, gamma_d, beta_d = part.to(d), gamma.detach().to(d), beta.detach().to(d)
    call("hkp_bn_finalize", c, m, 1, m, ctypes.c_void_p(part_d.data_ptr()), ctypes.c_void_p(gamma_d.data_ptr()),
         ctypes.c_void_p(beta_d.data_ptr()), 0.1, 1e-5, None, None, None, ctypes.c_void_p(ss.data_ptr()),
         ctypes.c_void_p(mi.data_ptr()), ops._stream())
    out_d = ops.bn_apply(y_d, ss, relu=mask)
    dy, dgamma, dbeta, dz = ops.bn_bwd(nhwc(g).to(d), out_d if mask else None, y_d, mi, gamma.detach().to(d),
                                       want_dz=True, want_amax=True)
    assert torch.equal(dy._hkp_amax, ops.absmax(dy))     # fused max|dy| == the separate pass
    assert (nchw(dy.cpu()) - y.grad).abs().max() < 1e-5 * max(1, y.grad.abs().max().item())
    assert (dgamma.cpu() - gamma.grad).abs().max() < 1e-4 * max(1, gamma.grad.abs().max().item())
    assert (dbeta.cpu() - beta.grad).abs().max() < 1e-4 * max(1, beta.grad.abs().max().item())
    ref_dz = g * (out.detach() > 0) if mask else g
    assert torch.equal(nchw(dz.cpu()), ref_dz)
    if c % 32 == 0:   # split-only dy: bound >= max|dy|, and exactly split_pack_x3(dy, bound)
        dys, dg2, db2, _ = ops.bn_bwd(nhwc(g).to(d), out_d if mask else None, y_d, mi, gamma.detach().to(d),
                                      split_only=True)
        bound = dys._hkp_amax
        assert dys.dtype == torch.float16 and dys._hkp_split_passes == 3
        assert bound.view(torch.float32).item() >= dy.abs().max().item()
        assert bound.view(torch.float32).item() <= 8 * dy.abs().max().item() + 1e-30
        assert torch.equal(dys, ops.split_pack_x3(dy, bound))
        assert torch.equal(dg2, dgamma) and torch.equal(db2, dbeta)
    if mask:            # mask recomputed from y and the forward's scale/shift: the same bits
        dy3, dg3, db3, dz3 = ops.bn_bwd(nhwc(g).to(d), None, y_d, mi, gamma.detach().to(d), want_dz=True,
                                        want_amax=True, relu_ss=ss)
        assert torch.equal(dy3, dy) and torch.equal(dz3, dz) and torch.equal(dg3, dgamma) and torch.equal(db3, dbeta)
        if c % 32 == 0:
            dys3, _, _, _ = ops.bn_bwd(nhwc(g).to(d), None, y_d, mi, gamma.detach().to(d), split_only=True,
                                       relu_ss=ss)
            assert torch.equal(dys3, dys)


def test_maxpool_backward(cuda_device):
    from hkp import ops
    c = 64
    y = rand(2, c, 25, 31, seed=10).requires_grad_(True)
    a, b = rand(c, seed=11), rand(c, seed=12)
    a[:4] = 0.0  # constant channels → all-zero / tied windows
    t = y * a[None, :, None, None] + b[None, :, None, None]
    p = F.max_pool2d(F.relu(t), 3, 2, 1)
    g = rand(*p.shape, seed=13)
    p.backward(g)
    ref = y.grad / torch.where(a == 0, torch.ones_like(a), a)[None, :, None, None]  # dL/dt
    ss = torch.cat([a, b]).to(cuda_device)
    yd = nhwc(y.detach()).to(cuda_device)
    pool = ops.bn_relu_maxpool(yd, ss, route=True)
    assert torch.equal(nchw(pool.cpu()), p.detach())
    rt = pool._hkp_route
    assert rt.dtype == torch.uint8 and int(rt[rt != 255].max()) <= 8
    dz = ops.maxpool_bwd(nhwc(g).to(cuda_device), rt, tuple(yd.shape))
    got = nchw(dz.cpu())
    live = a != 0
    assert (got[:, live] - ref[:, live]).abs().max() < 1e-5
    # constant channels (a = 0): the ReLU passes nothing where relu(b) == 0, and
    # the whole window's gradient goes to the first tap where b > 0
    assert torch.equal(got[:, ~live & (b <= 0)], torch.zeros_like(got[:, ~live & (b <= 0)]))


def test_heat_loss_matches_reference_golden(cuda_device, golden):
    from hkp import ops
    g = golden("bce")
    p = torch.from_numpy(g["p"]).reshape(1, 1, 8, 8).to(cuda_device)
    y = torch.from_numpy(g["y"]).reshape(1, 1, 8, 8).to(cuda_device)
    loss, dheat = ops.heat_loss(p, target=y, kind="bce")
    assert abs(loss.item() - float(g["loss"])) <= 1e-14 * abs(float(g["loss"]))
    np.testing.assert_array_equal(dheat.cpu().numpy().reshape(-1), g["grad"])
    loss, dheat = ops.heat_loss(p, target=y, kind="mse")
    assert abs(loss.item() - float(g["mse"])) <= 1e-14 * abs(float(g["mse"]))
    np.testing.assert_array_equal(dheat.cpu().numpy().reshape(-1), g["mse_grad"])


def test_heat_loss_uv_recompute_equals_dense(cuda_device):
    from hkp import ops
    B, K, H, W = 2, 4, 48, 64
    uv = torch.from_numpy(recipe.seeded_keypoints(B, K, H, W, 3)).to(cuda_device)
    p = torch.rand(B, K, H, W, generator=torch.Generator().manual_seed(4)).to(cuda_device)
    dense = ops.gauss_target(uv, H, W, 8)
    l1, g1 = ops.heat_loss(p, target=dense)
    l2, g2 = ops.heat_loss(p, uv=uv, sigma=8)
    assert l1.item() == l2.item() and torch.equal(g1, g2)
    ref = cpu_ref.bce_loss(p.cpu(), cpu_ref.gauss_target(uv.cpu(), H, W, 8))
    # expf (GPU) vs Sleef exp (CPU) in the target: ≤1 ulp per element
    assert abs(l1.item() - ref.item()) < 1e-10 * abs(ref.item())


@pytest.mark.parametrize("shape", [(2, 4, 12, 16, 96, 128), (1, 2, 10, 13, 75, 100), (1, 4, 60, 80, 480, 640)])
def test_head_backward(cuda_device, shape):
    from hkp import ops
    n, k, h, w, H, W = shape
    low = rand(n, k, h, w, seed=14).requires_grad_(True)
    heat = torch.sigmoid(F.interpolate(low, size=(H, W), mode="bilinear", align_corners=True))
    g = rand(n, k, H, W, seed=15)
    heat.backward(g)
    dlow = ops.head_bwd(g.to(cuda_device), heat.detach().to(cuda_device), h, w)
    assert (dlow.cpu() - low.grad).abs().max() < 2e-5 * max(1, low.grad.abs().max().item())


def test_head_fc_backward(cuda_device):
    from hkp import ops
    n, h, w, c, k = 2, 6, 7, 512, 4
    feat = rand(n, c, h, w, seed=16).requires_grad_(True)
    wt = (rand(k, c, 1, 1, seed=17) * 0.01).requires_grad_(True)
    b = rand(k, seed=18).requires_grad_(True)
    low = F.conv2d(feat, wt, b)
    g = rand(*low.shape, seed=19)
    low.backward(g)
    dfeat, dw, db = ops.head_fc_bwd(g.to(cuda_device), nhwc(feat.detach()).to(cuda_device),
                                    wt.detach().reshape(k, c).contiguous().to(cuda_device))
    assert (nchw(dfeat.cpu()) - feat.grad).abs().max() < 1e-5
    assert (dw.cpu() - wt.grad.reshape(k, c)).abs().max() < 1e-4
    assert (db.cpu() - b.grad).abs().max() < 1e-4


def _model(bb, k, wseed, dev):
    from src.model import KeypointsGauss
    m = KeypointsGauss(k, backbone=bb, pretrained=False)
    m.load_state_dict(recipe.seeded_state_dict(bb, wseed))
    return m.to(dev)


# Tolerances per fixture (see the comment in the test): step-0 grad |.| sums
# (rtol), step-1 grad sums, fc rows and stem gradient (atol relative to the
# reference's max), step-1 loss (relative), post-step |param| sums, running stats.
# R50@96x128: CPU fp32 vs fp64 on the same inputs differs by 6.3e-3 in the
# |grad| sums, 1.0e-5 in the fc rows, 2.1e-2 in the stem gradient, and after
# one Adam step its step-1 loss differs by 5.7e-4 relative (0.690897 vs 0.690503);
# after two steps the |param| sums by 9.1e-5 (GPU: loss 9.4e-4, params 1.7e-4).
TRAIN_TOL = {
    "train_r18_k2_64x80": dict(g0=1e-4, fc=1e-5, stem=1e-4, loss1=1e-6, param=1e-5, run=1e-4),
    "train_r34_k4_48x64": dict(g0=5e-2, fc=5e-3, stem=5e-2, loss1=2e-4, param=1e-4, run=1e-3),
    "train_r50_k8_96x128": dict(g0=2e-2, fc=1e-4, stem=5e-2, loss1=2e-3, param=5e-4, run=1e-3),
}


@pytest.mark.parametrize("optimizer", ["torch", "fused"])
@pytest.mark.parametrize("case", sorted(TRAIN_TOL))
def test_train_step_matches_reference_golden(cuda_device, golden, case, optimizer):
    """Reference idiom (train.py:33-36) end to end on the GPU path: heatmaps →
    .double() → nn.BCELoss → backward → Adam(lr 1e-4, wd 1e-4), two iterations
    (torch.optim.Adam, and hkp.optim.FusedAdam in its place)."""
    g = golden(case)
    bb, k = str(g["backbone"]), int(g["k"])
    m = _model(bb, k, int(g["wseed"]), cuda_device)
    x = recipe.to_tensor_nchw(g["images_u8"]).to(cuda_device)
    uv = torch.from_numpy(g["uv"]).to(cuda_device)
    from hkp import ops
    gt = ops.gauss_target(uv, x.shape[2], x.shape[3], 8)
    from hkp.optim import FusedAdam
    opt = (torch.optim.Adam if optimizer == "torch" else FusedAdam)(m.parameters(), lr=1.0e-4, weight_decay=1.0e-4)
    names = list(g["param_names"])
    params = dict(m.named_parameters())
    # Tolerances follow the problem's own conditioning, measured on the CPU
    # oracle (fp32 vs fp64, same inputs): R18@64x80 gradients agree to 6e-6,
    # R34@48x64 only to 1.5e-2 (train-mode BN over 96 values per channel makes
    # ReLU-mask flips from 1e-7 forward differences visible).  Kernel exactness
    # for the deep nets is pinned call by call in test_backward_calls_exact.
    # After an Adam step (update ≈ lr*sign(g)) near-zero gradient elements whose
    # sign differs move by 2*lr, so step-1 trajectories diverge further: measured
    # (tools/diag_grads.py two_step_report) GPU/CPU step-1 grad errors 3e-2 (R18)
    # and 4e-1 (R34) per element, loss 7e-9 (R18) and 4e-5 (R34).
    tol = TRAIN_TOL[case]
    for s in range(int(g["steps"])):
        opt.zero_grad()
        pred = m.forward(x).double()
        loss = torch.nn.BCELoss()(pred, gt)
        loss.backward()
        ltol = 1e-6 if s == 0 else tol["loss1"]
        print("%s step %d loss %.12f ref %.12f" % (case, s, loss.item(), float(g["loss%d" % s])))
        assert abs(loss.item() - float(g["loss%d" % s])) < ltol * float(g["loss%d" % s])
        if s > 0:
            opt.step()
            continue
        # gradients in the reference layout (OIHW) for comparison
        ga = np.array([float(params[n].grad.double().abs().sum()) for n in names])
        print("  grad |.| sums: max rel err %.3g" % (np.abs(ga - g["grad_abs0"]) / g["grad_abs0"]).max())
        np.testing.assert_allclose(ga, g["grad_abs%d" % s], rtol=tol["g0"], atol=1e-9)
        fcw = params["resnet.%s_8s.fc.weight" % bb].grad
        fref = g["fc_grad_rows%d" % s]
        np.testing.assert_allclose(fcw[:k].reshape(k, -1).cpu().numpy(), fref, rtol=0,
                                   atol=tol["fc"] * np.abs(fref).max())
        assert fcw[k:].abs().sum().item() == 0.0
        st = params["resnet.%s_8s.conv1.weight" % bb].grad.cpu().numpy()
        sref = g["stem_grad%d" % s]
        np.testing.assert_allclose(st, sref, rtol=0, atol=tol["stem"] * np.abs(sref).max())
        opt.step()
    sd = m.state_dict()
    pa = np.array([float(sd[n].double().abs().sum()) for n in names])
    np.testing.assert_allclose(pa, g["param_abs"], rtol=tol["param"])
    rc = [sum(float(v.double().sum()) for kk, v in sd.items() if kk.endswith(sfx))
          for sfx in ("running_mean", "running_var")]
    np.testing.assert_allclose(rc, g["running_checksum"][:2], rtol=tol["run"])


def test_fused_adam_matches_torch_adam(cuda_device):
    """hkp_adam_step == torch.optim.Adam (multi-tensor, L2 wd) to fp32 rounding over
    several steps: vector and scalar (odd length / misaligned view) tensors, a
    zero-gradient block (wd still moves it), state_dict round trip both ways."""
    from hkp.optim import FusedAdam
    gen = torch.Generator().manual_seed(5)
    shapes = [(64, 3, 3, 64), (1000, 512), (1000,), (37,), (4097,), (64,)]
    base = [torch.randn(*s, generator=gen) for s in shapes]
    big = torch.randn(4099, generator=gen)
    p1 = [b.clone().to(cuda_device).requires_grad_(True) for b in base] + \
        [big.to(cuda_device)[1:].clone().requires_grad_(True)]
    p2 = [b.clone().to(cuda_device).requires_grad_(True) for b in base]
    # misaligned (non-16-B) data pointer: a view starting one float in
    store = big.clone().to(cuda_device)
    p2.append(torch.nn.Parameter(store[1:]))
    o1 = torch.optim.Adam(p1, lr=1e-3, weight_decay=1e-4, foreach=True)
    o2 = FusedAdam(p2, lr=1e-3, weight_decay=1e-4)
    for step in range(4):
        for a, b in zip(p1, p2):
            g = torch.randn(a.shape, generator=gen).to(cuda_device) * (10.0 ** (step - 3))
            if a.shape == (1000, 512):
                g[4:] = 0.0
            a.grad, b.grad = g.clone(), g.clone()
        o1.step()
        v0 = [b._version for b in p2]
        o2.step()
        assert all(b._version > v for b, v in zip(p2, v0))   # in-place update is visible
        # fp32 rounding of each quantity's own scale (elements produced by a
        # cancellation, e.g. m = lerp(m, g) with g ~ m, differ relatively more)
        def close(x, y):
            torch.testing.assert_close(x, y, rtol=2e-6, atol=2e-7 * float(y.detach().abs().max()))
        for a, b in zip(p1, p2):
            close(b, a)
            s1, s2 = o1.state[a], o2.state[b]
            close(s2["exp_avg"], s1["exp_avg"])
            close(s2["exp_avg_sq"], s1["exp_avg_sq"])
            assert float(s2["step"]) == float(s1["step"])
    sd = o2.state_dict()
    assert set(sd["state"][0]) == set(o1.state_dict()["state"][0])
    o3 = torch.optim.Adam(p2, lr=1e-3, weight_decay=1e-4)
    o3.load_state_dict(sd)                       # FusedAdam state → torch Adam, and back
    FusedAdam(p2, lr=1e-3, weight_decay=1e-4).load_state_dict(o3.state_dict())


def test_trainer_fused_loss_equals_autograd_path(cuda_device):
    from hkp import train
    B, K, H, W = 2, 2, 64, 80
    x = recipe.to_tensor_nchw(recipe.seeded_images_u8(B, H, W, 21)).to(cuda_device)
    uv = torch.from_numpy(recipe.seeded_keypoints(B, K, H, W, 22)).to(cuda_device)
    m1 = _model("resnet18", K, 23, cuda_device)
    m2 = _model("resnet18", K, 23, cuda_device)
    t = train.Trainer(m1)
    l1 = t.forward_backward(x, uv=uv)
    from hkp import ops
    gt = ops.gauss_target(uv, H, W, 8)
    l2 = torch.nn.BCELoss()(m2(x).double(), gt)
    l2.backward()
    assert abs(l1.item() - l2.item()) < 1e-12
    for p1, p2 in zip(m1.parameters(), m2.parameters()):
        assert torch.allclose(p1.grad, p2.grad, rtol=1e-5, atol=1e-9)


def test_backward_deterministic(cuda_device):
    from hkp import train
    B, K, H, W = 2, 2, 64, 80
    x = recipe.to_tensor_nchw(recipe.seeded_images_u8(B, H, W, 31)).to(cuda_device)
    uv = torch.from_numpy(recipe.seeded_keypoints(B, K, H, W, 32)).to(cuda_device)
    m = _model("resnet18", K, 33, cuda_device)
    t = train.Trainer(m)
    t.forward_backward(x, uv=uv)
    g1 = [p.grad.clone() for p in m.parameters()]
    t.forward_backward(x, uv=uv)
    for a, b in zip(g1, m.parameters()):
        assert torch.equal(a, b.grad)


def test_dp_bucket_path_equals_plain(cuda_device):
    """The DP gradient path (bucket copies on the stream each gradient is made on,
    one join per bucket; forced at world size 1) hands the optimizer exactly the
    gradients of the plain path, with the side-stream wgrad on and off."""
    from hkp import train
    from hkp.policy import DEFAULT
    B, K, H, W = 2, 2, 64, 80
    x = recipe.to_tensor_nchw(recipe.seeded_images_u8(B, H, W, 41)).to(cuda_device)
    uv = torch.from_numpy(recipe.seeded_keypoints(B, K, H, W, 42)).to(cuda_device)
    m = _model("resnet34", K, 43, cuda_device)
    for overlap in (True, False):    # (off: dgrad may take stream-K — another fp32 order)
        m.policy = DEFAULT.with_(overlap_wgrad=overlap)
        train.Trainer(m).forward_backward(x, uv=uv)
        ref = [p.grad.clone() for p in m.parameters()]
        t = train.Trainer(m, force_buckets=True)
        assert t.bucketer is not None and len(t.bucketer.buckets) >= 2
        for _ in range(2):                       # buckets reused across steps
            t.forward_backward(x, uv=uv)
            torch.cuda.synchronize()
            for a, p in zip(ref, m.parameters()):
                assert torch.equal(a, p.grad)


@pytest.mark.parametrize("bb,k", [("resnet34", 4), ("resnet50", 8)])
def test_backward_calls_exact(cuda_device, bb, k):
    """Every conv (dgrad, wgrad) and BN backward call of a full training step,
    re-done in fp64 on the CPU from that call's own GPU inputs: kernel error only,
    free of the forward-rounding discontinuities a deep train-mode-BN net has."""
    from _spy import spy_calls
    from hkp import net, train
    B, H, W = 2, 64, 96
    x = recipe.to_tensor_nchw(recipe.seeded_images_u8(B, H, W, 41)).to(cuda_device)
    uv = torch.from_numpy(recipe.seeded_keypoints(B, k, H, W, 42)).to(cuda_device)
    m = _model(bb, k, 43, cuda_device)
    log = []

    def conv_spy(conv, xx, dy, add, dx, dw):
        log.append(("conv", conv, xx, dy, add, dx, dw))

    def bn_spy(bn, gr, mask, relu_ss, y, mi, dy, dgamma, dbeta):
        if relu_ss is not None:          # the mask the kernel recomputes: round(round(y*a) + b) > 0
            c = y.shape[-1]
            mask = (y.float() * relu_ss[:c]) + relu_ss[c:]
        log.append(("bn", bn, gr, mask, y, mi, dy, dgamma, dbeta))

    with spy_calls(on_conv_bwd=conv_spy, on_bn_bwd=bn_spy):
        train.Trainer(m).forward_backward(x, uv=uv)
    n_conv = sum(1 for r in log if r[0] == "conv")
    assert n_conv == len([mm for mm in m.modules() if mm.__class__.__name__ == "KRSCConv2d"])

    def rel(a, b):
        return ((a.double().cpu() - b).abs().max() / (b.abs().max() + 1e-30)).item()

    n_split = 0

    def dense(dy):
        """fp32 view of a dy: a split-only dy (packed hi|lo of dy * 2^e, 2^e from the
        bound in _hkp_amax) is decoded as (hi + lo) / 2^e (2^-22 relative)."""
        nonlocal n_split
        if dy.dtype != torch.float16:
            return dy
        n_split += 1
        g = dy.reshape(*dy.shape[:-1], dy.shape[-1] // 64, 2, 32).double()
        v = (g[..., 0, :] + g[..., 1, :]).reshape(*dy.shape[:-1], -1)
        bound = dy._hkp_amax.view(torch.float32).item()
        assert bound > 0
        _, e = np.frexp(bound)
        return v / 2.0 ** (14 - int(e))

    for rec in log:
        if rec[0] == "conv":
            _, conv, xx, dy, add, dx, dw = rec
            dy = dense(dy)
            if xx.dtype == torch.float16:    # split-only activation: x = hi + lo (unscaled)
                g16 = xx.reshape(*xx.shape[:-1], xx.shape[-1] // 64, 2, 32).double()
                xx = (g16[..., 0, :] + g16[..., 1, :]).reshape(*xx.shape[:-1], -1)
            st, pd, dl = net._i(conv.stride), net._i(conv.padding), net._i(conv.dilation)
            w = conv.weight.detach().double().cpu().permute(0, 3, 1, 2)
            xc, dyc = xx.double().cpu().permute(0, 3, 1, 2), dy.double().cpu().permute(0, 3, 1, 2)
            assert rel(dw.permute(0, 3, 1, 2), torch.nn.grad.conv2d_weight(xc, w.shape, dyc, st, pd, dl)) < 1e-5
            rdx = torch.nn.grad.conv2d_input(xc.shape, w, dyc, st, pd, dl)
            if add is not None:
                rdx = rdx + add.double().cpu().permute(0, 3, 1, 2)
            assert rel(dx.permute(0, 3, 1, 2), rdx) < 1e-5
        else:
            _, bn, gr, mask, y, mi, dy, dgam, dbet = rec
            c = y.shape[-1]
            gc, yc = gr.double().cpu().reshape(-1, c), y.double().cpu().reshape(-1, c)
            dz = gc * (mask.double().cpu().reshape(-1, c) > 0) if mask is not None else gc
            mean, inv = mi[:c].double().cpu(), mi[c:].double().cpu()
            xh = (yc - mean) * inv
            n = yc.shape[0]
            db, dgm = dz.sum(0), (dz * xh).sum(0)
            rdy = bn.weight.detach().double().cpu() * inv * (dz - db / n - xh * dgm / n)
            dyd = dense(dy)
            assert rel(dyd.reshape(-1, c), rdy) < 1e-5
            if dy.dtype == torch.float16:        # the bound really bounds max|dy|
                assert dy._hkp_amax.view(torch.float32).item() >= rdy.abs().max().item()
            assert rel(dgam, dgm) < 1e-5 and rel(dbet, db) < 1e-5
    assert n_split > 0                           # the fused split-only BN backward was exercised


@pytest.mark.parametrize("c,rows", [(64, 130 * 128 - 37), (96, 300 * 128), (512, 1200 * 128 - 5), (2048, 260 * 128)])
def test_bn_finalize_two_level(cuda_device, c, rows):
    """hkp_bn_finalize_ws (chunks of 128 tiles, then a per-channel merge) vs the
    one-kernel merge and an fp64 reference over the raw rows: mean/invstd and
    running statistics; partials built per 128-row tile as the conv epilogue does
    (sum, M2 about the tile mean), a ragged last tile included."""
    from hkp import ops
    d = cuda_device
    g = torch.Generator(device=d).manual_seed(c + rows)
    y = torch.randn(rows, c, device=d, generator=g, dtype=torch.float64) * 3 + 1.5
    tiles = (rows + 127) // 128
    pad = torch.zeros(tiles * 128, c, device=d, dtype=torch.float64)
    pad[:rows] = y
    n_t = torch.clamp(rows - torch.arange(tiles, device=d) * 128, max=128).to(torch.float64)
    yt = pad.view(tiles, 128, c)
    s = yt.sum(1)
    valid = (torch.arange(128, device=d)[None, :] < n_t[:, None]).to(torch.float64)
    m2 = (((yt - (s / n_t[:, None])[:, None, :]) ** 2) * valid[:, :, None]).sum(1)
    part = torch.stack([s, m2], -1).float().contiguous()
    gamma = torch.rand(c, device=d, generator=g) + 0.5
    beta = torch.rand(c, device=d, generator=g) - 0.5
    outs = []
    for two_level in (1 << 40, 129):        # the one-kernel merge, then the two-level form for every case
        rm, rv = torch.zeros(c, device=d), torch.ones(c, device=d)
        nbt = torch.zeros(1, device=d, dtype=torch.int64)
        ss, mi = ops.bn_finalize(part, rows, gamma, beta, rm, rv, nbt, two_level_tiles=two_level)
        outs.append((ss, mi, rm, rv, nbt))
    torch.cuda.synchronize()
    # the two forms: fp64 merges in different orders, rounded to fp32 -> at most 1 ulp apart
    for a, b in zip(outs[0][:4], outs[1][:4]):
        assert torch.allclose(a, b, rtol=2.5e-7, atol=0)
    assert outs[1][4].item() == 1
    # fp64 reference over the rows (the partials are fp32-rounded: 1e-6 relative)
    mean = y.mean(0)
    var = y.var(0, unbiased=False)
    ss, mi, rm, rv, _ = outs[1]
    assert torch.allclose(mi[:c].double(), mean, rtol=1e-5, atol=1e-6)
    assert torch.allclose(mi[c:].double(), 1 / torch.sqrt(var + 1e-5), rtol=1e-5)
    assert torch.allclose(rv.double(), 0.9 + 0.1 * y.var(0, unbiased=True), rtol=1e-5)
    # deterministic run to run
    ss2, mi2 = ops.bn_finalize(part, rows, gamma, beta, two_level_tiles=129)
    assert torch.equal(ss2, ss) and torch.equal(mi2, mi)


def test_bn_finalize_register_form_same_bits():
    """The finalize merges' register-held form (a tile lane's partials loaded in one
    round, kept for the second pass) gives the batched-load loops' bits, forward and
    backward (tools/fin_regs_check.py; the switch between the two forms is an A/B
    knob that only the tools build has, so the check runs in a child process on
    tools/ab_lib/libhulkkp_ab.so)."""
    import subprocess
    import sys
    from hkp import _lib
    if not os.path.exists(_lib.AB_LIB_PATH):
        pytest.skip("the A/B build is not built (make -C hulk-keypoints_amd/csrc ab)")
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "fin_regs_check.py")], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0 and "fin_regs_check ok" in r.stdout, r.stdout + r.stderr
