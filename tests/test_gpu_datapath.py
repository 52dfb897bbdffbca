"""SURVEY §8(f1) device data path and §8(f3) on-GPU visualisation.

* uint8 HWC (BGR, as cv2.imread gives) batches go straight into the stem: the
  heatmaps, argmax and training gradients are bit-identical to feeding the
  reference's ToTensor output (x = u8 / 255, dataset.py:16,71).
* DeviceBatches yields exactly the images / labels the dataset holds.
* Prediction.overlays (GPU) == Prediction.plot's numpy restatement, bit for bit.
"""
import os

import numpy as np
import pytest
import torch

from oracle import recipe

pytestmark = pytest.mark.gpu


def _model(bb, k, wseed, dev):
    from src.model import KeypointsGauss
    m = KeypointsGauss(k, backbone=bb, pretrained=False)
    m.load_state_dict(recipe.seeded_state_dict(bb, wseed))
    return m.to(dev)


def test_images_u8_to_nchw_is_to_tensor(cuda_device):
    from hkp import ops
    from src.dataset import transform
    imgs = recipe.seeded_images_u8(3, 37, 53, 7)                      # [B,H,W,3] uint8
    got = ops.images_u8_to_nchw(torch.from_numpy(imgs).to(cuda_device)).cpu()
    ref = torch.stack([transform(im) for im in imgs])
    assert torch.equal(got, ref)


@pytest.mark.parametrize("bb,k,hw", [("resnet34", 4, (96, 128)), ("resnet18", 2, (75, 100))])
def test_u8_input_bit_identical(cuda_device, bb, k, hw):
    """Inference and a training step from the uint8 batch == from ToTensor's fp32."""
    from hkp import train
    H, W = hw
    u8 = recipe.seeded_images_u8(2, H, W, 11)
    x32 = recipe.to_tensor_nchw(u8).to(cuda_device)
    x8 = torch.from_numpy(u8).to(cuda_device)
    m = _model(bb, k, 12, cuda_device)
    with torch.no_grad():
        h32, y32 = m.heatmaps_and_keypoints(x32)
        h8, y8 = m.heatmaps_and_keypoints(x8)
    assert torch.equal(h8, h32) and torch.equal(y8, y32)
    assert torch.equal(m.predict_keypoints(x8), y32)
    uv = torch.from_numpy(recipe.seeded_keypoints(2, k, H, W, 13)).to(cuda_device)
    m1, m2 = _model(bb, k, 12, cuda_device), _model(bb, k, 12, cuda_device)
    l1 = train.Trainer(m1).forward_backward(x32, uv=uv)
    l2 = train.Trainer(m2).forward_backward(x8, uv=uv)
    assert l1.item() == l2.item()
    for p1, p2 in zip(m1.parameters(), m2.parameters()):
        assert torch.equal(p1.grad, p2.grad)


def test_device_batches(cuda_device, tmp_path):
    from PIL import Image
    from src.dataset import DeviceBatches, KeypointsDataset, transform
    K, H, W, n = 2, 24, 32, 5
    imgs = recipe.seeded_images_u8(n, H, W, 21)
    os.makedirs(tmp_path / "images")
    os.makedirs(tmp_path / "labels")
    for i in range(n):
        # PNG content under the reference's %05d.jpg names: lossless, decoded by content
        Image.fromarray(imgs[i][:, :, ::-1]).save(tmp_path / "images" / ("%05d.jpg" % i), format="PNG")
        np.save(tmp_path / "labels" / ("%05d.npy" % i), np.array([[3.5 + i, 40.0], [-2.0, 7.25]]))
    ds = KeypointsDataset(str(tmp_path / "images"), str(tmp_path / "labels"), K, H, W, transform)
    seen = []
    for img, uv in DeviceBatches(ds, 2, shuffle=True, seed=3):
        assert img.dtype == torch.uint8 and img.is_cuda and img.shape[1:] == (H, W, 3)
        assert uv.shape[1:] == (K, 2)
        seen.append((img.cpu(), uv.cpu()))
    got = torch.cat([s[0] for s in seen])
    order = np.random.default_rng(3).permutation(n)
    assert torch.equal(got, torch.from_numpy(imgs[order]))
    uvs = torch.cat([s[1] for s in seen])
    assert float(uvs[0, 0, 0]) == min(3.5 + order[0], W - 1) and float(uvs[0, 1, 0]) == 0.0   # clipped (dataset.py:65)
    # decode workers (DataLoader processes): the same batches in the same order
    for workers in (1, 3):
        again = [(i.cpu(), u.cpu()) for i, u in DeviceBatches(ds, 2, shuffle=True, seed=3, workers=workers)]
        assert len(again) == len(seen)
        for (a, ua), (b, ub) in zip(again, seen):
            assert torch.equal(a, b) and torch.equal(ua, ub)


@pytest.mark.parametrize("k", [4, 1])
def test_overlays_match_plot(cuda_device, k, tmp_path):
    from src.prediction import Prediction
    H, W = 48, 64
    m = _model("resnet18", k, 31, cuda_device)
    u8 = recipe.seeded_images_u8(2, H, W, 32)
    x8 = torch.from_numpy(u8).to(cuda_device)
    pred = Prediction(m, k, H, W, True)
    with torch.no_grad():
        heat, yx = m.heatmaps_and_keypoints(x8)
    ov = pred.overlays(x8, heat, yx).cpu().numpy()
    for b in range(2):
        ref = pred.plot(u8[b], heat[b:b + 1].cpu().numpy(), image_id=b, keypoints=yx[b:b + 1].cpu().numpy(),
                        out_dir=str(tmp_path))
        assert ov[b].shape == ref.shape
        assert np.array_equal(ov[b], ref)
    # a flat heatmap (span 0) normalises to 0 everywhere, like the numpy path
    flat = torch.full((1, k, H, W), 0.5, device=cuda_device)
    yx0 = torch.zeros((1, k, 2), dtype=torch.int32, device=cuda_device)
    ov0 = pred.overlays(x8[:1], flat, yx0).cpu().numpy()[0]
    ref0 = pred.plot(u8[0], flat.cpu().numpy(), keypoints=yx0.cpu().numpy(), out_dir=str(tmp_path))
    assert np.array_equal(ov0, ref0)


def test_soft_argmax_fixed(cuda_device):
    """hkp_soft_argmax = Prediction.expectation (prediction.py:31-38) with the axis
    mix-up fixed, against its numpy restatement; a sharp peak lands on the argmax."""
    from src.prediction import Prediction
    g = torch.Generator().manual_seed(5)
    heat = torch.rand(2, 3, 37, 53, generator=g)
    heat[1, 2, 20, 7] = 30.0
    p = Prediction(None, 3, 37, 53, True)
    for beta in (1.0, 40.0):
        got = p.soft_argmax(heat.to(cuda_device), beta).cpu().numpy()
        for b in range(2):
            for k in range(3):
                ref = p.expectation_fixed(heat[b, k].numpy(), beta)
                np.testing.assert_allclose(got[b, k], ref, rtol=1e-5, atol=1e-4)
    assert np.allclose(p.soft_argmax(heat.to(cuda_device), 40.0).cpu().numpy()[1, 2], [7.0, 20.0], atol=1e-3)
