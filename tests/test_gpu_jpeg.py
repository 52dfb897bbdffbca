"""Hybrid JPEG decode, device half (hkp_jpeg_reconstruct, csrc/jpeg.hip) — the
replacement of the reference's cv2.imread (dataset.py:71) in the device data
path:

* GPU reconstruct == Pillow's libjpeg-turbo decode (BGR), bit for bit, over the
  subsamplings, sizes, restart intervals and tables of tests/test_jpeg_cpu.py
  (whose oracle pins the same arithmetic on the CPU);
* a batch of same-geometry images with different quantisation tables;
* DeviceBatches(decode="device") yields the same batches as decode="host",
  in the calling thread and with loader workers; a progressive file in the set
  falls back to the host decode for its batch.
"""
import io
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from test_jpeg_cpu import CASES, _image, _jpeg, _pil_bgr  # noqa: E402


def _decode_gpu(datas, dev):
    from hkp import jpeg
    parts = [jpeg.entropy_decode(d) for d in datas]
    g = parts[0][2]
    coefs = torch.from_numpy(np.stack([p[0] for p in parts])).to(dev)
    qt = torch.from_numpy(np.stack([p[1] for p in parts]).view(np.int16)).to(dev)
    return jpeg.reconstruct(coefs, qt, g, len(parts)).cpu().numpy()


@pytest.mark.parametrize("case", CASES, ids=lambda c: "%dx%d%s-%s" % (c[0], c[1], "g" if c[2] else "",
                                                                       "-".join("%s%s" % kv for kv in c[3].items())))
def test_reconstruct_equals_libjpeg(cuda_device, case):
    h, w, gray, kw = case
    data = _jpeg(_image(h, w, h * w, gray), **kw)
    got = _decode_gpu([data], cuda_device)[0]
    ref = _pil_bgr(data)
    diff = np.abs(got.astype(int) - ref.astype(int))
    assert diff.max() == 0, "max diff %d at %s" % (diff.max(), np.unravel_index(diff.argmax(), diff.shape))


def test_batch_of_tables_and_bench_size(cuda_device):
    """8 images at the bench's 640x480, 4:2:0, each with its own quality (own
    quantisation tables) and optimised Huffman tables, reconstructed in one launch."""
    datas = [_jpeg(_image(480, 640, 50 + i), quality=40 + 8 * i, subsampling=2, optimize=bool(i & 1))
             for i in range(8)]
    got = _decode_gpu(datas, cuda_device)
    for i, d in enumerate(datas):
        assert np.array_equal(got[i], _pil_bgr(d)), i


def test_randomised_configs_equal_libjpeg(cuda_device):
    rng = np.random.default_rng(77)
    for i in range(24):
        h, w = int(rng.integers(1, 70)), int(rng.integers(1, 70))
        kw = dict(quality=int(rng.integers(5, 101)), subsampling=int(rng.integers(0, 3)))
        if rng.integers(0, 3) == 0:
            kw["restart_marker_blocks"] = int(rng.integers(1, 9))
        gray = rng.integers(0, 6) == 0
        data = _jpeg(_image(h, w, 300 + i, gray), **kw)
        assert np.array_equal(_decode_gpu([data], cuda_device)[0], _pil_bgr(data)), (i, h, w, gray, kw)


def test_reconstruct_rejects_bad_shapes(cuda_device):
    from hkp import jpeg
    coefs, qt, g = jpeg.entropy_decode(_jpeg(_image(16, 16, 1), quality=80))
    c = torch.from_numpy(coefs).to(cuda_device)
    q = torch.from_numpy(qt.view(np.int16)).to(cuda_device)
    with pytest.raises(jpeg.JpegError):
        jpeg.reconstruct(c[:-1], q, g, 1)
    with pytest.raises(jpeg.JpegError):
        jpeg.reconstruct(c.cpu(), q, g, 1)


def test_device_batches_device_decode(cuda_device, tmp_path):
    from src.dataset import DeviceBatches, KeypointsDataset, transform
    K, H, W, n = 2, 48, 64, 7
    os.makedirs(tmp_path / "images")
    os.makedirs(tmp_path / "labels")
    for i in range(n):
        kw = dict(quality=60 + 5 * i, subsampling=2)
        if i == 4:
            kw["progressive"] = True                      # outside the hybrid decoder: host-decoded batch
        (tmp_path / "images" / ("%05d.jpg" % i)).write_bytes(_jpeg(_image(H, W, 900 + i), **kw))
        np.save(tmp_path / "labels" / ("%05d.npy" % i), np.array([[3.5 + i, 40.0], [-2.0, 7.25]]))
    ds = KeypointsDataset(str(tmp_path / "images"), str(tmp_path / "labels"), K, H, W, transform)
    host = [(i.cpu(), u.cpu()) for i, u in DeviceBatches(ds, 2, shuffle=True, seed=5)]
    for workers in (0, 2):
        dev = [(i.cpu(), u.cpu()) for i, u in DeviceBatches(ds, 2, shuffle=True, seed=5, workers=workers,
                                                            decode="device")]
        assert len(dev) == len(host)
        for (a, ua), (b, ub) in zip(dev, host):
            assert a.dtype == torch.uint8 and torch.equal(a, b) and torch.equal(ua, ub)
