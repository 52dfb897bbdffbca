"""CPU tests of the host-side logic: DP gradient bucketing over a real
2-process gloo group, the dataset / transform surface, and Prediction helpers."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, REPO


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bucket_worker(rank, world, port, q):
    import sys
    sys.path[:0] = [REPO, PKG]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hkp.train import GradBucketer
    torch.manual_seed(0)
    params = [torch.nn.Parameter(torch.randn(n)) for n in (1000, 3, 70000, 17, 250000, 5)]
    b = GradBucketer(params, bucket_bytes=300 * 1024)
    assert len(b.buckets) >= 2
    for step in range(2):
        grads = {p: torch.full_like(p, float(rank + 1 + step)) * (i + 1) for i, p in enumerate(params)}
        for p in reversed(params):          # backward order
            b.ready(p, grads[p])
        b.finish()
        expect = [(sum(r + 1 + step for r in range(world)) / world) * (i + 1) for i in range(len(params))]
        ok = all(torch.allclose(p.grad, torch.full_like(p, e)) for p, e in zip(params, expect))
        q.put((rank, step, ok))
    dist.destroy_process_group()


def test_grad_bucketer_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bucket_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    res = [q.get(timeout=5) for _ in range(2 * world)]
    assert all(p.exitcode == 0 for p in procs)
    assert all(ok for _, _, ok in res), res


def test_bucketer_single_process_passthrough():
    from hkp.train import GradBucketer
    params = [torch.nn.Parameter(torch.randn(5)), torch.nn.Parameter(torch.randn(7))]
    b = GradBucketer(params)
    for p in params:
        b.ready(p, torch.ones_like(p) * 3)
    b.finish()
    assert all(torch.equal(p.grad, torch.ones_like(p) * 3) for p in params)
    b.ready(params[0], torch.ones(5))
    with pytest.raises(RuntimeError, match="missing"):
        b.finish()


def test_transform_matches_totensor_semantics():
    from oracle import recipe
    from src.dataset import transform
    img = recipe.seeded_images_u8(1, 6, 9, 3)[0]
    assert torch.equal(transform(img), recipe.to_tensor_nchw(img[None])[0])


def test_dataset_reads_reference_layout(tmp_path):
    from PIL import Image
    from src.dataset import KeypointsDataset, transform
    (tmp_path / "img").mkdir()
    (tmp_path / "kp").mkdir()
    rng = np.random.default_rng(0)
    for i in range(3):
        Image.fromarray(rng.integers(0, 255, (12, 16, 3), dtype=np.uint8)).save(tmp_path / "img" / ("%05d.jpg" % i))
        np.save(tmp_path / "kp" / ("%05d.npy" % i), np.array([[-3.0, 5.0], [20.0, 40.0]]).reshape(-1))
    ds = KeypointsDataset(str(tmp_path / "img"), str(tmp_path / "kp"), 2, 12, 16, transform, return_uv=True,
                          device="cpu")
    assert len(ds) == 3
    img, uv = ds[1]
    assert img.shape == (3, 12, 16) and img.dtype == torch.float32 and 0 <= img.min() and img.max() <= 1
    # labels clipped to the image like dataset.py:65-66
    assert uv.tolist() == [[0.0, 5.0], [15.0, 11.0]]


def test_prediction_expectation_and_plot(tmp_path):
    from src.prediction import Prediction
    p = Prediction(None, 4, 10, 12, False)
    h = np.random.default_rng(1).random((10, 12)).astype(np.float32)
    # the reference's loop form (prediction.py:31-38)
    width, height = h.T.shape
    d = h.T.ravel()
    dn = p.softmax(d)
    ref = [int(np.dot(dn, np.array([i % width for i in range(width * height)]))),
           int(np.dot(dn, np.array([i // width for i in range(width * height)])))]
    assert p.expectation(h) == ref
    img = np.zeros((10, 12, 3), np.uint8)
    heat = np.random.default_rng(2).random((1, 4, 10, 12)).astype(np.float32)
    out = p.plot(img, heat, image_id=3, out_dir=str(tmp_path))
    assert out.shape == (20, 24, 3) and (tmp_path / "out0003.png").exists()


def test_split_weight_cache_tracks_versions_and_lifetimes():
    import gc
    from hkp import net
    calls = []

    def make(t):
        calls.append(1)
        return t.clone(), t.clone()
    p = torch.nn.Parameter(torch.randn(3))
    net._cached_split(p, "a", make)
    net._cached_split(p, "a", make)
    assert len(calls) == 1
    with torch.no_grad():
        p.add_(1)                    # optimizer-style in-place update → re-split
    net._cached_split(p, "a", make)
    assert len(calls) == 2
    pid = id(p)
    del p
    gc.collect()
    assert pid not in net._split_cache


def test_entry_modules_import():
    import importlib
    for mod in ("config", "train", "analysis", "src.model", "src.dataset", "src.prediction", "src.resnet_dilated"):
        importlib.import_module(mod)
    import config
    assert (config.NUM_KEYPOINTS, config.IMG_HEIGHT, config.IMG_WIDTH, config.GAUSS_SIGMA, config.epochs,
            config.batch_size) == (4, 480, 640, 8, 25, 4)
