"""CPU tests of the host-side logic: DP gradient bucketing over a real
2-process gloo group, the dataset / transform surface, and Prediction helpers."""
import os
import sys
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


def _trainer_worker(rank, world, port, q):
    """One rank of a world-2 gloo group running hkp.train.Trainer with its
    per-rank compute (net.keypoints_forward / ops.heat_loss /
    net.keypoints_backward) replaced by the oracle's CPU autograd restatement."""
    import sys
    sys.path[:0] = [REPO, PKG]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hkp import net, ops, train
    from oracle import cpu_ref, recipe
    from src.model import KeypointsGauss
    bb, K, B, H, W = "resnet18", 2, 2, 32, 48
    torch.manual_seed(100 + rank)                      # replicas start DIFFERENT ...
    m = KeypointsGauss(K, H, W, backbone=bb, pretrained=False)
    with torch.no_grad():
        for p in m.parameters():
            p.add_(0.01 * rank)
        for n_, b in m.named_buffers():
            if "running" in n_:
                b.add_(0.1 * (rank + 1))
    t = train.Trainer(m, distributed=True, optimizer="torch", bucket_mb=1)
    # ... and the Trainer broadcast rank 0's parameters and buffers
    state = torch.cat([v.detach().reshape(-1).double() for v in m.state_dict().values()])
    states = [torch.empty_like(state) for _ in range(world)]
    dist.all_gather(states, state)
    same_start = all(torch.equal(s, states[0]) for s in states)
    start_sd = {k: v.clone() for k, v in m.state_dict().items()}       # reference layout (OIHW)

    def oracle_forward(resnet, x, k, heat=True, argmax=False, trace=None):
        sd = m.state_dict(keep_vars=True)            # conv weights: differentiable OIHW views of KRSC params
        hm = cpu_ref.forward(sd, x, bb, k)
        trace.head = hm
        return hm, None, None

    def oracle_loss(hm, target, uv, sigma, kind, want_grad=True):
        gt = cpu_ref.gauss_target(uv, hm.shape[2], hm.shape[3], sigma)
        L = cpu_ref.bce_loss(hm, gt)
        (dheat,) = torch.autograd.grad(L, hm, retain_graph=True)
        return L.detach(), dheat

    def oracle_backward(resnet, trace, dheat, grads):
        ps = list(m.parameters())
        gs = torch.autograd.grad(trace.head, ps, dheat)
        for p, g in reversed(list(zip(ps, gs))):     # backward order: the bucketer fills from the fc side
            grads.put(p, g)
        return grads

    net.keypoints_forward, net.keypoints_backward, ops.heat_loss = oracle_forward, oracle_backward, oracle_loss
    imgs = recipe.seeded_images_u8(B * world, H, W, 7)
    uvs = recipe.seeded_keypoints(B * world, K, H, W, 8)
    x = recipe.to_tensor_nchw(imgs[rank * B:(rank + 1) * B])
    t.forward_backward(x, uv=torch.from_numpy(uvs[rank * B:(rank + 1) * B]))
    # reference: each shard's gradient from the common start, averaged
    ref = None
    for r in range(world):
        sd = {k: v.clone() for k, v in start_sd.items()}
        _, g, _ = cpu_ref.train_step(sd, recipe.to_tensor_nchw(imgs[r * B:(r + 1) * B]), uvs[r * B:(r + 1) * B], bb,
                                     K)
        ref = g if ref is None else {k: ref[k] + g[k] for k in g}
    names = [n_ for n_, _ in m.named_parameters()]
    err = 0.0
    for n_, p in zip(names, m.parameters()):
        want = ref[n_] / world
        got = p.grad if p.grad.shape == want.shape else p.grad.permute(0, 3, 1, 2)   # KRSC → OIHW
        err = max(err, ((got - want).abs().max() / (want.abs().max() + 1e-30)).item())
    grads_same = torch.cat([p.grad.reshape(-1) for p in m.parameters()])
    allg = [torch.empty_like(grads_same) for _ in range(world)]
    dist.all_gather(allg, grads_same)
    q.put((rank, same_start, err, all(torch.equal(a, allg[0]) for a in allg), len(t.bucketer.buckets)))
    dist.destroy_process_group()


def test_trainer_dp_gloo_world2():
    """Trainer(distributed=True) wiring over a real 2-process gloo group:
    parameters/buffers broadcast from rank 0 at construction, gradients
    all-reduced through the bucketer equal the mean of the per-shard oracle
    gradients, identical on both ranks."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_trainer_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    res = [q.get(timeout=5) for _ in range(world)]
    assert all(p.exitcode == 0 for p in procs)
    for rank, same_start, err, grads_same, nb in res:
        assert same_start, "replicas did not start from rank 0's state"
        assert err < 1e-5, "rank %d: DP gradient differs from the mean of per-shard gradients by %g" % (rank, err)
        assert grads_same and nb >= 2


def test_shard_range_and_gather_single():
    from hkp import parallel
    spans = [parallel.shard_range(10, r, 4) for r in range(4)]
    assert spans == [(0, 3), (3, 6), (6, 8), (8, 10)]
    yx = torch.zeros((3, 2, 2), dtype=torch.int32)
    assert parallel.gather_keypoints(yx) is yx
    with pytest.raises(ValueError):
        parallel.gather_keypoints(yx.float())


def _gather_worker(rank, world, port, q):
    import sys
    sys.path[:0] = [REPO, PKG]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hkp import parallel
    n = 7
    lo, hi = parallel.shard_range(n, rank, world)
    mine = torch.arange(lo * 6, hi * 6, dtype=torch.int32).reshape(-1, 3, 2)
    allk = parallel.gather_keypoints(mine)
    fixed = parallel.gather_keypoints_fixed(torch.full((2, 3, 2), rank, dtype=torch.int32))
    q.put((rank, torch.equal(allk, torch.arange(n * 6, dtype=torch.int32).reshape(n, 3, 2)),
           fixed[:, 0, 0].tolist()))
    dist.destroy_process_group()


def test_gather_keypoints_gloo_world3():
    """Inference DP: ragged shards' int32 keypoints all-gathered in rank order."""
    world, port = 3, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    res = [q.get(timeout=5) for _ in range(world)]
    assert all(p.exitcode == 0 for p in procs)
    assert all(ok for _, ok, _ in res)
    assert all(f == [0, 0, 1, 1, 2, 2] for _, _, f in res)


def test_bench_gpus_must_match_world_size():
    """bench.py --gpus N under a torchrun environment of another size refuses to
    run (exit 2) instead of silently reporting n_gpus = WORLD_SIZE."""
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr, r.stderr


def test_local_pretrained_import(tmp_path, monkeypatch):
    """pretrained=True reads a torchvision-format ImageNet checkpoint from
    $TORCH_HOME/hub/checkpoints (resnet.py:237-238 fetches the same file from
    download.pytorch.org): backbone weights and BN buffers land in the model
    (conv weights stored KRSC, state_dict OIHW), the 1000-way Linear fc of the
    file is ignored and the 1x1 scoring conv keeps its N(0, 0.01) init
    (resnet_dilated.py:15-22, applied after the load)."""
    from oracle import cpu_ref, recipe
    from src.model import KeypointsGauss
    from src.resnet import model_files
    sd = recipe.seeded_state_dict("resnet34", 77)
    pre = "resnet.resnet34_8s."
    tv = {k[len(pre):]: v for k, v in sd.items() if not k.endswith("num_batches_tracked")}
    tv["fc.weight"] = torch.randn(1000, 512)          # torchvision: nn.Linear(512, 1000)
    tv["fc.bias"] = torch.randn(1000)
    ck = tmp_path / "hub" / "checkpoints"
    ck.mkdir(parents=True)
    torch.save(tv, ck / model_files["resnet34"])
    monkeypatch.setenv("TORCH_HOME", str(tmp_path))
    torch.manual_seed(0)
    m = KeypointsGauss(4, pretrained=True)
    got = m.state_dict()
    for k, v in tv.items():
        if k.startswith("fc."):
            continue
        assert torch.equal(got[pre + k], v), k
    fc = got[pre + "fc.weight"]
    assert fc.shape == (1000, 512, 1, 1) and abs(fc.std().item() - 0.01) < 1e-3 and got[pre + "fc.bias"].abs().max() == 0
    # without the file: a warning, random init kept
    monkeypatch.setenv("TORCH_HOME", str(tmp_path / "none"))
    with pytest.warns(UserWarning, match="not found"):
        KeypointsGauss(4, pretrained=True)


def test_cv2_circle_disc_halfwidths():
    """cv2.circle(img, c, 4, color, -1) as OpenCV's midpoint Circle rasteriser
    (LINE_8) fills it: rows |dy| = 0..4 span ±4, ±3, ±3, ±2, ±0 — 49 pixels
    (prediction.py:52; cv2 absent here, so pixel parity stays unpinned)."""
    from src.prediction import Prediction
    hw = Prediction.disc_halfwidths(4)
    assert hw == [4, 3, 3, 2, 0]
    assert sum(2 * h + 1 for h in hw[1:]) * 2 + 2 * hw[0] + 1 == 49


def test_bench_pmc_traffic_folds_split_k_tail():
    """The dominant 256x256 conv's event pair also brackets its split-K tail
    launch: bench.pmc_traffic folds the tail's bytes and rocprof time in per main
    dispatch, and the folded average equals main + tail * (tail / main dispatches)
    of the committed summary it read."""
    import json
    sys.path.insert(0, REPO)
    import bench
    sym = "conv_x3_kernel<256, false, false, 16, false, 3>"
    nbytes, src, ms, folded = bench.pmc_traffic(sym, "infer_c2")
    if src is None:
        pytest.skip("no committed C2 PMC summary")
    data = json.load(open(os.path.join(REPO, "profiles", src)))
    main = next(c for n, c in data.items() if "::" + sym.replace(" ", "") + "(" in n.replace(" ", ""))
    plain = (main["FETCH_SIZE"] * 2 + main["WRITE_SIZE"]) * 1024
    if folded is None:
        assert nbytes == plain
    else:
        t = data[folded]
        per = t["dispatches"] / main["dispatches"]
        assert nbytes == pytest.approx(plain + (t["FETCH_SIZE"] * 2 + t["WRITE_SIZE"]) * 1024 * per)
        assert ms == pytest.approx((main["avg_duration_ns"] + t["avg_duration_ns"] * per) * 1e-6)
    assert bench._tail_of("conv_x3_a3_kernel<1>") == "::conv_x3_tail_kernel<256,1>("
    assert bench._tail_of(sym) == "::conv_x3_tail_kernel<256,3>("
    # kernels without a tail are looked up unchanged
    nb2, _, _, f2 = bench.pmc_traffic("wgrad_x3_kernel<256>", "train_c3")
    assert f2 is None


def _fit_worker(rank, world, port, out_dir, q):
    """One rank of a world-2 gloo group running the drop-in train.fit (the
    reference's loop: zero_grad, forward, loss.backward(), step) with DP wired by
    train.setup_data_parallel; the per-rank compute is the oracle's CPU autograd
    (net.keypoints_forward / keypoints_backward / ops.heat_loss replaced), so the
    test sees the order in which backward hands out gradients and the bucketer
    launches its all-reduces."""
    import sys
    sys.path[:0] = [REPO, PKG]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.Tensor.cuda = lambda self, *a, **k: self        # CPU-only rehearsal of train.forward's .cuda()
        import train as train_mod
        from hkp import net, ops
        from oracle import cpu_ref, recipe
        from src.model import KeypointsGauss
        bb, K, B, H, W = "resnet18", 2, 2, 32, 48
        torch.manual_seed(200 + rank)
        m = KeypointsGauss(K, H, W, backbone=bb, pretrained=False)
        with torch.no_grad():
            for p in m.parameters():
                p.add_(0.01 * rank)                          # replicas start different
        start_sd = None
        events = []
        orig_ar = dist.all_reduce

        def logged_all_reduce(t, *a, **k):
            events.append("all_reduce")
            return orig_ar(t, *a, **k)
        dist.all_reduce = logged_all_reduce

        def oracle_forward(resnet, x, k, heat=True, argmax=False, trace=None, pol=None):
            with torch.enable_grad():
                hm = cpu_ref.forward(m.state_dict(keep_vars=True), x, bb, k)
            trace.head = hm
            return hm.detach(), None, None

        def oracle_loss(hm, target, uv, sigma, kind, want_grad=True):
            h = hm.detach().requires_grad_(True)
            with torch.enable_grad():
                L = cpu_ref.bce_loss(h, cpu_ref.gauss_target(uv, hm.shape[2], hm.shape[3], sigma))
                (dheat,) = torch.autograd.grad(L, h)
            return L.detach(), dheat

        def oracle_backward(resnet, trace, dheat, grads):
            ps = list(m.parameters())
            gs = torch.autograd.grad(trace.head, ps, dheat)
            for p, g in reversed(list(zip(ps, gs))):         # backward order: fc side first
                grads.put(p, g)
                events.append("grad")
            events.append("backward_end")
            return grads

        net.keypoints_forward, net.keypoints_backward, ops.heat_loss = oracle_forward, oracle_backward, oracle_loss
        train_mod.setup_data_parallel(m, bucket_mb=4)
        start_sd = {k: v.clone() for k, v in m.state_dict().items()}        # after the broadcast
        lr = 1e-4
        train_mod.optimizer = torch.optim.SGD(m.parameters(), lr=lr)       # a plain step: p -= lr * grad
        imgs = recipe.seeded_images_u8(B * world, H, W, 9)
        uvs = recipe.seeded_keypoints(B * world, K, H, W, 10)
        batch = (recipe.to_tensor_nchw(imgs[rank * B:(rank + 1) * B]), torch.from_numpy(uvs[rank * B:(rank + 1) * B]))
        train_mod.fit([batch], [batch], m, epochs=1, checkpoint_path=out_dir)
        # reference: the mean of the per-shard oracle gradients from the common start
        ref = None
        for r in range(world):
            sd = {k: v.clone() for k, v in start_sd.items()}
            _, g, _ = cpu_ref.train_step(sd, recipe.to_tensor_nchw(imgs[r * B:(r + 1) * B]),
                                         uvs[r * B:(r + 1) * B], bb, K)
            ref = g if ref is None else {k: ref[k] + g[k] for k in g}
        err = 0.0
        for n_, p in m.named_parameters():
            want = ref[n_] / world
            got = p.grad if p.grad.shape == want.shape else p.grad.permute(0, 3, 1, 2)
            err = max(err, ((got - want).abs().max() / (want.abs().max() + 1e-30)).item())
        first_ar = events.index("all_reduce")
        q.put(dict(rank=rank, err=err, launched_before_end=first_ar < events.index("backward_end"),
                   n_all_reduce=events.count("all_reduce"), n_buckets=len(train_mod._bucketer.buckets),
                   grads_before_first=events[:first_ar].count("grad"), n_grads=events.count("grad")))
    except Exception as e:
        q.put(dict(rank=rank, error=repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def test_dropin_fit_dp_overlaps_allreduce_gloo_world2(tmp_path):
    """The drop-in train.fit over a 2-process gloo group: bucket all-reduces start
    while the backward is still producing gradients (not after loss.backward()
    returns), and the averaged gradients equal the mean of the per-shard oracle
    gradients."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_fit_worker, args=(r, world, port, str(tmp_path), q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(60)
    print(res)
    assert all("error" not in r for r in res), res
    for r in res:
        assert r["err"] < 1e-5, r
        assert r["launched_before_end"] and r["grads_before_first"] < r["n_grads"], r
        assert r["n_all_reduce"] == r["n_buckets"] >= 3, r
    assert os.path.exists(os.path.join(tmp_path, "model_2_1_0.pth"))


def test_bench_names_each_config():
    """bench.py names the BASELINE config a line measures (every line said C2)."""
    sys.path.insert(0, REPO)
    import bench
    n = bench.workload_name
    assert n("infer", "resnet34", 4, 480, 640, "f16x3", 32).startswith("C2")
    assert n("train", "resnet34", 4, 480, 640, "f16x3", 8).startswith("C3")
    assert n("infer", "resnet50", 8, 480, 640, "f16", 128).startswith("C4")
    assert n("train", "resnet50", 8, 960, 1280, "f16x3", 32).startswith("C5")
    assert n("train", "resnet18", 2, 240, 320, "f16x3", 4).startswith("C1")
    assert n("infer", "resnet50", 8, 480, 640, "f16x3", 128).startswith("custom")
    # the two-product precision modes are not fp32-class: never reported as C2
    assert n("infer", "resnet34", 4, 480, 640, "f16x2w", 32).startswith("custom")
    assert n("infer", "resnet34", 4, 480, 640, "f16x2a", 32).startswith("custom")
    # north_star's strong-scaling workload: C2 on a 64-image batch split over the ranks
    assert n("infer", "resnet34", 4, 480, 640, "f16x3", 8, 64, 8).startswith("north_star scaling: C2 batch 64 over 8")
    assert n("infer", "resnet34", 4, 480, 640, "f16", 8, 64, 8).startswith("custom strong")
