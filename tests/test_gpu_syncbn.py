"""SyncBN for data-parallel inference (caveat D5).

Train-mode BN (the reference never calls .eval()) makes a shard's outputs depend
on the shard: N ranks with per-rank statistics do not reproduce the reference's
forward over the global batch.  With SyncBN (Policy(sync_bn=True)) each rank's BN
statistics block (hkp_bn_stats) is all-gathered and merged in fixed rank order
(hkp_bn_finalize_ranks), and the sharded run matches the reference at the
global batch:

* kernel level: the rank merge of tile-aligned row shards == hkp_bn_finalize
  over all tiles (one-kernel and two-level forms; R = 1 bit-identical);
* end to end: 2 ranks (gloo, both on cuda:0) x 16 images of the C2 workload
  (R34-8s, K=4, 640x480) against the reference fixture for the whole batch of
  32 (tests/golden/make_golden.py fwd_r34_k4_480x640_b32): low-res logits,
  heatmap of image 0, argmax bit-exact, BN running statistics; and per-rank BN
  visibly misses that fixture.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "hulk-keypoints_amd")


def _partials(y, rows=128):
    """[tiles, C, 2] fp32 (sum, M2 about the tile mean) of 128-row tiles of y [M, C]
    — what the conv epilogues write."""
    m, c = y.shape
    full = m // rows
    parts = []
    if full:
        blk = y[:full * rows].double().reshape(full, rows, c)
        parts.append(torch.stack([blk.sum(1), ((blk - blk.mean(1, keepdim=True)) ** 2).sum(1)], -1))
    if m % rows:
        blk = y[full * rows:].double()
        parts.append(torch.stack([blk.sum(0), ((blk - blk.mean(0)) ** 2).sum(0)], -1)[None])
    return torch.cat(parts).float().contiguous()


def _bn_state(c, dev):
    g = torch.Generator().manual_seed(c)
    gamma = (1 + 0.1 * torch.randn(c, generator=g)).to(dev)
    beta = (0.1 * torch.randn(c, generator=g)).to(dev)
    rm = (0.05 * torch.randn(c, generator=g)).to(dev)
    rv = (1 + 0.1 * torch.rand(c, generator=g)).to(dev)
    return gamma, beta, rm, rv, torch.zeros(1, dtype=torch.int64, device=dev)


@pytest.mark.parametrize("m,c,cuts", [(2000, 96, [1024]), (1000, 64, []), (300_000, 64, [102_400, 204_800])])
def test_bn_finalize_ranks_matches_global(cuda_device, m, c, cuts):
    from hkp import ops
    torch.manual_seed(m)
    y = (torch.randn(m, c, device=cuda_device) * 3 + torch.linspace(-2, 2, c, device=cuda_device)).float()
    part = _partials(y)
    gamma, beta, rm, rv, nbt = _bn_state(c, cuda_device)
    ref_state = [t.clone() for t in (rm, rv, nbt)]
    ss_ref, mi_ref = ops.bn_finalize(part, m, gamma, beta, *ref_state)
    bounds = [0] + cuts + [m]
    blocks = []
    for lo, hi in zip(bounds[:-1], bounds[1:]):
        assert lo % 128 == 0
        blocks.append(ops.bn_stats(part[lo // 128:(hi + 127) // 128].contiguous(), hi - lo))
    st = torch.stack(blocks)
    assert st[:, -1].tolist() == [float(hi - lo) for lo, hi in zip(bounds[:-1], bounds[1:])]
    state = [t.clone() for t in (rm, rv, nbt)]
    ss, mi = ops.bn_finalize_ranks(st, gamma, beta, *state)
    torch.cuda.synchronize()
    if len(blocks) == 1:                       # one rank: the same bits as bn_finalize
        assert torch.equal(ss, ss_ref) and torch.equal(mi, mi_ref)
        assert all(torch.equal(a, b) for a, b in zip(state, ref_state))
    # fp64 merges in another order, rounded to fp32: at most an ulp or two apart
    torch.testing.assert_close(ss, ss_ref, rtol=3e-7, atol=1e-7)
    torch.testing.assert_close(mi, mi_ref, rtol=3e-7, atol=1e-7)
    torch.testing.assert_close(state[0], ref_state[0], rtol=3e-7, atol=1e-8)
    torch.testing.assert_close(state[1], ref_state[1], rtol=3e-7, atol=1e-8)
    assert int(state[2]) == int(ref_state[2]) == 1
    # and both against fp64 torch over the whole tensor
    yd = y.double()
    mean, var = yd.mean(0), yd.var(0, unbiased=False)
    torch.testing.assert_close(mi[:c].double(), mean, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(mi[c:].double(), 1 / torch.sqrt(var + 1e-5), rtol=1e-6, atol=1e-6)


def test_bn_finalize_ranks_bad_args(cuda_device):
    from hkp import ops
    with pytest.raises(ops.HkpError):
        ops.bn_finalize_ranks(torch.zeros(2, 10, dtype=torch.float64, device=cuda_device), None, None)
    with pytest.raises(ops.HkpError):
        ops.bn_finalize_ranks(torch.zeros(2, 9, dtype=torch.float32, device=cuda_device), None, None)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dp_worker(rank, world, port, q):
    import sys
    sys.path[:0] = [REPO, PKG]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from hkp import net, parallel
        from oracle import recipe
        from src.model import KeypointsGauss
        dev = torch.device("cuda:0")
        g = np.load(os.path.join(REPO, "tests", "golden", "fwd_r34_k4_480x640_b32.npz"), allow_pickle=False)
        B, H, W, K = int(g["batch"]), int(g["height"]), int(g["width"]), int(g["k"])
        lo, hi = parallel.shard_range(B, rank, world)
        imgs = recipe.seeded_images_u8(B, H, W, int(g["iseed"]))[lo:hi]
        x = torch.from_numpy(imgs).to(dev)

        def model():
            m = KeypointsGauss(K, backbone="resnet34", pretrained=False)
            m.load_state_dict(recipe.seeded_state_dict("resnet34", int(g["wseed"])))
            return m.to(dev)
        m = model()
        with torch.no_grad():
            hm, yx, low = net.keypoints_forward(m.resnet.net, x, K, heat=True, argmax=True,
                                                pol=m.policy.with_(sync_bn=True))
        yx_all = parallel.gather_keypoints(yx.to(torch.int32).cpu())        # gloo: host tensors
        res = dict(rank=rank,
                   low_err=float(np.abs(low.cpu().numpy() - g["lowres"][lo:hi]).max()),
                   rowsum_err=float(np.abs(hm.double().sum(3).cpu().numpy() / g["heat_row_sum"][lo:hi] - 1).max()),
                   argmax_ok=bool(np.array_equal(yx_all.cpu().numpy(), g["argmax_yx"])))
        if lo == 0:
            res["heat0_err"] = float(np.abs(hm[0].cpu().numpy() - g["heat0"]).max())
        sd = m.state_dict()
        res["rv_err"] = float(np.abs(sd["resnet.resnet34_8s.bn1.running_var"].cpu().numpy() / g["bn1_running_var"]
                                     - 1).max())
        rm = sum(float(v.double().sum()) for kk, v in sd.items() if kk.endswith("running_mean"))
        res["rm_err"] = abs(rm - float(g["running_checksum"][0])) / max(1.0, abs(rm))
        m3 = model()                          # the Prediction-level DP entry point with SyncBN
        yx3, _ = parallel.predict_keypoints_dp(m3, x, sync=True)
        res["predict_dp_ok"] = bool(np.array_equal(yx3.cpu().numpy(), g["argmax_yx"]))
        m2 = model()                          # per-rank BN (the default): the shard's own statistics
        with torch.no_grad():
            _, _, low2 = net.keypoints_forward(m2.resnet.net, x, K, heat=True, argmax=True)
        res["low_err_per_rank_bn"] = float(np.abs(low2.cpu().numpy() - g["lowres"][lo:hi]).max())
        torch.cuda.synchronize()
        q.put(res)
        dist.destroy_process_group()
    except Exception as e:            # report instead of hanging the parent on q.get
        q.put(dict(rank=rank, error=repr(e)))
        raise


def test_syncbn_dp_inference_matches_reference_global_batch(cuda_device):
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(60)
    print(res)
    assert all("error" not in r for r in res), res
    assert all(p.exitcode == 0 for p in procs)
    for r in res:
        assert r["low_err"] < 1e-4, r
        assert r["rowsum_err"] < 1e-4, r
        assert r["argmax_ok"], r                       # all 128 keypoints, bit-exact
        assert r["predict_dp_ok"], r                   # parallel.predict_keypoints_dp(sync=True)
        assert r["rv_err"] < 1e-4 and r["rm_err"] < 1e-4, r
        assert r["low_err_per_rank_bn"] > 1e-3, r      # without SyncBN the shard misses the batch-32 fixture
    assert [r for r in res if "heat0_err" in r][0]["heat0_err"] < 1e-3


# ---------------------------------------------------------------- training


def _train_worker(rank, world, port, out_dir, q):
    import sys
    sys.path[:0] = [REPO, PKG, os.path.join(REPO, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from hkp import parallel, train
        from oracle import recipe
        from src.model import KeypointsGauss
        from test_gpu_scale import _sampled_train_step
        dev = torch.device("cuda:0")
        B, H, W, K = TRAIN_SHAPE
        lo, hi = parallel.shard_range(B, rank, world)
        imgs = recipe.seeded_images_u8(B, H, W, 21)
        uv_all = recipe.seeded_keypoints(B, K, H, W, 22)

        n_gathers = [0]
        orig_gather = parallel.gather_bn_stats

        def counting_gather(st, group=None):
            n_gathers[0] += 1
            return orig_gather(st, group)
        parallel.gather_bn_stats = counting_gather

        def grads_of(x, uv, sync, distributed=False):
            m = KeypointsGauss(K, backbone="resnet18", pretrained=False)
            m.load_state_dict(recipe.seeded_state_dict("resnet18", 23))
            m = m.to(dev)
            t = train.Trainer(m, distributed=distributed, sync_bn=sync)
            if distributed:
                # the BN gathers run on their own communicator, the buckets on the world's
                res["groups_differ"] = (t.bn_group is not t.group and t.policy.sync_group is t.bn_group
                                        and t.bucketer is not None and t.bucketer.group is t.group)
            n_gathers[0] = 0
            loss = t.forward_backward(x, uv=uv)
            if sync and not distributed:
                res["gathers"] = n_gathers[0]
            torch.cuda.synchronize()
            g = {n: p.grad.detach().cpu() for n, p in m.named_parameters()}
            rm = {n: b.detach().cpu() for n, b in m.named_buffers() if n.endswith("running_mean")}
            return float(loss), g, rm
        x = torch.from_numpy(imgs[lo:hi]).to(dev)
        uv = torch.from_numpy(uv_all[lo:hi]).to(dev)
        res = {}
        res["sync"] = grads_of(x, uv, True)
        res["local"] = grads_of(x, uv, False)
        res["dp_sync"] = grads_of(x, uv, True, distributed=True)      # + the bucketed gradient all-reduce
        # the same SyncBN step with every conv forward / dgrad / wgrad call and every
        # BN backward's dgamma / dbeta checked against fp64 from the call's own inputs
        # (mask flips cannot hide a kernel error here: each call is checked alone)
        loss_s, counts, stats, _, _ = _sampled_train_step(dev, "resnet18", K, H, W, hi - lo, (21, 22, 23, 77 + rank),
                                                          x=x, uv=uv, sync_bn=True)
        res["spy"] = (float(loss_s), counts, stats)
        if rank == 0:
            res["global"] = grads_of(torch.from_numpy(imgs).to(dev), torch.from_numpy(uv_all).to(dev), False)
        torch.save(res, os.path.join(out_dir, "rank%d.pt" % rank))
        q.put(dict(rank=rank))
        dist.destroy_process_group()
    except Exception as e:
        q.put(dict(rank=rank, error=repr(e)))
        raise


TRAIN_SHAPE = (4, 96, 128, 2)          # global batch, H, W, K (R18-8s)


def _rel(a, b):
    return float((a.double() - b.double()).norm() / max(float(b.double().norm()), 1e-30))


def _oracle_grads(dtype):
    """The reference's step over the whole 4-image batch (oracle, CPU) in `dtype`."""
    from oracle import cpu_ref, recipe
    B, H, W, K = TRAIN_SHAPE
    sd = {k: (v.clone().to(dtype) if v.is_floating_point() else v.clone())
          for k, v in recipe.seeded_state_dict("resnet18", 23).items()}
    x = recipe.to_tensor_nchw(recipe.seeded_images_u8(B, H, W, 21)).to(dtype)
    L, g, _ = cpu_ref.train_step(sd, x, recipe.seeded_keypoints(B, K, H, W, 22), "resnet18", K, adam_state=None)
    return float(L), g


def _as_ref_layout(g, ref):
    """KRSC conv gradients → the reference's OIHW for comparison."""
    return {n: (t if t.shape == ref[n].shape else t.permute(0, 3, 1, 2)) for n, t in g.items()}


def test_syncbn_training_step_equals_global_batch(cuda_device, tmp_path):
    """2 ranks x 2 images with SyncBN == one step over all 4 images (R18-8s, 96x128).

    Gradient tolerance from the problem's measured conditioning.  This step has a
    ReLU kink inside fp32 noise: in the reference's own fp32 run exactly one element
    of layer4.0's output (image 2, channel 218, (7, 6)), whose pre-ReLU sum is
    ~1e-6 from zero, falls on the other side of the kink than in fp64 — and that one
    element carries all of the fp32-vs-fp64 gradient difference (0.6 % at layer4,
    ~1 % upstream; DESIGN "SyncBN step parity").  Two correct fp32-class
    computations that round differently (another tile shape / MFMA order) can
    therefore differ by that much, so the bound is 2x the reference's own fp32
    distance from its fp64 step (measured here, ~1.1e-2), each path is checked
    against fp64, and kernel exactness is pinned call by call (spy harness) instead.
    Per-rank BN misses by ~1.0, far outside the bound."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_train_worker, args=(r, world, port, str(tmp_path), q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(60)
    assert all("error" not in r for r in res), res
    assert all(p.exitcode == 0 for p in procs)
    r0 = torch.load(os.path.join(tmp_path, "rank0.pt"), weights_only=True)
    r1 = torch.load(os.path.join(tmp_path, "rank1.pt"), weights_only=True)
    lg, gg, rmg = r0["global"]
    l64, g64 = _oracle_grads(torch.float64)
    l32, g32 = _oracle_grads(torch.float32)
    cond = max(_rel(g32[n], g64[n]) for n in g64)          # the reference's own fp32 distance from fp64
    bound = 2 * cond
    gg = _as_ref_layout(gg, g64)
    print("conditioning: reference fp32 vs fp64 worst grad rel %.3g -> bound %.3g" % (cond, bound))
    assert 1e-4 < cond < 5e-2, cond                          # the kink is there (and nothing else is off)
    # R18: 20 BN layers, 3 downsample blocks whose last BN and downsample BN share
    # one gather in each direction -> 17 forward + 17 backward statistics gathers
    assert r0["gathers"] == r1["gathers"] == 34, (r0["gathers"], r1["gathers"])
    assert r0["groups_differ"] and r1["groups_differ"]
    # every call of the SyncBN step exact vs fp64 from its own inputs (asserted in the
    # worker; the counts and worst ratios come back for the log)
    for r in (r0, r1):
        print("spy: loss %.9f calls %s worst %s" % (r["spy"][0], r["spy"][1],
                                                   {k: round(v, 4) for k, v in r["spy"][2].items()}))
        assert r["spy"][1]["fwd"] > 0 and r["spy"][1]["bwd"] > 0 and r["spy"][1]["bn"] > 0
        assert max(r["spy"][2].values()) <= 1.0
    glob_err = max(_rel(gg[n], g64[n]) for n in g64)
    print("global 4-image GPU step vs fp64: worst grad rel %.3g; loss %.3g" % (glob_err, abs(lg - l64) / l64))
    assert glob_err < bound and abs(lg - l64) < 1e-6 * l64
    for kind in ("sync", "local"):
        l0, g0, rm0 = r0[kind]
        l1, g1, rm1 = r1[kind]
        mean_g = _as_ref_layout({n: (g0[n] + g1[n]) / 2 for n in g0}, g64)
        loss_err = abs((l0 + l1) / 2 - lg) / abs(lg)
        grad_err = max(_rel(mean_g[n], gg[n]) for n in gg)
        exact_err = max(_rel(mean_g[n], g64[n]) for n in g64)
        rm_err = max(_rel(rm0[n], rmg[n]) for n in rmg)
        print("%s: loss rel err %.3g, worst grad rel err vs global GPU %.3g, vs fp64 %.3g, running-mean rel err %.3g"
              % (kind, loss_err, grad_err, exact_err, rm_err))
        if kind == "sync":
            assert loss_err < 1e-6
            assert grad_err < bound and exact_err < bound
            assert rm_err < 1e-5
            assert all(torch.equal(rm0[n], rm1[n]) for n in rm0)      # every rank holds the same statistics
        else:
            assert exact_err > 20 * bound                               # per-rank BN: another computation
    # Trainer(distributed=True, sync_bn=True): the all-reduced gradients on each rank
    # are the global-batch step's, within the same bound
    for r in (r0, r1):
        ld, gd, rmd = r["dp_sync"]
        gd = _as_ref_layout(gd, g64)
        dp_err = max(_rel(gd[n], g64[n]) for n in g64)
        print("dp_sync rank: worst grad rel err vs fp64 %.3g" % dp_err)
        assert dp_err < bound
        assert max(_rel(rmd[n], rmg[n]) for n in rmg) < 1e-5
    assert all(torch.equal(r0["dp_sync"][1][n], r1["dp_sync"][1][n]) for n in r0["dp_sync"][1])
