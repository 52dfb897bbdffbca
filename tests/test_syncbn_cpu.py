"""SyncBN host logic on CPU (the kernels are checked by tests/test_gpu_syncbn.py).

* the fixed-order rank merge hkp_bn_finalize_ranks implements
  (mean = sum n_r mean_r / N, M2 = sum M2_r + n_r (mean_r - mean)^2), restated in
  numpy, equals the statistics of the whole batch (ragged shards included);
* hkp.parallel.gather_bn_stats over a gloo world of 2 returns the blocks in rank
  order on every rank; a Policy(sync_bn=True) switches it on (active_sync_group),
  per policy — no process-global state; check_shards makes every rank raise
  when one holds no image (instead of hanging in a gather).
"""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "hulk-keypoints_amd")


def _rank_block(y):
    """[mean | M2 | count] of rows y [n, C] (hkp_bn_stats' layout), fp64."""
    mean = y.mean(0)
    return np.concatenate([mean, ((y - mean) ** 2).sum(0), [float(len(y))]])


def _merge(blocks):
    """numpy restatement of bn_fin_ranks_kernel (csrc/bn.hip)."""
    st = np.stack(blocks)
    c = (st.shape[1] - 1) // 2
    n = st[:, 2 * c]
    if len(st) == 1:
        mean = st[0, :c]
    else:
        mean = (n[:, None] * st[:, :c]).sum(0) / n.sum()
    m2 = (st[:, c:2 * c] + n[:, None] * (st[:, :c] - mean) ** 2).sum(0)
    return n.sum(), mean, m2


def test_rank_merge_formula_matches_whole_batch():
    rng = np.random.default_rng(5)
    y = rng.normal(3.0, 2.0, size=(1000, 17)) + np.linspace(-50, 50, 17)
    for cuts in ([], [512], [1, 999], [100, 350, 351, 800]):
        b = [0] + cuts + [len(y)]
        n, mean, m2 = _merge([_rank_block(y[lo:hi]) for lo, hi in zip(b[:-1], b[1:])])
        assert n == len(y)
        np.testing.assert_allclose(mean, y.mean(0), rtol=1e-13, atol=1e-12)
        np.testing.assert_allclose(m2 / n, y.var(0), rtol=1e-12)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gather_worker(rank, world, port, q):
    import sys
    sys.path[:0] = [REPO, PKG]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hkp import parallel
    from hkp.policy import DEFAULT
    on = DEFAULT.with_(sync_bn=True)
    ok = parallel.active_sync_group(DEFAULT) is None           # off by default
    ok &= parallel.active_sync_group(on) is not None
    st = torch.arange(7, dtype=torch.float64) + 100.0 * rank
    g = parallel.gather_bn_stats(st, parallel.active_sync_group(on)[0])
    ok &= tuple(g.shape) == (world, 7) and g.dtype == torch.float64
    ok &= all(torch.equal(g[r], torch.arange(7, dtype=torch.float64) + 100.0 * r) for r in range(world))
    ok &= DEFAULT.sync_bn is False                            # the default is untouched
    parallel.check_shards(1 + rank)                            # every rank holds images: passes
    try:                                                       # rank 1 empty: EVERY rank raises (no hang)
        parallel.check_shards(1 - rank)
        ok = False
    except ValueError:
        pass
    q.put((rank, bool(ok)))
    dist.destroy_process_group()


def test_gather_bn_stats_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    res = [q.get(timeout=5) for _ in range(world)]
    assert all(p.exitcode == 0 for p in procs)
    assert all(ok for _, ok in res), res


def _groups_worker(rank, world, port, q):
    import sys
    sys.path[:0] = [REPO, PKG]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hkp import parallel, train
    from src.model import KeypointsGauss
    m = KeypointsGauss(2, 32, 48, backbone="resnet18", pretrained=False)
    t = train.Trainer(m, distributed=True, optimizer="torch", sync_bn=True, bucket_mb=1)
    ok = t.bn_group is not None and t.bn_group is not t.group            # SyncBN: its own communicator
    ok &= t.policy.sync_group is t.bn_group and t.bucketer.group is t.group
    ok &= parallel.active_sync_group(t.policy) == (t.bn_group,)
    ok &= dist.get_process_group_ranks(t.bn_group) == list(range(world))
    # the BN group carries collectives independently of the default group
    st = torch.full((3,), float(rank), dtype=torch.float64)
    g = parallel.gather_bn_stats(st, t.bn_group)
    ok &= torch.equal(g[:, 0], torch.arange(world, dtype=torch.float64))
    ok &= not t.bucketer.avg_in_collective        # gloo has no ReduceOp.AVG: sum, then 1/world
    t2 = train.Trainer(m, distributed=True, optimizer="torch", sync_bn=False, bucket_mb=1)
    ok &= t2.bn_group is t2.group is None          # no SyncBN: no extra communicator
    t3 = train.Trainer(m, distributed=True, optimizer="torch", sync_bn=True, bucket_mb=1)
    ok &= t3.bn_group is t.bn_group                # one cached communicator per rank set, not one per Trainer
    # the empty-shard guard: no host collective over N SyncBN steps that name their
    # global batch (shard_range shares: 7 images -> 4 + 3), one per step otherwise
    for _ in range(5):
        t.shard_check(4 - rank, global_batch=7)
    ok &= t.shard_check.collectives == 0
    for _ in range(2):
        t.shard_check(4 - rank)
    ok &= t.shard_check.collectives == 2
    try:                                        # global batch < world: every rank raises
        t.shard_check(1 - rank, 1)
        ok = False
    except ValueError:
        pass
    # only rank 1's size differs from its shard_range share (a sampler that does not
    # pad its last batch): no rank raises, both go on into the gathers, which carry
    # the counts (a raise on one rank left the other waiting in them)
    t.shard_check(4 if rank == 0 else 2, global_batch=7)
    ok &= t.shard_check.mismatches == rank
    st = torch.tensor([float(rank), 0.0, 4.0 if rank == 0 else 2.0], dtype=torch.float64)
    g = parallel.gather_bn_stats(st, t.bn_group)
    ok &= g[:, 2].tolist() == [4.0, 2.0]
    q.put((rank, bool(ok)))
    dist.destroy_process_group()


def _empty_shard_worker(rank, world, port, q):
    import sys
    sys.path[:0] = [REPO, PKG]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hkp import parallel
    chk = parallel.ShardCheck()
    grp = parallel.new_group_like()
    q.put((rank, "checking"))
    chk(0 if rank == 1 else 4, global_batch=7)      # rank 1: no image although 7 >= world
    try:                                            # rank 0 goes on into a SyncBN gather
        parallel.gather_bn_stats(torch.zeros(3, dtype=torch.float64), grp)
        q.put((rank, "gathered"))
    except Exception as e:                          # the peer exited: the gather fails, it does not wait
        q.put((rank, "failed: %s" % type(e).__name__))


def test_shard_check_empty_rank_does_not_hang_peers_gloo_world2():
    """a rank whose shard is empty while the declared global batch covers
    every rank exits (status 3) instead of raising, so its peer's next SyncBN gather
    fails instead of waiting for it forever."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_empty_shard_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode is not None for p in procs), "a rank hung"
    assert procs[1].exitcode == 3
    msgs = []
    while len(msgs) < 3:                            # (rank 1's os._exit may drop its queued message)
        try:
            msgs.append(q.get(timeout=5))
        except Exception:
            break
    assert (0, "gathered") not in msgs and any(r == 0 and m.startswith("failed") for r, m in msgs), msgs


def test_trainer_syncbn_own_communicator_gloo_world2():
    """Trainer(sync_bn=True) gives the BN gathers a communicator of their own
    (RCCL runs one communicator's collectives in issue order: a backward BN gather
    must not queue behind an in-flight gradient bucket); the step equality itself
    is checked on the GPU (test_gpu_syncbn.py, dp_sync)."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_groups_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    res = [q.get(timeout=5) for _ in range(world)]
    assert all(p.exitcode == 0 for p in procs)
    assert all(ok for _, ok in res), res


def test_sync_bn_single_process_is_off():
    import sys
    sys.path[:0] = [REPO, PKG]
    from hkp import parallel
    from hkp.policy import DEFAULT
    assert parallel.active_sync_group(DEFAULT.with_(sync_bn=True)) is None     # one rank: nothing to sync
    st = torch.ones(5, dtype=torch.float64)
    assert torch.equal(parallel.gather_bn_stats(st), st[None])
    parallel.check_shards(0)                                   # one rank: nothing to check
