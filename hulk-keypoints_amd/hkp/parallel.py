"""Data parallelism over the GPUs of a node: sharded inference
and SyncBN (training's gradient all-reduce is hkp.train.GradBucketer).

Inference shards by image: every rank runs the fused forward + argmax on its
own slice of the batch (no collective on the data path; train-mode BN
statistics are per shard, exactly as a per-shard run of the reference's
analysis.py would compute them, SURVEY D5 — unless SyncBN is on), then the int32 [b, K, 2] (y, x)
keypoints — 8 bytes per keypoint — are all-gathered so every rank (and in
particular rank 0, which writes results) holds the global [B, K, 2] in rank
order.  One process per GPU, torch.distributed "nccl" = RCCL over xGMI (gloo
for the CPU tests).
"""
import torch
import torch.distributed as dist


def world():
    return dist.get_world_size() if dist.is_initialized() else 1


def rank():
    return dist.get_rank() if dist.is_initialized() else 0


def shard_range(n, rank_, world_):
    """Contiguous [lo, hi) slice of n items owned by rank_ (the first n % world_
    ranks take one extra item)."""
    base, extra = divmod(n, world_)
    lo = rank_ * base + min(rank_, extra)
    return lo, lo + base + (1 if rank_ < extra else 0)


def gather_keypoints(yx, group=None):
    """all_gather of each rank's int32 [b_r, K, 2] keypoints → [sum b_r, K, 2] in
    rank order, on every rank.  Shards may differ in size (padded to the largest
    for the collective, trimmed after)."""
    if yx.dtype != torch.int32 or yx.dim() != 3 or yx.shape[2] != 2:
        raise ValueError("gather_keypoints: expected int32 [b, K, 2], got %s %s" % (yx.dtype, tuple(yx.shape)))
    n = dist.get_world_size(group) if dist.is_initialized() else 1
    if n == 1:
        return yx
    yx = yx.contiguous()
    sizes = torch.tensor([yx.shape[0]], device=yx.device, dtype=torch.int64)
    all_sizes = [torch.empty_like(sizes) for _ in range(n)]
    dist.all_gather(all_sizes, sizes, group=group)
    counts = [int(s.item()) for s in all_sizes]
    bmax = max(counts)
    if yx.shape[0] < bmax:
        pad = torch.zeros((bmax - yx.shape[0],) + tuple(yx.shape[1:]), device=yx.device, dtype=yx.dtype)
        yx = torch.cat([yx, pad])
    parts = [torch.empty_like(yx) for _ in range(n)]
    dist.all_gather(parts, yx, group=group)
    return torch.cat([p[:c] for p, c in zip(parts, counts)])


def gather_keypoints_fixed(yx, out=None, group=None):
    """gather_keypoints for equal shards (the bench's steady state): one
    all_gather_into_tensor, no size exchange; out: a [world*b, K, 2] int32 buffer
    reused across steps."""
    n = dist.get_world_size(group) if dist.is_initialized() else 1
    if n == 1:
        return yx
    if out is None:
        out = torch.empty((n * yx.shape[0],) + tuple(yx.shape[1:]), device=yx.device, dtype=yx.dtype)
    dist.all_gather_into_tensor(out, yx.contiguous(), group=group)
    return out


_HOST_GROUPS = {}


def _ranks(group):
    return list(range(dist.get_world_size())) if group is None else list(dist.get_process_group_ranks(group))


def host_group(group=None):
    """A gloo group over the ranks of `group` (the group itself when it is gloo),
    created once per rank set and cached.  Host-side checks (check_shards) run on
    it so they never wait for the GPU queue: an RCCL collective followed by
    .item() would block the host until every kernel queued before it had run.
    Like dist.new_group, the first call for a rank set is collective over the
    default group."""
    if dist.get_backend(group) == "gloo":
        return group
    key = tuple(_ranks(group))
    if key not in _HOST_GROUPS:
        _HOST_GROUPS[key] = dist.new_group(list(key), backend="gloo")
    return _HOST_GROUPS[key]


_LIKE_GROUPS = {}


def new_group_like(group=None):
    """A separate communicator over the same ranks and backend as `group`, created
    once per (rank set, backend) and cached (every Trainer(sync_bn=True) over the
    same ranks shares it; communicators are never leaked per Trainer).
    Trainer(sync_bn=True) runs the SyncBN statistics gathers on one: RCCL runs the
    collectives of one communicator in issue order, so on the gradient buckets'
    communicator every backward BN gather would queue behind the in-flight 32 MB
    bucket all-reduce and put it back on the critical path.  The first call for a
    rank set is collective over the default group (dist.new_group)."""
    key = (tuple(_ranks(group)), str(dist.get_backend(group)))
    if key not in _LIKE_GROUPS:
        _LIKE_GROUPS[key] = dist.new_group(list(key[0]), backend=key[1])
    return _LIKE_GROUPS[key]


class ShardCheck:
    """The SyncBN empty-shard guard of a Trainer.  Given the job's batch size
    (`global_batch`: the same on every rank, sharded by shard_range) it needs no
    collective at all — each outcome is one that every rank reaches, or one that
    cannot leave a peer waiting:
      * global_batch < world: some rank's shard is empty; every rank computes the
        same verdict and raises;
      * this rank holds >= 1 image: it enters every SyncBN gather, whose merge
        weights each rank by the row count it gathered (hkp_bn_finalize_ranks,
        hkp_bn_bwd_finalize_ranks), so the statistics are the global batch's even
        if the size differs from its shard_range share (a sampler that does not
        pad its last batch): the step proceeds, with a warning;
      * this rank holds no image although the global batch covers every rank: it
        alone would skip the gathers and leave its peers waiting in them, and an
        exception can be caught and the process kept alive — so the process exits
        (status 3) after writing why to stderr; the peers' collectives then fail
        (gloo: connection closed; RCCL: the watchdog) instead of hanging.
    Without global_batch, one check_shards collective per step: a rank cannot skip
    on its own (a cache of "sizes already seen" would let the ranks whose size did
    not change skip while the one whose did waits in the collective forever)."""

    def __init__(self, group=None):
        self.group = group
        self.collectives = 0            # host collectives run (tests)
        self.mismatches = 0             # steps whose local size was not the shard_range share

    def __call__(self, n_local, global_batch=None):
        if not dist.is_initialized() or dist.get_world_size(self.group) == 1:
            return
        n = dist.get_world_size(self.group)
        if global_batch is not None:
            if int(global_batch) < n:
                raise ValueError("SyncBN needs at least one image on every rank (global batch %d < world size %d)"
                                 % (global_batch, n))
            lo, hi = shard_range(int(global_batch), _ranks(self.group).index(dist.get_rank()), n)
            if int(n_local) < 1:
                import os
                import sys
                sys.stderr.write("hkp.parallel.ShardCheck: rank %d holds no image of the global batch %d (its "
                                 "shard_range share is %d); exiting so that the other ranks' SyncBN gathers fail "
                                 "instead of waiting for it\n" % (dist.get_rank(), global_batch, hi - lo))
                sys.stderr.flush()
                os._exit(3)
            if int(n_local) != hi - lo:
                if self.mismatches == 0:
                    import warnings
                    warnings.warn("SyncBN: rank %d holds %d images, its shard_range share of the global batch %d "
                                  "is %d; the BN statistics weight each rank by its own count"
                                  % (dist.get_rank(), n_local, global_batch, hi - lo))
                self.mismatches += 1
            return
        check_shards(n_local, self.group)
        self.collectives += 1


def check_shards(n_local, group=None):
    """Every rank holds at least one image (one tiny host collective: the shard
    sizes all-gathered).  A SyncBN forward or backward with an empty shard would
    leave the other ranks waiting in their statistics gathers forever, so every
    rank raises instead.  The gather runs on a gloo group over host memory
    (host_group): no GPU sync, so the host keeps queuing the step's kernels ahead
    of the GPU.  Returns every rank's size, in rank order."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return [int(n_local)]
    n = dist.get_world_size(group)
    t = torch.tensor([int(n_local)], dtype=torch.int64)
    parts = [torch.empty_like(t) for _ in range(n)]
    dist.all_gather(parts, t, group=host_group(group))
    sizes = [int(p.item()) for p in parts]
    if min(sizes) < 1:
        raise ValueError("SyncBN needs at least one image on every rank (global batch < world size %d)" % n)
    return sizes


@torch.no_grad()
def predict_keypoints_dp(model, x_shard, heat=False, sync=False, group=None, global_batch=None):
    """Each rank's shard through the fused forward (+ argmax); keypoints gathered.
    sync: BN statistics over the whole sharded batch of `group` (SyncBN, below) —
    the result then equals one forward over the global batch.  global_batch (the
    same on every rank; x_shard its shard_range share) spares the empty-shard
    guard its host collective (ShardCheck).
    Returns (global int32 [B, K, 2], this rank's heatmaps or None)."""
    pol = model.policy.with_(sync_bn=True, sync_group=group) if sync else model.policy
    if sync:
        ShardCheck(group)(x_shard.shape[0], global_batch)
    if heat:
        hm, yx = model.heatmaps_and_keypoints(x_shard, policy=pol)
    else:
        hm, yx = None, model.predict_keypoints(x_shard, policy=pol)
    return gather_keypoints(yx, group), hm


# ---- SyncBN (caveat D5) ----------------------------------------
# Off by default: per-rank BN statistics (standard DDP semantics, as above).  On
# (Policy(sync_bn=True, sync_group=...), carried by the model or the Trainer):
# every train-mode BN layer's batch statistics are taken over the whole sharded
# batch — each rank's [mean | M2 | count] block (hkp_bn_stats, fp64) is
# all-gathered in rank order and merged in fixed order (hkp_bn_finalize_ranks),
# so every rank applies the same scale/shift and a DP forward over N ranks gives
# the outputs of one forward over the global batch (torch SyncBatchNorm's
# forward).  In training the BN backward's channel sums are gathered the same
# way (hkp_bn_bwd_stats / hkp_bn_bwd_finalize_ranks: torch SyncBatchNorm's
# all-reduced sum_dy / sum_dy_xmu), so a step equals one step over the global
# batch.  A block's downsample BN and its last BN share one gather in each
# direction (hkp.net); DESIGN.md gives the per-step count.


def active_sync_group(policy):
    """(group,) while `policy` synchronises BN and more than one rank takes part,
    else None."""
    if policy is None or not policy.sync_bn or not dist.is_initialized() \
            or dist.get_world_size(policy.sync_group) == 1:
        return None
    return (policy.sync_group,)


def gather_bn_stats(st, group=None):
    """all_gather of each rank's fp64 statistics block ([2C+1] forward, [4C+1]
    backward, or several blocks concatenated) → [world, len] in rank order.  RCCL gathers on the device; other backends (gloo) through host
    copies (the blocks are a few KB)."""
    n = dist.get_world_size(group) if dist.is_initialized() else 1
    if n == 1:
        return st.reshape(1, -1)
    if st.is_cuda and dist.get_backend(group) == "nccl":
        out = torch.empty((n, st.numel()), device=st.device, dtype=st.dtype)
        dist.all_gather_into_tensor(out, st.contiguous(), group=group)
        return out
    host = st.detach().cpu().contiguous()
    parts = [torch.empty_like(host) for _ in range(n)]
    dist.all_gather(parts, host, group=group)
    return torch.stack(parts).to(st.device)
