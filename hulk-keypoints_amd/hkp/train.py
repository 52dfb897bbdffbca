"""Training step (train.py:32-36 restated for the MI355X path) and data parallelism.

Trainer.step = forward (kernel walk, Trace kept) → fused fp64 loss kernel
(dL/dheat) → backward kernels (net.keypoints_backward) → [RCCL all-reduce of
gradients, bucketed and overlapped with the rest of backward] → Adam
(lr 1e-4, weight_decay 1e-4, train.py:79): the optimizer loop stays a PyTorch
optimizer object as the north star asks; its update is either hkp.optim.FusedAdam
(default: one HIP pass over all parameters) or torch.optim.Adam.

Data parallelism: one process per GPU (torchrun), torch.distributed backend
"nccl" = RCCL over xGMI.  Gradients land in flat per-bucket buffers in the
order backward produces them (fc, layer4, …, stem); as soon as a bucket is
complete its all-reduce is launched asynchronously, so communication of the
late layers overlaps the backward of the early ones.  BatchNorm statistics
stay per rank (standard DDP semantics) unless Trainer(sync_bn=True): then the
BN statistics and the BN backward sums are taken over every rank's shard
(Policy(sync_bn=True), hkp.parallel), and a step equals one step over the
global batch.
Parameters and buffers are broadcast from rank 0 when the Trainer is built
(broadcast_state).
"""
import torch
import torch.distributed as dist

from . import net, ops, parallel
from .optim import FusedAdam


class GradBucketer:
    """Bucketed, overlapped gradient all-reduce (mean over ranks)."""

    def __init__(self, params, bucket_bytes=32 << 20, group=None, last_bucket_bytes=None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        # RCCL averages inside the all-reduce (ReduceOp.AVG); gloo has no AVG, so
        # there the sum is scaled by 1/world after the wait
        self.avg_in_collective = self.world > 1 and dist.get_backend(group) == "nccl"
        self.op = dist.ReduceOp.AVG if self.avg_in_collective else dist.ReduceOp.SUM
        # backward produces grads roughly in reverse parameter order; buckets are cut
        # from the END of that order (the stem side), the first of them (the last
        # to fill, its all-reduce exposed after backward) capped at
        # last_bucket_bytes (bucket_bytes / 8 by default): for R34 the tail bucket
        # is layer2 + layer1 + stem (~6 MB) instead of a 23 MB remainder
        if last_bucket_bytes is None:
            last_bucket_bytes = bucket_bytes // 8
        order = list(reversed(list(params)))
        tail_first = []
        cur, cur_bytes, cap = [], 0, last_bucket_bytes
        for p in reversed(order):
            if cur and cur_bytes + p.numel() * 4 > cap:
                tail_first.append(cur)
                cur, cur_bytes, cap = [], 0, bucket_bytes
            cur.insert(0, p)
            cur_bytes += p.numel() * 4
        if cur:
            tail_first.append(cur)
        self.buckets = list(reversed(tail_first))
        self.slot = {}
        self.flat = []
        for bi, ps in enumerate(self.buckets):
            n = sum(p.numel() for p in ps)
            flat = torch.zeros(n, device=ps[0].device, dtype=torch.float32)
            off = 0
            for p in ps:
                self.slot[p] = (bi, off)
                off += p.numel()
            self.flat.append(flat)
        self._reset()

    def _reset(self):
        self.pending = [len(ps) for ps in self.buckets]
        self.works = [None] * len(self.buckets)
        self.streams = [set() for _ in self.buckets]

    def ready(self, p, g):
        """Copy g into its bucket on the CURRENT stream (the one that produced g:
        main, or the side stream a wgrad ran on); a full bucket's all-reduce is
        launched after the current stream joins the other streams that copied
        into it (once per bucket, not per gradient)."""
        bi, off = self.slot[p]
        cur = torch.cuda.current_stream(g.device) if g.is_cuda else None    # (gloo tests: CPU tensors)
        self.flat[bi][off:off + p.numel()].copy_(g.reshape(-1))
        self.streams[bi].add(cur)
        self.pending[bi] -= 1
        if self.pending[bi] == 0:
            for s in self.streams[bi]:
                if s is not None and s != cur:
                    cur.wait_stream(s)
            if self.world > 1:
                self.works[bi] = dist.all_reduce(self.flat[bi], op=self.op, group=self.group, async_op=True)

    def finish(self):
        """Wait for every bucket; average; point p.grad at the flat buffers."""
        if any(self.pending):
            raise RuntimeError("gradient missing for %d parameters" % sum(self.pending))
        for bi, w in enumerate(self.works):
            if w is not None:
                w.wait()
            else:                              # world 1: the copies themselves
                for s in self.streams[bi]:
                    if s is not None and s != torch.cuda.current_stream(s.device):
                        torch.cuda.current_stream(s.device).wait_stream(s)
            if self.world > 1 and not self.avg_in_collective:
                self.flat[bi].mul_(1.0 / self.world)
        for p, (bi, off) in self.slot.items():
            p.grad = self.flat[bi][off:off + p.numel()].view_as(p)
        self._reset()


def broadcast_state(model, src=0, group=None):
    """Copy rank src's parameters and buffers (BN running stats and counters) to
    every rank, in place — what DDP does at construction.  Tensors are flattened
    per dtype into one buffer each, so a whole network costs a few collectives."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    tensors = [t.data for t in list(model.parameters()) + list(model.buffers())]
    by_dtype = {}
    for t in tensors:
        by_dtype.setdefault((t.dtype, t.device), []).append(t)
    for (dtype, dev), ts in by_dtype.items():
        flat = torch.cat([t.reshape(-1) for t in ts])
        dist.broadcast(flat, src, group=group)
        off = 0
        for t in ts:
            t.copy_(flat[off:off + t.numel()].view_as(t))
            off += t.numel()


class Trainer:
    """One optimizer step per call, reference semantics (train.py:33-36)."""

    def __init__(self, model, lr=1e-4, weight_decay=1e-4, loss="bce", sigma=8.0, distributed=False,
                 bucket_mb=32, optimizer="fused", sync_bn=False, group=None, force_buckets=False):
        """sync_bn: BN statistics and their backward sums over every rank of
        `group` (default: the world; the step then equals one step over the
        global batch), instead of per-rank BN (DDP semantics, the default).
        force_buckets: the DP gradient path (bucket copies, stream joins) at world
        size 1, to time its overhead on one GPU."""
        self.model = model
        self.group = group
        self.sync_bn = sync_bn
        # SyncBN gathers on their own communicator over the same ranks (RCCL orders
        # the collectives of one communicator by issue, so the 33 + 33 per-step R34
        # BN gathers would otherwise wait behind in-flight gradient buckets)
        multi = sync_bn and dist.is_initialized() and dist.get_world_size(group) > 1
        self.bn_group = parallel.new_group_like(group) if multi else group
        # the empty-shard check's host (gloo) group, created here — collectively, on
        # every rank, next to the communicator above — never lazily inside a step
        # (dist.new_group is collective over the default group: ranks outside a
        # subgroup would never make the call)
        if multi:
            parallel.host_group(group)
        self.shard_check = parallel.ShardCheck(group)
        self.policy = model.policy.with_(sync_bn=True, sync_group=self.bn_group) if sync_bn else model.policy
        self.params = list(model.parameters())
        self.loss_kind = loss
        self.sigma = sigma
        if optimizer not in ("fused", "torch"):
            raise ValueError("optimizer must be 'fused' or 'torch'")
        opt_cls = FusedAdam if optimizer == "fused" else torch.optim.Adam
        self.opt = opt_cls(self.params, lr=lr, weight_decay=weight_decay)
        use_dp = distributed and dist.is_initialized() and dist.get_world_size(group) > 1
        if use_dp:
            broadcast_state(model, group=group)   # every replica starts from rank 0's weights and BN buffers
        self.bucketer = GradBucketer(self.params, bucket_mb << 20, group=group) if (use_dp or force_buckets) \
            else None

    def forward_backward(self, x, uv=None, target=None, global_batch=None):
        """global_batch (SyncBN): the job's batch size — the same on every rank, x
        being this rank's hkp.parallel.shard_range share of it; lets the empty-shard
        guard run without a host collective (parallel.ShardCheck)."""
        if self.sync_bn:
            self.shard_check(x.shape[0], global_batch)
        m = self.model
        trace = net.Trace(self.policy)
        hm, _, _ = net.keypoints_forward(m.resnet.net, x, m.num_keypoints, heat=True, trace=trace)
        loss, dheat = ops.heat_loss(hm, target, uv, self.sigma, self.loss_kind, want_grad=True)
        grads = net.Grads(on_ready=self.bucketer.ready if self.bucketer else None)
        net.keypoints_backward(m.resnet.net, trace, dheat, grads)
        if self.bucketer is not None:
            self.bucketer.finish()
        else:
            for p in self.params:
                p.grad = grads[p]
        return loss

    def step(self, x, uv=None, target=None, global_batch=None):
        loss = self.forward_backward(x, uv, target, global_batch)
        self.opt.step()
        return loss
