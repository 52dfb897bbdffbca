"""FusedAdam: torch.optim.Adam's interface and state (train.py:79 constructs
``optim.Adam(params, lr=1e-4, weight_decay=1e-4)``), one HIP pass over every
parameter per step (hkp_adam_step, csrc/adam.hip).

Same constructor, ``step()``, ``zero_grad()``, ``state_dict()`` / ``load_state_dict()``
and per-parameter state keys (``step``, ``exp_avg``, ``exp_avg_sq``) as
torch.optim.Adam, so checkpoints move between the two.  Options the reference
never uses (amsgrad, maximize, capturable, differentiable, fused, foreach,
decoupled weight decay) are rejected rather than silently ignored.  No CPU path:
parameters must be fp32 CUDA tensors.
"""
import ctypes
import math

import torch

from ._lib import AdamTensor, HkpError, call


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False, *,
                 maximize=False, foreach=None, capturable=False, differentiable=False, fused=None):
        if amsgrad or maximize or capturable or differentiable or fused:
            raise HkpError("FusedAdam: amsgrad/maximize/capturable/differentiable/fused are not supported")
        if not 0.0 <= lr or not 0.0 <= eps or not 0.0 <= weight_decay:
            raise ValueError("FusedAdam: invalid lr/eps/weight_decay")
        if not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError("FusedAdam: invalid betas %s" % (betas,))
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False, maximize=False,
                        foreach=None, capturable=False, differentiable=False, fused=None)
        super().__init__(params, defaults)
        # per param group: the launch table of the last step (parameter / moment
        # pointers fixed; gradient pointers refreshed each step) and the common step
        # count — rebuilding it per parameter in Python left the GPU idle ~1.4 ms per
        # training step.  Invalidated by load_state_dict / add_param_group.
        self._fast = {}

    def load_state_dict(self, state_dict):
        self._fast = {}
        super().load_state_dict(state_dict)

    def add_param_group(self, param_group):
        self._fast = {}
        super().add_param_group(param_group)

    def _fast_step(self, gi, group):
        """One launch from the cached table, or False (cache miss: slow path)."""
        fc = self._fast.get(gi)
        if fc is None:
            return False
        ps = [p for p in group["params"] if p.grad is not None]
        if len(ps) != len(fc["ps"]) or any(a is not b for a, b in zip(ps, fc["ps"])):
            return False
        arr = fc["arr"]
        for i, p in enumerate(ps):
            g = p.grad
            if g.dtype != torch.float32 or g.is_sparse or not g.is_contiguous() or g.device != p.device:
                raise HkpError("FusedAdam: fp32 contiguous CUDA gradients only")
            arr[i].grad = g.data_ptr()
        torch._foreach_add_(fc["steps"], 1.0)
        fc["step"] += 1
        self._launch(group, ps, arr, fc["step"])
        return True

    def _launch(self, group, ps, arr, step):
        b1, b2 = group["betas"]
        bc1 = 1.0 - b1 ** step
        bc2 = 1.0 - b2 ** step
        call("hkp_adam_step", len(ps), arr, b2, 1.0 - b1, 1.0 - b2, group["eps"], group["weight_decay"],
             -group["lr"] / bc1, math.sqrt(bc2), ctypes.c_void_p(torch.cuda.current_stream(ps[0].device).cuda_stream))
        # the kernel wrote p, exp_avg, exp_avg_sq behind autograd's back: bump
        # their version counters as torch's in-place Adam ops do (operand caches
        # keyed on the version — the packed conv weights — see the change)
        torch.autograd.graph.increment_version(ps + [self.state[p][k] for p in ps for k in ("exp_avg", "exp_avg_sq")])

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            if self._fast_step(gi, group):
                continue
            self._fast.pop(gi, None)
            # one launch set per distinct step count (all equal in practice)
            by_step = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.dtype != torch.float32 or p.device.type != "cuda" or p.grad.dtype != torch.float32:
                    raise HkpError("FusedAdam: fp32 CUDA parameters and gradients only")
                if p.grad.is_sparse:
                    raise HkpError("FusedAdam: sparse gradients are not supported")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                for t, name in ((p, "param"), (p.grad, "grad"), (st["exp_avg"], "exp_avg"),
                                (st["exp_avg_sq"], "exp_avg_sq")):
                    if not t.is_contiguous():
                        raise HkpError("FusedAdam: %s must be contiguous" % name)
                st["step"] += 1
                by_step.setdefault(int(st["step"].item()), []).append(p)
            for step, ps in by_step.items():
                arr = (AdamTensor * len(ps))()
                for i, p in enumerate(ps):
                    st = self.state[p]
                    arr[i].param, arr[i].grad = p.data_ptr(), p.grad.data_ptr()
                    arr[i].exp_avg, arr[i].exp_avg_sq = st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr()
                    arr[i].n = p.numel()
                self._launch(group, ps, arr, step)
                if len(by_step) == 1:      # every parameter of the group at one step count: cacheable
                    self._fast[gi] = dict(ps=ps, arr=arr, step=step, steps=[self.state[p]["step"] for p in ps])
        return loss
