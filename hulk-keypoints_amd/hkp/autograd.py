"""autograd bridge: the whole keypoint network is ONE torch.autograd.Function.

forward runs hkp.net's kernel walk keeping a Trace of the activations the
backward needs; backward runs the hand-written backward kernels and returns
every parameter gradient at once.  This is what makes the reference's
training idiom (train.py:21,25,35: ``model.forward(img).double()`` →
``nn.BCELoss()`` → ``loss.backward()``) work unchanged on this path.

HeatmapLoss is the fused fp64 BCE/MSE (train.py:25 / :13) as a Function too.
"""
import torch

from . import net, ops


class _KeypointsFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, model, *params):
        trace = net.Trace(model.policy)
        hm, _, _ = net.keypoints_forward(model.resnet.net, x, model.num_keypoints, heat=True, trace=trace)
        ctx.trace, ctx.model = trace, model
        return hm

    @staticmethod
    def backward(ctx, d_heat):
        model = ctx.model
        # model.grad_ready (DP: GradBucketer.ready) sees each gradient as soon as it
        # exists, so bucket all-reduces overlap the rest of this backward
        grads = net.keypoints_backward(model.resnet.net, ctx.trace, d_heat.contiguous(),
                                       net.Grads(on_ready=getattr(model, "grad_ready", None)))
        ctx.trace = None
        out = [None, None]
        for p in model.parameters():
            out.append(grads.get(p))
        return tuple(out)


def keypoints_heatmaps(model, x):
    return _KeypointsFn.apply(x, model, *model.parameters())


class _HeatLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, heat, target, uv, sigma, kind):
        loss, dheat = ops.heat_loss(heat.contiguous(), target, uv, sigma, kind,
                                    want_grad=torch.is_grad_enabled() or heat.requires_grad)
        ctx.save_for_backward(dheat)
        return loss

    @staticmethod
    def backward(ctx, g):
        (dheat,) = ctx.saved_tensors
        return dheat * g.to(dheat.dtype), None, None, None, None


def heatmap_loss(heat, target=None, uv=None, sigma=8.0, kind="bce"):
    """mean BCE (default) or MSE between fp32 heatmaps and the fp64 Gaussian target
    (dense ``target`` or recomputed from ``uv``), returned as a 0-dim fp64 tensor."""
    return _HeatLossFn.apply(heat, target, uv, sigma, kind)


class HeatmapBCELoss(torch.nn.Module):
    """Drop-in for ``nn.BCELoss()(pred.double(), gt)`` (train.py:25) on GPU heatmaps."""

    def forward(self, pred, gt):
        if pred.dtype == torch.float64:
            raise TypeError("pass the fp32 heatmaps (the kernel performs the .double() itself)")
        return heatmap_loss(pred, target=gt, kind="bce")


class HeatmapMSELoss(torch.nn.Module):
    def forward(self, pred, gt):
        return heatmap_loss(pred, target=gt, kind="mse")
