"""autograd bridge: one Function for the whole keypoint network (placeholder until backward lands)."""
import torch

from . import net


class _KeypointsFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, model, *params):
        trace = net.Trace()
        hm, _, _ = net.keypoints_forward(model.resnet.net, x, model.num_keypoints, heat=True, trace=trace)
        ctx.trace, ctx.model = trace, model
        return hm

    @staticmethod
    def backward(ctx, d_heat):
        raise NotImplementedError("backward kernels not built yet")


def keypoints_heatmaps(model, x):
    return _KeypointsFn.apply(x, model, *model.parameters())
