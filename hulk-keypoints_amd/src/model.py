"""MI355X-native restatement of src/model.py (KeypointsGauss, :10-22).

``forward(x)`` returns sigmoid heatmaps [B,K,H,W] exactly like the reference,
computed by the fused K-channel head (only the K kept fc rows are evaluated;
SURVEY D8).  Autograd flows through it (train.py:21,35 call pattern) via one
autograd.Function that runs the hand-written backward kernels.
``backbone`` selects resnet18 / resnet34 (default, the reference) / resnet50.
``precision`` (or a whole hkp.policy.Policy as ``policy``) selects the conv
arithmetic: "f16x3" (default, fp32-accurate), "fp32" (exact) or "f16" (config
C4, inference only); it is per model, not process-global.
"""
import torch
import torch.nn as nn

from hkp import autograd as hkp_autograd
from hkp import net
from hkp.policy import DEFAULT
from src.resnet_dilated import ResnetDilated8s


class KeypointsGauss(nn.Module):
    def __init__(self, num_keypoints, img_height=480, img_width=640, backbone="resnet34", pretrained=True,
                 precision=None, policy=None):
        super().__init__()
        if policy is None:
            policy = DEFAULT if precision is None else DEFAULT.with_(precision=precision)
        elif precision is not None:
            policy = policy.with_(precision=precision)
        self.num_keypoints = num_keypoints
        self.num_outputs = self.num_keypoints
        self.img_height = img_height
        self.img_width = img_width
        self.resnet = ResnetDilated8s(backbone, pretrained=pretrained, policy=policy)
        self.sigmoid = torch.nn.Sigmoid()
        # DP training through autograd (train.py): called as grad_ready(param, grad)
        # for each gradient as the backward kernels produce it (GradBucketer.ready)
        self.grad_ready = None

    @property
    def policy(self):
        return self.resnet.policy

    @policy.setter
    def policy(self, p):
        self.resnet.policy = p

    def forward(self, x):
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            return hkp_autograd.keypoints_heatmaps(self, x)
        hm, _, _ = net.keypoints_forward(self.resnet.net, x, self.num_keypoints, heat=True, argmax=False,
                                         pol=self.policy)
        return hm

    @torch.no_grad()
    def predict_keypoints(self, x, policy=None):
        """Fused decode: argmax (y, x) int32 [B,K,2] without materialising the heatmap
        (src/prediction.py:46 semantics, first max wins)."""
        _, yx, _ = net.keypoints_forward(self.resnet.net, x, self.num_keypoints, heat=False, argmax=True,
                                         pol=policy or self.policy)
        return yx

    @torch.no_grad()
    def heatmaps_and_keypoints(self, x, policy=None):
        hm, yx, _ = net.keypoints_forward(self.resnet.net, x, self.num_keypoints, heat=True, argmax=True,
                                          pol=policy or self.policy)
        return hm, yx
