"""MI355X-native restatement of src/resnet_dilated.py (Resnet34_8s, :5-28),
plus the same wrapper around resnet18 / resnet50 (BASELINE configs C1, C4, C5;
SURVEY D2).  Attribute name ``<backbone>_8s`` keeps the reference's
state_dict prefix (``resnet.resnet34_8s.*`` for the default backbone)."""
import torch.nn as nn

from hkp import net
from hkp.policy import DEFAULT, Policy
from src import resnet as _resnet


class ResnetDilated8s(nn.Module):
    """``policy`` (hkp.policy.Policy): how the kernels compute this network —
    conv arithmetic (default f16x3), SyncBN group, tuning; a plain attribute, so
    two models with different policies coexist."""

    def __init__(self, backbone="resnet34", num_classes=1000, pretrained=True, policy=None):
        super().__init__()
        self.policy = DEFAULT if policy is None else policy
        if not isinstance(self.policy, Policy):
            raise TypeError("policy must be an hkp.policy.Policy")
        # load (local) pretrained weights, remove avg pool, output stride 8 (resnet_dilated.py:8-13)
        model = getattr(_resnet, backbone)(fully_conv=True, pretrained=pretrained, output_stride=8,
                                           remove_avg_pool_layer=True)
        # randomly initialise the 1x1 scoring conv (resnet_dilated.py:15-22)
        model.fc = nn.Conv2d(model.inplanes, num_classes, 1)
        self.backbone = backbone
        setattr(self, backbone + "_8s", model)
        self._normal_initialization(model.fc)

    @property
    def net(self):
        return getattr(self, self.backbone + "_8s")

    def _normal_initialization(self, layer):
        layer.weight.data.normal_(0, 0.01)
        layer.bias.data.zero_()

    def forward(self, x):
        """Upsampled raw logits [B,1000,H,W] (resnet_dilated.py:24-28)."""
        return net.logits_forward(self.net, x, pol=self.policy)


class Resnet34_8s(ResnetDilated8s):
    def __init__(self, num_classes=1000, pretrained=True):
        super().__init__("resnet34", num_classes, pretrained)


class Resnet18_8s(ResnetDilated8s):
    def __init__(self, num_classes=1000, pretrained=True):
        super().__init__("resnet18", num_classes, pretrained)


class Resnet50_8s(ResnetDilated8s):
    def __init__(self, num_classes=1000, pretrained=True):
        super().__init__("resnet50", num_classes, pretrained)
