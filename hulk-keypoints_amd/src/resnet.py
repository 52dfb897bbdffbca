"""MI355X-native restatement of the reference's src/resnet.py call surface.

Same constructors, module tree, parameter names/order and state_dict as the
reference (so checkpoints move both ways), but the modules are parameter
holders: compute runs in libhulkkp through hkp.net.  Conv weights are stored
KRSC ([Cout][R][S][Cin], the layout the NHWC implicit-GEMM kernel reads) and
converted to/from the reference's OIHW at state_dict()/load_state_dict() time.

  conv3x3              src/resnet.py:20-37   (padding = dilation)
  BasicBlock           src/resnet.py:40-69
  Bottleneck           src/resnet.py:72-112
  ResNet               src/resnet.py:115-217 (_make_layer OS logic :163-196)
  resnet18/34/50/...   src/resnet.py:220-272
"""
import math
import os
import warnings

import torch
import torch.nn as nn

from hkp import net

__all__ = ["ResNet", "resnet18", "resnet34", "resnet50", "resnet101", "resnet152", "conv3x3", "KRSCConv2d"]

# file names the reference's model_zoo URLs point at (src/resnet.py:11-17); looked up locally only
model_files = {
    "resnet18": "resnet18-5c106cde.pth",
    "resnet34": "resnet34-333f7ec4.pth",
    "resnet50": "resnet50-19c8e357.pth",
    "resnet101": "resnet101-5d3b4d8f.pth",
    "resnet152": "resnet152-b121ed2d.pth",
}


class KRSCConv2d(nn.Module):
    """Bias-free conv whose weight lives as KRSC; state_dict speaks OIHW."""

    def __init__(self, in_planes, out_planes, kernel_size, stride=1, padding=0, dilation=1):
        super().__init__()
        self.in_channels, self.out_channels = in_planes, out_planes
        self.kernel_size = (kernel_size, kernel_size)
        self.stride, self.padding, self.dilation = stride, padding, dilation
        self.weight = nn.Parameter(torch.empty(out_planes, kernel_size, kernel_size, in_planes))
        self._register_state_dict_hook(KRSCConv2d._to_oihw)
        self._register_load_state_dict_pre_hook(KRSCConv2d._from_oihw)

    @staticmethod
    def _to_oihw(module, state_dict, prefix, local_metadata):
        k = prefix + "weight"
        if k in state_dict:
            state_dict[k] = state_dict[k].permute(0, 3, 1, 2).contiguous()
        return state_dict

    @staticmethod
    def _from_oihw(state_dict, prefix, local_metadata, strict, missing, unexpected, errors):
        # checkpoints always carry the reference's OIHW layout (state_dict() emits it too)
        k = prefix + "weight"
        if k in state_dict and state_dict[k].dim() == 4:
            state_dict[k] = state_dict[k].permute(0, 2, 3, 1).contiguous()

    def extra_repr(self):
        return "%d, %d, kernel_size=%s, stride=%d, padding=%d, dilation=%d, layout=KRSC" % (
            self.in_channels, self.out_channels, self.kernel_size, self.stride, self.padding, self.dilation)


def conv3x3(in_planes, out_planes, stride=1, dilation=1):
    "3x3 convolution with full padding (padding = dilation), src/resnet.py:20-37"
    return KRSCConv2d(in_planes, out_planes, 3, stride=stride, padding=dilation, dilation=dilation)


class BasicBlock(nn.Module):
    expansion = 1
    kind = "basic"

    def __init__(self, inplanes, planes, stride=1, downsample=None, dilation=1):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride, dilation=dilation)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes, dilation=dilation)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x_nhwc):
        """Operates on NHWC activations (the framework's internal layout)."""
        return net.block_forward(self, x_nhwc, final=True)


class Bottleneck(nn.Module):
    expansion = 4
    kind = "bottleneck"

    def __init__(self, inplanes, planes, stride=1, downsample=None, dilation=1):
        super().__init__()
        self.conv1 = KRSCConv2d(inplanes, planes, 1)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = conv3x3(planes, planes, stride=stride, dilation=dilation)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = KRSCConv2d(planes, planes * 4, 1)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x_nhwc):
        return net.block_forward(self, x_nhwc, final=True)


class ResNet(nn.Module):
    def __init__(self, block, layers, num_classes=1000, fully_conv=False, remove_avg_pool_layer=False,
                 output_stride=32):
        super().__init__()
        if not fully_conv or not remove_avg_pool_layer:
            raise NotImplementedError("only the fully-convolutional, avg-pool-free form the keypoint path uses "
                                      "(resnet_dilated.py:10-13) is implemented")
        self.output_stride = output_stride
        self.current_stride = 4
        self.current_dilation = 1
        self.remove_avg_pool_layer = remove_avg_pool_layer
        self.inplanes = 64
        self.fully_conv = fully_conv
        # the stem reads the reference's NCHW image directly with an OIHW weight
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AvgPool2d(7, padding=3, stride=1)
        # reference: nn.Linear here, replaced by a 1x1 Conv2d in Resnet34_8s (resnet_dilated.py:16)
        self.fc = nn.Conv2d(512 * block.expansion, num_classes, 1)
        for m in self.modules():  # src/resnet.py:155-161
            if isinstance(m, (nn.Conv2d, KRSCConv2d)):
                n = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
                m.weight.data.normal_(0, math.sqrt(2.0 / n))
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()

    def _make_layer(self, block, planes, blocks, stride=1, dilation=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            if self.current_stride == self.output_stride:
                self.current_dilation = self.current_dilation * stride
                stride = 1
            else:
                self.current_stride = self.current_stride * stride
            downsample = nn.Sequential(KRSCConv2d(self.inplanes, planes * block.expansion, 1, stride=stride),
                                       nn.BatchNorm2d(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample, dilation=self.current_dilation)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, dilation=self.current_dilation))
        return nn.Sequential(*layers)

    def forward(self, x):
        """[B,3,H,W] → raw fc logits at output stride 8, NCHW [B,1000,h,w]."""
        feat = net.backbone_forward(self, x)
        from hkp import ops
        W2 = self.fc.weight.reshape(self.fc.weight.shape[0], -1)
        outs = [ops.head_fc(feat, W2[c0:c0 + 16].contiguous(), self.fc.bias[c0:c0 + 16].contiguous())
                for c0 in range(0, W2.shape[0], 16)]
        return torch.cat(outs, 1)


def _load_local_pretrained(model, name):
    """pretrained=True: the reference downloads from download.pytorch.org
    (src/resnet.py:226-227 …); offline we only look in $TORCH_HOME/hub/checkpoints."""
    home = os.environ.get("TORCH_HOME", os.path.expanduser("~/.cache/torch"))
    path = os.path.join(home, "hub", "checkpoints", model_files[name])
    if not os.path.exists(path):
        warnings.warn("pretrained %s weights not found at %s (no network); keeping random init" % (name, path))
        return model
    sd = torch.load(path, map_location="cpu", weights_only=True)
    sd = {k: v for k, v in sd.items() if not k.startswith("fc.")}  # classifier is replaced anyway
    model.load_state_dict(sd, strict=False)
    return model


def _make(name, block, layers, pretrained, kwargs):
    model = ResNet(block, layers, **kwargs)
    return _load_local_pretrained(model, name) if pretrained else model


def resnet18(pretrained=False, **kwargs):
    return _make("resnet18", BasicBlock, [2, 2, 2, 2], pretrained, kwargs)


def resnet34(pretrained=False, **kwargs):
    return _make("resnet34", BasicBlock, [3, 4, 6, 3], pretrained, kwargs)


def resnet50(pretrained=False, **kwargs):
    return _make("resnet50", Bottleneck, [3, 4, 6, 3], pretrained, kwargs)


def resnet101(pretrained=False, **kwargs):
    return _make("resnet101", Bottleneck, [3, 4, 23, 3], pretrained, kwargs)


def resnet152(pretrained=False, **kwargs):
    return _make("resnet152", Bottleneck, [3, 8, 36, 3], pretrained, kwargs)
