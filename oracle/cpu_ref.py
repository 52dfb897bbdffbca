"""ORACLE — test infrastructure only (see oracle/__init__.py).

CPU restatement of the reference hot path, in plain ``torch.nn.functional`` on
CPU, NCHW, fp32 network / fp64 loss — exactly the reference's semantics:

  * backbone plan      resnet.py:115-217 (_make_layer output-stride logic :163-196)
  * conv3x3 padding    resnet.py:20-37   (padding = dilation)
  * BasicBlock         resnet.py:40-69
  * Bottleneck         resnet.py:72-112
  * 1000-ch fc + bilinear(align_corners=True) upsample   resnet_dilated.py:16,24-28
  * slice [:K] + sigmoid                                   model.py:19-22
  * Gaussian target    dataset.py:36-44
  * BCE on .double()   train.py:21,25
  * argmax decode      prediction.py:46
  * Adam(lr=1e-4, weight_decay=1e-4) step                 train.py:79,33-36

BatchNorm runs in TRAIN mode by default, because the reference never calls
``.eval()``.  Pinned against goldens produced by importing the
reference itself (tests/golden/make_golden.py → tests/golden/*.npz, checked in
tests/test_oracle_golden.py).
"""
from collections import OrderedDict

import numpy as np
import torch
import torch.nn.functional as F

BACKBONES = {
    "resnet18": ("basic", [2, 2, 2, 2]),    # resnet.py:225
    "resnet34": ("basic", [3, 4, 6, 3]),    # resnet.py:236
    "resnet50": ("bottleneck", [3, 4, 6, 3]),  # resnet.py:247
}
EXPANSION = {"basic": 1, "bottleneck": 4}
NUM_CLASSES = 1000  # resnet_dilated.py:6,16
BN_EPS = 1e-5
BN_MOMENTUM = 0.1


def layer_plan(backbone, output_stride=8):
    """Restates ResNet._make_layer (resnet.py:163-196) for fully_conv OS=8.

    Returns a list of block dicts with keys: name, kind, inplanes, planes,
    stride, dilation, downsample (None or (cin, cout, stride)).
    """
    kind, layers = BACKBONES[backbone]
    exp = EXPANSION[kind]
    current_stride, current_dilation, inplanes = 4, 1, 64  # resnet.py:129-134
    blocks = []
    for li, (planes, stride) in enumerate([(64, 1), (128, 2), (256, 2), (512, 2)]):
        downsample = None
        if stride != 1 or inplanes != planes * exp:       # :166
            if current_stride == output_stride:           # :170
                current_dilation *= stride                # :174
                stride = 1
            else:
                current_stride *= stride                  # :180
            downsample = (inplanes, planes * exp, stride)  # :184-188 (1x1 never dilated)
        for bi in range(layers[li]):
            blocks.append(dict(
                name="layer%d.%d" % (li + 1, bi), kind=kind,
                inplanes=inplanes if bi == 0 else planes * exp, planes=planes,
                stride=stride if bi == 0 else 1, dilation=current_dilation,
                downsample=downsample if bi == 0 else None))
        inplanes = planes * exp
    return blocks


def key_prefix(backbone):
    # model.py:17 (self.resnet) → resnet_dilated.py:17 (self.resnet34_8s)
    return "resnet.%s_8s." % backbone


def state_dict_spec(backbone):
    """[(key, shape, kind)] in the reference's state_dict order."""
    p = key_prefix(backbone)
    spec = []

    def bn(name, c):
        spec.extend([(p + name + ".weight", (c,), "bn_weight"), (p + name + ".bias", (c,), "bn_bias"),
                     (p + name + ".running_mean", (c,), "bn_mean"), (p + name + ".running_var", (c,), "bn_var"),
                     (p + name + ".num_batches_tracked", (), "bn_count")])

    spec.append((p + "conv1.weight", (64, 3, 7, 7), "conv"))
    bn("bn1", 64)
    for b in layer_plan(backbone):
        n, cin, pl = b["name"], b["inplanes"], b["planes"]
        if b["kind"] == "basic":
            spec.append((p + n + ".conv1.weight", (pl, cin, 3, 3), "conv")); bn(n + ".bn1", pl)
            spec.append((p + n + ".conv2.weight", (pl, pl, 3, 3), "conv")); bn(n + ".bn2", pl)
        else:
            spec.append((p + n + ".conv1.weight", (pl, cin, 1, 1), "conv")); bn(n + ".bn1", pl)
            spec.append((p + n + ".conv2.weight", (pl, pl, 3, 3), "conv")); bn(n + ".bn2", pl)
            spec.append((p + n + ".conv3.weight", (pl * 4, pl, 1, 1), "conv")); bn(n + ".bn3", pl * 4)
        if b["downsample"] is not None:
            ci, co, _ = b["downsample"]
            spec.append((p + n + ".downsample.0.weight", (co, ci, 1, 1), "conv")); bn(n + ".downsample.1", co)
    c_last = 512 * EXPANSION[BACKBONES[backbone][0]]
    spec.append((p + "fc.weight", (NUM_CLASSES, c_last, 1, 1), "fc_weight"))
    spec.append((p + "fc.bias", (NUM_CLASSES,), "fc_bias"))
    return spec


def _bn(x, sd, name, bn_mode):
    training = bn_mode == "train"
    y = F.batch_norm(x, sd[name + ".running_mean"], sd[name + ".running_var"], sd[name + ".weight"],
                     sd[name + ".bias"], training=training, momentum=BN_MOMENTUM, eps=BN_EPS)
    if training:
        with torch.no_grad():
            sd[name + ".num_batches_tracked"].add_(1)
    return y


def _conv(x, w, stride=1, padding=0, dilation=1):
    return F.conv2d(x, w, None, stride, padding, dilation)


def backbone_forward(sd, x, backbone, bn_mode="train"):
    """ResNet.forward up to (excluding) fc: resnet.py:198-213."""
    p = key_prefix(backbone)
    x = _conv(x, sd[p + "conv1.weight"], 2, 3)
    x = F.relu(_bn(x, sd, p + "bn1", bn_mode))
    x = F.max_pool2d(x, 3, 2, 1)
    for b in layer_plan(backbone):
        n, d = p + b["name"], b["dilation"]
        res = x
        if b["kind"] == "basic":   # resnet.py:53-69
            out = F.relu(_bn(_conv(x, sd[n + ".conv1.weight"], b["stride"], d, d), sd, n + ".bn1", bn_mode))
            out = _bn(_conv(out, sd[n + ".conv2.weight"], 1, d, d), sd, n + ".bn2", bn_mode)
        else:                      # resnet.py:92-112
            out = F.relu(_bn(_conv(x, sd[n + ".conv1.weight"]), sd, n + ".bn1", bn_mode))
            out = F.relu(_bn(_conv(out, sd[n + ".conv2.weight"], b["stride"], d, d), sd, n + ".bn2", bn_mode))
            out = _bn(_conv(out, sd[n + ".conv3.weight"]), sd, n + ".bn3", bn_mode)
        if b["downsample"] is not None:
            res = _bn(_conv(x, sd[n + ".downsample.0.weight"], b["downsample"][2]), sd, n + ".downsample.1", bn_mode)
        x = F.relu(out + res)
    return x


def forward(sd, x, backbone="resnet34", num_keypoints=4, bn_mode="train", head="faithful",
            return_lowres=False):
    """KeypointsGauss.forward (model.py:19-22) → [B,K,H,W] sigmoid heatmaps.

    head="faithful": 1000-channel fc, 1000-channel upsample, then slice (the
    reference as written, resnet_dilated.py:16,27 + model.py:21).
    head="k_only": slice the fc to K rows first (bit-identical per channel).
    """
    p = key_prefix(backbone)
    feat = backbone_forward(sd, x, backbone, bn_mode)
    w, bias = sd[p + "fc.weight"], sd[p + "fc.bias"]
    if head == "k_only":
        w, bias = w[:num_keypoints], bias[:num_keypoints]
    lowres = F.conv2d(feat, w, bias)
    up = F.interpolate(lowres, size=x.shape[2:], mode="bilinear", align_corners=True)
    heat = torch.sigmoid(up[:, :num_keypoints])
    if return_lowres:
        return heat, lowres[:, :num_keypoints]
    return heat


def gauss_2d_batch(width, height, sigma, U, V):
    """dataset.py:36-44 (normalize_dist=False): [K] U,V → [K,H,W] float64.

    Unlike the reference it does not mutate U/V in place (dataset.py:37-38)."""
    U = torch.as_tensor(U).reshape(-1, 1, 1).float()
    V = torch.as_tensor(V).reshape(-1, 1, 1).float()
    X, Y = torch.meshgrid([torch.arange(0., width), torch.arange(0., height)], indexing="ij")
    X, Y = X.t(), Y.t()
    G = torch.exp(-((X - U) ** 2 + (Y - V) ** 2) / (2.0 * sigma ** 2))
    return G.double()


def gauss_target(uv, height, width, sigma):
    """Batched dataset target: uv [B,K,2] (u=x, v=y) → [B,K,H,W] f64."""
    uv = torch.as_tensor(uv)
    return torch.stack([gauss_2d_batch(width, height, sigma, uv[b, :, 0], uv[b, :, 1])
                        for b in range(uv.shape[0])])


def bce_loss(pred_f32, gt_f64):
    """train.py:21,25 — nn.BCELoss()(pred.double(), gt), mean reduction."""
    return F.binary_cross_entropy(pred_f32.double(), gt_f64)


def mse_loss(pred_f32, gt_f64):
    """train.py:13 MSE (defined, unused by the reference) on the same .double() pred."""
    return F.mse_loss(pred_f32.double(), gt_f64)


def argmax_yx(heat):
    """prediction.py:46 — np.unravel_index(h.argmax(), h.shape) per (b,k) → int32 [B,K,2] (y,x)."""
    h = np.asarray(heat.detach().cpu().numpy() if torch.is_tensor(heat) else heat)
    B, K = h.shape[:2]
    out = np.zeros((B, K, 2), dtype=np.int32)
    for b in range(B):
        for k in range(K):
            out[b, k] = np.unravel_index(h[b, k].argmax(), h[b, k].shape)
    return out


def top2_margin(heat):
    """max - second max per (b,k): how robust the argmax is to rounding."""
    h = heat.detach().reshape(heat.shape[0], heat.shape[1], -1)
    t = torch.topk(h, 2, dim=-1).values
    return (t[..., 0] - t[..., 1]).numpy()


def param_keys(backbone):
    return [k for k, _, kind in state_dict_spec(backbone) if not kind.startswith("bn_") or kind in ("bn_weight", "bn_bias")]


class OracleTrainer:
    """Stateful fit loop (train.py:32-36): persistent parameters and Adam state."""

    def __init__(self, sd, backbone, num_keypoints, lr=1e-4, weight_decay=1e-4, head="faithful"):
        self.sd, self.bb, self.k, self.head = sd, backbone, num_keypoints, head
        self.keys = param_keys(backbone)
        self.params = OrderedDict((k, sd[k].detach().clone().requires_grad_(True)) for k in self.keys)
        self.opt = torch.optim.Adam(list(self.params.values()), lr=lr, weight_decay=weight_decay)

    def step(self, x, uv, sigma=8, loss="bce"):
        work = OrderedDict(self.sd)
        work.update(self.params)
        self.opt.zero_grad()
        pred = forward(work, x, self.bb, self.k, "train", self.head)
        gt = gauss_target(uv, x.shape[2], x.shape[3], sigma).to(pred.dtype if pred.dtype == torch.float64
                                                                 else torch.float64)
        L = bce_loss(pred, gt) if loss == "bce" else mse_loss(pred, gt)
        L.backward()
        grads = OrderedDict((k, self.params[k].grad.detach().clone()) for k in self.keys)
        self.opt.step()
        return L.detach(), grads


def train_step(sd, x, uv, backbone="resnet18", num_keypoints=2, sigma=8, loss="bce", lr=1e-4,
               weight_decay=1e-4, adam_state=None, head="faithful"):
    """One reference training iteration (train.py:33-36): zero_grad → forward →
    BCE → backward → Adam(lr=1e-4, weight_decay=1e-4).step().

    Mutates ``sd`` (params and BN running stats).  Returns (loss, grads dict, optimizer)."""
    keys = param_keys(backbone)
    params = OrderedDict()
    for k in keys:
        t = sd[k].detach().clone().requires_grad_(True)
        params[k] = t
    work = OrderedDict(sd)
    work.update(params)
    opt = adam_state or torch.optim.Adam(list(params.values()), lr=lr, weight_decay=weight_decay)
    opt.zero_grad()
    pred = forward(work, x, backbone, num_keypoints, "train", head)
    gt = gauss_target(uv, x.shape[2], x.shape[3], sigma)
    L = bce_loss(pred, gt) if loss == "bce" else mse_loss(pred, gt)
    L.backward()
    grads = OrderedDict((k, params[k].grad.detach().clone()) for k in keys)
    opt.step()
    with torch.no_grad():
        for k in keys:
            sd[k] = params[k].detach().clone()
    return L.detach(), grads, opt
