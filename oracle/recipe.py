"""ORACLE — test infrastructure only (see oracle/__init__.py).

Deterministic weight / input recipe shared by the golden-fixture generator,
the parity tests and bench.py's cpu_baseline leg.  Pretrained ImageNet weights
(``resnet.py:237-238`` → ``model_zoo.load_url``) cannot be fetched offline
(SURVEY D7), so every parity case runs on weights drawn here from numpy
``PCG64(seed)`` and loaded into both sides through the reference's own
state_dict key format.

Distributions follow the reference's init where it has one:
  * conv weights ~ N(0, sqrt(2 / (kh*kw*Cout)))          resnet.py:155-158
  * fc (1x1 scoring conv) weight ~ N(0, 0.01)             resnet_dilated.py:20-22
and are perturbed where the reference's init is degenerate for testing
(BN gamma=1/beta=0, fc bias=0 would leave whole code paths unexercised):
  * BN gamma ~ U(0.5, 1.5), beta ~ N(0, 0.1), running_mean ~ N(0, 0.1),
    running_var ~ U(0.5, 1.5), num_batches_tracked = 0
  * fc bias ~ N(0, 0.01)
"""
import math
from collections import OrderedDict

import numpy as np
import torch

from .cpu_ref import state_dict_spec


def seeded_state_dict(backbone="resnet34", seed=0):
    """Return an OrderedDict in the reference key format (``resnet.<bb>_8s.*``)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    sd = OrderedDict()
    for key, shape, kind in state_dict_spec(backbone):
        if kind == "conv":
            cout, _, kh, kw = shape
            std = math.sqrt(2.0 / (kh * kw * cout))
            v = rng.standard_normal(shape, dtype=np.float64) * std
        elif kind == "fc_weight":
            v = rng.standard_normal(shape, dtype=np.float64) * 0.01
        elif kind == "fc_bias":
            v = rng.standard_normal(shape, dtype=np.float64) * 0.01
        elif kind == "bn_weight":
            v = rng.uniform(0.5, 1.5, shape)
        elif kind in ("bn_bias", "bn_mean"):
            v = rng.standard_normal(shape, dtype=np.float64) * 0.1
        elif kind == "bn_var":
            v = rng.uniform(0.5, 1.5, shape)
        elif kind == "bn_count":
            sd[key] = torch.tensor(0, dtype=torch.int64)
            continue
        else:  # pragma: no cover
            raise ValueError(kind)
        sd[key] = torch.from_numpy(np.ascontiguousarray(v, dtype=np.float32))
    return sd


def seeded_images_u8(batch, height, width, seed=1234):
    """uint8 BGR HWC images [B,H,W,3] (SURVEY §8(d) synthetic inputs)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.integers(0, 256, size=(batch, height, width, 3), dtype=np.uint8)


def to_tensor_nchw(imgs_u8):
    """torchvision ``ToTensor`` semantics (dataset.py:16): HWC uint8 → CHW f32 / 255."""
    t = torch.from_numpy(np.ascontiguousarray(imgs_u8)).permute(0, 3, 1, 2).contiguous()
    return t.to(torch.float32).div_(255.0)


def seeded_keypoints(batch, num_keypoints, height, width, seed=99, edge_cases=True):
    """(u, v) float32 [B,K,2] with u~U[0,W-1], v~U[0,H-1]; optionally a few
    integer, edge-clipped and out-of-range labels (clipped as dataset.py:65-66)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    uv = np.empty((batch, num_keypoints, 2), dtype=np.float64)
    uv[..., 0] = rng.uniform(0, width - 1, (batch, num_keypoints))
    uv[..., 1] = rng.uniform(0, height - 1, (batch, num_keypoints))
    if edge_cases and batch * num_keypoints >= 4:
        flat = uv.reshape(-1, 2)
        flat[0] = (np.round(flat[0, 0]), np.round(flat[0, 1]))   # integer keypoint → peak exactly 1
        flat[1] = (-7.5, height + 3.0)                             # out of range → clipped to the border
        flat[2] = (width - 1, 0.0)                                 # exact corner
        flat[3] = (0.25, height - 1.75)                            # fractional near the edge
    uv[..., 0] = np.clip(uv[..., 0], 0, width - 1)
    uv[..., 1] = np.clip(uv[..., 1], 0, height - 1)
    return uv.astype(np.float32)
