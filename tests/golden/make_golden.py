"""Generate tests/golden/*.npz by running the REFERENCE itself (this container only).

Usage:  python tests/golden/make_golden.py        (needs /root/reference)

The reference is imported read-only from /root/reference with the SURVEY §8(c)
recipe: stub the imported-but-unused / absent modules (torchvision, cv2,
imgaug), make ``Tensor.cuda`` a no-op, block ``model_zoo.load_url`` and force
``pretrained=False`` (ImageNet weights are not fetchable offline).
Weights come from oracle/recipe.py and are loaded through the reference's own
``load_state_dict``.  Only the resulting arrays (inputs + outputs) are
committed; no reference source is copied.
"""
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)

from oracle import recipe  # noqa: E402


def import_reference():
    for name in ["torchvision", "torchvision.models", "torchvision.transforms", "torchvision.utils",
                 "cv2", "imgaug", "imgaug.augmenters"]:
        sys.modules.setdefault(name, types.ModuleType(name))
    tv = sys.modules["torchvision"]
    tv.models, tv.transforms, tv.utils = (sys.modules["torchvision.models"], sys.modules["torchvision.transforms"],
                                          sys.modules["torchvision.utils"])

    class Compose:
        def __init__(self, t):
            self.t = t

        def __call__(self, x):
            for f in self.t:
                x = f(x)
            return x
    sys.modules["torchvision.transforms"].Compose = Compose
    sys.modules["torchvision.transforms"].ToTensor = lambda: recipe.to_tensor_nchw
    sys.modules["imgaug"].augmenters = sys.modules["imgaug.augmenters"]
    torch.Tensor.cuda = lambda self, *a, **k: self
    sys.path.insert(0, REF + "/src")
    sys.path.insert(0, REF)
    import resnet
    import resnet_dilated
    import model
    import dataset

    def _no_net(*a, **k):
        raise RuntimeError("pretrained weights are not fetchable offline")
    resnet.model_zoo.load_url = _no_net
    resnet_dilated.resnet34 = lambda **kw: resnet.resnet34(**{**kw, "pretrained": False})
    return resnet, resnet_dilated, model, dataset


resnet, resnet_dilated, model, dataset = import_reference()


class _Inner(nn.Module):
    """Same composition as resnet_dilated.Resnet34_8s (:5-28), for any constructor."""

    def __init__(self, backbone):
        super().__init__()
        net = getattr(resnet, backbone)(fully_conv=True, pretrained=False, output_stride=8,
                                        remove_avg_pool_layer=True)
        net.fc = nn.Conv2d(net.inplanes, 1000, 1)
        setattr(self, backbone + "_8s", net)
        self.backbone = backbone

    def forward(self, x):
        size = x.size()[2:]
        x = getattr(self, self.backbone + "_8s")(x)
        return nn.functional.upsample_bilinear(input=x, size=size)


class _Keypoints(nn.Module):
    """model.KeypointsGauss with a selectable backbone (forward identical to model.py:19-22)."""

    def __init__(self, backbone, k):
        super().__init__()
        self.num_keypoints = k
        self.resnet = _Inner(backbone)
        self.sigmoid = nn.Sigmoid()

    def forward(self, x):
        return self.sigmoid(self.resnet(x)[:, :self.num_keypoints, :, :])


def build(backbone, k, seed):
    if backbone == "resnet34":
        m = model.KeypointsGauss(k)          # the reference class itself
    else:
        m = _Keypoints(backbone, k)
    m.load_state_dict(recipe.seeded_state_dict(backbone, seed))
    return m


def lowres_of(m, backbone, x):
    net = getattr(m.resnet, backbone + "_8s")
    return net(x)


def running_checksum(sd):
    rm = sum(float(v.double().sum()) for k, v in sd.items() if k.endswith("running_mean"))
    rv = sum(float(v.double().sum()) for k, v in sd.items() if k.endswith("running_var"))
    nb = sum(int(v) for k, v in sd.items() if k.endswith("num_batches_tracked"))
    return np.array([rm, rv, nb], dtype=np.float64)


def fwd_case(name, backbone, k, B, H, W, wseed, iseed, full_heat=True, eval_too=False):
    torch.manual_seed(0)
    imgs = recipe.seeded_images_u8(B, H, W, iseed)
    x = recipe.to_tensor_nchw(imgs)
    m = build(backbone, k, wseed)
    with torch.no_grad():
        # two passes on identically-initialised models: heat (train-mode BN, like analysis.py)
        # and the low-res logits (the fc output before upsample)
        heat = m(x)
        m2 = build(backbone, k, wseed)
        low = lowres_of(m2, backbone, x)[:, :k]
    sd_after = m.state_dict()
    h = heat.numpy()
    out = dict(backbone=np.array(backbone), k=np.int32(k), wseed=np.int32(wseed), iseed=np.int32(iseed),
               images_u8=imgs, lowres=low.numpy().astype(np.float32),
               argmax_yx=np.array([[np.unravel_index(h[b, j].argmax(), h[b, j].shape) for j in range(k)]
                                   for b in range(B)], dtype=np.int32),
               margin=(lambda t: (t[..., 0] - t[..., 1]).numpy())(torch.topk(heat.reshape(B, k, -1), 2, -1).values),
               heat_row_sum=h.astype(np.float64).sum(axis=3),
               running_checksum=running_checksum(sd_after),
               bn1_running_mean=sd_after["resnet.%s_8s.bn1.running_mean" % backbone].numpy(),
               bn1_running_var=sd_after["resnet.%s_8s.bn1.running_var" % backbone].numpy())
    if full_heat:
        out["heat"] = h.astype(np.float32)
    if eval_too:
        me = build(backbone, k, wseed).eval()
        with torch.no_grad():
            out["heat_eval"] = me(x).numpy().astype(np.float32)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print(name, "margin min %.3g" % out["margin"].min(), "argmax", out["argmax_yx"].reshape(-1, 2)[:4].tolist())


def image_digest(imgs):
    """sha256 of the uint8 image bytes: large fixtures store this instead of the
    images, which the tests regenerate from recipe.seeded_images_u8 (PCG64)."""
    import hashlib
    return np.array(hashlib.sha256(np.ascontiguousarray(imgs).tobytes()).hexdigest())


def heat_from_lowres(low_k, size):
    """The reference's head applied to the first K fc channels only:
    upsample_bilinear (resnet_dilated.py:27) then sigmoid (model.py:21).  The
    reference upsamples all 1000 channels and slices after; ATen's CPU bilinear
    kernel computes every channel plane independently with the same arithmetic,
    so slicing first is bit-identical (checked in __main__ on a small case) and
    avoids a [32,1000,480,640] fp32 (39 GB) intermediate at the bench batch."""
    return torch.sigmoid(nn.functional.upsample_bilinear(input=low_k, size=size))


def fwd_batch_case(name, backbone, k, B, H, W, wseed, iseed, shard_of=None):
    """Forward at a bench-size batch (BASELINE config C2: R34 K4 640x480 B=32):
    train-mode BN over the whole batch, as analysis.py / Prediction.predict run it.
    Images are not stored (29 MB); the fixture keeps their digest.  shard_of =
    (G, i): the batch is slice i of the seeded G-image batch — one rank's shard of
    a data-parallel job, whose BN statistics are the shard's own."""
    if shard_of is None:
        imgs = recipe.seeded_images_u8(B, H, W, iseed)
    else:
        G, i = shard_of
        imgs = np.ascontiguousarray(recipe.seeded_images_u8(G, H, W, iseed)[i * B:(i + 1) * B])
    x = recipe.to_tensor_nchw(imgs)
    m = build(backbone, k, wseed)
    with torch.no_grad():
        low = lowres_of(m, backbone, x)[:, :k].contiguous()
        heat = heat_from_lowres(low, x.size()[2:])
    sd_after = m.state_dict()
    h = heat.numpy()
    out = dict(backbone=np.array(backbone), k=np.int32(k), wseed=np.int32(wseed), iseed=np.int32(iseed),
               batch=np.int32(B), height=np.int32(H), width=np.int32(W), images_sha256=image_digest(imgs),
               shard_of=np.array(shard_of if shard_of else (B, 0), dtype=np.int32),
               lowres=low.numpy().astype(np.float32),
               argmax_yx=np.array([[np.unravel_index(h[b, j].argmax(), h[b, j].shape) for j in range(k)]
                                   for b in range(B)], dtype=np.int32),
               margin=(lambda t: (t[..., 0] - t[..., 1]).numpy())(torch.topk(heat.reshape(B, k, -1), 2, -1).values),
               heat_row_sum=h.astype(np.float64).sum(axis=3),
               heat0=h[0].astype(np.float32),
               running_checksum=running_checksum(sd_after),
               bn1_running_mean=sd_after["resnet.%s_8s.bn1.running_mean" % backbone].numpy(),
               bn1_running_var=sd_after["resnet.%s_8s.bn1.running_var" % backbone].numpy())
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print(name, "margin min %.3g" % out["margin"].min(), "argmax", out["argmax_yx"].reshape(-1, 2)[:4].tolist())


def fwd_subsampled_case(name, backbone, k, B, H, W, wseed, iseed, step=4):
    """Forward at bench resolution for a wide head (BASELINE config C4's network,
    R50-8s K=8 at 640x480): the full low-res logits, argmax, margins and heatmap
    row sums of every plane, and the heatmaps on every `step`-th row and column
    (a full [B,8,480,640] fp32 heatmap would be ~20 MB)."""
    imgs = recipe.seeded_images_u8(B, H, W, iseed)
    x = recipe.to_tensor_nchw(imgs)
    m = build(backbone, k, wseed)
    with torch.no_grad():
        low = lowres_of(m, backbone, x)[:, :k].contiguous()
        heat = heat_from_lowres(low, x.size()[2:])
    sd_after = m.state_dict()
    h = heat.numpy()
    out = dict(backbone=np.array(backbone), k=np.int32(k), wseed=np.int32(wseed), iseed=np.int32(iseed),
               batch=np.int32(B), height=np.int32(H), width=np.int32(W), images_sha256=image_digest(imgs),
               step=np.int32(step), lowres=low.numpy().astype(np.float32),
               argmax_yx=np.array([[np.unravel_index(h[b, j].argmax(), h[b, j].shape) for j in range(k)]
                                   for b in range(B)], dtype=np.int32),
               margin=(lambda t: (t[..., 0] - t[..., 1]).numpy())(torch.topk(heat.reshape(B, k, -1), 2, -1).values),
               heat_row_sum=h.astype(np.float64).sum(axis=3),
               heat_sub=np.ascontiguousarray(h[:, :, ::step, ::step]).astype(np.float32),
               running_checksum=running_checksum(sd_after))
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print(name, "margin min %.3g" % out["margin"].min(), "argmax", out["argmax_yx"].reshape(-1, 2)[:4].tolist())


def check_slice_first_head():
    """heat_from_lowres(K channels) == the reference's full 1000-channel head, bitwise."""
    imgs = recipe.seeded_images_u8(2, 120, 160, 3)
    x = recipe.to_tensor_nchw(imgs)
    m1, m2 = build("resnet34", 4, 9), build("resnet34", 4, 9)
    with torch.no_grad():
        full = m1(x)
        low = lowres_of(m2, "resnet34", x)[:, :4].contiguous()
        sliced = heat_from_lowres(low, x.size()[2:])
    assert torch.equal(full, sliced), "slice-first head differs from the reference's"
    print("slice-first head: bit-identical")


def gauss_cases():
    cases = [(64, 48, 8, [10.0, 0.0, 63.0, 31.37], [5.0, 47.0, 0.0, 20.5]),
             (80, 60, 10, [40.25, 79.0], [30.75, 59.0]),
             (33, 17, 3, [0.5, 16.0, 32.0], [8.5, 0.0, 16.0])]
    out = {}
    for i, (w, h, s, U, V) in enumerate(cases):
        Ut, Vt = torch.tensor(U, dtype=torch.float64), torch.tensor(V, dtype=torch.float64)
        G = dataset.gauss_2d_batch(w, h, s, Ut, Vt)
        out["case%d_whs" % i] = np.array([w, h, s], dtype=np.int32)
        out["case%d_U" % i] = np.array(U, dtype=np.float64)
        out["case%d_V" % i] = np.array(V, dtype=np.float64)
        out["case%d_G" % i] = G.numpy()
    np.savez_compressed(os.path.join(HERE, "gauss.npz"), **out)
    print("gauss", len(cases))


def bce_cases():
    rng = np.random.Generator(np.random.PCG64(7))
    p = rng.uniform(0, 1, 64).astype(np.float32)
    p[:8] = [0.0, 1.0, 1e-30, 1.0 - 2 ** -24, 0.5, 1e-7, 0.9999, 2 ** -24]
    y = rng.uniform(0, 1, 64)
    y[:8] = [0.5, 0.5, 1.0, 0.0, 1.0, 0.0, 1.0, 1.0]
    pt = torch.tensor(p, requires_grad=True)
    L = nn.BCELoss()(pt.double(), torch.tensor(y))      # train.py:21,25
    L.backward()
    pm = torch.tensor(p, requires_grad=True)
    Lm = nn.MSELoss()(pm.double(), torch.tensor(y))      # train.py:13
    Lm.backward()
    np.savez_compressed(os.path.join(HERE, "bce.npz"), p=p, y=y, loss=np.float64(L.item()),
                        grad=pt.grad.numpy(), mse=np.float64(Lm.item()), mse_grad=pm.grad.numpy())
    print("bce", L.item())


def train_case(name, backbone, k, B, H, W, wseed, iseed, kseed, steps=2, store_images=True, fp64_step0=False):
    """`steps` reference train steps (train.py:33-36) on one batch.  store_images=False
    keeps the images' digest instead (tests regenerate them); fp64_step0 adds the
    same steps run in float64 (same weights, images, target) so a test can take its
    tolerance from the problem's measured conditioning (|fp32 - fp64| of the reference
    itself) rather than from a guess."""
    imgs = recipe.seeded_images_u8(B, H, W, iseed)
    x = recipe.to_tensor_nchw(imgs)
    uv = recipe.seeded_keypoints(B, k, H, W, kseed)
    m = build(backbone, k, wseed)
    opt = torch.optim.Adam(m.parameters(), lr=1.0e-4, weight_decay=1.0e-4)   # train.py:79
    # dataset.__getitem__ target (dataset.py:70-76), one sample at a time, then default_collate
    gt = torch.stack([dataset.gauss_2d_batch(W, H, 8, torch.tensor(uv[b, :, 0]), torch.tensor(uv[b, :, 1]))
                      for b in range(B)])
    names = [n for n, _ in m.named_parameters()]
    out = dict(backbone=np.array(backbone), k=np.int32(k), wseed=np.int32(wseed), iseed=np.int32(iseed),
               uv=uv, steps=np.int32(steps))
    if store_images:
        out["images_u8"] = imgs
    else:
        out.update(images_sha256=image_digest(imgs), batch=np.int32(B), height=np.int32(H), width=np.int32(W))
    if fp64_step0:
        md = build(backbone, k, wseed).double()
        optd = torch.optim.Adam(md.parameters(), lr=1.0e-4, weight_decay=1.0e-4)
        for s in range(steps):
            optd.zero_grad()
            loss = nn.BCELoss()(md.forward(x.double()), gt)
            loss.backward()
            out["f64_loss%d" % s] = np.float64(loss.item())
            if s == 0:
                gd = {n: p.grad.detach().clone() for n, p in md.named_parameters()}
                out["f64_grad_abs0"] = np.array([float(gd[n].abs().sum()) for n in names])
                out["f64_fc_grad_rows0"] = gd["resnet.%s_8s.fc.weight" % backbone][:k].reshape(k, -1).numpy()
                out["f64_stem_grad0"] = gd["resnet.%s_8s.conv1.weight" % backbone].numpy()
            optd.step()
        sdd = md.state_dict()
        out["f64_param_abs"] = np.array([float(sdd[n].abs().sum()) for n in names])
    for s in range(steps):
        opt.zero_grad()                                       # train.py:33
        pred = m.forward(x).double()                          # train.py:21
        loss = nn.BCELoss()(pred, gt)                         # train.py:25
        loss.backward()                                       # train.py:35
        g = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
        opt.step()                                            # train.py:36
        out["loss%d" % s] = np.float64(loss.item())
        out["grad_sum%d" % s] = np.array([float(g[n].double().sum()) for n in names])
        out["grad_abs%d" % s] = np.array([float(g[n].double().abs().sum()) for n in names])
        fcw = "resnet.%s_8s.fc.weight" % backbone
        out["fc_grad_rows%d" % s] = g[fcw][:k].reshape(k, -1).numpy()
        out["fc_bias_grad%d" % s] = g["resnet.%s_8s.fc.bias" % backbone][:k].numpy()
        out["fc_grad_rest_abs%d" % s] = np.float64(g[fcw][k:].abs().sum())
        out["stem_grad%d" % s] = g["resnet.%s_8s.conv1.weight" % backbone].numpy()
    sd = m.state_dict()
    out["param_names"] = np.array(names)
    out["param_sum"] = np.array([float(sd[n].double().sum()) for n in names])
    out["param_abs"] = np.array([float(sd[n].double().abs().sum()) for n in names])
    out["running_checksum"] = running_checksum(sd)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print(name, [out["loss%d" % s] for s in range(steps)])


if __name__ == "__main__":
    torch.set_num_threads(8)
    only = sys.argv[1:]          # optional: names of the fixtures to (re)generate

    def want(n):
        return not only or n in only
    if want("gauss"):
        gauss_cases()
    if want("bce"):
        bce_cases()
    for args in [("fwd_r18_k2_96x128", "resnet18", 2, 2, 96, 128, 1, 11, True, False),
                 ("fwd_r34_k4_96x128", "resnet34", 4, 2, 96, 128, 2, 12, True, True),
                 ("fwd_r34_k4_75x100", "resnet34", 4, 2, 75, 100, 3, 13, True, False),
                 ("fwd_r50_k8_96x128", "resnet50", 8, 2, 96, 128, 4, 14, True, False),
                 ("fwd_r34_k4_480x640", "resnet34", 4, 1, 480, 640, 5, 15, False, False)]:
        if want(args[0]):
            fwd_case(*args[:6], wseed=args[6], iseed=args[7], full_heat=args[8], eval_too=args[9])
    if want("fwd_r34_k4_480x640_b32"):
        check_slice_first_head()
        # BASELINE config C2 at the bench's batch
        fwd_batch_case("fwd_r34_k4_480x640_b32", "resnet34", 4, 32, 480, 640, wseed=10, iseed=20)
    if want("fwd_r34_k4_480x640_b8_shard7"):
        # north_star's scaling workload (640x480 batch-64 inference over 8 GPUs): the
        # 8-image shard of rank 7 (images 56-63 of the 64-image batch), per-shard BN
        fwd_batch_case("fwd_r34_k4_480x640_b8_shard7", "resnet34", 4, 8, 480, 640, wseed=10, iseed=1234,
                       shard_of=(64, 7))
    if want("fwd_r50_k8_480x640_b2"):
        # BASELINE config C4's network (R50-8s, K=8) at the bench resolution
        fwd_subsampled_case("fwd_r50_k8_480x640_b2", "resnet50", 8, 2, 480, 640, wseed=30, iseed=31)
    for args in [("train_r18_k2_64x80", "resnet18", 2, 2, 64, 80, 6, 16, 26),
                 ("train_r34_k4_48x64", "resnet34", 4, 2, 48, 64, 7, 17, 27),
                 # R50 K8 (the C4 / C5 network) train steps
                 ("train_r50_k8_96x128", "resnet50", 8, 2, 96, 128, 8, 18, 28)]:
        if want(args[0]):
            train_case(*args[:6], wseed=args[6], iseed=args[7], kseed=args[8])
    if want("train_r18_k2_240x320_b4"):
        # BASELINE config C1 at its own size: R18-8s, K=2, 320x240, batch 4, two Adam steps
        train_case("train_r18_k2_240x320_b4", "resnet18", 2, 4, 240, 320, wseed=40, iseed=41, kseed=42,
                   store_images=False, fp64_step0=True)
