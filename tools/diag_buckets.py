#!/usr/bin/env python3
"""Which gradients differ between the plain and the DP-bucket training paths
(world size 1, HKP_FORCE_BUCKETS) with the side-stream wgrad on / off."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "hulk-keypoints_amd")]
import torch  # noqa: E402

from oracle import recipe  # noqa: E402


def main():
    from hkp import net, train
    from src.model import KeypointsGauss
    dev = torch.device("cuda", 0)
    B, K, H, W = 2, 2, 64, 80
    x = recipe.to_tensor_nchw(recipe.seeded_images_u8(B, H, W, 41)).to(dev)
    uv = torch.from_numpy(recipe.seeded_keypoints(B, K, H, W, 42)).to(dev)
    m = KeypointsGauss(K, backbone="resnet34", pretrained=False)
    m.load_state_dict(recipe.seeded_state_dict("resnet34", 43))
    m = m.to(dev)
    names = [n for n, _ in m.named_parameters()]
    res = {}
    for buckets in (False, True):
        for overlap in (True, False):
            os.environ["HKP_FORCE_BUCKETS"] = "1" if buckets else "0"
            net.OVERLAP_WGRAD = overlap
            t = train.Trainer(m)
            for rep in range(2):
                t.forward_backward(x, uv=uv)
                torch.cuda.synchronize()
                res[(buckets, overlap, rep)] = [p.grad.clone() for p in m.parameters()]
    ref = res[(False, True, 0)]
    for key, gs in res.items():
        bad = [(n, (a - b).abs().max().item()) for n, a, b in zip(names, ref, gs) if not torch.equal(a, b)]
        print(key, "differs in %d params" % len(bad), bad[:6])


if __name__ == "__main__":
    main()
