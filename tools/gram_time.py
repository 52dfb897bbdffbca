#!/usr/bin/env python3
"""HIP-event time of hkp_bn_from_gram (the bn3 statistics of C4's Bottlenecks from
conv3's input moments) at R50's shapes, median of `--iters` calls; run once per
library build (`--lib`) and compare (also prints a checksum of scale/shift)."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "hulk-keypoints_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--iters", type=int, default=30)
    args = ap.parse_args()
    if args.lib:
        from hkp import _lib
        _lib.use_library(os.path.abspath(args.lib))
    from hkp import ops
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    for c, k in ((64, 256), (128, 512), (256, 1024), (512, 2048)):
        a = torch.relu(torch.randn(8192, c, device=dev, generator=g)).half()
        mean, e2 = ops.gram_f16(a)
        wp = ops.weight_pack_f16(torch.randn(k, 1, 1, c, device=dev, generator=g) * 0.05)
        gam = torch.rand(k, device=dev, generator=g) + 0.5
        bet = torch.randn(k, device=dev, generator=g)
        for _ in range(3):
            ss, _ = ops.bn_from_gram(mean, e2, wp, 8192, gam, bet)
        ts = []
        for _ in range(args.iters):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ops.bn_from_gram(mean, e2, wp, 8192, gam, bet)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        print("C=%4d K=%4d lib=%s median %.1f us min %.1f us  checksum %.9e" % (
            c, k, os.path.basename(args.lib or "libhulkkp.so"), ts[len(ts) // 2] * 1e3, ts[0] * 1e3,
            ss.double().abs().sum().item()), flush=True)


if __name__ == "__main__":
    main()
