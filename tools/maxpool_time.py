#!/usr/bin/env python3
"""HIP-event time of hkp_bn_relu_maxpool on the C4 stem map (128 x 240 x 320 x 64 fp32
-> fp16 split-1 output) and the C2 one (32 images, split-3 output), median of
`--iters` launches; run once per library build (`--lib`) and compare."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "hulk-keypoints_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    if args.lib:
        from hkp import _lib
        _lib.use_library(os.path.abspath(args.lib))
    from hkp import ops
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    for name, n, split in (("c4_stem", 128, 1), ("c2_stem", 32, 3)):
        y = torch.randn(n, 240, 320, 64, device=dev, generator=g)
        ss = torch.cat([torch.rand(64, device=dev, generator=g) + 0.5, torch.randn(64, device=dev, generator=g)])
        for _ in range(3):
            o = ops.bn_relu_maxpool(y, ss, split=split, keep_fp32=False)
        ts = []
        for _ in range(args.iters):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ops.bn_relu_maxpool(y, ss, split=split, keep_fp32=False)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        print("%s lib=%s median %.3f ms min %.3f ms" % (name, os.path.basename(args.lib or "libhulkkp.so"),
                                                        ts[len(ts) // 2], ts[0]), flush=True)


if __name__ == "__main__":
    main()
