#!/usr/bin/env python3
"""HIP-event time of hkp_bn_apply_head on the C4 tail (R50 K8 640x480 B128: y and
the raw residual fp16, C = 2048) and the C2 tail (R34 K4 B32: fp32 y, packed
split residual, C = 512), median of `--iters` launches after a warm-up.  Run it
once per library build (`--lib`) in one box call and compare.

    python tools/head_time.py [--lib tools/ab_lib/libhulkkp_a.so] [--iters 20]
"""
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
    cases = {"c4_tail": (128, 60, 80, 2048, 8, torch.float16), "c2_tail": (32, 60, 80, 512, 4, torch.float32)}
    for name, (n, h, w, c, k, dt) in cases.items():
        y = torch.randn(n, h, w, c, device=dev, generator=g).to(dt)
        ss = torch.cat([torch.rand(c, device=dev, generator=g) + 0.5, torch.randn(c, device=dev, generator=g) * 0.3])
        if dt == torch.float16:
            res = torch.randn(n, h, w, c, device=dev, generator=g).to(dt)
            nbytes = y.numel() * 4
        else:
            res = ops.split_pack_x3(torch.randn(n, h, w, c, device=dev, generator=g))
            nbytes = y.numel() * 8
        wk = torch.randn(k, c, device=dev, generator=g) * 0.02
        bk = torch.randn(k, device=dev, generator=g)
        for _ in range(3):
            low = ops.bn_apply_head(y, ss, res, None, wk, bk)
        ts = []
        for _ in range(args.iters):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ops.bn_apply_head(y, ss, res, None, wk, bk)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        med = ts[len(ts) // 2]
        print("%s lib=%s median %.3f ms min %.3f ms  %.2f TB/s  checksum %.6e" %
              (name, os.path.basename(args.lib or "libhulkkp.so"), med, ts[0], nbytes / med / 1e9,
               low.double().sum().item()), flush=True)


if __name__ == "__main__":
    main()
