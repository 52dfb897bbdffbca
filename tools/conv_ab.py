#!/usr/bin/env python3
"""In-process A/B of conv_x3 schedule variants (hkp_set_conv_variant) on the
C2 conv shapes: variants interleaved round-robin, HIP-event timed, median and
min per variant (cdna_hip_programming.md §5.4 rule 24: never compare separate
processes).  Reports the largest output difference between variants (fp32 summation order).

    python tools/conv_ab.py [--variants 0,1] [--rounds 7] [--iters 10]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "hulk-keypoints_amd"))

import torch  # noqa: E402

SHAPES = {   # name: (N, H, W, Cin, Cout, k, stride, pad, dil) — R34-8s @640x480, batch 32
    "layer4": (32, 60, 80, 512, 512, 3, 1, 4, 4),
    "layer3": (32, 60, 80, 256, 256, 3, 1, 2, 2),
    "layer2": (32, 60, 80, 128, 128, 3, 1, 1, 1),
    "layer1": (32, 120, 160, 64, 64, 3, 1, 1, 1),
    "t4": (8, 60, 80, 512, 512, 3, 1, 4, 4),             # training shard (batch 8)
    "t3": (8, 60, 80, 256, 256, 3, 1, 2, 2),
    "t2": (8, 60, 80, 128, 128, 3, 1, 1, 1),
    "t1": (8, 120, 160, 64, 64, 3, 1, 1, 1),
    "layer4_n2": (2, 60, 80, 512, 512, 3, 1, 4, 4),     # 4.9 MB operand: L2/MALL-resident
    "layer3_n4": (4, 60, 80, 256, 256, 3, 1, 2, 2),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,1,2")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    args = ap.parse_args()
    from hkp import ops
    from hkp._lib import call
    variants = [int(v) for v in args.variants.split(",")]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    for name in args.shapes.split(","):
        n, h, w, ci, co, k, st, pd, dl = SHAPES[name]
        x = torch.relu(torch.randn(n, h, w, ci, device=dev, generator=g))
        wt = torch.randn(co, k, k, ci, device=dev, generator=g) * (2.0 / (k * k * co)) ** 0.5
        ss = torch.cat([torch.ones(ci, device=dev), torch.zeros(ci, device=dev)])
        xs = ops.bn_apply(x, ss, relu=False, split=3, keep_fp32=False)
        ws = ops.weight_pack_x3(wt)
        outs, times = {}, {v: [] for v in variants}
        for r in range(args.rounds):
            for v in variants:
                call("hkp_set_conv_variant", v)
                y, _ = ops.conv2d_fwd_x3(xs, ws, st, pd, dl)      # warm / result
                if r == 0:
                    outs[v] = y.clone()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(args.iters):
                    ops.conv2d_fwd_x3(xs, ws, st, pd, dl)
                e.record()
                torch.cuda.synchronize()
                times[v].append(s.elapsed_time(e) / args.iters)
        call("hkp_set_conv_variant", 0)
        flops = 2.0 * n * h * w * co * ci * k * k * 3
        ref = outs[variants[0]]
        same = max((outs[v] - ref).abs().max().item() / ref.abs().max().item() for v in variants)
        for v in variants:
            t = sorted(times[v])
            print("%-7s var %d: median %.3f ms  min %.3f ms  (%.0f TF/s issued)  max rel diff=%.1e" % (
                name, v, t[len(t) // 2], t[0], flops / (t[len(t) // 2] * 1e-3) / 1e12, same))


if __name__ == "__main__":
    main()
