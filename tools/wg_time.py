#!/usr/bin/env python3
"""Standalone timing of the f16x3 wgrad (wgrad_x3_kernel + wg_x3_reduce) on the
C3-shard shapes, HIP-event timed on the launching stream, with no dgrad sharing
the CUs (the training step overlaps them, so its per-kernel trace times include
the sharing).  Optional in-process A/B against an alternative build of the same
ABI (--lib) is done by running this twice in one call.

    python tools/wg_time.py [--shapes t3,t4] [--rounds 7] [--iters 10]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "hulk-keypoints_amd"))

import torch  # noqa: E402

# name: (N, H, W, Cin, Cout, k, stride, pad, dil) — R34-8s @640x480
SHAPES = {
    "t4": (8, 60, 80, 512, 512, 3, 1, 4, 4),
    "t3": (8, 60, 80, 256, 256, 3, 1, 2, 2),
    "t2": (8, 60, 80, 128, 128, 3, 1, 1, 1),
    "t1": (8, 120, 160, 64, 64, 3, 1, 1, 1),
    "b4": (32, 60, 80, 512, 512, 3, 1, 4, 4),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="t4,t3,t2,t1")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--lib", default=None, help="another build of libhulkkp.so (A/B)")
    ap.add_argument("--variants", default="0", help="CU budgets (d->tile) to time per shape: 0 = the planner, "
                    "-1 = the tiled body (no halo body)")
    args = ap.parse_args()
    if args.lib:
        from hkp import _lib
        _lib.use_library(os.path.abspath(args.lib))
    from hkp import ops
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    for name in args.shapes.split(","):
        n, h, w, ci, co, k, st, pd, dl = SHAPES[name]
        x = torch.relu(torch.randn(n, h, w, ci, device=dev, generator=g))
        ss = torch.cat([torch.ones(ci, device=dev), torch.zeros(ci, device=dev)])
        xs = ops.bn_apply(x, ss, relu=False, split=3, keep_fp32=False)
        ho, wo = ops.conv_out_hw(h, w, k, k, st, pd, dl)
        dy = torch.randn(n, ho, wo, co, device=dev, generator=g) * 1e-3
        amax = ops.absmax(dy)
        dys = ops.split_pack_x3(dy, amax)
        del x, dy

        from hkp._lib import HKP_KOP_WGRAD_X3
        first = None
        for v in [int(t) for t in args.variants.split(",")]:
            def run():
                return ops.conv2d_bwd_filter_x3(xs, dys, (co, k, k, ci), st, pd, dl, amax=amax, cus=v)

            ref = run()
            first = ref if first is None else first
            times = []
            for _ in range(args.rounds):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(args.iters):
                    run()
                e.record()
                torch.cuda.synchronize()
                times.append(s.elapsed_time(e) / args.iters)
            times.sort()
            med = times[len(times) // 2]
            flops = 2.0 * n * ho * wo * co * ci * k * k * 3
            d = ops._fwd_desc((n, h, w, ci), (co, k, k, ci), st, pd, dl, "nhwc")
            d.tile = v
            rel = ((ref - first).abs().max() / first.abs().max()).item()
            print("%-4s %-24s median %.4f ms  min %.4f ms  (%.0f TF/s issued = %.3f of 2.5 PF)  vs first %.2e" % (
                name, ops.kernel_name(d, HKP_KOP_WGRAD_X3), med, times[0], flops / (med * 1e-3) / 1e12,
                flops / (med * 1e-3) / 2.5e15, rel), flush=True)


if __name__ == "__main__":
    main()
