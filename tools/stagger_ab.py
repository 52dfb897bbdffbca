#!/usr/bin/env python3
"""In-process A/B of the first-round stagger of the one-tile conv launches
(hkp_debug_x3_stagger): half the CUs of every XCD start their first block late,
so the rounds' HBM-bound epilogues stop coinciding.  Values interleaved
round-robin, HIP-event timed, median per value.

    python tools/stagger_ab.py [--ns 0,4000,8000] [--shapes c4_l4_c3,...] [--rounds 7] [--iters 10]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "hulk-keypoints_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))

import torch  # noqa: E402

from conv_ab import SHAPES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="0,3000,6000,9000,12000")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--shapes", default="c4_l4_c3,c4_l4_c1,c4_l3_c3,c4_l3_c1,c4_l1_c3,c4_l4_c2,layer4,layer3")
    args = ap.parse_args()
    from hkp import ops
    from hkp import _lib
    _lib.use_ab_library()                       # the hkp_debug_* knobs (include/hulkkp_ab.h)
    from hkp._lib import lib
    vals = [int(v) for v in args.ns.split(",")]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    for name in args.shapes.split(","):
        prec, n, h, w, ci, co, k, st, pd, dl = SHAPES[name]
        x = torch.relu(torch.randn(n, h, w, ci, device=dev, generator=g))
        wt = torch.randn(co, k, k, ci, device=dev, generator=g) * (2.0 / (k * k * co)) ** 0.5
        if prec == "x3":
            ss = torch.cat([torch.ones(ci, device=dev), torch.zeros(ci, device=dev)])
            xs = ops.bn_apply(x, ss, relu=False, split=3, keep_fp32=False)
            ws = ops.weight_pack_x3(wt)

            def run():
                return ops.conv2d_fwd_x3(xs, ws, st, pd, dl)[0]
        else:
            xs = x.half()
            ws = ops.weight_pack_f16(wt)

            def run():
                return ops.conv2d_fwd_f16(xs, ws, st, pd, dl)[0]
        del x
        times = {v: [] for v in vals}
        ref = None
        for r in range(args.rounds):
            for v in vals:
                lib().hkp_debug_x3_stagger(v)
                y = run()
                if r == 0:
                    if ref is None:
                        ref = y.clone()
                    assert torch.equal(y, ref), "stagger changed the output"
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(args.iters):
                    run()
                e.record()
                torch.cuda.synchronize()
                times[v].append(s.elapsed_time(e) / args.iters)
        lib().hkp_debug_x3_stagger(0)
        base = sorted(times[vals[0]])[len(times[vals[0]]) // 2]
        for v in vals:
            ts = sorted(times[v])
            print("%-9s stagger %6d ns: median %.3f ms  min %.3f ms  (%+.1f %%)" % (
                name, v, ts[len(ts) // 2], ts[0], 100 * (ts[len(ts) // 2] / base - 1)), flush=True)


if __name__ == "__main__":
    main()
