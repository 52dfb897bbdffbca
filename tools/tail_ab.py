#!/usr/bin/env python3
"""In-process A/B of an A3 grid's split-K tail in the same launch (default) vs as
a second launch (hkp_debug_x3_split_tail), on the shapes with a partial last
round: C2 layer3 (600 tiles), the C3 shard's layer4 forward (300 tiles), C4
l4_c2 (4800 tiles).  Interleaved, HIP-event timed, median per form; outputs
must be bit-identical (same segments, same order).

    python tools/tail_ab.py [--rounds 7] [--iters 10]
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
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--shapes", default="layer3,t4,t3,c4_l4_c2,c4_l3_c2")
    args = ap.parse_args()
    from hkp import ops
    from hkp import _lib
    _lib.use_ab_library()                       # the hkp_debug_* knobs (include/hulkkp_ab.h)
    from hkp._lib import lib
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
        times = {0: [], 1: []}
        outs = {}
        for r in range(args.rounds):
            for v in (0, 1):
                lib().hkp_debug_x3_split_tail(v)
                y = run()
                if r == 0:
                    outs[v] = y.clone()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(args.iters):
                    run()
                e.record()
                torch.cuda.synchronize()
                times[v].append(s.elapsed_time(e) / args.iters)
        lib().hkp_debug_x3_split_tail(0)
        same = torch.equal(outs[0], outs[1])
        med = {v: sorted(t)[len(t) // 2] for v, t in times.items()}
        print("%-9s one launch %.3f ms, two launches %.3f ms (%+.1f %%), bit-identical %s" % (
            name, med[0], med[1], 100 * (med[0] / med[1] - 1), same), flush=True)


if __name__ == "__main__":
    main()
