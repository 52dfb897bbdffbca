#!/usr/bin/env python3
"""Which HKP_TILE_* each forward conv of one inference step launches with (the
measured tile plan's choice, or 0 = the C planner), the plan misses, and the
kernel names — for bench.py's model at a given batch.

    python tools/plan_check.py --batch 8
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "hulk-keypoints_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--backbone", default="resnet34")
    ap.add_argument("--keypoints", type=int, default=4)
    ap.add_argument("--precision", default="f16x3")
    args = ap.parse_args()
    from hkp import net, ops
    from hkp.policy import Policy
    from src.model import KeypointsGauss
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    m = KeypointsGauss(args.keypoints, 480, 640, backbone=args.backbone, pretrained=False,
                       policy=Policy(precision=args.precision)).to(dev)
    x = torch.rand(args.batch, 3, 480, 640, device=dev)
    seen = []

    def observe(sym, flops, nbytes, launch):
        seen.append(sym)
        launch()
    orig = ops.conv2d_fwd_x3

    def wrap(xs, wp, stride=1, pad=0, dil=1, **kw):
        print("conv2d_fwd_x3 x%s w%s s%d p%d d%d tile=%s" % (tuple(xs.shape), tuple(wp[0].shape), stride, pad, dil,
                                                           kw.get("tile")))
        return orig(xs, wp, stride, pad, dil, **kw)
    ops.conv2d_fwd_x3 = wrap
    ops.set_observer(observe)
    with torch.no_grad():
        m.heatmaps_and_keypoints(x)
    ops.set_observer(None)
    ops.conv2d_fwd_x3 = orig
    torch.cuda.synchronize()
    print("kernels:", sorted(set(seen)))
    print("plan misses:", net.PLAN_MISSES)
    print("plan entries:", len(net._tile_plan_table()))


if __name__ == "__main__":
    main()
