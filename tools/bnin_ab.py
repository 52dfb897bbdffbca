#!/usr/bin/env python3
"""In-process A/B of the fused input BN on the 256-wide convs (C2 layer3/4 conv2):
  apply  bn_apply(relu, split 3) then the A3 conv   (the unfused pair)
  conv   the A3 conv alone on the applied operand   (what the fusion must beat)
  fused  hkp_conv2d_fwd_x3_bnin (conv_x3_a3_bnin_kernel<3>)
interleaved round-robin, HIP-event timed, median per form; the fused output must
equal the unfused one bit for bit.

    python tools/bnin_ab.py [--shapes layer3,layer4] [--rounds 7] [--iters 10]
"""
import argparse
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "hulk-keypoints_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))

import torch  # noqa: E402

from conv_ab import SHAPES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="layer3,layer4")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--lib", default=None, help="another build of libhulkkp.so (A/B instrument builds)")
    args = ap.parse_args()
    if args.lib:
        from hkp import _lib
        _lib.use_library(os.path.abspath(args.lib))
    from hkp import ops
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(5)
    for name in args.shapes.split(","):
        prec, n, h, w, c, k, r, st, pad, dil = SHAPES[name]
        assert prec == "x3"
        y = (torch.randn(n, h, w, c, generator=g) * 2 + 0.5).to(dev)
        ss = torch.cat([torch.randn(c, generator=g) * 0.5, torch.randn(c, generator=g)]).to(dev)
        wt = (torch.randn(k, r, r, c, generator=g) * (2.0 / (r * r * k)) ** 0.5).to(dev)
        wp = ops.weight_pack_x3(wt)
        name_f = ops.bnin_kernel(n, h, w, c, k, r, r, st, pad, dil)
        a = ops.bn_apply(y, ss, relu=True, split=3, keep_fp32=False)

        def f_apply():
            aa = ops.bn_apply(y, ss, relu=True, split=3, keep_fp32=False)
            return ops.conv2d_fwd_x3(aa, wp, st, pad, dil)

        def f_conv():
            return ops.conv2d_fwd_x3(a, wp, st, pad, dil)

        def f_fused():
            return ops.conv2d_fwd_bnin(y, ss, wp, st, pad, dil)

        forms = {"apply": f_apply, "conv": f_conv, "fused": f_fused}
        ref = f_conv()
        got = f_fused()
        torch.cuda.synchronize()
        same = torch.equal(ref[0], got[0]) and torch.equal(ref[1], got[1])
        times = {f: [] for f in forms}
        for _ in range(args.rounds):
            for f, fn in forms.items():
                fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                times[f].append(e0.elapsed_time(e1) / args.iters)
        med = {f: statistics.median(v) for f, v in times.items()}
        print("%-7s %s  apply+conv %.3f ms  conv %.3f ms  fused %.3f ms  (fused vs conv %+.1f %%, vs apply+conv "
              "%+.1f %%)  bit-identical %s" % (name, name_f, med["apply"], med["conv"], med["fused"],
                                               100 * (med["fused"] / med["conv"] - 1),
                                               100 * (med["fused"] / med["apply"] - 1), same), flush=True)


if __name__ == "__main__":
    main()
