#!/usr/bin/env python3
"""In-process A/B of conv tile policies (hkp_conv_desc.tile) on the C2 (f16x3)
and C4 (plain fp16) conv shapes: policies interleaved round-robin, HIP-event
timed, median and min per policy (cdna_hip_programming.md §5.4 rule 24: never
compare separate processes).  Reports the kernel each policy runs and the
largest output difference between policies (fp32 summation order).

    python tools/conv_ab.py [--tiles 0,3,4] [--shapes c4_l4_c1,...] [--rounds 7] [--iters 10]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "hulk-keypoints_amd"))

import torch  # noqa: E402

# name: (precision, N, H, W, Cin, Cout, k, stride, pad, dil)
SHAPES = {
    # R34-8s @640x480, batch 32 (C2, f16x3)
    "layer4": ("x3", 32, 60, 80, 512, 512, 3, 1, 4, 4),
    "layer3": ("x3", 32, 60, 80, 256, 256, 3, 1, 2, 2),
    "layer2": ("x3", 32, 60, 80, 128, 128, 3, 1, 1, 1),
    "layer1": ("x3", 32, 120, 160, 64, 64, 3, 1, 1, 1),
    "l2c1": ("x3", 32, 120, 160, 64, 128, 3, 2, 1, 1),          # layer2 conv1 (stride 2)
    "l2ds": ("x3", 32, 120, 160, 64, 128, 1, 2, 0, 1),          # layer2 downsample
    "l3c1": ("x3", 32, 60, 80, 128, 256, 3, 1, 1, 1),           # layer3 conv1 (128 -> 256)
    "l3ds": ("x3", 32, 60, 80, 128, 256, 1, 1, 0, 1),
    "t2": ("x3", 8, 60, 80, 128, 128, 3, 1, 1, 1),             # layer2 at batch 8
    "t1": ("x3", 8, 120, 160, 64, 64, 3, 1, 1, 1),             # layer1 at batch 8
    "l4c1": ("x3", 32, 60, 80, 256, 512, 3, 1, 2, 2),           # layer4 conv1 (256 -> 512)
    "l4ds": ("x3", 32, 60, 80, 256, 512, 1, 1, 0, 1),
    "t2c1": ("x3", 8, 120, 160, 64, 128, 3, 2, 1, 1),           # batch 8: layer2 conv1, downsamples
    "t2ds": ("x3", 8, 120, 160, 64, 128, 1, 2, 0, 1),
    "t3ds": ("x3", 8, 60, 80, 128, 256, 1, 1, 0, 1),
    "h128": ("x3", 4, 240, 320, 128, 128, 3, 1, 1, 1),           # halo body at 128 channels
    "t4": ("x3", 8, 60, 80, 512, 512, 3, 1, 4, 4),             # training shard (batch 8)
    "t3": ("x3", 8, 60, 80, 256, 256, 3, 1, 2, 2),
    "t2": ("x3", 8, 60, 80, 128, 128, 3, 1, 1, 1),             # layer2 3x3 at batch 8 (128-wide)
    "c2_l3": ("x3", 32, 60, 80, 256, 256, 3, 1, 2, 2),         # C2 layer3 3x3 (dilation 2)
    "c2_l3a": ("x3", 32, 60, 80, 128, 256, 3, 1, 2, 2),        # C2 layer3 conv1
    "t2s": ("x3", 8, 120, 160, 64, 128, 3, 2, 1, 1),           # layer2 conv1, stride 2
    "t3a": ("x3", 8, 60, 80, 128, 256, 3, 1, 2, 2),            # layer3 conv1 at batch 8 (dilated, stride 1)
    "t4ds": ("x3", 8, 60, 80, 256, 512, 1, 1, 0, 1),
    # R50-8s @1280x960, batch 32 (C5 training, f16x3): short-K 1x1s
    "c5_l3_c3": ("x3", 32, 120, 160, 256, 1024, 1, 1, 0, 1),
    "c5_l2_c3": ("x3", 32, 120, 160, 128, 512, 1, 1, 0, 1),
    "c5_l1_c3": ("x3", 32, 240, 320, 64, 256, 1, 1, 0, 1),
    "c5_l2_ds": ("x3", 32, 240, 320, 256, 512, 1, 2, 0, 1),
    "c5_l2_c2": ("x3", 32, 120, 160, 128, 128, 3, 1, 1, 1),
    # R50-8s @640x480, batch 128 (C4, plain fp16)
    "c4_l4_c2": ("f16", 128, 60, 80, 512, 512, 3, 1, 4, 4),
    "c4_l4_c1": ("f16", 128, 60, 80, 2048, 512, 1, 1, 0, 1),
    "c4_l4_c3": ("f16", 128, 60, 80, 512, 2048, 1, 1, 0, 1),
    "c4_l4_ds": ("f16", 128, 60, 80, 1024, 2048, 1, 1, 0, 1),
    "c4_l1_ds": ("f16", 128, 120, 160, 64, 256, 1, 1, 0, 1),
    "c4_l3_c2": ("f16", 128, 60, 80, 256, 256, 3, 1, 2, 2),
    "c4_l3_c1": ("f16", 128, 60, 80, 1024, 256, 1, 1, 0, 1),
    "c4_l3_c3": ("f16", 128, 60, 80, 256, 1024, 1, 1, 0, 1),
    "c4_l1_c3": ("f16", 128, 120, 160, 64, 256, 1, 1, 0, 1),
    "c4_l1_c2": ("f16", 128, 120, 160, 64, 64, 3, 1, 1, 1),
    "c4_l1_c1": ("f16", 128, 120, 160, 256, 64, 1, 1, 0, 1),
    "c4_l1_c1a": ("f16", 128, 120, 160, 64, 64, 1, 1, 0, 1),
    "c4_l2_c1a": ("f16", 128, 120, 160, 256, 128, 1, 1, 0, 1),
    "c4_l2_c2": ("f16", 128, 60, 80, 128, 128, 3, 1, 1, 1),
    "c4_l2_c1": ("f16", 128, 60, 80, 512, 128, 1, 1, 0, 1),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default="0,3,4,5")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--nostats", action="store_true", help="no BN partials (epilogue cost A/B)")
    ap.add_argument("--lib", default=None, help="another build of libhulkkp.so (A/B)")
    ap.add_argument("--duo-staggers", default="-1", help="DUO first-round stagger(s) in ns to cross with the "
                    "tiles (hkp_debug_duo_stagger: 0 off, -1 the default estimate)")
    ap.add_argument("--a-wraps", default="0", help="A-row wraps to cross with the tiles (hkp_debug_x3_a_wrap: "
                    "0 off; e.g. 2048 = every tile reads the first 8 m-tiles' A rows, an L2-resident stream)")
    ap.add_argument("--stores", default="0", help="epilogue store flavours to cross with the tiles "
                    "(hkp_debug_x3_store: 0 default, 1 plain, 2 nt, 3 sc1, 4 sc0 sc1)")
    args = ap.parse_args()
    from hkp import _lib
    if args.lib:
        _lib.use_library(os.path.abspath(args.lib))
    elif os.path.exists(_lib.AB_LIB_PATH):
        _lib.use_ab_library()                   # its hkp_debug_* knobs (include/hulkkp_ab.h)
    from hkp import ops
    from hkp._lib import HKP_KOP_FWD_F16, HKP_KOP_FWD_X3, ConvDesc
    from hkp._lib import lib
    forms = [(int(t), int(k), int(d), int(aw)) for t in args.tiles.split(",") for k in args.stores.split(",")
             for d in args.duo_staggers.split(",") for aw in args.a_wraps.split(",")]

    def set_store(k, d=-1, aw=0):
        if hasattr(lib(), "hkp_debug_x3_store"):
            lib().hkp_debug_x3_store(k)
            lib().hkp_debug_duo_stagger(d)
            lib().hkp_debug_x3_a_wrap(aw)
        elif (k, d, aw) != (0, -1, 0):
            raise SystemExit("--stores / --duo-staggers / --a-wraps need the A/B build: make -C hulk-keypoints_amd/csrc ab")
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
            passes, op = 3, HKP_KOP_FWD_X3

            def run(t):
                return ops.conv2d_fwd_x3(xs, ws, st, pd, dl, stats=not args.nostats, tile=t)[0]
        else:
            xs = x.half()
            ws = ops.weight_pack_f16(wt)
            passes, op = 1, HKP_KOP_FWD_F16

            def run(t):
                return ops.conv2d_fwd_f16(xs, ws, st, pd, dl, stats=not args.nostats, tile=t)[0]
        del x
        outs, times = {}, {f: [] for f in forms}
        for r in range(args.rounds):
            for f in forms:
                t = f[0]
                set_store(f[1], f[2], f[3])
                y = run(t)
                if r == 0:
                    outs[f] = y.float()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(args.iters):
                    run(t)
                e.record()
                torch.cuda.synchronize()
                times[f].append(s.elapsed_time(e) / args.iters)
        set_store(0)
        ho, wo = ops.conv_out_hw(h, w, k, k, st, pd, dl)
        flops = 2.0 * n * ho * wo * co * ci * k * k * passes
        ref = outs[forms[0]]
        same = max((outs[f] - ref).abs().max().item() / max(ref.abs().max().item(), 1e-30) for f in forms)
        for f in forms:
            t = f[0]
            ts = sorted(times[f])
            set_store(f[1], f[2], f[3])
            kn = ops.kernel_name(ConvDesc(n, h, w, ci, co, k, k, st, pd, dl, 0, t), op)
            set_store(0)
            print("%-9s tile %d store %d stagger %d a_wrap %d: median %.3f ms  min %.3f ms  (%.0f TF/s issued)  %s  "
                  "max rel diff=%.1e" % (name, t, f[1], f[2], f[3], ts[len(ts) // 2], ts[0],
                                         flops / (ts[len(ts) // 2] * 1e-3) / 1e12, kn, same), flush=True)


if __name__ == "__main__":
    main()
