#!/usr/bin/env python3
"""Measured tile-plan table (verdict r5 item 4): record every forward conv launch
of the C2 / B=8-shard / C3-shard / C4 / C5 networks (kind, shape), time each conv
under every live tile policy (hkp_conv_desc.tile) in one process (policies
interleaved round-robin, HIP events, median of rounds), and write the table the
network reads (hulk-keypoints_amd/hkp/tile_plan.json: per shape the policies'
median ms and the chosen one — the fastest, kept at the planner (0) unless the
fastest beats it by more than HYST).

    python tools/tile_sweep.py [--workloads c2,b8,c4,c5] [--rounds 5] [--iters 4] [--out PATH]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "hulk-keypoints_amd")]

import torch  # noqa: E402

# every live HKP_TILE_* (7, 8, 14 retired; 12 = AUTO_A3, the round-4 planner; 15 / 16 = 192- / 160-row A3, x3 only)
TILES = {"x3": (0, 1, 2, 3, 4, 5, 6, 9, 11, 12, 15, 16), "f16": (0, 1, 2, 3, 4, 5, 6, 9, 11, 12, 13),
         "f16bn": (0, 3, 4, 5, 6, 11, 13)}
HYST = 0.015

WORKLOADS = {   # name: (backbone, keypoints, batch, height, width, precision, mode)
    "c2": ("resnet34", 4, 32, 480, 640, "f16x3", "infer"),
    "b8": ("resnet34", 4, 8, 480, 640, "f16x3", "infer"),
    "b16": ("resnet34", 4, 16, 480, 640, "f16x3", "infer"),    # north_star batch 64 over 4 GPUs
    "c3": ("resnet34", 4, 8, 480, 640, "f16x3", "train"),
    "c4": ("resnet50", 8, 128, 480, 640, "f16", "infer"),
    "c5": ("resnet50", 8, 32, 960, 1280, "f16x3", "train"),
}


def record(name):
    """(kind, n, h, w, cin, cout, k, stride, pad, dil) of every forward conv of one
    step of the workload whose tile the plan table may choose (the fused-input-BN
    halo convs have none)."""
    from hkp import ops
    from src.model import KeypointsGauss
    bb, K, B, H, W, prec, mode = WORKLOADS[name]
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = KeypointsGauss(K, H, W, backbone=bb, pretrained=False, precision=prec).to(dev)
    x = torch.rand(B, 3, H, W, device=dev)
    seen = []
    orig = {n: getattr(ops, n) for n in ("conv2d_fwd_x3", "conv2d_fwd_f16", "conv2d_fwd_f16_bn")}

    def wrap(fname, kind):
        def f(x_, wp, stride=1, pad=0, dil=1, *a, **kw):
            ws = wp[0]
            n, h, w, c = x_.shape
            cin = c // 2 if kind == "x3" else c
            seen.append((kind, n, h, w, cin, ws.shape[0], ws.shape[1], stride, pad, dil))
            return orig[fname](x_, wp, stride, pad, dil, *a, **kw)
        return f
    ops.conv2d_fwd_x3 = wrap("conv2d_fwd_x3", "x3")
    ops.conv2d_fwd_f16 = wrap("conv2d_fwd_f16", "f16")

    def bn_wrap(x16, wp, ss, res=None, res_ss=None, relu=True, stride=1, pad=0, dil=1, **kw):
        n, h, w, c = x16.shape
        seen.append(("f16bn", n, h, w, c, wp[0].shape[0], wp[0].shape[1], stride, pad, dil))
        return orig["conv2d_fwd_f16_bn"](x16, wp, ss, res=res, res_ss=res_ss, relu=relu, stride=stride, pad=pad,
                                         dil=dil, **kw)
    ops.conv2d_fwd_f16_bn = bn_wrap
    try:
        if mode == "infer":
            with torch.no_grad():
                m.heatmaps_and_keypoints(x, policy=m.policy.with_(tile_plan=False))
        else:
            from hkp import train as hkp_train
            uv = torch.stack([torch.rand(B, K) * (W - 1), torch.rand(B, K) * (H - 1)], -1).to(dev)
            m.policy = m.policy.with_(tile_plan=False)
            hkp_train.Trainer(m, lr=1e-4).step(x, uv)
    finally:
        for n, f in orig.items():
            setattr(ops, n, f)
    del m, x
    torch.cuda.empty_cache()
    return sorted(set(seen))


def key_of(s):
    return "|".join(str(v) for v in s)


def time_shape(s, rounds, iters):
    from hkp import ops
    kind, n, h, w, cin, cout, k, st, pd, dl = s
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.relu(torch.randn(n, h, w, cin, device=dev, generator=g))
    wt = torch.randn(cout, k, k, cin, device=dev, generator=g) * (2.0 / (k * k * cout)) ** 0.5
    if kind == "x3":
        ss = torch.cat([torch.ones(cin, device=dev), torch.zeros(cin, device=dev)])
        xs = ops.bn_apply(x, ss, relu=False, split=3, keep_fp32=False)
        wp = ops.weight_pack_x3(wt)

        def run(t):
            ops.conv2d_fwd_x3(xs, wp, st, pd, dl, tile=t)
    else:
        xs, wp = x.half(), ops.weight_pack_f16(wt)
        if kind == "f16":
            def run(t):
                ops.conv2d_fwd_f16(xs, wp, st, pd, dl, tile=t)
        else:
            ho, wo = ops.conv_out_hw(h, w, k, k, st, pd, dl)
            res = torch.relu(torch.randn(n, ho, wo, cout, device=dev, generator=g)).half()
            bss = torch.cat([torch.rand(cout, device=dev, generator=g) + 0.5, torch.rand(cout, device=dev) - 0.5])

            def run(t):
                ops.conv2d_fwd_f16_bn(xs, wp, bss, res=res, relu=True, stride=st, pad=pd, dil=dl, tile=t)
    del x
    # only the policies that launch another kernel than the planner's (a policy the
    # shape does not take plans as AUTO: timing it again would only sample noise)
    from hkp._lib import HKP_KOP_FWD_F16, HKP_KOP_FWD_X3, ConvDesc
    kop = HKP_KOP_FWD_X3 if kind == "x3" else HKP_KOP_FWD_F16
    names = {t: ops.kernel_name(ConvDesc(n, h, w, cin, cout, k, k, st, pd, dl, 0, t), kop) for t in TILES[kind]}
    tiles = [t for t in TILES[kind] if t == 0 or names[t] != names[0] or kind == "f16bn"]
    # the halo body stays where the planner puts it: the fused-input-BN conv runs where
    # the unfused one runs it (same tiles, same bits — test_fused_input_bn_network_bitexact)
    if names[0].startswith("conv_x3_halo"):
        tiles = [0]
    times = {t: [] for t in tiles}
    for _ in range(rounds):
        for t in tiles:
            run(t)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                run(t)
            e1.record()
            torch.cuda.synchronize()
            times[t].append(e0.elapsed_time(e1) / iters)
    return {t: sorted(v)[len(v) // 2] for t, v in times.items()}


def choose(med):
    """The plan's tile of one shape: the fastest policy, the planner (0) unless the
    fastest beats it by more than HYST (box-to-box noise is ~1-2 %)."""
    best = min(med, key=lambda t: (med[t], t))
    return best if med[best] < med[0] * (1.0 - HYST) else 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="c2,b8,c3,c4,c5")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=4)
    ap.add_argument("--out", default=os.path.join(REPO, "hulk-keypoints_amd", "hkp", "tile_plan.json"))
    args = ap.parse_args()
    table = {}
    if os.path.exists(args.out):
        table = json.load(open(args.out)).get("shapes", {})
    for wl in args.workloads.split(","):
        shapes = record(wl)
        print("%s: %d conv shapes" % (wl, len(shapes)), flush=True)
        for s in shapes:
            med = time_shape(s, args.rounds, args.iters)
            pick = choose(med)
            table[key_of(s)] = {"ms": {str(t): round(v, 5) for t, v in med.items()}, "tile": pick,
                                "workloads": sorted(set(table.get(key_of(s), {}).get("workloads", []) + [wl]))}
            print("  %-48s planner %.3f ms  best %2d %.3f ms  -> tile %d" % (key_of(s), med[0], min(med, key=med.get),
                                                                           min(med.values()), pick), flush=True)
    doc = {"about": "measured forward tile plan (tools/tile_sweep.py): key = kind|n|h|w|cin|cout|k|stride|pad|dil; "
                    "ms = median per HKP_TILE_* policy; tile = the policy the network uses (hkp.net._planned_tile)",
           "hysteresis": HYST, "shapes": table}
    json.dump(doc, open(args.out, "w"), indent=1, sort_keys=True)
    print("wrote %s (%d shapes)" % (args.out, len(table)))


if __name__ == "__main__":
    main()
