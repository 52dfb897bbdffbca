#!/usr/bin/env python3
"""Per-stage precision study at config C4 (verdict r5 item 7): promote one stage at
a time (layer1..layer4; the stem conv is fp32-class in both modes, the head
follows layer4) from plain fp16 to f16x3 (Policy.stage_precision) and report, for
each plan, the heatmap error and argmax agreement against the reference's R50-8s
K=8 640x480 fixture (tests/golden/fwd_r50_k8_480x640_b2) and the C4 throughput
(batch 128, plans interleaved round-robin in one process, HIP-event timed).

    python tests/precision_study.py [--rounds 3] [--iters 3]

(Under tests/: it regenerates the fixture's inputs with oracle.recipe, as the GPU tests do;
not collected by pytest.)
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "hulk-keypoints_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

PLANS = [
    ("f16", ()),
    ("f16 | layer1 f16x3", ("f16x3", "f16", "f16", "f16")),
    ("f16 | layer2 f16x3", ("f16", "f16x3", "f16", "f16")),
    ("f16 | layer3 f16x3", ("f16", "f16", "f16x3", "f16")),
    ("f16 | layer4+head f16x3", ("f16", "f16", "f16", "f16x3")),
    ("f16 | layer3-4 f16x3", ("f16", "f16", "f16x3", "f16x3")),
    ("f16 | layer1-2 f16x3", ("f16x3", "f16x3", "f16", "f16")),
    ("f16x3", None),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--batch", type=int, default=128)
    args = ap.parse_args()
    from oracle import recipe
    from src.model import KeypointsGauss
    dev = torch.device("cuda", 0)
    g = np.load(os.path.join(REPO, "tests", "golden", "fwd_r50_k8_480x640_b2.npz"), allow_pickle=False)
    B, H, W, K, st = int(g["batch"]), int(g["height"]), int(g["width"]), int(g["k"]), int(g["step"])
    m = KeypointsGauss(K, H, W, backbone="resnet50", pretrained=False, precision="f16")
    m.load_state_dict(recipe.seeded_state_dict("resnet50", int(g["wseed"])))
    m = m.to(dev)
    xg = recipe.to_tensor_nchw(recipe.seeded_images_u8(B, H, W, int(g["iseed"]))).to(dev)
    xb = recipe.to_tensor_nchw(recipe.seeded_images_u8(args.batch, H, W, 1234)).to(dev)

    def pol_of(plan):
        if plan is None:
            return m.policy.with_(precision="f16x3")
        return m.policy.with_(precision="f16", stage_precision=plan)
    rows = []
    for name, plan in PLANS:
        with torch.no_grad():
            hm, yx = m.heatmaps_and_keypoints(xg, policy=pol_of(plan))
        err = float(np.abs(hm[:, :, ::st, ::st].cpu().numpy() - g["heat_sub"]).max())
        agree = int((yx.cpu().numpy() == g["argmax_yx"]).all(-1).sum())
        rows.append([name, err, agree, []])
    for _ in range(args.rounds):
        for r, (name, plan) in zip(rows, PLANS):
            pol = pol_of(plan)
            with torch.no_grad():
                m.heatmaps_and_keypoints(xb, policy=pol)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(args.iters):
                    m.heatmaps_and_keypoints(xb, policy=pol)
                e.record()
            torch.cuda.synchronize()
            r[3].append(args.batch * args.iters / (s.elapsed_time(e) * 1e-3))
    f16_ips = sorted(rows[0][3])[len(rows[0][3]) // 2]
    x3_ips = sorted(rows[-1][3])[len(rows[-1][3]) // 2]
    print("R50-8s K=8 640x480: fixture fwd_r50_k8_480x640_b2 (%d keypoints, min top-2 margin %.2g); "
          "C4 batch %d img/s, median of %d rounds" % (B * K, float(g["margin"].min()), args.batch, args.rounds))
    print("%-26s %10s %8s %9s %7s %9s" % ("plan", "heat err", "argmax", "img/s", "x f16", "x f16x3"))
    for name, err, agree, ips in rows:
        med = sorted(ips)[len(ips) // 2]
        print("%-26s %10.3g %5d/%d %9.0f %7.2f %9.2f" % (name, err, agree, B * K, med, med / f16_ips, med / x3_ips),
              flush=True)


if __name__ == "__main__":
    main()
