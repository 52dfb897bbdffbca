#!/usr/bin/env python3
"""Host cost of one step: the time the CPU spends enqueueing a C2 inference /
C3-shard training step (bench.py's workloads), measured with the GPU drained
before each step so the host never waits on a full queue — if it is near the
GPU's step time, the step is launch-bound and the GPU idles in the short-kernel
stretches (layer1/2 backward).  --profile adds a cProfile of the enqueue
(top functions by own time).

    python tools/host_cost.py [--mode train|infer] [--steps 10] [--profile]
"""
import argparse
import cProfile
import os
import pstats
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "hulk-keypoints_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="train")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--profile", action="store_true")
    args = ap.parse_args()
    import hkp
    from hkp.policy import Policy
    from oracle import recipe
    from src.model import KeypointsGauss
    hkp.lib()
    dev = torch.device("cuda", 0)
    B = args.batch or (8 if args.mode == "train" else 32)
    K, H, W = 4, 480, 640
    torch.manual_seed(1234)
    model = KeypointsGauss(K, H, W, backbone="resnet34", pretrained=False, policy=Policy()).to(dev)
    x = recipe.to_tensor_nchw(recipe.seeded_images_u8(B, H, W, 1234)).to(dev)
    uv = torch.from_numpy(recipe.seeded_keypoints(B, K, H, W, 99)).to(dev)
    if args.mode == "train":
        from hkp import train as hkp_train
        trainer = hkp_train.Trainer(model, lr=1e-4, weight_decay=1e-4)

        def step():
            return trainer.step(x, uv)
    else:
        def step():
            with torch.no_grad():
                return model.heatmaps_and_keypoints(x)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    host, wall = [], []
    for _ in range(args.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        host.append((t1 - t0) * 1e3)
        wall.append((t2 - t0) * 1e3)
    print("%s B=%d: host enqueue %.2f ms (min %.2f), enqueue+drain %.2f ms per step" %
          (args.mode, B, statistics.median(host), min(host), statistics.median(wall)), flush=True)
    if args.profile:
        torch.cuda.synchronize()
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(args.steps):
            step()
        pr.disable()
        torch.cuda.synchronize()
        st = pstats.Stats(pr)
        st.sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
