#!/usr/bin/env python3
"""Upper bound for multi-stream inference: one B=32 C2 forward vs two B=16
forwards issued on two streams (independent: no shared BN statistics), HIP-event
timed in one process.  python tools/lane_probe.py"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "hulk-keypoints_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    from src.model import KeypointsGauss
    from oracle import recipe
    dev = torch.device("cuda", 0)
    m = KeypointsGauss(4, 480, 640, pretrained=False).to(dev)
    x = recipe.to_tensor_nchw(recipe.seeded_images_u8(32, 480, 640, 1)).to(dev)
    xa, xb = x[:16].contiguous(), x[16:].contiguous()
    s2 = torch.cuda.Stream(dev)

    def one():
        with torch.no_grad():
            m.heatmaps_and_keypoints(x)

    def two():
        with torch.no_grad():
            main = torch.cuda.current_stream(dev)
            s2.wait_stream(main)
            m.heatmaps_and_keypoints(xa)
            with torch.cuda.stream(s2):
                m.heatmaps_and_keypoints(xb)
            main.wait_stream(s2)

    def seq():
        with torch.no_grad():
            m.heatmaps_and_keypoints(xa)
            m.heatmaps_and_keypoints(xb)

    for f in (one, two, seq):
        for _ in range(3):
            f()
    torch.cuda.synchronize()
    for rnd in range(3):
        for name, f in (("B32", one), ("2x16 streams", two), ("2x16 serial", seq)):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                f()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 10
            print("%-14s %.2f ms  %.0f img/s" % (name, dt * 1e3, 32 / dt), flush=True)


if __name__ == "__main__":
    main()
