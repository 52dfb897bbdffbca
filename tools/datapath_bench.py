#!/usr/bin/env python3
"""Data-path throughput: images/s that DeviceBatches delivers to
the GPU from a folder of 640x480 JPEGs in the reference's dataset layout, with
the reference's per-image decode in the training process (workers=0,
dataset.py:71 / train.py:51) and with N DataLoader decode workers, vs the
compute rate of the C2 inference step.  Synthetic images (smooth gradients +
noise, JPEG quality 95), written to a temp dir.

    python tools/datapath_bench.py [--n 512] [--batch 32] [--workers 0,4,8,15] [--decode host,device]

--decode device: the hybrid decode (hkp.jpeg) — workers only entropy-decode, the
IDCT / upsampling / colour conversion run on the GPU on the copy stream.
"""
import argparse
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "hulk-keypoints_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def write_dataset(root, n, H, W, K):
    from PIL import Image
    os.makedirs(os.path.join(root, "images"))
    os.makedirs(os.path.join(root, "keypoints"))
    rng = np.random.default_rng(0)
    yy, xx = np.mgrid[0:H, 0:W]
    for i in range(n):
        base = np.stack([(xx * (i % 7 + 1)) % 256, (yy * (i % 5 + 1)) % 256, (xx + yy + 9 * i) % 256], -1)
        img = np.clip(base + rng.normal(0, 8, base.shape), 0, 255).astype(np.uint8)
        Image.fromarray(img).save(os.path.join(root, "images", "%05d.jpg" % i), quality=95)
        np.save(os.path.join(root, "keypoints", "%05d.npy" % i), rng.uniform(0, [W - 1, H - 1], (K, 2)).reshape(-1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2048)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--workers", default="0,4,8,15")
    ap.add_argument("--decode", default="host,device")
    args = ap.parse_args()
    from src.dataset import DeviceBatches, KeypointsDataset, transform
    H, W, K = 480, 640, 4
    with tempfile.TemporaryDirectory() as root:
        write_dataset(root, args.n, H, W, K)
        ds = KeypointsDataset(os.path.join(root, "images"), os.path.join(root, "keypoints"), K, H, W, transform)
        cpus = len(os.sched_getaffinity(0))
        try:
            q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
            cpus = min(cpus, int(q) // int(per)) if q != "max" else cpus
        except (OSError, ValueError):
            pass
        for w, dec in [(int(v), d) for d in args.decode.split(",") for v in args.workers.split(",")]:
            it = DeviceBatches(ds, args.batch, shuffle=True, workers=w, decode=dec)
            for _ in it:                       # warm epoch: page cache, persistent worker start-up
                pass
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            n = 0
            for img, uv in it:
                n += img.shape[0]
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(json.dumps({"decode": dec, "workers": w, "images": n, "seconds": round(dt, 3), "images_per_sec": round(n / dt, 1),
                              "batch": args.batch, "image": "%dx%d JPEG q95" % (W, H),
                              "host_cpu_share": cpus}), flush=True)


if __name__ == "__main__":
    main()
