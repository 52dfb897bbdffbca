#!/usr/bin/env python3
"""Where a training step waits for the host: at every conv launch of one step
(started from an idle GPU) record the host clock and a HIP event on the launch
stream; GPU time at a launch minus host time at its enqueue is the queue's lead
there — near the launch latency means the GPU had drained and was waiting.
python tools/host_lag.py [batch]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "hulk-keypoints_amd")]
import torch  # noqa: E402


def main():
    from src.model import KeypointsGauss
    from oracle import recipe
    from hkp import ops, train
    dev = torch.device("cuda", 0)
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    K, H, W = 4, 480, 640
    m = KeypointsGauss(K, H, W, pretrained=False).to(dev)
    x = recipe.to_tensor_nchw(recipe.seeded_images_u8(B, H, W, 1)).to(dev)
    uv = torch.from_numpy(recipe.seeded_keypoints(B, K, H, W, 2)).to(dev)
    t = train.Trainer(m)
    for _ in range(3):
        t.step(x, uv)
    torch.cuda.synchronize()
    rec = []

    def obs(sym, flops, nbytes, launch):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        rec.append((sym, time.perf_counter(), e))
        launch()

    for rnd in range(3):
        rec.clear()
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        h0 = time.perf_counter()
        ops.set_observer(obs)
        t.step(x, uv)
        ops.set_observer(None)
        h_end = time.perf_counter()
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        torch.cuda.synchronize()
        total = e0.elapsed_time(e1)
        lead = [(s, (h - h0) * 1e3, e0.elapsed_time(e)) for s, h, e in rec]
        starved = [(s, hh, g) for s, hh, g in lead if g - hh < 0.05]
        print("step %.2f ms GPU, host enqueue %.2f ms; %d conv launches, %d with < 50 us of queued work ahead" % (
            total, (h_end - h0) * 1e3, len(lead), len(starved)), flush=True)
        if rnd == 2:
            for i, (s, hh, g) in enumerate(lead):
                print("  %3d host %7.2f  gpu %7.2f  lead %6.2f ms  %s" % (i, hh, g, g - hh, s[:60]))


if __name__ == "__main__":
    main()
