#!/usr/bin/env python3
"""How much host time shows in a training step: eager forward+backward+Adam vs
the same forward+backward captured once in a HIP graph and replayed (Adam eager).
python tools/graph_probe.py"""
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
    B, K, H, W = 8, 4, 480, 640
    m = KeypointsGauss(K, H, W, pretrained=False).to(dev)
    x = recipe.to_tensor_nchw(recipe.seeded_images_u8(B, H, W, 1)).to(dev)
    uv = torch.from_numpy(recipe.seeded_keypoints(B, K, H, W, 2)).to(dev)
    t = train.Trainer(m)
    for _ in range(3):
        t.step(x, uv)
    torch.cuda.synchronize()

    def eager(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            t.step(x, uv)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n

    def host_only(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            t.step(x, uv)
        dt = (time.perf_counter() - t0) / n
        torch.cuda.synchronize()
        return dt

    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops._sk_workspace()                  # stream-K workspace of the capture stream, outside the graph
        t.forward_backward(x, uv=uv)         # warm the capture stream's caches
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        t.forward_backward(x, uv=uv)
    torch.cuda.synchronize()

    def graphed(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            g.replay()
            t.opt.step()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n

    for rnd in range(3):
        e = eager(20)
        h = host_only(20)
        gr = graphed(20)
        print("eager %.3f ms (%.1f img/s)  host enqueue %.3f ms  graph+adam %.3f ms (%.1f img/s)" % (
            e * 1e3, B / e, h * 1e3, gr * 1e3, B / gr), flush=True)


if __name__ == "__main__":
    main()
