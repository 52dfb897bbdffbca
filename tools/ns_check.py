#!/usr/bin/env python3
"""bench.py's north_star leg step by step (the 64-image batch, then rank 7's
8-image shard), printing each leg's img/s, its event-timed conv kernels and the
tile-plan misses — to see what the shard leg launches after the batch-64 leg.

    python tools/ns_check.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "hulk-keypoints_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    from hkp import net
    sys.argv = ["bench.py"]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    for name, b, shard in (("b64", 64, (64, 0)), ("b8-shard7", 8, (64, 7)), ("b8-own", 8, None)):
        leg = bench.run_leg("infer", "f16x3", b, args, dev, 0, 1, 10, 3, shard_of=shard)
        r = leg["roofline"]
        print("%-10s %.1f img/s  dominant %s  launches/step %s" % (name, leg["value"], r["kernel"],
                                                                   r.get("launches_per_step")), flush=True)
        print("   plan misses so far:", len(net.PLAN_MISSES), flush=True)


if __name__ == "__main__":
    main()
