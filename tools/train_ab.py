#!/usr/bin/env python3
"""In-process A/B of training-step policies (bench.py's C3-shard step by
default: R34-8s K=4 640x480 B=8): one model and Trainer, the Policy switched
between rounds, forms interleaved round-robin, wall time of `--iters` steps
between two synchronisations; median per form (img/s).

    python tools/train_ab.py "overlap_min_gflop=0" "overlap_min_gflop=20" "overlap_wgrad=0"
"""
import argparse
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "hulk-keypoints_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


from infer_ab import KNOBS, knobs, set_knobs  # noqa: E402  (tools/ is on sys.path when run as a script)


# pseudo-fields handled here: mainprio=P runs the step on a stream of priority P
# (torch: lower = higher priority; 0 = the default stream's), sideprio=P recreates
# the wgrad side stream with priority P
STREAM_KNOBS = ("mainprio", "sideprio")


def stream_knobs(form):
    d = dict(item.partition("=")[::2] for item in filter(None, form.split(",")))
    return {k: int(d[k]) for k in STREAM_KNOBS if k in d}


def parse(form):
    """Policy overrides of a form; the pseudo-fields store=K, prio=K and stem_pair=K
    are library debug knobs (infer_ab.KNOBS), not Policy fields."""
    from hkp.policy import DEFAULT
    kw = {}
    for item in filter(None, form.split(",")):
        k, _, v = item.partition("=")
        if k in KNOBS or k in STREAM_KNOBS:
            continue
        cur = getattr(DEFAULT, k)
        kw[k] = (v.lower() in ("1", "true", "yes")) if isinstance(cur, bool) else type(cur)(v)
    return kw


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("forms", nargs="+", help="comma-separated FIELD=VALUE Policy overrides per form ('' = default)")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--backbone", default="resnet34")
    ap.add_argument("--keypoints", type=int, default=4)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--ab", action="store_true", help="load the A/B build (tools/ab_lib, its hkp_debug_* knobs)")
    args = ap.parse_args()
    if args.ab:
        from hkp import _lib
        _lib.use_ab_library()
    import hkp
    from hkp import train as hkp_train
    from hkp.policy import Policy
    from oracle import recipe
    from src.model import KeypointsGauss
    hkp.lib()
    dev = torch.device("cuda", 0)
    B, K, H, W = args.batch, args.keypoints, args.height, args.width
    torch.manual_seed(1234)
    base = Policy()
    model = KeypointsGauss(K, H, W, backbone=args.backbone, pretrained=False, policy=base).to(dev)
    x = recipe.to_tensor_nchw(recipe.seeded_images_u8(B, H, W, 1234)).to(dev)
    uv = torch.from_numpy(recipe.seeded_keypoints(B, K, H, W, 99)).to(dev)
    trainer = hkp_train.Trainer(model, lr=1e-4, weight_decay=1e-4)
    pols = [base.with_(**parse(f)) for f in args.forms]
    kns = [knobs(f) for f in args.forms]
    from hkp import net as hkp_net
    default_side = hkp_net._side_stream(dev)
    sks = []
    for f in args.forms:
        sk = stream_knobs(f)
        main = torch.cuda.Stream(dev, priority=sk["mainprio"]) if "mainprio" in sk else torch.cuda.current_stream(dev)
        side = torch.cuda.Stream(dev, priority=sk["sideprio"]) if "sideprio" in sk else default_side
        sks.append((main, side))

    def run(n, ms):
        main, side = ms
        hkp_net._side_streams[dev] = side
        main.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(main):
            for _ in range(n):
                trainer.step(x, uv)
        torch.cuda.current_stream(dev).wait_stream(main)

    print("stream priority range", torch.cuda.Stream.priority_range(), flush=True)
    for p, kv, ms in zip(pols, kns, sks):      # warm every form (kernels, caches, plans)
        model.policy = trainer.policy = p
        set_knobs(hkp.lib(), kv)
        run(3, ms)
    torch.cuda.synchronize()
    res = {f: [] for f in args.forms}
    for _ in range(args.rounds):
        for f, p, kv, ms in zip(args.forms, pols, kns, sks):
            model.policy = trainer.policy = p
            set_knobs(hkp.lib(), kv)
            run(1, ms)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(args.iters, ms)
            torch.cuda.synchronize()
            res[f].append(B * args.iters / (time.perf_counter() - t0))
    set_knobs(hkp.lib(), knobs(""))
    for f in args.forms:
        print("%-40s %.1f img/s  (%s)" % (f or "(default)", statistics.median(res[f]),
                                          " ".join("%.1f" % v for v in res[f])), flush=True)


if __name__ == "__main__":
    main()
