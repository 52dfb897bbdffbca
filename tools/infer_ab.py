#!/usr/bin/env python3
"""In-process A/B of inference policies (bench.py's C2 step by default: R34-8s
K=4 640x480 B=32, f16x3; --backbone resnet50 --keypoints 8 --batch 128
--precision f16 for C4): one model, the Policy switched between rounds, forms
interleaved round-robin, wall time of `--iters` forwards (heatmaps + argmax)
between two synchronisations; median per form (img/s).

    python tools/infer_ab.py "" "x3_tile=9"
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


KNOBS = {"store": ("hkp_debug_x3_store", 0), "prio": ("hkp_debug_x3_prio", 0), "stem_pair": ("hkp_debug_stem_pair", 0),
         "finregs": ("hkp_debug_fin_regs", 1), "pair128": ("hkp_debug_x3_pair128", 1),
         "stem_img": (None, 1)}


def knobs(form):
    d = dict(i.partition("=")[::2] for i in filter(None, form.split(",")))
    return {k: int(d.get(k, dflt)) for k, (_, dflt) in KNOBS.items()}


def set_knobs(lib, kv):
    for k, v in kv.items():
        if k == "stem_img":                     # a Python-side switch (hkp.ops), not a library knob
            from hkp import ops
            ops.STEM_IMAGE_DIRECT = bool(v)
        elif hasattr(lib, KNOBS[k][0]):
            getattr(lib, KNOBS[k][0])(v)
        elif v != KNOBS[k][1]:      # the product library has no knobs (include/hulkkp_ab.h)
            raise SystemExit("knob %s=%d needs the A/B build: make -C hulk-keypoints_amd/csrc ab, then --ab"
                             % (k, v))


def parse(form):
    """Policy overrides of a form; the pseudo-fields store=K, prio=K and stem_pair=K
    are library debug knobs (hkp_debug_x3_store / _x3_prio / _stem_pair), not
    Policy fields."""
    from hkp.policy import DEFAULT
    kw = {}
    for item in filter(None, form.split(",")):
        k, _, v = item.partition("=")
        if k in KNOBS:
            continue
        cur = getattr(DEFAULT, k)
        kw[k] = (v.lower() in ("1", "true", "yes")) if isinstance(cur, bool) else type(cur)(v)
    return kw


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("forms", nargs="+", help="comma-separated FIELD=VALUE Policy overrides per form ('' = default)")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--backbone", default="resnet34")
    ap.add_argument("--keypoints", type=int, default=4)
    ap.add_argument("--precision", default="f16x3")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--ab", action="store_true", help="load the A/B build (tools/ab_lib, its hkp_debug_* knobs)")
    args = ap.parse_args()
    if args.ab:
        from hkp import _lib
        _lib.use_ab_library()
    import hkp
    from hkp.policy import Policy
    from oracle import recipe
    from src.model import KeypointsGauss
    hkp.lib()
    dev = torch.device("cuda", 0)
    B, K, H, W = args.batch, args.keypoints, 480, 640
    torch.manual_seed(1234)
    base = Policy(precision=args.precision)
    model = KeypointsGauss(K, H, W, backbone=args.backbone, pretrained=False, policy=base).to(dev)
    x = recipe.to_tensor_nchw(recipe.seeded_images_u8(B, H, W, 1234)).to(dev)

    def step():
        with torch.no_grad():
            return model.heatmaps_and_keypoints(x)
    pols = [base.with_(**parse(f)) for f in args.forms]
    kns = [knobs(f) for f in args.forms]
    for p, kv in zip(pols, kns):      # warm every form (kernels, caches, plans)
        model.policy = p
        set_knobs(hkp.lib(), kv)
        for _ in range(3):
            step()
    torch.cuda.synchronize()
    res = {f: [] for f in args.forms}
    for _ in range(args.rounds):
        for f, p, kv in zip(args.forms, pols, kns):
            model.policy = p
            set_knobs(hkp.lib(), kv)
            step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.iters):
                step()
            torch.cuda.synchronize()
            res[f].append(B * args.iters / (time.perf_counter() - t0))
    set_knobs(hkp.lib(), knobs(""))
    for f in args.forms:
        print("%-40s %.1f img/s  (%s)" % (f or "(default)", statistics.median(res[f]),
                                          " ".join("%.1f" % v for v in res[f])), flush=True)


if __name__ == "__main__":
    main()
