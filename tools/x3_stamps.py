#!/usr/bin/env python3
"""Per-block phase timeline of the one-tile x3/fp16 conv (hkp_debug_x3_stamps):
runs a conv shape once warm, then once with stamps, and prints the median
per-block phase durations (us) and the launch span.

    python tools/x3_stamps.py c4_l4_c3 [c4_l1_c3 ...]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "hulk-keypoints_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))

import torch  # noqa: E402

from conv_ab import SHAPES  # noqa: E402

PHASES = ["fill", "kloop", "partials|stores(x3)", "stage|partials(x3)", "store"]


def main():
    from hkp import ops
    from hkp import _lib
    _lib.use_ab_library()                       # the hkp_debug_* knobs (include/hulkkp_ab.h)
    from hkp._lib import lib
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    args = sys.argv[1:]
    tile = 0
    if "--tile" in args:                 # HKP_TILE_* (e.g. 13: the DUO body)
        i = args.index("--tile")
        tile = int(args[i + 1])
        del args[i:i + 2]
    if "--duo-stagger" in args:          # hkp_debug_duo_stagger (ns; 0 off, < 0 default)
        i = args.index("--duo-stagger")
        lib().hkp_debug_duo_stagger(int(args[i + 1]))
        del args[i:i + 2]
    for name in args:
        if name.startswith("stem"):          # stem[:N]: the 7x7/s2 stem (hkp_conv2d_fwd_stem_x3), batch N (32)
            n = int(name.partition(":")[2] or 32)
            prec, h, w, ci, co, k, st, pd, dl = "stem", 480, 640, 3, 64, 7, 2, 3, 1
        else:
            prec, n, h, w, ci, co, k, st, pd, dl = SHAPES[name]
        if prec == "stem":
            img = torch.randint(0, 256, (n, h, w, 3), device=dev, dtype=torch.uint8, generator=g)
            wp = ops.stem_weight_pack_x3(torch.randn(co, ci, k, k, device=dev, generator=g) * 0.05)
            run = lambda: ops.conv2d_fwd_stem_x3(img, wp, co, tile=tile)  # noqa: E731
        elif prec == "x3":
            x = torch.relu(torch.randn(n, h, w, ci, device=dev, generator=g))
            wt = torch.randn(co, k, k, ci, device=dev, generator=g) * (2.0 / (k * k * co)) ** 0.5
            ss = torch.cat([torch.ones(ci, device=dev), torch.zeros(ci, device=dev)])
            xs = ops.bn_apply(x, ss, relu=False, split=3, keep_fp32=False)
            ws = ops.weight_pack_x3(wt)
            run = lambda: ops.conv2d_fwd_x3(xs, ws, st, pd, dl, sk=False, tile=tile)  # noqa: E731
        else:
            x = torch.relu(torch.randn(n, h, w, ci, device=dev, generator=g))
            wt = torch.randn(co, k, k, ci, device=dev, generator=g) * (2.0 / (k * k * co)) ** 0.5
            xs = x.half()
            ws = ops.weight_pack_f16(wt)
            run = lambda: ops.conv2d_fwd_f16(xs, ws, st, pd, dl, sk=False, tile=tile)  # noqa: E731
        for _ in range(3):
            run()
        ho, wo = ops.conv_out_hw(h, w, k, k, st, pd, dl)
        blocks = ((n * ho * wo + 255) // 256) * (co // 64) * 2 + 64
        buf = torch.zeros(blocks * 8, dtype=torch.int64, device=dev)
        lib().hkp_debug_x3_stamps(buf.data_ptr())
        run()
        torch.cuda.synchronize()
        lib().hkp_debug_x3_stamps(None)
        s = buf.view(-1, 8).cpu()
        s = s[s[:, 0] != 0].double()
        t0 = s[:, 0].min()
        span = (s[:, 5].max() - t0) / 100.0
        out = []
        for i, ph in enumerate(PHASES):
            d = (s[:, i + 1] - s[:, i]) / 100.0
            out.append("%s %.2f" % (ph, d.median().item()))
        tot = ((s[:, 5] - s[:, 0]) / 100.0).median().item()
        print("%-9s tile %d blocks %d  span %.1f us  per-block median total %.2f us: %s" % (
            name, tile, s.shape[0], span.item(), tot, ", ".join(out)), flush=True)
        if tile == 13:
            # DUO (two blocks per CU): which first-round blocks share a CU (slot 6 = HW_ID,
            # slot 7 = XCC_ID, recorded by the DUO body), and how far apart they start
            full = buf.view(-1, 8).cpu()
            idx = torch.nonzero(full[:, 0] != 0).flatten()
            st0 = full[idx, 0].double()
            first = idx[(st0 - st0.min()) / 100.0 < 2.0]             # blocks started within 2 us
            cu = {}
            for b in first.tolist():
                hw, xcc = int(full[b, 6]), int(full[b, 7])
                key = (xcc & 0xF, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 0xF)
                cu.setdefault(key, []).append(b)
            pairs = [sorted(v) for v in cu.values() if len(v) == 2]
            diffs = {}
            for p in pairs:
                diffs[p[1] - p[0]] = diffs.get(p[1] - p[0], 0) + 1
            print("          first-round blocks %d on %d CUs; blocks per CU %s; pair index gaps (count) %s"
                  % (len(first), len(cu), sorted({len(v) for v in cu.values()}),
                     sorted(diffs.items(), key=lambda kv: -kv[1])[:6]))
            print("          sample pairs %s" % pairs[:8])
            # phase of the two slots of a CU over the whole launch: gap between
            # consecutive block starts on one CU / block lifetime (0 = in lockstep,
            # 0.5 = half a block apart)
            allcu = {}
            for b in idx.tolist():
                hw, xcc = int(full[b, 6]), int(full[b, 7])
                key = (xcc & 0xF, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 0xF)
                allcu.setdefault(key, []).append(int(full[b, 0]))
            life = float(((full[idx, 5] - full[idx, 0]) / 100.0).median())
            ph = []
            for v in allcu.values():
                v.sort()
                ph += [min(1.0, (v[i + 1] - v[i]) / 100.0 / life) for i in range(len(v) - 1)]
            ph = torch.tensor(ph)
            print("          start gap on a CU / lifetime: p10 %.2f p50 %.2f p90 %.2f" % (
                ph.quantile(0.1).item(), ph.median().item(), ph.quantile(0.9).item()))
        # start-time spread of consecutive waves of blocks
        starts = ((s[:, 0] - t0) / 100.0).sort().values
        print("          block starts: p10 %.1f p50 %.1f p90 %.1f us" % (
            starts[int(0.1 * len(starts))].item(), starts[len(starts) // 2].item(),
            starts[int(0.9 * len(starts))].item()))


if __name__ == "__main__":
    main()
