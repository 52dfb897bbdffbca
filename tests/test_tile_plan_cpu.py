"""The measured forward tile plan (hulk-keypoints_amd/hkp/tile_plan.json, written
by tools/tile_sweep.py from in-process timings of every live HKP_TILE_* policy
per conv shape): every entry's chosen policy is its measured argmin under the
sweep's hysteresis (the C planner kept unless beaten by more than it), the
table covers the C2 / B=8-shard / C3-shard / C4 / C5 workloads, and the network
reads it (hkp.net._planned_tile)."""
import json
import os

import pytest

from conftest import PKG

TABLE = os.path.join(PKG, "hkp", "tile_plan.json")
KINDS = ("x3", "f16", "f16bn")


def _doc():
    if not os.path.exists(TABLE):
        pytest.skip("no tile plan table")
    return json.load(open(TABLE))


def test_plan_is_the_measured_argmin():
    doc = _doc()
    hyst = float(doc["hysteresis"])
    assert doc["shapes"]
    for key, ent in doc["shapes"].items():
        f = key.split("|")
        assert len(f) == 10 and f[0] in KINDS and all(v.isdigit() for v in f[1:]), key
        ms = {int(t): v for t, v in ent["ms"].items()}
        assert 0 in ms and all(v > 0 for v in ms.values()), key
        best = min(ms, key=lambda t: (ms[t], t))
        want = best if ms[best] < ms[0] * (1.0 - hyst) else 0
        assert ent["tile"] == want, (key, ent)


def test_plan_keeps_the_planners_distinct_kernels():
    """A planned policy launches another kernel than the planner's (a policy a shape
    does not take plans as AUTO), and shapes the planner puts on the halo body stay
    there: the fused-input-BN conv runs exactly where the unfused one runs it."""
    import ctypes  # noqa: F401
    import sys
    sys.path.insert(0, PKG)
    from hkp import ops
    from hkp._lib import HKP_KOP_FWD_F16, HKP_KOP_FWD_X3, ConvDesc
    doc = _doc()
    for key, ent in doc["shapes"].items():
        kind, n, h, w, cin, cout, k, st, pd, dl = key.split("|")
        if kind == "f16bn" or ent["tile"] == 0:
            continue
        kop = HKP_KOP_FWD_X3 if kind == "x3" else HKP_KOP_FWD_F16
        args = [int(v) for v in (n, h, w, cin, cout, k, k, st, pd, dl)] + [0]
        planner = ops.kernel_name(ConvDesc(*args, 0), kop)
        planned = ops.kernel_name(ConvDesc(*args, ent["tile"]), kop)
        assert planned != planner and not planner.startswith("conv_x3_halo"), (key, planner, planned)


def test_plan_covers_the_workloads():
    doc = _doc()
    seen = set()
    for ent in doc["shapes"].values():
        seen.update(ent["workloads"])
    assert {"c2", "b8", "c3", "c4", "c5"} <= seen, seen


def test_network_reads_the_plan():
    import sys
    sys.path.insert(0, PKG)
    import torch
    from hkp import net
    from hkp.policy import DEFAULT
    doc = _doc()
    key, ent = next(iter(doc["shapes"].items()))
    kind, n, h, w, cin, cout, k, st, pd, dl = key.split("|")

    class Conv:
        weight = torch.empty(int(cout), int(k), int(k), int(cin))
        stride, padding, dilation = int(st), int(pd), int(dl)
    c = int(cin) * (2 if kind == "x3" else 1)
    shape = (int(n), int(h), int(w), c)
    assert net.plan_key(kind, shape, Conv) == key
    assert net._planned_tile(kind, shape, Conv, DEFAULT, 0) == ent["tile"]
    assert net._planned_tile(kind, shape, Conv, DEFAULT, 5) == 5                   # a forced policy wins
    assert net._planned_tile(kind, shape, Conv, DEFAULT.with_(tile_plan=False), 0) == 0
