#!/usr/bin/env python3
"""Merge rocprofv3 --pmc passes (rocpd SQLite DBs under DIR/pass*/) into one
JSON: {kernel: {counter: mean value per dispatch, ..., "dispatches": n,
"avg_duration_ns": d}} and print derived ratios for the conv kernels.

    python tools/pmc_summary.py gpurun_out/pmc16i profiles/r01_infer_c2_pmc_v3_x3.json

HBM bytes per dispatch on gfx950 = (FETCH_SIZE * 2 + WRITE_SIZE) * 1024
(FETCH_SIZE counts half of a wide read; MI355X_MICROARCH.md §HBM).
"""
import glob
import json
import os
import sqlite3
import sys


def collect(d):
    out = {}
    for db in sorted(glob.glob(os.path.join(d, "pass*", "*.db"))):
        con = sqlite3.connect(db)
        for name, ctr, val, n in con.execute(
                "select kernel_name, counter_name, sum(value), count(distinct dispatch_id) "
                "from counters_collection group by kernel_name, counter_name"):
            k = out.setdefault(name, {})
            k[ctr] = val / n
            k["dispatches"] = max(k.get("dispatches", 0), n)
        for name, dur in con.execute("select name, avg(duration) from kernels group by name"):
            if name in out:
                out[name].setdefault("avg_duration_ns", dur)
    return out


def main():
    data = collect(sys.argv[1])
    if len(sys.argv) > 2:
        json.dump(data, open(sys.argv[2], "w"), indent=1, sort_keys=True)
    for name, c in data.items():
        print(name[:80], "x%d" % c.get("dispatches", 0))
        g = c.get
        if g("SQ_WAVE_CYCLES"):
            wc = c["SQ_WAVE_CYCLES"]
            print("  wait_any %.2f  wait_inst %.2f  active %.2f (of wave cycles)" % (
                g("SQ_WAIT_ANY", 0) / wc, g("SQ_WAIT_INST_ANY", 0) / wc, g("SQ_ACTIVE_INST_ANY", 0) / wc))
        if g("SQ_VALU_MFMA_BUSY_CYCLES") and g("GRBM_GUI_ACTIVE"):
            # SQ_VALU_MFMA_BUSY_CYCLES sums over all 1024 SIMDs; GRBM_GUI_ACTIVE over the 8 XCDs
            print("  mfma busy %.3f of SIMD-cycles" % (c["SQ_VALU_MFMA_BUSY_CYCLES"] /
                                                     (1024 * c["GRBM_GUI_ACTIVE"] / 8)))
        if g("SQ_LDS_IDX_ACTIVE"):
            print("  lds bank-conflict %.3f of LDS cycles" % (g("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"]))
        if g("FETCH_SIZE") is not None and g("WRITE_SIZE") is not None:
            print("  HBM %.1f MB per dispatch" % ((c["FETCH_SIZE"] * 2 + c["WRITE_SIZE"]) * 1024 / 1e6))
        if g("TCC_HIT_sum") is not None:
            print("  L2 hit %.3f" % (c["TCC_HIT_sum"] / max(1, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])))


if __name__ == "__main__":
    main()
