#!/usr/bin/env python3
"""Per-kernel time and HBM rate of one bench workload: joins a rocprofv3
--kernel-trace --stats CSV (tools/rocpd_stats.py: calls, average duration) with a
PMC summary of the same command (tools/pmc_summary.py: FETCH_SIZE, WRITE_SIZE,
L2 hits, MFMA busy per dispatch).  HBM bytes per dispatch = (FETCH_SIZE * 2 +
WRITE_SIZE) * 1024 (gfx950: FETCH_SIZE counts half of a wide read,
MI355X_MICROARCH.md §HBM); the rate uses the trace's duration (the PMC passes
serialise kernels and run at another clock).  Achievable HBM: 6.3 TB/s (the
guide's measured float4 copy).

    python tools/hbm_table.py STATS.csv PMC.json --steps 3 [--top 30]
"""
import argparse
import csv
import json

ACHIEVABLE_GBS = 6300.0


def short(name):
    n = name.replace("void ", "").replace("hkp::", "")
    return n.split("(")[0][:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats")
    ap.add_argument("pmc")
    ap.add_argument("--steps", type=int, required=True, help="bench steps the trace covers (timed + warmup + roofline)")
    ap.add_argument("--top", type=int, default=30)
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.stats)))
    pmc = json.load(open(args.pmc))
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    print("%-60s %7s %9s %7s %9s %8s %6s %6s %6s" % ("kernel", "calls", "avg us", "share", "MB/disp", "GB/s",
                                                      "x6.3TB", "L2hit", "mfma"))
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:args.top]:
        name, calls, avg = r["Name"], int(r["Calls"]), float(r["AverageNs"])
        c = pmc.get(name)
        if c is None:       # the trace demangles some names the PMC pass keeps mangled, or vice versa
            c = next((v for k, v in pmc.items() if short(k) == short(name)), None)
        mb = gbs = frac = hit = busy = None
        if c and "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            nb = (c["FETCH_SIZE"] * 2 + c["WRITE_SIZE"]) * 1024
            mb = nb / 1e6
            gbs = nb / (avg * 1e-9) / 1e9
            frac = gbs / ACHIEVABLE_GBS
        if c and c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0) > 0:
            hit = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
        if c and c.get("SQ_VALU_MFMA_BUSY_CYCLES") and c.get("GRBM_GUI_ACTIVE"):
            # sums over the 1024 SIMDs / GRBM_GUI_ACTIVE over the 8 XCDs (tools/pmc_summary.py)
            busy = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * c["GRBM_GUI_ACTIVE"] / 8)

        def f(v, fmt):
            return fmt % v if v is not None else "-"
        print("%-60s %7.1f %9.1f %6.1f%% %9s %8s %6s %6s %6s" % (
            short(name), calls / args.steps, avg / 1e3, 100.0 * float(r["TotalDurationNs"]) / total,
            f(mb, "%.1f"), f(gbs, "%.0f"), f(frac, "%.2f"), f(hit, "%.2f"), f(busy, "%.2f")))


if __name__ == "__main__":
    main()
