#!/usr/bin/env python3
"""Per-kernel statistics (calls, total/avg ns, share) from a rocprofv3 rocpd
SQLite database (rocprofv3 --kernel-trace output), written as the CSV layout of
rocprofv3 --stats (Name,Calls,TotalDurationNs,AverageNs,Percentage,MinNs,MaxNs).

    python tools/rocpd_stats.py gpurun_out/p/run_results.db [out.csv] [--top N]
"""
import csv
import sqlite3
import sys


def kernel_stats(db):
    con = sqlite3.connect(db)
    rows = con.execute("select name, count(*), sum(end - start), min(end - start), max(end - start) "
                       "from kernels group by name").fetchall()
    total = sum(r[2] for r in rows) or 1
    out = [dict(Name=n, Calls=c, TotalDurationNs=t, AverageNs=t / c, Percentage=100.0 * t / total, MinNs=mn,
                MaxNs=mx) for n, c, t, mn, mx in rows]
    return sorted(out, key=lambda r: -r["TotalDurationNs"])


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 25
    if "--top" in sys.argv:
        args = [a for a in args if a != str(top)]
    st = kernel_stats(args[0])
    if len(args) > 1:
        with open(args[1], "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(st[0].keys()))
            w.writeheader()
            w.writerows(st)
    for r in st[:top]:
        print("%6.2f%% %6d %10.1f us  %s" % (r["Percentage"], r["Calls"], r["AverageNs"] / 1e3, r["Name"][:110]))


if __name__ == "__main__":
    main()
