#!/usr/bin/env python3
"""One step's kernel sequence from a rocprofv3 --kernel-trace rocpd database:
the last `--per-step` launches' names, grids and durations, in launch order, so
each conv launch can be mapped to its layer.

    python tools/step_breakdown.py gpurun_out/prof_infer/run_results.db [--match conv_x3] [--steps 10]
"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else ""
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 25
    con = sqlite3.connect(db)
    rows = con.execute("select name, grid_x, grid_y, grid_z, workgroup_x, duration, stream_id from kernels "
                       "order by start").fetchall()
    per = len(rows) // steps
    last = rows[-per:]
    tot = sum(r[5] for r in last)
    print("launches/step %d, kernel time/step %.3f ms" % (per, tot / 1e6))
    for n, gx, gy, gz, wx, d, s in last:
        if match in n:
            short = n.replace("void ", "").replace("hkp::", "").split("(")[0][:48]
            print("%-48s grid %7d x%4d x%3d wg %4d  s%d %8.1f us" % (short, gx // max(wx, 1), gy, gz, wx, s, d / 1e3))


if __name__ == "__main__":
    main()
