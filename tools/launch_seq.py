#!/usr/bin/env python3
"""Print the kernel launch sequence (name, duration, grid) of one step from a
rocprofv3 rocpd database: the launches between the n-th and (n+1)-th
occurrence of a marker kernel (default: the stem pack, first kernel of a step).

    python tools/launch_seq.py gpurun_out/prof_c4_v1/run_results.db [step] [marker]
"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    step = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    marker = sys.argv[3] if len(sys.argv) > 3 else "stem_pack"
    con = sqlite3.connect(db)
    rows = con.execute("select name, start, end, grid_x, workgroup_x from kernels order by start").fetchall()
    starts = [i for i, r in enumerate(rows) if marker in r[0]]
    a, b = starts[step], starts[step + 1] if step + 1 < len(starts) else len(rows)
    tot = 0
    for name, s, e, gx, wx in rows[a:b]:
        tot += e - s
        print("%9.1f us  grid %8d  %s" % ((e - s) / 1e3, gx // max(wx, 1), name[:100]))
    print("total %.3f ms over %d launches" % (tot / 1e6, b - a))


if __name__ == "__main__":
    main()
