#!/usr/bin/env python3
"""One step's kernel sequence from a rocprofv3 --kernel-trace rocpd database:
the last `--per-step` launches' names, grids and durations, in launch order, so
each conv launch can be mapped to its layer.

    python tools/step_breakdown.py gpurun_out/prof_infer/run_results.db [--match conv_x3] [--steps 10]

With --walls: the last step's launches with their start offset from the step's
first launch, stream and duration (wall-clock order; concurrent side-stream
kernels show as overlapping intervals).

With --timeline: per-step wall (first start to last end of the step's launches),
the union of kernel intervals (GPU busy), idle gaps, and how much kernel time ran
concurrently (side-stream overlap), by stream; plus the largest idle gaps and the
kernels that precede them.
"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else ""
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 25
    con = sqlite3.connect(db)
    if "--timeline" in sys.argv:
        return timeline(con, steps)
    if "--last-step" in sys.argv:
        return last_step(con, match)
    if "--walls" in sys.argv:
        return walls(con, match)
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


def _marker(rows):
    if "--marker" in sys.argv:
        return sys.argv[sys.argv.index("--marker") + 1]
    return "heat_loss_kernel" if any("heat_loss_kernel" in r[0] for r in rows) else "argmax_decode_kernel"


def last_step(con, match):
    """Every launch of the last complete step (between the last two marker
    launches), in launch order, with a running total."""
    rows = con.execute("select name, grid_x, workgroup_x, end - start from kernels order by start").fetchall()
    marker = _marker(rows)
    idx = [i for i, r in enumerate(rows) if marker in r[0]]
    if len(idx) < 2:
        raise SystemExit("fewer than two %s launches" % marker)
    last = rows[idx[-2] + 1:idx[-1] + 1]
    tot, run = sum(r[3] for r in last), 0
    print("launches/step %d, kernel time/step %.3f ms" % (len(last), tot / 1e6))
    for n, gx, wx, d in last:
        run += d
        if match in n:
            short = n.replace("void ", "").replace("hkp::", "").split("(")[0][:56]
            print("%-56s grid %7d wg %4d %8.1f us  cum %7.3f ms" % (short, gx // max(wx, 1), wx, d / 1e3, run / 1e6))


def walls(con, match):
    rows = con.execute("select name, start, end, stream_id, grid_x, workgroup_x from kernels order by start").fetchall()
    marker = _marker(rows)
    idx = [i for i, r in enumerate(rows) if marker in r[0]]
    if len(idx) < 2:
        raise SystemExit("fewer than two %s launches" % marker)
    last = rows[idx[-2] + 1:idx[-1] + 1]
    t0 = last[0][1]
    print("step wall %.3f ms; start / end offsets (us), stream, duration" % ((max(r[2] for r in last) - t0) / 1e6))
    for n, s_, e, st, gx, wx in last:
        if match in n:
            short = n.replace("void ", "").replace("hkp::", "").split("(")[0][:52]
            print("%9.1f %9.1f  s%-2s %8.1f us  grid %6d  %s" % ((s_ - t0) / 1e3, (e - t0) / 1e3, st, (e - s_) / 1e3,
                                                               gx // max(wx, 1), short))


def timeline(con, steps):
    """The step is the launches after the second-to-last marker kernel (one per
    step: heat_loss_kernel in training, argmax_decode_kernel in
    inference) through the last one."""
    rows = con.execute("select name, start, end, stream_id from kernels order by start").fetchall()
    marker = sys.argv[sys.argv.index("--marker") + 1] if "--marker" in sys.argv else None
    if marker is None:
        marker = "heat_loss_kernel" if any("heat_loss_kernel" in r[0] for r in rows) else "argmax_decode_kernel"
    idx = [i for i, r in enumerate(rows) if marker in r[0]]
    if len(idx) < 2:
        raise SystemExit("fewer than two %s launches" % marker)
    last = rows[idx[-2] + 1:idx[-1] + 1]
    per = len(last)
    t0, t1 = last[0][1], max(r[2] for r in last)
    busy, cur_s, cur_e, gaps = 0, None, None, []
    prev_name = None
    for n, s, e, _ in last:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append((s - cur_e, prev_name))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        prev_name = n
    busy += cur_e - cur_s
    tot = sum(e - s for _, s, e, _ in last)
    by_stream = {}
    for n, s, e, st in last:
        by_stream[st] = by_stream.get(st, 0) + (e - s)
    wall = t1 - t0
    print("launches/step %d; step wall %.3f ms, GPU busy %.3f ms (%.1f %%), idle %.3f ms in %d gaps; "
          "kernel time %.3f ms (%.2fx the busy time)" % (per, wall / 1e6, busy / 1e6, 100 * busy / wall,
                                                           (wall - busy) / 1e6, len(gaps), tot / 1e6, tot / busy))
    for st, t in sorted(by_stream.items()):
        print("  stream %s: %.3f ms of kernels" % (st, t / 1e6))
    gaps.sort(key=lambda g: -g[0])
    print("largest idle gaps:")
    for g, n in gaps[:12]:
        print("  %7.1f us after %s" % (g / 1e3, n.replace("void ", "").replace("hkp::", "").split("(")[0][:70]))


if __name__ == "__main__":
    main()
