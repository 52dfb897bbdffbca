#!/bin/bash
# Interleaved bench.py A/B in one gpurun call (separate processes, same box):
#   tools/bench_ab.sh <tag> "<bench args A>" "<bench args B>" [reps]
# Lines go to gpurun_out/ab_<tag>/{A,B}_<rep>.log; a summary to gpurun_out/ab_<tag>/summary.txt.
set -o pipefail
tag=$1; A=$2; B=$3; reps=${4:-2}
out=gpurun_out/ab_$tag; mkdir -p $out
for r in $(seq 1 $reps); do
    for v in A B; do
        args=$A; [ $v = B ] && args=$B
        timeout -k 10 300 python bench.py --no-extras --no-cpu-baseline $args > $out/${v}_$r.log 2>&1 || exit $?
    done
done
python - "$out" <<'PY'
import json, sys, glob, os
out = sys.argv[1]
for v in "AB":
    vals = []
    for f in sorted(glob.glob(os.path.join(out, v + "_*.log"))):
        for l in open(f):
            if l.startswith("{"):
                vals.append(json.loads(l)["value"])
    print(v, " ".join("%.1f" % x for x in vals), file=open(os.path.join(out, "summary.txt"), "a"))
PY
cat $out/summary.txt
