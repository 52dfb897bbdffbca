#!/bin/bash
# Bench A/B of environment settings on one box, interleaved, twice; prints value per setting:
#   tools/ab.sh "BENCH ARGS" "ENV_A" "ENV_B" ...   (use "X=0" for the default)
set -e
O=gpurun_out/ab
mkdir -p $O
ARGS=$1; shift
for rep in 1 2; do
  i=0
  for e in "$@"; do
    env $e timeout -k 10 200 python -u bench.py $ARGS --no-extras --no-cpu-baseline > $O/${i}_$rep.log 2>&1
    python3 -c "import json,sys; d=json.loads(open('$O/${i}_$rep.log').read().strip().splitlines()[-1]); print('%-40s rep $rep  %8.1f img/s  %7.3f ms  %s %.3f' % ('$e', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac']))"
    i=$((i+1))
  done
done
