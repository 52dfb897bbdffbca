#!/bin/bash
# Bench A/B of variants on one box, interleaved, twice; prints value per variant:
#   tools/ab.sh "BENCH ARGS" "VARIANT A ARGS" "VARIANT B ARGS" ...
# A variant is extra bench.py arguments: "" (the default policy),
# "--tune overlap_wgrad=0" (a non-default hkp.policy.Policy tuning field),
# "--lib tools/bin/libhulkkp_x.so" (another build of the library).
set -e
O=gpurun_out/ab
mkdir -p $O
ARGS=$1; shift
for rep in 1 2; do
  i=0
  for v in "$@"; do
    timeout -k 10 200 python -u bench.py $ARGS $v --no-extras --no-cpu-baseline > $O/${i}_$rep.log 2>&1
    python3 -c "import json,sys; d=json.loads(open('$O/${i}_$rep.log').read().strip().splitlines()[-1]); print('%-40s rep $rep  %8.1f img/s  %7.3f ms  %s %.3f' % ('$v', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac']))"
    i=$((i+1))
  done
done
