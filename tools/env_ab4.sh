#!/bin/bash
# Bench of up to four environment settings on one box, interleaved, twice:
#   tools/env_ab4.sh MODE "A=1 B=2" "A=0" ...   -> gpurun_out/envab4/<i>_<rep>.log
set -e
O=gpurun_out/envab4
mkdir -p $O
MODE=$1; shift
for rep in 1 2; do
  i=0
  for e in "$@"; do
    env $e timeout -k 10 200 python -u bench.py --mode $MODE --no-cpu-baseline > $O/${i}_$rep.log 2>&1
    i=$((i+1))
  done
done
