#!/bin/bash
# Bench A/B of two environment settings on one box, interleaved, twice:
#   tools/env_ab.sh "HKP_X=1" "HKP_X=0" [train|infer]
set -e
mkdir -p gpurun_out/envab
MODE=${3:-train}
for rep in 1 2; do
  env $1 timeout -k 10 200 python -u bench.py --mode $MODE --no-cpu-baseline > gpurun_out/envab/A_$rep.log 2>&1
  env $2 timeout -k 10 200 python -u bench.py --mode $MODE --no-cpu-baseline > gpurun_out/envab/B_$rep.log 2>&1
done
