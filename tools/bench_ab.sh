#!/bin/bash
# Bench A/B on one box: tools/bench_ab.sh KNOB_A KNOB_B — C2 inference and
# C3-shard training, each under HKP_X3_VARIANT=A then B, twice, interleaved.
set -e
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for v in $1 $2; do
    HKP_X3_VARIANT=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/ab/infer_v${v}_$rep.log 2>&1
    HKP_X3_VARIANT=$v timeout -k 10 200 python -u bench.py --mode train --no-cpu-baseline > gpurun_out/ab/train_v${v}_$rep.log 2>&1
  done
done
