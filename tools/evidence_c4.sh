#!/bin/bash
# C4 evidence pass (tag $1): bench line, kernel-trace stats, PMC passes of the conv kernels.
set -e
T=${1:?tag}
O=gpurun_out/$T
export TMPDIR=/tmp
mkdir -p $O
A="--backbone resnet50 --keypoints 8 --batch 128 --precision f16"
timeout -k 10 300 python -u bench.py $A --no-cpu-baseline > $O/bench_c4.log 2>&1
echo "bench ok"
bash tools/prof_c4.sh $T/prof_c4
echo "trace ok"
bash tools/pmc_passes.sh $O/pmc_c4 "$A --steps 3 --warmup 1 --no-extras" "conv_x3"
echo "pmc ok"
