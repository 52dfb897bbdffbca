#!/bin/bash
# Round-4 extra measurements (one gpurun call): training dgrad-overlap tile A/B
# (2-stage 256x256 + tail vs the A3 body + tail) and the C5 bench line.
set -o pipefail
O=gpurun_out/r04_extra; mkdir -p $O
bash tools/bench_ab.sh train_a3 "--mode train" "--mode train --tune dgrad_overlap_tile=11" 2 || exit $?
timeout -k 10 600 python -u bench.py --mode train --backbone resnet50 --keypoints 8 --height 960 --width 1280 \
    --batch 32 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_c5.log 2>&1 || exit $?
echo "extra ok"
