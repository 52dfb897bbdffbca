#!/bin/bash
# C4 iteration: precision tests, C4 bench, C4 kernel trace.
set -o pipefail
export TMPDIR=/tmp
T=${1:-c4}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_precision.py -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$T/pytest.log; exit 1; }
timeout -k 10 300 python -u bench.py --backbone resnet50 --keypoints 8 --batch 128 --precision f16 --no-extras --no-cpu-baseline > gpurun_out/$T/bench.log 2>&1 || exit 1
bash tools/prof_c4.sh $T/prof
