#!/bin/bash
# GPU-box A/B pass: x3 conv parity tests, then the in-process conv variant A/B.
#   tools/ab_run.sh "<conv_ab.py args>"
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_precision.py -x -q --timeout 120 --timeout-method thread -k "x3" > gpurun_out/ab_pytest.log 2>&1
timeout -k 10 400 python -u tools/conv_ab.py $1 > gpurun_out/ab.log 2>&1
