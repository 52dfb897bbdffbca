#!/bin/bash
# x3 parity tests + in-process conv A/B:  tools/sk_ab.sh VARIANTS SHAPES
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_precision.py -x -q --timeout 120 --timeout-method thread -k "x3 or stem" > gpurun_out/sk_pytest.log 2>&1
timeout -k 10 300 python -u tools/conv_ab.py --variants $1 --shapes $2 > gpurun_out/ab_sk.log 2>&1
