#!/bin/bash
# One GPU-box pass: gpu tests, C2 inference + C3-shard training bench, kernel-trace stats of both.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_infer.log 2>&1
timeout -k 10 300 python -u bench.py --mode train --no-cpu-baseline > gpurun_out/bench_train.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_infer -o run -- python3 bench.py --steps 10 --no-cpu-baseline > gpurun_out/prof_infer.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -o run -- python3 bench.py --mode train --steps 10 --no-cpu-baseline > gpurun_out/prof_train.log 2>&1
