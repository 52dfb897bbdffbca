#!/bin/bash
# forward tests, then C2 inference bench with two lanes (default) vs one (HKP_LANES=1), interleaved.
set -e
mkdir -p gpurun_out/lanes
timeout -k 10 400 python -u -m pytest tests/test_gpu_forward.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lanes/fwd.log 2>&1
for rep in 1 2; do
  HKP_LANES=2 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/lanes/two_$rep.log 2>  timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/lanes/two_$rep.log 2>&11
  HKP_LANES=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/lanes/one_$rep.log 2>&1
done
