#!/bin/bash
# Host-path A/B of the training step (cached Adam table / prepack launch on vs off).
set -e
mkdir -p gpurun_out/host
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py --mode train --no-cpu-baseline > gpurun_out/host/fast_$rep.log 2>&1
  HKP_ADAM_NO_FAST=1 HKP_NO_PREPACK_PLAN=1 timeout -k 10 200 python -u bench.py --mode train --no-cpu-baseline > gpurun_out/host/slow_$rep.log 2>&1
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/host/prof -o run -- python3 bench.py --mode train --steps 10 --no-cpu-baseline > gpurun_out/host/prof.log 2>&1
