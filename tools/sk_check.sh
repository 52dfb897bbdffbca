#!/bin/bash
# Stream-K check on the box: x3 parity tests, in-process conv A/B (knob 9 = never
# stream-K vs 0 = policy), training + inference bench with either knob.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_precision.py -x -q --timeout 120 --timeout-method thread -k "x3" > gpurun_out/sk_pytest.log 2>&1
timeout -k 10 300 python -u tools/conv_ab.py --variants 9,0 --shapes t4,t3,t2,layer3 > gpurun_out/ab_sk.log 2>&1
HKP_X3_VARIANT=9 timeout -k 10 200 python -u bench.py --mode train --no-cpu-baseline > gpurun_out/sk_train_v9.log 2>&1
timeout -k 10 200 python -u bench.py --mode train --no-cpu-baseline > gpurun_out/sk_train_v0.log 2>&1
HKP_X3_VARIANT=9 timeout -k 10 200 python -u bench.py --mode train --no-cpu-baseline > gpurun_out/sk_train_v9b.log 2>&1
timeout -k 10 200 python -u bench.py --mode train --no-cpu-baseline > gpurun_out/sk_train_v0b.log 2>&1
HKP_X3_VARIANT=9 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/sk_infer_v9.log 2>&1
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/sk_infer_v0.log 2>&1
