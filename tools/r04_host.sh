#!/bin/bash
# Host enqueue cost per step (tools/host_cost.py) for C3-shard training and C2
# inference, with a cProfile of the training enqueue; bench lines without the
# launch observer in the timed region.  Output under gpurun_out/host/.
set -e
O=gpurun_out/host; mkdir -p $O
timeout -k 10 300 python -u tools/host_cost.py --mode train --steps 10 --profile > $O/train.log 2>&1
head -1 $O/train.log
timeout -k 10 300 python -u tools/host_cost.py --mode infer --steps 10 > $O/infer.log 2>&1
head -1 $O/infer.log
timeout -k 10 300 python -u bench.py --mode train --no-cpu-baseline > $O/bench_train.log 2>&1
timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline > $O/bench_infer.log 2>&1
grep -o '"value": [0-9.]*' $O/bench_train.log $O/bench_infer.log
