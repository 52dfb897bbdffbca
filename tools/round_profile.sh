#!/bin/bash
# Full evidence pass on the box (tag $1, e.g. r01_v5): GPU tests, C2 inference and
# C3-shard training bench lines, rocprofv3 kernel-trace stats of both, PMC passes
# of both.  Everything lands under gpurun_out/$1/; copy what is judged to profiles/.
set -e
T=${1:?tag}
O=gpurun_out/$T
export TMPDIR=/tmp
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo "pytest ok"
timeout -k 10 300 python -u bench.py > $O/bench_infer.log 2>&1
timeout -k 10 300 python -u bench.py --mode train --no-cpu-baseline > $O/bench_train.log 2>&1
echo "bench ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_infer -o run -- python3 bench.py --steps 10 --no-extras --no-cpu-baseline > $O/prof_infer.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_train -o run -- python3 bench.py --mode train --steps 10 --no-cpu-baseline > $O/prof_train.log 2>&1
echo "kernel trace ok"
bash tools/pmc_passes.sh $O/pmc_infer "--steps 5 --no-extras" "conv_x3"
bash tools/pmc_passes.sh $O/pmc_train "--mode train --steps 5" "conv_x3|wgrad_x3"
echo "pmc ok"
