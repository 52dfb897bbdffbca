#!/bin/bash
# Per-launch breakdown of one C4 (R50 K8 B128 fp16) and one C2 step on the box:
# GPU suite first (the tree is green), then rocprofv3 kernel traces whose last
# step tools/step_breakdown.py lists launch by launch.  Output under gpurun_out/$1/.
set -e
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
export TMPDIR=/tmp
mkdir -p $O
C4="--backbone resnet50 --keypoints 8 --batch 128 --precision f16"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo "pytest ok: $(tail -1 $O/pytest_gpu.log)"
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_c4 -o run -- python3 bench.py $C4 --steps 3 --warmup 2 --no-extras --no-cpu-baseline > $O/prof_c4.log 2>&1
python3 tools/step_breakdown.py $O/prof_c4/run_results.db --last-step > $O/c4_breakdown.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_c2 -o run -- python3 bench.py --steps 3 --warmup 2 --no-extras --no-cpu-baseline > $O/prof_c2.log 2>&1
python3 tools/step_breakdown.py $O/prof_c2/run_results.db --last-step > $O/c2_breakdown.txt
rm -rf $O/prof_c4 $O/prof_c2
echo "breakdown ok"
