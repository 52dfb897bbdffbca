#!/bin/bash
# Full evidence pass on the box (tag $1, e.g. r03_v1), in two calls that each fit
# gpurun's limit:
#   tools/round_profile.sh TAG        GPU tests; C2 inference, C3-shard training and
#                                     C4 (R50 fp16) bench lines; rocprofv3
#                                     kernel-trace stats of all three
#   tools/round_profile.sh TAG pmc    PMC passes of all three (tools/pmc_passes.sh)
# Everything lands under gpurun_out/$1/; copy what is judged to profiles/.
set -e
T=${1:?tag}
O=gpurun_out/$T
export TMPDIR=/tmp
mkdir -p $O
C4="--backbone resnet50 --keypoints 8 --batch 128 --precision f16"
if [ "${2:-}" = "pmc" ]; then
    bash tools/pmc_passes.sh $O/pmc_infer "--steps 5 --no-extras" "conv_x3"
    bash tools/pmc_passes.sh $O/pmc_train "--mode train --steps 5" "conv_x3|wgrad_x3"
    bash tools/pmc_passes.sh $O/pmc_c4 "$C4 --steps 3 --no-extras" "conv_x3"
    echo "pmc ok"
    exit 0
fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo "pytest ok: $(tail -1 $O/pytest_gpu.log)"
timeout -k 10 300 python -u bench.py > $O/bench_infer.log 2>&1
timeout -k 10 300 python -u bench.py --mode train --no-cpu-baseline > $O/bench_train.log 2>&1
timeout -k 10 300 python -u bench.py $C4 --no-cpu-baseline > $O/bench_c4.log 2>&1
timeout -k 10 400 python -u tools/datapath_bench.py --n 1024 --workers 0,8,15 --decode host,device > $O/datapath.log 2>&1
echo "bench ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_infer -o run -- python3 bench.py --steps 10 --no-extras --no-cpu-baseline > $O/prof_infer.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_train -o run -- python3 bench.py --mode train --steps 10 --no-cpu-baseline > $O/prof_train.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o run -- python3 bench.py $C4 --steps 5 --no-extras --no-cpu-baseline > $O/prof_c4.log 2>&1
echo "kernel trace ok"
# per-kernel stats CSV + top list + step timeline of each trace (the files profiles/ keeps)
for L in infer train c4; do
    DB=$O/prof_$L/run_results.db
    [ -f $DB ] || DB=$(ls $O/prof_$L/*/run_results.db 2>/dev/null | head -1)
    python3 tools/rocpd_stats.py $DB $O/${L}_kernel_stats.csv --top 25 > $O/${L}_kernel_top.txt
    python3 tools/step_breakdown.py $DB --timeline > $O/${L}_timeline.txt
    python3 tools/step_breakdown.py $DB --last-step > $O/${L}_last_step.txt
    python3 tools/step_breakdown.py $DB --walls > $O/${L}_walls.txt
done
rm -rf $O/prof_infer $O/prof_train $O/prof_c4
echo "stats ok"
