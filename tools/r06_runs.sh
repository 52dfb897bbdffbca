#!/bin/bash
# The round-6 GPU recipes behind DESIGN's numbers, one per subcommand (each one
# gpurun call; outputs under gpurun_out/<name>/).
#   hbm       per-kernel HBM tables (kernel trace + PMC passes over every kernel) of
#             C2 (batch 32) and the north_star shard (batch 8), and the default bench line
#   check     GPU suite + the default bench line
#   final     GPU suite, smoke(), default bench line
set -e
export TMPDIR=/tmp
cmd=${1:?subcommand}
O=gpurun_out/$cmd; mkdir -p $O
C4="--backbone resnet50 --keypoints 8 --batch 128 --precision f16"

# kernel trace + per-kernel stats of one bench workload: trace NAME "bench args"
trace() {
    local name=$1 args=$2
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$name -o run -- python3 bench.py $args \
        --no-extras --no-cpu-baseline > $O/prof_$name.log 2>&1
    local DB=$O/prof_$name/run_results.db
    [ -f $DB ] || DB=$(ls $O/prof_$name/*/run_results.db 2>/dev/null | head -1)
    python3 tools/rocpd_stats.py $DB $O/${name}_kernel_stats.csv --top 40 > $O/${name}_kernel_top.txt
    python3 tools/step_breakdown.py $DB --walls > $O/${name}_walls.txt
    rm -rf $O/prof_$name
}

case $cmd in
hbm)
    timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
    echo "bench ok"
    trace c2 "--steps 5 --warmup 2"
    bash tools/pmc_passes.sh $O/pmc_c2 "--steps 2 --warmup 1 --no-extras" "."
    python3 tools/hbm_table.py $O/c2_kernel_stats.csv $O/pmc_c2/pmc_summary.json --steps 12 --top 40 > $O/c2_hbm_table.txt
    echo "c2 ok"
    trace b8 "--batch 8 --steps 10 --warmup 2"
    bash tools/pmc_passes.sh $O/pmc_b8 "--batch 8 --steps 2 --warmup 1 --no-extras" "."
    python3 tools/hbm_table.py $O/b8_kernel_stats.csv $O/pmc_b8/pmc_summary.json --steps 22 --top 40 > $O/b8_hbm_table.txt
    echo "b8 ok"
    ;;
check)
    timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
    echo "pytest: $(tail -1 $O/pytest_gpu.log)"
    timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
    ;;
final)
    timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
    timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
    ;;
*)
    echo "unknown subcommand $cmd" >&2
    exit 2
    ;;
esac
echo "$cmd ok"
