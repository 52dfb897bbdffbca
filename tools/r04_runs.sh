#!/bin/bash
# The round-4 GPU recipes behind DESIGN's numbers, one per subcommand (each one
# gpurun call; outputs under gpurun_out/<name>/):
#   profile   round profile (tools/round_profile.sh r04_v2) + fused-BN per-conv A/B
#             + training dgrad-tile A/B + C5 line
#   fb        fused-input-BN parity tests, per-conv A/B (tools/bnin_ab.py), C2 A/B
#   fb_prof   C2 kernel traces: A3 + fused BN, A3, the round-3 body
#   host      host enqueue cost per step (tools/host_cost.py) + bench lines
#   train_ab  training-step policy A/Bs in one process (tools/train_ab.py)
#   train_check  GPU suite, C3-shard bench line and kernel trace (the default policy)
#   c4_fuse   C4 with / without the halo-stage fused input BN (tools/infer_ab.py)
#   knobs     C2 / C4 BN-finalize two-level threshold A/B (tools/infer_ab.py)
#   infer_ab  C2 / C4 inference policy A/Bs in one process (tools/infer_ab.py): the A3
#             body vs the 2-stage body + tail launch, the fused input BN on / off
#   final     GPU suite, smoke(), default bench line
# Retired (round 5): the fused-BN A3 body (FB), tools/bnin_ab.py and the
# Policy.fuse_input_bn_a3 field were removed; the profile / fb / fb_prof recipes
# are kept as the record of how the round-4 profiles were made and refuse to run.
set -e
export TMPDIR=/tmp
cmd=${1:?subcommand}
O=gpurun_out/$cmd; mkdir -p $O
case $cmd in
profile)
    echo "$cmd: retired recipe (its tool / Policy field no longer exists)" >&2; exit 2
    bash tools/round_profile.sh r04_v2
    timeout -k 10 300 python -u tools/bnin_ab.py > gpurun_out/r04_v2/bnin_ab.log 2>&1
    bash tools/bench_ab.sh train_a3 "--mode train" "--mode train --tune dgrad_overlap_tile=11" 2
    timeout -k 10 600 python -u bench.py --mode train --backbone resnet50 --keypoints 8 --height 960 --width 1280 \
        --batch 32 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_c5.log 2>&1
    ;;
fb)
    echo "$cmd: retired recipe (its tool / Policy field no longer exists)" >&2; exit 2
    timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
        tests/test_gpu_precision.py -k "fused_input_bn" > $O/pytest_fb.log 2>&1
    timeout -k 10 300 python -u tools/bnin_ab.py > $O/bnin_ab.log 2>&1
    bash tools/bench_ab.sh fb_fuse "--tune fuse_input_bn_a3=1" "" 3 > $O/ab_fuse.txt 2>&1
    ;;
fb_prof)
    echo "$cmd: retired recipe (its tool / Policy field no longer exists)" >&2; exit 2
    i=0
    for cfg in "--tune fuse_input_bn_a3=1" "" "--tune x3_tile=9"; do
        i=$((i + 1))
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p$i -o run -- python3 bench.py --steps 10 \
            --no-extras --no-cpu-baseline $cfg > $O/p$i.log 2>&1
        DB=$O/p$i/run_results.db
        [ -f $DB ] || DB=$(ls $O/p$i/*/run_results.db 2>/dev/null | head -1)
        python3 tools/rocpd_stats.py $DB $O/k$i.csv --top 30 > $O/top$i.txt
        rm -rf $O/p$i
    done
    ;;
host)
    timeout -k 10 300 python -u tools/host_cost.py --mode train --steps 10 --profile > $O/train.log 2>&1
    timeout -k 10 300 python -u tools/host_cost.py --mode infer --steps 10 > $O/infer.log 2>&1
    timeout -k 10 300 python -u bench.py --mode train --no-cpu-baseline > $O/bench_train.log 2>&1
    ;;
train_ab)
    timeout -k 10 500 python -u tools/train_ab.py "" "overlap_min_gflop=20" "overlap_min_gflop=60" "overlap_wgrad=0" \
        --rounds 5 --iters 10 > $O/ab_overlap.log 2>&1
    timeout -k 10 500 python -u tools/train_ab.py "dgrad_overlap_tile=9" "" "dgrad_overlap_tile=0" \
        --rounds 7 --iters 10 > $O/ab_dgrad_tile.log 2>&1
    ;;
train_ab_sk)
    timeout -k 10 500 python -u tools/train_ab.py "" "dgrad_overlap_sk=1" --rounds 7 --iters 10 > $O/ab_dgrad_sk.log 2>&1
    ;;
infer_ab)
    timeout -k 10 400 python -u tools/infer_ab.py "" "x3_tile=9" "fuse_input_bn=0" --rounds 7 --iters 10 \
        > $O/ab_c2.log 2>&1
    timeout -k 10 400 python -u tools/infer_ab.py "" "f16_tile_1x1=9,f16_tile_kxk=9" --backbone resnet50 --keypoints 8 \
        --batch 128 --precision f16 --rounds 5 --iters 5 > $O/ab_c4.log 2>&1
    ;;
knobs)
    timeout -k 10 400 python -u tools/infer_ab.py "" "fin_two_level_tiles=512" "fin_two_level_tiles=8192" \
        --rounds 5 --iters 10 > $O/ab_c2_fin.log 2>&1
    timeout -k 10 400 python -u tools/infer_ab.py "" "fin_two_level_tiles=512" "fin_two_level_tiles=8192" \
        --backbone resnet50 --keypoints 8 --batch 128 --precision f16 --rounds 5 --iters 5 > $O/ab_c4_fin.log 2>&1
    ;;
c4_fuse)
    timeout -k 10 400 python -u tools/infer_ab.py "" "fuse_input_bn=0" --backbone resnet50 --keypoints 8 --batch 128 \
        --precision f16 --rounds 5 --iters 5 > $O/ab_c4_fuse.log 2>&1
    ;;
train_check)
    timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
    timeout -k 10 300 python -u bench.py --mode train --no-cpu-baseline > $O/bench_train.log 2>&1
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --mode train --steps 10 \
        --no-cpu-baseline > $O/prof.log 2>&1
    DB=$O/prof/run_results.db
    [ -f $DB ] || DB=$(ls $O/prof/*/run_results.db 2>/dev/null | head -1)
    python3 tools/rocpd_stats.py $DB $O/train_kernel_stats.csv --top 25 > $O/train_kernel_top.txt
    python3 tools/step_breakdown.py $DB --walls > $O/train_walls.txt
    rm -rf $O/prof
    ;;
final)
    timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
    timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1
    ;;
*)
    echo "unknown subcommand $cmd" >&2
    exit 2
    ;;
esac
echo "$cmd ok"
