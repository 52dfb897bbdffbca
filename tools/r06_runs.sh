#!/bin/bash
# The round-6 GPU recipes behind DESIGN's numbers, one per subcommand (each one
# gpurun call; outputs under gpurun_out/<name>/).
#   hbm       per-kernel HBM tables (kernel trace + PMC passes over every kernel) of
#             C2 (batch 32) and the north_star shard (batch 8), and the default bench line
#   (fold / fold2, the folded BN finalize A/Bs, ran against the experiment's commit
#   0a6ba20 and went with it; their logs are profiles/r06_fold_v*)
#   awrap     C4 1x1 convs with an L2-resident A window (AB build): what bounds the K loop
#   prec      per-stage precision plans at C4 (Policy.stage_precision): tests + study table
#   plan      the measured tile plan (tools/tile_sweep.py) and its A/B against the C planner
#   prof      the final tree's traces (C2 + PMC, B=8, C4, C3 train) and bench lines
#   pmc       PMC passes of the final tree for C4 and C3 training
#   a192      the 192-row A3 tiles: tests and per-conv timing on the B=8 shapes
#   dg        the overlapped dgrad's tile (C3 training) with the 160-row forms
#   plan16    the batch-16 shard (north_star at N = 4) added to the plan
#   c5        C5 training: the plan vs the C planner
#   h12       the 12x20 halo-staged A3 body: tests and per-conv timing (ran against commit 5d8eaa7;
#             measured slower and removed with it: profiles/r06_h12_*)
#   bnr/bnrt  BN backward reduce with batched row loads: tests, C3 old vs new build, traces
#             (measured slower when sharing CUs with the wgrad; not kept: profiles/r06_bnr_*)
#   wab       the overlapped wgrad behind the next BN backward: C3 A/B (ran with a Policy field
#             that was not kept: 471 vs 480 img/s, profiles/r06_wgrad_after_bn_ab_train.log)
#   wgh       the halo wgrad body (3x3 stride-1 layers of <= 128 channels): tests, standalone
#             timing vs the tiled body, C3 training A/B
#   gap       C3 traces with the halo wgrads on 64 vs 160 CUs (the cross-stream gaps)
#   trainab   this build vs tools/ab_lib/libhulkkp_base.so: backward tests, C3 bench lines
#   proftrain the C3 training trace, PMC and bench line after the halo wgrad
#   wgh2      a halo wgrad build vs the previous build (tests, timing, C3 bench lines)
#   wghpmc    PMC passes over the standalone halo and tiled wgrads (layer1 shape)
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
awrap)
    # verdict item 1 probe (AB build): C4's 1x1 convs with their A rows wrapped to an
    # L2-resident window (hkp_debug_x3_a_wrap) — if the K loop speeds up to the MFMA
    # rate, the stream of A from HBM (not the LDS / MFMA schedule) bounds it
    timeout -k 10 500 python -u tools/conv_ab.py --tiles 0 --a-wraps 0,4096,1024,256 --rounds 5 --iters 10 \
        --shapes c4_l4_c3,c4_l4_ds,c4_l4_c1,c4_l3_c3,c4_l3_c1 > $O/conv_ab.log 2>&1
    ;;
prec)
    # per-stage precision at C4 (Policy.stage_precision): the plan tests, then the study table
    timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_precision.py \
        -k "stage_precision or r50" tests/test_gpu_scale.py > $O/pytest_prec.log 2>&1
    echo "pytest prec: $(tail -1 $O/pytest_prec.log)"
    timeout -k 10 600 python -u tests/precision_study.py --rounds 3 --iters 3 > $O/precision_study.log 2>&1
    ;;
plan)
    # the measured tile plan: sweep every live tile policy over the workloads' forward
    # conv shapes (writes hulk-keypoints_amd/hkp/tile_plan.json, copied back), then the
    # plan vs the C planner in one process (Policy.tile_plan)
    timeout -k 10 900 python -u tools/tile_sweep.py --workloads ${WL:-c2,b8,c3,c4,c5} --rounds 5 --iters 4 \
        --out $O/tile_plan.json > $O/sweep.log 2>&1
    cp $O/tile_plan.json hulk-keypoints_amd/hkp/tile_plan.json
    timeout -k 10 400 python -u tools/infer_ab.py "" "tile_plan=0" --batch 8 --rounds 7 --iters 20 > $O/ab_b8.log 2>&1
    timeout -k 10 400 python -u tools/infer_ab.py "" "tile_plan=0" --rounds 7 --iters 10 > $O/ab_c2.log 2>&1
    timeout -k 10 500 python -u tools/infer_ab.py "" "tile_plan=0" $C4 --rounds 5 --iters 5 > $O/ab_c4.log 2>&1
    timeout -k 10 500 python -u tools/train_ab.py "" "tile_plan=0" "dgrad_overlap_tile=15" --rounds 5 --iters 10 \
        > $O/ab_train.log 2>&1
    ;;
prof)
    # the final tree's traces and C2 PMC passes (copied into profiles/ on the box so
    # the bench lines after them read this tree's trace), then the C2, B=8, C4 and
    # C3-train bench lines
    trace c2 "--steps 5 --warmup 2"
    cp $O/c2_kernel_stats.csv profiles/r06_infer_c2_kernel_stats_v3.csv
    bash tools/pmc_passes.sh $O/pmc_c2 "--steps 2 --warmup 1 --no-extras" "." > $O/pmc_c2.log 2>&1
    cp $O/pmc_c2/pmc_summary.json profiles/r06_infer_c2_pmc_v3.json
    python3 tools/hbm_table.py $O/c2_kernel_stats.csv $O/pmc_c2/pmc_summary.json --steps 12 --top 40 > $O/c2_hbm_table.txt
    echo "c2 ok"
    trace b8 "--batch 8 --steps 10 --warmup 2"
    cp $O/b8_kernel_stats.csv profiles/r06_b8_kernel_stats_v3.csv
    trace c4 "$C4 --steps 5 --warmup 2"
    cp $O/c4_kernel_stats.csv profiles/r06_infer_c4_kernel_stats_v2.csv
    trace train "--mode train --steps 5 --warmup 2"
    cp $O/train_kernel_stats.csv profiles/r06_train_c3_kernel_stats_v2.csv
    echo "traces ok"
    timeout -k 10 300 python -u bench.py > $O/bench_c2.log 2>&1
    timeout -k 10 300 python -u bench.py --batch 8 --no-cpu-baseline --no-extras > $O/bench_b8.log 2>&1
    timeout -k 10 300 python -u bench.py $C4 --no-cpu-baseline --no-extras > $O/bench_c4.log 2>&1
    timeout -k 10 300 python -u bench.py --mode train --no-cpu-baseline --no-extras > $O/bench_train.log 2>&1
    ;;
pmc)
    # PMC passes of the final tree for C4 and the C3 training shard (the C2 passes are
    # in "prof"); kernel traces from "prof" pair with them in the HBM tables
    bash tools/pmc_passes.sh $O/pmc_c4 "$C4 --steps 2 --warmup 1 --no-extras" "." > $O/pmc_c4.log 2>&1
    echo "c4 ok"
    bash tools/pmc_passes.sh $O/pmc_train "--mode train --steps 2 --warmup 1 --no-extras" "." > $O/pmc_train.log 2>&1
    echo "train ok"
    ;;
a192)
    # the 192-row A3 tiles (HKP_TILE_192_A3): their parity tests, the precision suite
    # around them, then per-conv timing on the B=8 shard's shapes against A3 / the planner
    timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_precision.py \
        > $O/pytest_prec.log 2>&1
    echo "pytest: $(tail -1 $O/pytest_prec.log)"
    timeout -k 10 500 python -u tools/conv_ab.py --tiles 0,11,15,16 --rounds 7 --iters 20 \
        --shapes t3,t3a,t2,t2s,t4,t4ds,t3ds > $O/conv_ab.log 2>&1
    ;;
dg)
    # training dgrad tile under the wgrad overlap (Policy.dgrad_overlap_tile) with the 160-row forms
    timeout -k 10 600 python -u tools/train_ab.py "" "dgrad_overlap_tile=16" "dgrad_overlap_tile=0" \
        --rounds 7 --iters 10 > $O/ab_train.log 2>&1
    timeout -k 10 600 python -u tools/train_ab.py "" "dgrad_overlap_tile=16,wgrad_overlap_cus=64" \
        "dgrad_overlap_tile=16,wgrad_overlap_cus=128" "overlap_wgrad=0" --rounds 5 --iters 10 > $O/ab_train2.log 2>&1
    ;;
plan16)
    # the north_star shard at N = 4 (batch 16 per rank) added to the committed plan
    cp hulk-keypoints_amd/hkp/tile_plan.json $O/tile_plan.json
    timeout -k 10 600 python -u tools/tile_sweep.py --workloads b16 --rounds 5 --iters 4 \
        --out $O/tile_plan.json > $O/sweep.log 2>&1
    cp $O/tile_plan.json hulk-keypoints_amd/hkp/tile_plan.json
    timeout -k 10 400 python -u tools/infer_ab.py "" "tile_plan=0" --batch 16 --rounds 7 --iters 20 > $O/ab_b16.log 2>&1
    ;;
c5)
    # config C5 (R50-8s K=8 1280x960, the 32-image shard of batch 256 over 8 GPUs): the
    # measured plan against the C planner in one process
    timeout -k 10 900 python -u tools/train_ab.py "" "tile_plan=0" --backbone resnet50 --keypoints 8 --height 960 \
        --width 1280 --batch 32 --rounds 3 --iters 2 > $O/ab_c5.log 2>&1
    ;;
h12)
    # the 12x20 halo-staged A3 body (HKP_TILE_HALO12): its tests, then per-conv timing
    timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_precision.py \
        > $O/pytest_prec.log 2>&1
    echo "pytest: $(tail -1 $O/pytest_prec.log)"
    timeout -k 10 500 python -u tools/conv_ab.py --tiles 0,11,17 --rounds 7 --iters 10 \
        --shapes c2_l3,c2_l3a,c4_l3_c2,t3 > $O/conv_ab.log 2>&1
    ;;
bnr)
    # the BN backward reduce with its rows' loads batched (8 in flight per thread):
    # the backward tests, then the C3 training bench line of the previous build
    # (tools/ab_lib/libhulkkp_base.so) against this one in alternating processes
    timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu \
        -k "backward or bwd or train or syncbn or c3 or grad" > $O/pytest_bwd.log 2>&1
    echo "pytest: $(tail -1 $O/pytest_bwd.log)"
    for i in 1 2; do
        timeout -k 10 300 python -u bench.py --mode train --no-extras --no-cpu-baseline \
            --lib tools/ab_lib/libhulkkp_base.so > $O/bench_base_$i.log 2>&1
        timeout -k 10 300 python -u bench.py --mode train --no-extras --no-cpu-baseline > $O/bench_new_$i.log 2>&1
    done
    ;;
bnrt)
    # kernel traces of the C3 step, previous build vs this one (BN backward reduce)
    trace train_new "--mode train --steps 5 --warmup 2"
    trace train_base "--mode train --steps 5 --warmup 2 --lib tools/ab_lib/libhulkkp_base.so"
    ;;
wab)
    # the overlapped wgrad launched behind the next BN backward (Policy.wgrad_after_bn)
    timeout -k 10 600 python -u tools/train_ab.py "" "wgrad_after_bn=1" --rounds 7 --iters 10 > $O/ab_train.log 2>&1
    timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu \
        -k "backward or bwd or train or c3 or grad" > $O/pytest_bwd.log 2>&1
    ;;
wgh)
    timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_precision.py \
        -k "wgrad" > $O/pytest_wgrad.log 2>&1
    echo "pytest: $(tail -1 $O/pytest_wgrad.log)"
    timeout -k 10 300 python -u tools/wg_time.py --shapes t1,t2 --variants 0,-1 > $O/wg_time.log 2>&1
    cat $O/wg_time.log
    timeout -k 10 600 python -u tools/train_ab.py "" "wgrad_halo=0" --rounds 7 --iters 10 > $O/ab_train.log 2>&1
    tail -4 $O/ab_train.log
    ;;
gap)
    # the layer1/2 cross-stream gaps: traces of the C3 step with the halo wgrads on 64
    # CUs (192 left to the dgrad) and on the default 160
    trace train_h64 "--mode train --steps 5 --warmup 2 --tune wgrad_halo_cus=64"
    trace train_h160 "--mode train --steps 5 --warmup 2"
    ;;
gapsk)
    # the overlapped dgrads without the stream-K workspace: A/B and a trace
    timeout -k 10 550 python -u tools/train_ab.py "" "dgrad_overlap_sk=0" --rounds 11 --iters 10 > $O/ab.log 2>&1
    tail -2 $O/ab.log
    trace train_nosk "--mode train --steps 5 --warmup 2 --tune dgrad_overlap_sk=0"
    ;;
trainab)
    # this build against tools/ab_lib/libhulkkp_base.so: the backward tests, then C3
    # training bench lines alternating
    timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu \
        -k "backward or bwd or train or c3 or grad or dgrad" > $O/pytest_bwd.log 2>&1
    echo "pytest: $(tail -1 $O/pytest_bwd.log)"
    for i in 1 2 3 4; do
        timeout -k 10 300 python -u bench.py --mode train --no-cpu-baseline --no-extras > $O/train_new_$i.log 2>&1
        timeout -k 10 300 python -u bench.py --mode train --no-cpu-baseline --no-extras \
            --lib tools/ab_lib/libhulkkp_base.so > $O/train_base_$i.log 2>&1
    done
    for f in $O/train_new_*.log $O/train_base_*.log; do
        echo "$f $(grep '^{' $f | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
    done
    ;;
proftrain)
    # the C3 training step after the halo wgrad / CU budgets: kernel trace (copied into
    # profiles/ on the box so the bench line after it reads it), PMC passes, bench line
    trace train "--mode train --steps 5 --warmup 2"
    cp $O/train_kernel_stats.csv profiles/r06_train_c3_kernel_stats_v4.csv
    bash tools/pmc_passes.sh $O/pmc_train "--mode train --steps 2 --warmup 1 --no-extras" "." > $O/pmc_train.log 2>&1
    cp $O/pmc_train/pmc_summary.json profiles/r06_train_c3_pmc_v3.json
    cp $O/pmc_train/pmc_summary.txt profiles/r06_train_c3_pmc_v3.txt
    python3 tools/hbm_table.py $O/train_kernel_stats.csv $O/pmc_train/pmc_summary.json --steps 7 --top 40 \
        > $O/train_hbm_table.txt
    timeout -k 10 300 python -u bench.py --mode train --no-cpu-baseline --no-extras > $O/bench_train.log 2>&1
    ;;
wgh2)
    # a halo wgrad build against the previous one (tools/ab_lib/libhulkkp_base.so):
    # tests, standalone timing per build, C3 training bench lines alternating
    timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_precision.py \
        -k "wgrad" > $O/pytest_wgrad.log 2>&1
    echo "pytest: $(tail -1 $O/pytest_wgrad.log)"
    for i in 1 2; do
        timeout -k 10 200 python -u tools/wg_time.py --shapes t1,t2 --variants 0 > $O/wg_new_$i.log 2>&1
        timeout -k 10 200 python -u tools/wg_time.py --shapes t1,t2 --variants 0 --lib tools/ab_lib/libhulkkp_base.so \
            > $O/wg_base_$i.log 2>&1
    done
    grep -h wgrad $O/wg_new_*.log $O/wg_base_*.log
    for i in 1 2 3; do
        timeout -k 10 300 python -u bench.py --mode train --no-extras --no-cpu-baseline > $O/train_new_$i.log 2>&1
        timeout -k 10 300 python -u bench.py --mode train --no-extras --no-cpu-baseline \
            --lib tools/ab_lib/libhulkkp_base.so > $O/train_base_$i.log 2>&1
    done
    for f in $O/train_new_*.log $O/train_base_*.log; do
        echo "$f $(grep '^{' $f | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
    done
    ;;
wghpmc)
    # PMC passes over the standalone halo wgrad (layer1 shape) and the tiled body
    PROG=tools/wg_time.py bash tools/pmc_passes.sh $O/halo "--shapes t1 --variants 0 --rounds 2 --iters 3" \
        "wgrad_x3_halo" > $O/halo.log 2>&1
    PROG=tools/wg_time.py bash tools/pmc_passes.sh $O/tiled "--shapes t1 --variants -1 --rounds 2 --iters 3" \
        "wgrad_x3_kernel" > $O/tiled.log 2>&1
    cat $O/halo/pmc_summary.txt $O/tiled/pmc_summary.txt
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
