#!/bin/bash
# The round-5 GPU recipes behind DESIGN's numbers, one per subcommand (each one
# gpurun call; outputs under gpurun_out/<name>/).  The recipes of variants removed
# after their measurement (frac, multi, tail128, stem4, fin, a4) stay as the record of
# how those profiles were made; their knobs no longer exist, so they do not re-run.
#   check     GPU suite + the default bench line (C2 + the north_star batch-64 leg)
#   duo       the DUO body (plain-fp16 256x128, two blocks per CU): its parity tests,
#             per-conv A/B vs the planner (tools/conv_ab.py), C4 A/B in one process
#             (tools/infer_ab.py), then the GPU suite and the default bench line
#   store     epilogue store flavour A/B (hkp_debug_x3_store: default / nt / sc1) per conv
#             and end to end on C4 and C2, in one process each
#   stamps    per-block phase clocks of the A3 and DUO bodies on C4's 1x1 shapes
#             (tools/x3_stamps.py); training store-flavour A/B (tools/train_ab.py)
#   duo_stagger  DUO with its first-round per-CU stagger: phase stamps, per-conv and
#             C4 A/B
#   verify    GPU suite, C4 planner A/B (DUO choices vs the round-4 planner), default
#             and C4 bench lines
#   halo      the conflict-free halo swizzle: bit-identity tests, per-conv A/B against the
#             previous build (tools/ab_lib/libhulkkp_a.so), LDS bank-conflict PMC on C2 / C4,
#             C2 bench A/B
#   syncbn    the SyncBN GPU tests (per-call global BN-backward checks) + a 2-rank gloo
#             rehearsal of bench.py --gpus 2 (relaunch, north_star leg, train leg)
#   a3p       the persistent A3 body (HKP_TILE_A3P): parity tests, per-conv and C4 / C2 A/B
#   c5        C5 shard (R50-8s K=8 1280x960 B=32 training step): bench line, kernel
#             trace stats, per-launch listing, PMC passes over every kernel
#   frac      the fractional A3 tail (conv_x3_a3sk_kernel; removed after this run): its parity tests,
#             per-conv A/B (hkp_debug_x3_frac_tail 0 / 1 / 2), C2 / B=8 shard / C4 / C3-train A/B
#   rehearse8 bench.py --gpus 4 and --gpus 8 as gloo rehearsals on the one GPU (the driver's
#             scaling run's relaunch, rendezvous, north_star and train legs; not a measurement)
#   stem      per-block phase clocks of the stem conv (C2 batch 32, C4 batch 128)
#   stem4     the 4-wave stem patch form (removed after this run): tests, phase clocks, C2 / C4 A/B
#   multi     the multi-round split-K tail (removed after this run): tail tests, per-conv A/B
#             (hkp_debug_x3_multi_tail 0 / 1),
#             B=8 shard / C2 / C3-train A/B in one process
#   tail128   the split-K tail on 256x128 grids (removed after this run): tests, C2 / C3 / C4 A/B
#   fin       the one-pass BN finalize (removed after this run): BN tests, B=8 / C2 / C4 / C3 A/B
#   stemimg   the stem straight from the image (no packed planes): stem / data-path tests, C2 / C4 A/B
#   a3pfused  the persistent A3 body on C4's fused-epilogue conv3s only (Policy.f16_tile_fused = 14)
#   duofused  the DUO body on C4's fused-epilogue conv3s only (Policy.f16_tile_fused = 13)
#   stemimg2  the image-direct stem with its loads batched: stem tests, phase clocks, C2 / C4 A/B
#   a4        the 4-wave A3 body (HKP_TILE_A4; removed after this run): parity tests, per-conv A/B, phase clocks
#   ups       the upsample + sigmoid + argmax kernel at 4 sub-chunks per block: its tests, kernel
#             trace of the C2 and C4 benches (upsample_sigmoid_kernel average vs r05_v2)
#   pair128   the planner's 256x64 pairs for short-K / 128-wide f16x3 convs: planner and
#             forward / backward tests, C2 / B=8 / C3-train A/B (hkp_debug_x3_pair128 0 / 1)
#   finregs   the register-held BN finalize form: BN tests, B=8 / C2 / C3-train A/B
#             (hkp_debug_fin_regs 0 / 1)
#   sprio     the training step on a high-priority stream / the wgrad side stream high
#   headdw    the head's fc weight gradient on the wgrad side stream (Policy.overlap_head_dw;
#             removed after this run: neutral)
#   final     GPU suite, smoke(), default bench line
set -e
export TMPDIR=/tmp
cmd=${1:?subcommand}
O=gpurun_out/$cmd; mkdir -p $O
C5="--mode train --backbone resnet50 --keypoints 8 --height 960 --width 1280 --batch 32"
case $cmd in
check)
    timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
    echo "pytest: $(tail -1 $O/pytest_gpu.log)"
    timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
    ;;
duo)
    timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_precision.py \
        -k "f16_conv_exact_products" tests/test_gpu_gram.py > $O/pytest_duo.log 2>&1
    echo "pytest duo: $(tail -1 $O/pytest_duo.log)"
    timeout -k 10 400 python -u tools/conv_ab.py --tiles 0,13 --rounds 5 --iters 5 \
        --shapes c4_l4_c3,c4_l4_ds,c4_l4_c1,c4_l4_c2,c4_l3_c1,c4_l3_c3,c4_l3_c2,c4_l2_c1,c4_l2_c2,c4_l1_ds > $O/conv_ab.log 2>&1
    echo "conv_ab ok"
    timeout -k 10 500 python -u tools/infer_ab.py "" "f16_tile_1x1=13" "f16_tile_1x1=13,f16_tile_kxk=13" \
        --backbone resnet50 --keypoints 8 --batch 128 --precision f16 --rounds 5 --iters 5 > $O/ab_c4.log 2>&1
    echo "infer_ab ok"
    timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
    echo "pytest: $(tail -1 $O/pytest_gpu.log)"
    timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
    ;;
store)
    timeout -k 10 500 python -u tools/conv_ab.py --tiles 0,13 --stores 0,2,3 --rounds 5 --iters 5 \
        --shapes c4_l4_c3,c4_l4_ds,c4_l3_c3,c4_l3_c1,c4_l1_ds,layer4,layer3 > $O/conv_ab.log 2>&1
    echo "conv_ab ok"
    timeout -k 10 500 python -u tools/infer_ab.py "" "store=2" "store=3" "f16_tile_1x1=13,store=3" \
        --backbone resnet50 --keypoints 8 --batch 128 --precision f16 --rounds 5 --iters 5 > $O/ab_c4.log 2>&1
    echo "infer_ab c4 ok"
    timeout -k 10 500 python -u tools/infer_ab.py "" "store=2" "store=3" --rounds 5 --iters 10 > $O/ab_c2.log 2>&1
    ;;
stamps)
    timeout -k 10 300 python -u tools/x3_stamps.py c4_l4_c3 c4_l4_ds c4_l3_c3 c4_l1_ds > $O/stamps_a3.log 2>&1
    timeout -k 10 300 python -u tools/x3_stamps.py --tile 13 c4_l4_c3 c4_l4_ds c4_l3_c3 c4_l1_ds > $O/stamps_duo.log 2>&1
    timeout -k 10 500 python -u tools/train_ab.py "" "store=2" "store=3" --rounds 5 --iters 10 > $O/ab_train.log 2>&1
    ;;
duo_stagger)
    for d in 0 -1 4000 10000; do
        timeout -k 10 300 python -u tools/x3_stamps.py --tile 13 --duo-stagger $d c4_l4_c3 c4_l3_c3 c4_l1_ds \
            > $O/stamps_duo_$d.log 2>&1
    done
    timeout -k 10 500 python -u tools/conv_ab.py --tiles 0,13 --duo-staggers 0,-1,4000,10000 --rounds 5 --iters 5 \
        --shapes c4_l4_c3,c4_l4_ds,c4_l4_c1,c4_l3_c3,c4_l3_c1,c4_l3_c2,c4_l2_c1,c4_l1_ds > $O/conv_ab.log 2>&1
    timeout -k 10 500 python -u tools/infer_ab.py "" "f16_tile_1x1=13" "f16_tile_1x1=13,f16_tile_kxk=13" \
        --backbone resnet50 --keypoints 8 --batch 128 --precision f16 --rounds 5 --iters 5 > $O/ab_c4.log 2>&1
    ;;
verify)
    timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
    echo "pytest: $(tail -1 $O/pytest_gpu.log)"
    timeout -k 10 500 python -u tools/infer_ab.py "" "f16_tile_1x1=12,f16_tile_kxk=12" \
        --backbone resnet50 --keypoints 8 --batch 128 --precision f16 --rounds 7 --iters 5 > $O/ab_c4.log 2>&1
    timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
    timeout -k 10 400 python -u bench.py --backbone resnet50 --keypoints 8 --batch 128 --precision f16 \
        --no-cpu-baseline > $O/bench_c4.log 2>&1
    ;;
halo)
    timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_precision.py \
        -k "halo or fused_input_bn" > $O/pytest_halo.log 2>&1
    echo "pytest halo: $(tail -1 $O/pytest_halo.log)"
    timeout -k 10 300 python -u tools/conv_ab.py --tiles 0 --shapes layer1,c4_l1_c2,h128 --rounds 7 --iters 10 \
        --lib tools/ab_lib/libhulkkp_a.so > $O/conv_a.log 2>&1
    timeout -k 10 300 python -u tools/conv_ab.py --tiles 0 --shapes layer1,c4_l1_c2,h128 --rounds 7 --iters 10 \
        > $O/conv_b.log 2>&1
    timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE \
        --kernel-include-regex "halo" -d $O/pmc/pass1 -o run -- python3 bench.py --steps 3 --no-extras \
        --no-cpu-baseline > $O/pmc1.log 2>&1
    timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE \
        --kernel-include-regex "halo" -d $O/pmc_c4/pass1 -o run -- python3 bench.py --steps 2 --no-extras \
        --no-cpu-baseline --backbone resnet50 --keypoints 8 --batch 128 --precision f16 > $O/pmc2.log 2>&1
    python3 tools/pmc_summary.py $O/pmc $O/pmc_c2.json > $O/pmc_c2.txt
    python3 tools/pmc_summary.py $O/pmc_c4 $O/pmc_c4.json > $O/pmc_c4.txt
    rm -rf $O/pmc $O/pmc_c4
    bash tools/ab.sh "" "--lib tools/ab_lib/libhulkkp_a.so" "" > $O/ab_c2.txt 2>&1
    ;;
syncbn)
    timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_syncbn.py \
        > $O/pytest_syncbn.log 2>&1
    echo "pytest syncbn: $(tail -1 $O/pytest_syncbn.log)"
    timeout -k 10 600 python -u bench.py --gpus 2 --rehearse-gloo --steps 3 --warmup 1 --no-cpu-baseline \
        > $O/rehearse_n2.log 2>&1
    echo "rehearsal ok"
    ;;
a3p)
    timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_precision.py \
        -k "a3p" > $O/pytest_a3p.log 2>&1
    echo "pytest a3p: $(tail -1 $O/pytest_a3p.log)"
    timeout -k 10 500 python -u tools/conv_ab.py --tiles 0,14 --rounds 5 --iters 5 \
        --shapes c4_l4_c3,c4_l4_ds,c4_l4_c1,c4_l4_c2,c4_l3_c3,c4_l3_c1,c4_l3_c2,c4_l1_ds,layer4,layer3 > $O/conv_ab.log 2>&1
    echo "conv_ab ok"
    timeout -k 10 500 python -u tools/infer_ab.py "" "f16_tile_1x1=14" "f16_tile_1x1=14,f16_tile_kxk=14" \
        --backbone resnet50 --keypoints 8 --batch 128 --precision f16 --rounds 5 --iters 5 > $O/ab_c4.log 2>&1
    timeout -k 10 500 python -u tools/infer_ab.py "" "x3_tile=14" --rounds 5 --iters 10 > $O/ab_c2.log 2>&1
    ;;
a3p_stamps)
    timeout -k 10 300 python -u tools/x3_stamps.py c4_l4_c3 c4_l3_c3 c4_l1_ds layer3 > $O/stamps_a3.log 2>&1
    timeout -k 10 300 python -u tools/x3_stamps.py --tile 14 c4_l4_c3 c4_l3_c3 c4_l1_ds layer3 > $O/stamps_a3p.log 2>&1
    ;;
prio)
    timeout -k 10 500 python -u tools/infer_ab.py "" "prio=1" "prio=2" --rounds 7 --iters 10 > $O/ab_c2.log 2>&1
    timeout -k 10 500 python -u tools/infer_ab.py "" "prio=1" "prio=2" --backbone resnet50 --keypoints 8 --batch 128 \
        --precision f16 --rounds 5 --iters 5 > $O/ab_c4.log 2>&1
    timeout -k 10 500 python -u tools/train_ab.py "" "prio=1" --rounds 5 --iters 10 > $O/ab_train.log 2>&1
    ;;
b8)
    # the north_star shard (C2 network, batch 8 on one GPU): bench line + kernel trace
    timeout -k 10 300 python -u bench.py --batch 8 --no-extras --no-cpu-baseline > $O/bench_b8.log 2>&1
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --batch 8 --steps 10 \
        --no-extras --no-cpu-baseline > $O/prof.log 2>&1
    DB=$O/prof/run_results.db
    [ -f $DB ] || DB=$(ls $O/prof/*/run_results.db 2>/dev/null | head -1)
    python3 tools/rocpd_stats.py $DB $O/b8_kernel_stats.csv --top 30 > $O/b8_kernel_top.txt
    python3 tools/step_breakdown.py $DB --last-step > $O/b8_last_step.txt
    python3 tools/step_breakdown.py $DB --timeline > $O/b8_timeline.txt
    rm -rf $O/prof
    ;;
c5)
    timeout -k 10 400 python -u bench.py $C5 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_c5.log 2>&1
    echo "bench ok"
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py $C5 --steps 3 \
        --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1
    DB=$O/prof/run_results.db
    [ -f $DB ] || DB=$(ls $O/prof/*/run_results.db 2>/dev/null | head -1)
    python3 tools/rocpd_stats.py $DB $O/c5_kernel_stats.csv --top 40 > $O/c5_kernel_top.txt
    python3 tools/step_breakdown.py $DB --last-step > $O/c5_last_step.txt
    python3 tools/step_breakdown.py $DB --walls > $O/c5_walls.txt
    rm -rf $O/prof
    echo "trace ok"
    bash tools/pmc_passes.sh $O/pmc "$C5 --steps 2 --warmup 1" "."
    ;;
frac)
    timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_precision.py \
        -k "fractional or split_k_tail" > $O/pytest_frac.log 2>&1
    echo "pytest frac: $(tail -1 $O/pytest_frac.log)"
    timeout -k 10 500 python -u tools/conv_ab.py --tiles 0 --fracs 0,1,2 --rounds 5 --iters 5 \
        --shapes t3,t4,t3a,t4ds,layer3,layer4,c4_l4_c2,c4_l3_c2,c4_l3_c1 > $O/conv_ab.log 2>&1
    echo "conv_ab ok"
    timeout -k 10 400 python -u tools/infer_ab.py "frac=0" "" "frac=2" --rounds 7 --iters 10 > $O/ab_c2.log 2>&1
    timeout -k 10 400 python -u tools/infer_ab.py "frac=0" "" "frac=2" --batch 8 --rounds 7 --iters 20 > $O/ab_b8.log 2>&1
    timeout -k 10 500 python -u tools/infer_ab.py "frac=0" "" "frac=2" --backbone resnet50 --keypoints 8 --batch 128 \
        --precision f16 --rounds 5 --iters 5 > $O/ab_c4.log 2>&1
    timeout -k 10 500 python -u tools/train_ab.py "frac=0" "" "frac=2" --rounds 5 --iters 10 > $O/ab_train.log 2>&1
    ;;
rehearse8)
    timeout -k 10 500 python -u bench.py --gpus 4 --rehearse-gloo --steps 2 --warmup 1 --no-cpu-baseline \
        > $O/rehearse_n4.log 2>&1
    echo "n4 ok"
    timeout -k 10 700 python -u bench.py --gpus 8 --rehearse-gloo --steps 2 --warmup 1 --no-cpu-baseline \
        > $O/rehearse_n8.log 2>&1
    echo "n8 ok"
    ;;
stem)
    timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_precision.py \
        -k "stem" tests/test_gpu_forward.py > $O/pytest_stem.log 2>&1
    echo "pytest stem: $(tail -1 $O/pytest_stem.log)"
    timeout -k 10 300 python -u tools/x3_stamps.py stem:32 stem:128 > $O/stamps_stem.log 2>&1
    timeout -k 10 300 python -u tools/x3_stamps.py --tile 6 stem:32 stem:128 > $O/stamps_stem_pair.log 2>&1
    timeout -k 10 400 python -u tools/infer_ab.py "stem_pair=1" "" --rounds 7 --iters 10 > $O/ab_c2.log 2>&1
    timeout -k 10 500 python -u tools/infer_ab.py "stem_pair=1" "" --backbone resnet50 --keypoints 8 --batch 128 \
        --precision f16 --rounds 5 --iters 5 > $O/ab_c4.log 2>&1
    ;;
stem4)
    timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_precision.py \
        -k "stem" > $O/pytest_stem4.log 2>&1
    echo "pytest stem4: $(tail -1 $O/pytest_stem4.log)"
    timeout -k 10 300 python -u tools/x3_stamps.py stem:32 stem4:32 stem:128 stem4:128 > $O/stamps.log 2>&1
    timeout -k 10 400 python -u tools/infer_ab.py "" "stem4=1" --rounds 7 --iters 10 > $O/ab_c2.log 2>&1
    timeout -k 10 500 python -u tools/infer_ab.py "" "stem4=1" --backbone resnet50 --keypoints 8 --batch 128 \
        --precision f16 --rounds 5 --iters 5 > $O/ab_c4.log 2>&1
    ;;
multi)
    timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_precision.py \
        -k "tail" > $O/pytest_multi.log 2>&1
    echo "pytest multi: $(tail -1 $O/pytest_multi.log)"
    timeout -k 10 500 python -u tools/conv_ab.py --tiles 0 --multis 0,1 --rounds 7 --iters 5 \
        --shapes t3,t3a,t4,layer3,layer4 > $O/conv_ab.log 2>&1
    echo "conv_ab ok"
    timeout -k 10 400 python -u tools/infer_ab.py "multi=0" "" --batch 8 --rounds 9 --iters 20 > $O/ab_b8.log 2>&1
    timeout -k 10 400 python -u tools/infer_ab.py "multi=0" "" --batch 64 --rounds 5 --iters 5 > $O/ab_b64.log 2>&1
    timeout -k 10 500 python -u tools/train_ab.py "multi=0" "" --rounds 5 --iters 10 > $O/ab_train.log 2>&1
    ;;
tail128)
    timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_precision.py \
        -k "tail" > $O/pytest_tail128.log 2>&1
    echo "pytest tail128: $(tail -1 $O/pytest_tail128.log)"
    timeout -k 10 400 python -u tools/infer_ab.py "tail128=0" "" "tail128=0" "" --rounds 9 --iters 10 > $O/ab_c2.log 2>&1
    timeout -k 10 500 python -u tools/train_ab.py "tail128=0" "" --rounds 5 --iters 10 > $O/ab_train.log 2>&1
    timeout -k 10 500 python -u tools/infer_ab.py "tail128=0" "" --backbone resnet50 --keypoints 8 --batch 128 \
        --precision f16 --rounds 5 --iters 5 > $O/ab_c4.log 2>&1
    ;;
fin)
    timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_backward.py \
        tests/test_gpu_forward.py tests/test_gpu_syncbn.py tests/test_gpu_gram.py > $O/pytest_fin.log 2>&1
    echo "pytest fin: $(tail -1 $O/pytest_fin.log)"
    timeout -k 10 400 python -u tools/infer_ab.py "fin2=1" "" --batch 8 --rounds 9 --iters 20 > $O/ab_b8.log 2>&1
    timeout -k 10 400 python -u tools/infer_ab.py "fin2=1" "" --rounds 9 --iters 10 > $O/ab_c2.log 2>&1
    timeout -k 10 500 python -u tools/train_ab.py "fin2=1" "" --rounds 5 --iters 10 > $O/ab_train.log 2>&1
    timeout -k 10 500 python -u tools/infer_ab.py "fin2=1" "" --backbone resnet50 --keypoints 8 --batch 128 \
        --precision f16 --rounds 5 --iters 5 > $O/ab_c4.log 2>&1
    ;;
stemimg)
    timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_precision.py \
        -k "stem" tests/test_gpu_datapath.py tests/test_gpu_forward.py > $O/pytest_stemimg.log 2>&1
    echo "pytest stemimg: $(tail -1 $O/pytest_stemimg.log)"
    timeout -k 10 400 python -u tools/infer_ab.py "stem_img=0" "" --rounds 9 --iters 10 > $O/ab_c2.log 2>&1
    timeout -k 10 500 python -u tools/infer_ab.py "stem_img=0" "" --backbone resnet50 --keypoints 8 --batch 128 \
        --precision f16 --rounds 5 --iters 5 > $O/ab_c4.log 2>&1
    ;;
a3pfused)
    timeout -k 10 500 python -u tools/infer_ab.py "" "f16_tile_fused=14" "" "f16_tile_fused=14" --backbone resnet50 \
        --keypoints 8 --batch 128 --precision f16 --rounds 4 --iters 5 > $O/ab_c4.log 2>&1
    ;;
duofused)
    timeout -k 10 500 python -u tools/infer_ab.py "" "f16_tile_fused=13" "" "f16_tile_fused=13" --backbone resnet50 \
        --keypoints 8 --batch 128 --precision f16 --rounds 4 --iters 5 > $O/ab_c4.log 2>&1
    ;;
stemimg2)
    timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_precision.py \
        -k "stem" > $O/pytest.log 2>&1
    echo "pytest: $(tail -1 $O/pytest.log)"
    timeout -k 10 400 python -u tools/infer_ab.py "stem_img=0" "" "stem_img=0" "" --rounds 5 --iters 10 > $O/ab_c2.log 2>&1
    timeout -k 10 500 python -u tools/infer_ab.py "stem_img=0" "" --backbone resnet50 --keypoints 8 --batch 128 \
        --precision f16 --rounds 5 --iters 5 > $O/ab_c4.log 2>&1
    ;;
a4)
    timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_precision.py \
        -k "a4_equals" > $O/pytest_a4.log 2>&1
    echo "pytest a4: $(tail -1 $O/pytest_a4.log)"
    timeout -k 10 500 python -u tools/conv_ab.py --tiles 11,15 --rounds 5 --iters 5 \
        --shapes layer4,layer3,t4,c4_l4_c2,c4_l4_c1,c4_l4_c3,c4_l3_c3 > $O/conv_ab.log 2>&1
    timeout -k 10 300 python -u tools/x3_stamps.py --tile 15 layer4 c4_l4_c3 > $O/stamps_a4.log 2>&1
    timeout -k 10 300 python -u tools/x3_stamps.py --tile 11 layer4 c4_l4_c3 > $O/stamps_a3.log 2>&1
    ;;
ups)
    timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_forward.py \
        tests/test_gpu_scale.py tests/test_gpu_dropin.py > $O/pytest_ups.log 2>&1
    echo "pytest ups: $(tail -1 $O/pytest_ups.log)"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 10 --no-extras \
        --no-cpu-baseline > $O/prof.log 2>&1
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof4 -o run -- python3 bench.py --steps 5 --no-extras \
        --no-cpu-baseline --backbone resnet50 --keypoints 8 --batch 128 --precision f16 > $O/prof4.log 2>&1
    for L in prof prof4; do
        DB=$O/$L/run_results.db
        [ -f $DB ] || DB=$(ls $O/$L/*/run_results.db 2>/dev/null | head -1)
        python3 tools/rocpd_stats.py $DB $O/${L}_stats.csv --top 40 > $O/${L}_top.txt
    done
    rm -rf $O/prof $O/prof4
    ;;
pair128)
    timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_precision.py \
        tests/test_gpu_forward.py tests/test_gpu_backward.py > $O/pytest_pair128.log 2>&1
    echo "pytest pair128: $(tail -1 $O/pytest_pair128.log)"
    timeout -k 10 400 python -u tools/infer_ab.py "pair128=0" "" --rounds 9 --iters 10 > $O/ab_c2.log 2>&1
    timeout -k 10 400 python -u tools/infer_ab.py "pair128=0" "" --batch 8 --rounds 9 --iters 20 > $O/ab_b8.log 2>&1
    timeout -k 10 500 python -u tools/train_ab.py "pair128=0" "" --rounds 5 --iters 10 > $O/ab_train.log 2>&1
    ;;
finregs)
    timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_backward.py \
        tests/test_gpu_forward.py tests/test_gpu_syncbn.py tests/test_gpu_gram.py > $O/pytest_finregs.log 2>&1
    echo "pytest finregs: $(tail -1 $O/pytest_finregs.log)"
    timeout -k 10 400 python -u tools/infer_ab.py "finregs=0" "" --batch 8 --rounds 9 --iters 20 > $O/ab_b8.log 2>&1
    timeout -k 10 400 python -u tools/infer_ab.py "finregs=0" "" --rounds 9 --iters 10 > $O/ab_c2.log 2>&1
    timeout -k 10 500 python -u tools/train_ab.py "finregs=0" "" --rounds 5 --iters 10 > $O/ab_train.log 2>&1
    ;;
headdw)
    timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_backward.py \
        tests/test_gpu_scale.py tests/test_gpu_dropin.py tests/test_gpu_syncbn.py > $O/pytest_headdw.log 2>&1
    echo "pytest headdw: $(tail -1 $O/pytest_headdw.log)"
    timeout -k 10 600 python -u tools/train_ab.py "overlap_head_dw=0" "" "overlap_head_dw=0" "" --rounds 5 \
        --iters 10 > $O/ab_train.log 2>&1
    ;;
sprio)
    timeout -k 10 500 python -u tools/train_ab.py "" "mainprio=-1" "" "mainprio=-1" "sideprio=-1" --rounds 5 \
        --iters 10 > $O/ab_train.log 2>&1
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
