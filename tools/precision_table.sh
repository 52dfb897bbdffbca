#!/bin/bash
# Precision modes on config C4's network (DESIGN "precision modes"): parity vs the
# reference fixture (pytest -s prints heat error / argmax agreement) and img/s at
# the C4 bench shape (R50-8s K=8 640x480 B=128) per mode.  Output: gpurun_out/prec/
set -o pipefail
out=gpurun_out/prec; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -s -v --timeout 240 --timeout-method thread tests/test_gpu_precision.py \
    -k "product_subsets or f16_forward_close" > $out/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -s -v --timeout 240 --timeout-method thread tests/test_gpu_scale.py \
    -k "r50_bench_resolution" >> $out/pytest.log 2>&1 || exit $?
for p in f16 f16x2a f16x2w f16x3; do
    timeout -k 10 300 python bench.py --backbone resnet50 --keypoints 8 --batch 128 --precision $p --steps 10 \
        --warmup 3 --no-extras --no-cpu-baseline > $out/bench_$p.log 2>&1 || exit $?
done
