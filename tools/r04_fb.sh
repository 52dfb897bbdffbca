#!/bin/bash
# Round-4 A3 fused-input-BN evidence (one gpurun call): its parity tests, then
# in-process / interleaved A/Bs — split-K tail in-launch vs second launch, C2 with
# and without the fused input BN, C2 on A3 vs the round-3 body (2-stage + tail
# launch, x3_tile=9).  Output under gpurun_out/fb/.
set -e
O=gpurun_out/fb; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_precision.py -k "fused_input_bn or sk_combine or tail" > $O/pytest_fb.log 2>&1
echo "fb tests ok: $(tail -1 $O/pytest_fb.log)"
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_gpu_scale.py -k "c2_bench_batch" > $O/pytest_c2.log 2>&1
echo "c2 test ok: $(tail -1 $O/pytest_c2.log)"
timeout -k 10 300 python -u tools/tail_ab.py --rounds 5 > $O/tail_ab.log 2>&1
echo "tail ab ok"
bash tools/bench_ab.sh fb_fuse "" "--tune fuse_input_bn=0" 3 > $O/ab_fuse.txt 2>&1
echo "fuse ab: $(cat $O/ab_fuse.txt | tr '\n' ' ')"
bash tools/bench_ab.sh fb_body "" "--tune x3_tile=9 --tune fuse_input_bn=0" 3 > $O/ab_body.txt 2>&1
echo "body ab: $(cat $O/ab_body.txt | tr '\n' ' ')"
