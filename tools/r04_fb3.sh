#!/bin/bash
# A3 fused-input-BN body with asm-ordered LDS traffic: parity tests, per-conv A/B,
# C2 bench A/B fused vs unfused.  Output under gpurun_out/fb3/.
set -e
O=gpurun_out/fb3; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_precision.py -k "fused_input_bn" > $O/pytest_fb.log 2>&1
echo "fb tests ok: $(tail -1 $O/pytest_fb.log)"
timeout -k 10 300 python -u tools/bnin_ab.py > $O/bnin_ab.log 2>&1
grep -v amdgpu.ids $O/bnin_ab.log
bash tools/bench_ab.sh fb3_fuse "--tune fuse_input_bn_a3=1" "" 3 > $O/ab_fuse.txt 2>&1
echo "fuse ab (A fused, B not): $(cat $O/ab_fuse.txt | tr '\n' ' ')"
