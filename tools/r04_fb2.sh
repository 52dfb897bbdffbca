#!/bin/bash
# A3 fused-input-BN body, second form: parity tests, per-conv in-process A/B
# (tools/bnin_ab.py), C2 bench A/B fused vs unfused.  Output under gpurun_out/fb2/.
set -e
O=gpurun_out/fb2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_precision.py -k "fused_input_bn" > $O/pytest_fb.log 2>&1
echo "fb tests ok: $(tail -1 $O/pytest_fb.log)"
timeout -k 10 300 python -u tools/bnin_ab.py > $O/bnin_ab.log 2>&1
cat $O/bnin_ab.log | grep -v amdgpu.ids
bash tools/bench_ab.sh fb2_fuse "" "--tune fuse_input_bn=0" 3 > $O/ab_fuse.txt 2>&1
echo "fuse ab: $(cat $O/ab_fuse.txt | tr '\n' ' ')"
