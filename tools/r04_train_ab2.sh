#!/bin/bash
# In-process A/B of the overlapped dgrad's tile policy (9: 2-stage 256x256 + a
# tail launch; 11: A3 with the tail in the same launch; 0: the planner).
set -e
O=gpurun_out/train_ab; mkdir -p $O
timeout -k 10 500 python -u tools/train_ab.py "" "dgrad_overlap_tile=11" "dgrad_overlap_tile=0" \
    --rounds 7 --iters 10 > $O/ab2.log 2>&1
grep -v amdgpu.ids $O/ab2.log
