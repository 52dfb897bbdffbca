#!/bin/bash
# Training-step policy A/B in one process (tools/train_ab.py): the wgrad
# side-stream overlap everywhere / above a size / nowhere, and the dgrad tile
# beside it.  Output under gpurun_out/train_ab/.
set -e
O=gpurun_out/train_ab; mkdir -p $O
timeout -k 10 500 python -u tools/train_ab.py "" "overlap_min_gflop=20" "overlap_min_gflop=60" "overlap_wgrad=0" \
    "overlap_min_gflop=20,dgrad_overlap_tile=11" --rounds 5 --iters 10 > $O/ab1.log 2>&1
grep -v amdgpu.ids $O/ab1.log
