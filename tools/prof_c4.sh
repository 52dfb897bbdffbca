#!/bin/bash
# Kernel-trace stats of the C4 (R50 K8 640x480 B128 fp16) inference bench.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-prof_c4}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o run -- python3 bench.py --backbone resnet50 --keypoints 8 --batch 128 --precision f16 --steps 5 --warmup 2 --no-extras --no-cpu-baseline > $O/log.txt 2>&1
python3 tools/rocpd_stats.py $(ls $O/*/*.db $O/*.db 2>/dev/null | head -1) $O/stats.csv --top 40 > $O/top.txt
