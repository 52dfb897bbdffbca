set -e
export TMPDIR=/tmp
O=gpurun_out/c5
mkdir -p $O
timeout -k 10 400 python -u bench.py --mode train --backbone resnet50 --keypoints 8 --height 960 --width 1280 --batch 32 --steps 5 --warmup 2 --no-extras --no-cpu-baseline > $O/c5.log 2>&1
tail -1 $O/c5.log | cut -c1-400
