set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"
timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1 && echo c2 ok
timeout -k 10 300 python -u bench.py --backbone resnet50 --keypoints 8 --batch 128 --precision f16 --no-extras --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1 && echo c4 ok
timeout -k 10 400 python -u bench.py --mode train --backbone resnet50 --keypoints 8 --height 960 --width 1280 --batch 32 --steps 5 --warmup 2 --no-extras --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1 && echo c5 ok
