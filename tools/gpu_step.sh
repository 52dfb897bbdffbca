set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
timeout -k 10 500 python -u -m pytest tests/test_gpu_precision.py tests/test_gpu_gram.py tests/test_gpu_scale.py -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r03/pytest_stem.log 2>&1 || { echo "pytest failed"; grep -E "Error|error|assert|FAILED" gpurun_out/r03/pytest_stem.log | head -30; tail -5 gpurun_out/r03/pytest_stem.log; exit 1; }
tail -1 gpurun_out/r03/pytest_stem.log
grep -E "C4 B=128|vs reference|fused vs unfused" gpurun_out/r03/pytest_stem.log | cut -c1-250
C4="--backbone resnet50 --keypoints 8 --batch 128 --precision f16"
timeout -k 10 300 python -u bench.py $C4 --no-extras --no-cpu-baseline > gpurun_out/r03/c4_stem.log 2>&1 && tail -1 gpurun_out/r03/c4_stem.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r03/prof_c4_stem -o run -- python3 bench.py $C4 --steps 5 --no-extras --no-cpu-baseline > gpurun_out/r03/prof_c4_stem.log 2>&1
echo done
