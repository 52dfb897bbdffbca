set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg.py tests/test_gpu_datapath.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03/pytest_jpeg.log 2>&1 || { echo "pytest failed"; grep -E "Error|error|assert|FAILED" gpurun_out/r03/pytest_jpeg.log | head -30; tail -5 gpurun_out/r03/pytest_jpeg.log; exit 1; }
tail -1 gpurun_out/r03/pytest_jpeg.log
