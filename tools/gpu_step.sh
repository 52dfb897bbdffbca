set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u -m pytest tests/test_gpu_precision.py -m gpu -x -q -k "wgrad" --timeout 120 --timeout-method thread > gpurun_out/r03/pytest_wg.log 2>&1 || { echo "pytest failed"; grep -E "Error|error|assert|FAILED" gpurun_out/r03/pytest_wg.log | head -20; tail -5 gpurun_out/r03/pytest_wg.log; exit 1; }
tail -1 gpurun_out/r03/pytest_wg.log
bash tools/ab.sh "--mode train" "" "--tune wgrad_overlap_cus=64" "--tune wgrad_overlap_cus=128" "--tune wgrad_overlap_cus=192"
