set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u -m pytest tests/test_gpu_backward.py -m gpu -x -q -k "priority or deterministic or bucket" --timeout 200 --timeout-method thread > gpurun_out/r03/pytest_prio.log 2>&1 || { echo "pytest failed"; grep -E "Error|error|assert|FAILED" gpurun_out/r03/pytest_prio.log | head -30; tail -5 gpurun_out/r03/pytest_prio.log; exit 1; }
tail -1 gpurun_out/r03/pytest_prio.log
bash tools/ab.sh "--mode train" "" "--tune priority_stream=1"
