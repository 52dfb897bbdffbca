set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/v3
timeout -k 10 300 python -u -m pytest tests/test_gpu_precision.py -x -q --timeout 120 --timeout-method thread -k "persistent" > gpurun_out/v3/pytest_p.log 2>&1 || { tail -30 gpurun_out/v3/pytest_p.log; exit 1; }
tail -2 gpurun_out/v3/pytest_p.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_precision.py -x -q --timeout 120 --timeout-method thread > gpurun_out/v3/pytest.log 2>&1 || { tail -30 gpurun_out/v3/pytest.log; exit 1; }
tail -2 gpurun_out/v3/pytest.log
bash tools/ab.sh "--backbone resnet50 --keypoints 8 --batch 128 --precision f16" "X=0" "HKP_F16_TILE_1X1=7" "HKP_F16_TILE_1X1=8"
