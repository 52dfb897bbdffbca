set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/v4
timeout -k 10 400 python -u -m pytest tests/test_gpu_precision.py tests/test_gpu_forward.py -x -q --timeout 120 --timeout-method thread > gpurun_out/v4/pytest.log 2>&1 || { tail -30 gpurun_out/v4/pytest.log; exit 1; }
tail -2 gpurun_out/v4/pytest.log
timeout -k 10 200 python -u tools/x3_stamps.py c4_l4_c3 c4_l1_c3 c4_l4_c1
bash tools/ab.sh "--backbone resnet50 --keypoints 8 --batch 128 --precision f16" "X=0"
bash tools/ab.sh "" "X=0"
