set -e
export TMPDIR=/tmp
O=gpurun_out/v6
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_precision.py tests/test_gpu_forward.py tests/test_gpu_backward.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python -u tools/x3_stamps.py c4_l4_c3 c4_l1_c3 layer4 layer3 layer1
bash tools/ab.sh "--backbone resnet50 --keypoints 8 --batch 128 --precision f16" "X=0"
bash tools/ab.sh "" "X=0"
