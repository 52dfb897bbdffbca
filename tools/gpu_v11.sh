set -e
export TMPDIR=/tmp
O=gpurun_out/v11
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_precision.py tests/test_gpu_forward.py tests/test_gpu_backward.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u tools/conv_ab.py --tiles 0,3,9 --shapes layer3,layer4,t3,t4,c4_l4_c2 --rounds 5 --iters 5 | grep tile
bash tools/ab.sh "" "X=0"
bash tools/ab.sh "--mode train" "X=0"
bash tools/ab.sh "--backbone resnet50 --keypoints 8 --batch 128 --precision f16" "X=0"
