set -e
export TMPDIR=/tmp
O=gpurun_out/nst3
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_precision.py tests/test_gpu_forward.py tests/test_gpu_backward.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u tools/conv_ab.py --tiles 0 --shapes layer2,t3,t4,c4_l2_c2,c4_l2_c1 --rounds 5 > $O/conv_new.log 2>&1
HKP_LIB_AB=tools/bin/libhulkkp_base.so timeout -k 10 200 python -u tools/conv_ab.py --tiles 0 --shapes layer2,t3,t4,c4_l2_c2,c4_l2_c1 --rounds 5 > $O/conv_base.log 2>&1
cat $O/conv_new.log $O/conv_base.log
bash tools/ab.sh "" "X=0" "HKP_LIB_AB=tools/bin/libhulkkp_base.so"
bash tools/ab.sh "--mode train" "X=0" "HKP_LIB_AB=tools/bin/libhulkkp_base.so"
bash tools/ab.sh "--backbone resnet50 --keypoints 8 --batch 128 --precision f16" "X=0" "HKP_LIB_AB=tools/bin/libhulkkp_base.so"
