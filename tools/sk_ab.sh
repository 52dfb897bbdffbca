set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_precision.py -x -q --timeout 120 --timeout-method thread -k "x3" > gpurun_out/sk_pytest.log 2>&1
timeout -k 10 300 python -u tools/conv_ab.py --variants 9,8 --shapes t4,t3,t2,t1,layer4,layer3,layer2,layer1 > gpurun_out/ab_sk.log 2>&1
