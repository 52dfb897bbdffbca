mkdir -p gpurun_out
timeout -k 10 300 python -u tools/conv_ab.py --tiles 0,3,4 --shapes layer4,layer3,t4,c4_l4_c2,c4_l4_c1,c4_l4_c3,c4_l3_c3,c4_l4_c3,c4_l3_c3,c4_l1_c3 --rounds 5 --iters 5 > gpurun_out/ab2.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --backbone resnet50 --keypoints 8 --batch 128 --precision f16 --no-extras --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --mode train --no-extras --no-cpu-baseline > gpurun_out/bench_train.log 2>&1 || exit 1
