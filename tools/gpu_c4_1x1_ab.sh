set -e
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ab1x1
S=c4_l1_c3,c4_l1_c1,c4_l1_c1a,c4_l2_c1a,c4_l3_c1,c4_l4_c1,c4_l4_c3
timeout -k 10 300 python -u tools/conv_ab.py --tiles 0,6,4 --shapes $S --rounds 5 --iters 5 > gpurun_out/ab1x1/stats.log 2>&1
cat gpurun_out/ab1x1/stats.log
timeout -k 10 300 python -u tools/conv_ab.py --tiles 0,6,4 --shapes $S --rounds 5 --iters 5 --nostats > gpurun_out/ab1x1/nostats.log 2>&1
cat gpurun_out/ab1x1/nostats.log
