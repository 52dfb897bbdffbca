#!/bin/bash
# conv_ab per-shape timings with the timing-probe builds (X3_PROBE: 1 no DMA in
# the K loop, 2 no MFMA) beside the product library
set -o pipefail
O=gpurun_out/probe
mkdir -p $O
S=${1:-layer4,layer3,c4_l4_c3,c4_l4_c2,c4_l3_c3}
for v in base p1 p2; do
  if [ $v = base ]; then L=""; else L=tools/bin/libhulkkp_$v.so; fi
  HKP_LIB_AB=$L timeout -k 10 240 python3 -u tools/conv_ab.py --tiles 3 --rounds 5 --iters 5 --shapes $S > $O/$v.log 2>&1 || exit 1
  echo "== $v"; cat $O/$v.log | grep tile
done
