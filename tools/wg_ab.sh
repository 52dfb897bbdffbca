#!/bin/bash
# Kernel-trace A/B of the wgrad tile (KA 256 vs 128) on the C3 training shard:
# per-kernel totals land in gpurun_out/wgab/{A,B}/.../run_kernel_stats.csv
set -e
O=gpurun_out/wgab
mkdir -p $O
for rep in A B; do
  if [ $rep = A ]; then export HKP_WG_KA256=1; else export HKP_WG_KA256=0; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$rep -o run -- python3 bench.py --mode train --steps 10 --no-cpu-baseline > $O/$rep.log 2>&1
done
