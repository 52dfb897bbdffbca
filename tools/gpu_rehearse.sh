# the N>1 bench path rehearsed with 2 ranks on the box's one GPU (gloo); not a measurement
set -e
export TMPDIR=/tmp
O=gpurun_out/rehearse
mkdir -p $O
HKP_DIST_REHEARSE=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline > $O/n2.log 2>&1 || { tail -40 $O/n2.log; exit 1; }
tail -1 $O/n2.log | cut -c1-400
HKP_DIST_REHEARSE=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-extras --sync-bn > $O/n2_sync.log 2>&1 || { tail -40 $O/n2_sync.log; exit 1; }
tail -1 $O/n2_sync.log | cut -c1-300
HKP_DIST_REHEARSE=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-extras --mode train --sync-bn > $O/n2_train_sync.log 2>&1 || { tail -40 $O/n2_train_sync.log; exit 1; }
tail -1 $O/n2_train_sync.log | cut -c1-300
