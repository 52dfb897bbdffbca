set -e
mkdir -p gpurun_out/bk
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py --mode train --no-cpu-baseline > gpurun_out/bk/plain_$rep.log 2>&1
  HKP_FORCE_BUCKETS=1 timeout -k 10 200 python -u bench.py --mode train --no-cpu-baseline > gpurun_out/bk/buckets_$rep.log 2>&1
  HKP_FORCE_BUCKETS=1 HKP_OVERLAP_WGRAD=0 timeout -k 10 200 python -u bench.py --mode train --no-cpu-baseline > gpurun_out/bk/serial_$rep.log 2>&1
done
