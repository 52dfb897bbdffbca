set -e
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/mp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "maxpool or stem or forward or golden or backward" > gpurun_out/mp/pytest.log 2>&1 || { tail -30 gpurun_out/mp/pytest.log; exit 1; }
tail -1 gpurun_out/mp/pytest.log
for r in 1 2; do
timeout -k 10 120 python -u tools/maxpool_time.py --lib tools/ab_lib/libhulkkp_a.so
timeout -k 10 120 python -u tools/maxpool_time.py
done
