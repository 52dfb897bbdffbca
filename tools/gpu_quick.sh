set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/v2
timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py -x -q --timeout 120 --timeout-method thread > gpurun_out/v2/pytest.log 2>&1 || { tail -40 gpurun_out/v2/pytest.log; exit 1; }
tail -2 gpurun_out/v2/pytest.log
timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline > gpurun_out/v2/c2.log 2>&1
timeout -k 10 300 python -u bench.py --backbone resnet50 --keypoints 8 --batch 128 --precision f16 --no-extras --no-cpu-baseline > gpurun_out/v2/c4.log 2>&1
python3 -c "
import json
for f in ['c2','c4']:
    d=json.loads(open('gpurun_out/v2/%s.log'%f).read().strip().splitlines()[-1]); print(f, round(d['value'],1), round(d['ms_per_step'],3), d['roofline']['kernel'], round(d['roofline']['frac'],3))
"
