# bench lines with the per-launch attainable roofline (C2 default, C4)
set -e
export TMPDIR=/tmp
O=gpurun_out/roof
mkdir -p $O
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/c2.log 2>&1 || { tail -20 $O/c2.log; exit 1; }
timeout -k 10 300 python -u bench.py --backbone resnet50 --keypoints 8 --batch 128 --precision f16 --no-extras --no-cpu-baseline > $O/c4.log 2>&1 || { tail -20 $O/c4.log; exit 1; }
for f in c2 c4; do python3 -c "
import json; d=json.loads(open('$O/$f.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$f', round(d['value'],1), r['kernel'], 'frac %.3f' % r['frac'], 'frac_of_roofline %.3f' % r['frac_of_roofline'], 'hbm share %.2f' % r['hbm_bound_share_of_attainable'])
t=d.get('train'); 
if t: print('train', round(t['value'],1), 'frac %.3f' % t['roofline']['frac'], 'roof %.3f' % t['roofline']['frac_of_roofline'])"; done
