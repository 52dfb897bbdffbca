#!/bin/bash
# Kernel traces of C2 under three forms: default (A3 + fused input BN), A3 with the
# apply pass (fuse_input_bn=0), the round-3 body (x3_tile=9: 2-stage ring + tail
# launch, no fusion).  Per-kernel stats CSV per form under gpurun_out/fbp/.
set -e
O=gpurun_out/fbp; mkdir -p $O
export TMPDIR=/tmp
i=0
for cfg in "" "--tune fuse_input_bn=0" "--tune x3_tile=9 --tune fuse_input_bn=0"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p$i -o run -- python3 bench.py --steps 10 --no-extras --no-cpu-baseline $cfg > $O/p$i.log 2>&1
    DB=$O/p$i/run_results.db
    [ -f $DB ] || DB=$(ls $O/p$i/*/run_results.db 2>/dev/null | head -1)
    python3 tools/rocpd_stats.py $DB $O/k$i.csv --top 30 > $O/top$i.txt
    python3 tools/step_breakdown.py $DB --walls > $O/walls$i.txt
    rm -rf $O/p$i
    echo "cfg $i ok: $(grep -o '"value": [0-9.]*' $O/p$i.log | head -1)"
done
