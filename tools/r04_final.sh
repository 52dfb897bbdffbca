#!/bin/bash
# Final-tree check (one call): GPU suite, smoke(), default bench line.
set -e
O=gpurun_out/r04_final; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo "pytest: $(tail -1 $O/pytest_gpu.log)"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1
grep -o '"value": [0-9.]*' $O/bench.log | head -1
