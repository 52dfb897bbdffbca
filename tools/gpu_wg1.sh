set -e
export TMPDIR=/tmp
O=gpurun_out/wg1
mkdir -p $O
timeout -k 10 200 python -u tools/wg_time.py > $O/wg_time.log 2>&1
cat $O/wg_time.log
HKP_OVERLAP_WGRAD=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_serial -o run -- python3 bench.py --mode train --steps 10 --no-cpu-baseline > $O/prof_serial.log 2>&1
python3 - <<'PY'
import csv, glob
f = sorted(glob.glob("gpurun_out/wg1/prof_serial/**/*kernel_stats.csv", recursive=True))[0]
rows = list(csv.DictReader(open(f)))
for r in rows[:16]:
    print("%6.2f%% %6s %10.1f us  %s" % (float(r["Percentage"]), r["Calls"], float(r["AverageNs"]) / 1e3, r["Name"][:90]))
PY
grep -o '"value": [0-9.]*' $O/prof_serial.log | head -1
