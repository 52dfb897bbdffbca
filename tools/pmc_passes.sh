#!/bin/bash
# PMC counter passes (one rocprofv3 run per counter group; --pmc is never
# combined with trace domains) for the kernels matching $KREGEX, over a short
# bench run.  Usage (on the GPU box, from the repo root):
#   tools/pmc_passes.sh OUTDIR "bench args..." [KREGEX]
# (PROG=tools/wg_time.py runs that script with the given args instead of bench.py)
# Writes OUTDIR/pmc_summary.json (tools/pmc_summary.py) and deletes the
# per-pass databases (they can exceed gpurun's 64 MiB copy-back limit).
set -u
OUT=$1
ARGS=$2
KREGEX=${3:-"conv_x3|wgrad_x3"}
export TMPDIR=/tmp
mkdir -p "$OUT"
NOCPU=--no-cpu-baseline
[ -n "${PROG:-}" ] && NOCPU=
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i + 1))
    timeout -k 10 240 rocprofv3 --pmc $grp --kernel-include-regex "$KREGEX" -d "$OUT/pass$i" -o run \
        -- python3 ${PROG:-bench.py} $ARGS $NOCPU > "$OUT/pass$i.log" 2>&1 || { echo "pass $i ($grp) failed: rc=$?"; exit 1; }
    echo "pass $i ok: $grp"
done
python3 tools/pmc_summary.py "$OUT" "$OUT/pmc_summary.json" > "$OUT/pmc_summary.txt" && rm -rf "$OUT"/pass*/
cat "$OUT/pmc_summary.txt"
