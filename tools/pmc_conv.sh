#!/bin/bash
# PMC counter passes over one conv_ab.py shape (one rocprofv3 --pmc run per
# counter group, never combined with trace domains):
#   tools/pmc_conv.sh OUTDIR SHAPE TILE
# Writes OUTDIR/pmc_summary.{json,txt} (tools/pmc_summary.py).
set -u
OUT=$1
SHAPE=$2
TILE=${3:-0}
export TMPDIR=/tmp
mkdir -p "$OUT"
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_SALU SQ_INSTS_VALU SQ_ACTIVE_INST_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "conv_x3_kernel" -d "$OUT/pass$i" -o run \
        -- python3 tools/conv_ab.py --tiles $TILE --shapes $SHAPE --rounds 2 --iters 3 > "$OUT/pass$i.log" 2>&1 \
        || { echo "pass $i ($grp) failed: rc=$?"; tail -5 "$OUT/pass$i.log"; exit 1; }
    echo "pass $i ok: $grp"
done
python3 tools/pmc_summary.py "$OUT" "$OUT/pmc_summary.json" > "$OUT/pmc_summary.txt" && rm -rf "$OUT"/pass*/
cat "$OUT/pmc_summary.txt"
