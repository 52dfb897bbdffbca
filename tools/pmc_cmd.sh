#!/bin/bash
# PMC counter passes of an arbitrary command (one rocprofv3 --pmc run per group,
# never combined with trace domains), summarized on the box.
#   tools/pmc_cmd.sh OUTDIR KREGEX "group1;group2;..." python3 tools/conv_ab.py ...
set -u
OUT=$1; KREGEX=$2; GROUPS_=$3; shift 3
export TMPDIR=/tmp
mkdir -p "$OUT"
i=0
IFS=';' read -ra GS <<< "$GROUPS_"
for grp in "${GS[@]}"; do
    i=$((i + 1))
    timeout -k 10 240 rocprofv3 --pmc $grp --kernel-include-regex "$KREGEX" -d "$OUT/pass$i" -o run -- "$@" \
        > "$OUT/pass$i.log" 2>&1 || { echo "pass $i ($grp) failed: rc=$?"; exit 1; }
    echo "pass $i ok: $grp"
done
python3 tools/pmc_summary.py "$OUT" "$OUT/pmc_summary.json" > "$OUT/pmc_summary.txt" && rm -rf "$OUT"/pass*/
cat "$OUT/pmc_summary.txt"
