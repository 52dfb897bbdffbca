#!/bin/bash
# Per-kernel resource usage (VGPRs, spills, LDS, occupancy) of one .hip file: tools/kres.sh csrc/conv_x3.hip
f=${1:?hip file}
cd /tmp && /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-function \
    -Wno-unused-variable -c "$f" -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import re, sys, subprocess
cur = None
rows = []
for line in sys.stdin:
    m = re.search(r"remark: +(Function Name|Name|VGPRs|AGPRs|VGPRs Spill|SGPRs Spill|LDS Size \[bytes/block\]|Occupancy \[waves/SIMD\]): (\S+)", line)
    if not m: continue
    k, v = m.groups()
    if k in ("Function Name", "Name"):
        cur = {"name": v}; rows.append(cur)
    elif cur is not None:
        cur[k] = v
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True).stdout.split("\n")
for r, n in zip(rows, names):
    print("%4s vgpr %3s spill %5s lds occ %s  %s" % (r.get("VGPRs"), r.get("VGPRs Spill"), r.get("LDS Size [bytes/block]"), r.get("Occupancy [waves/SIMD]"), n[:110]))
'
