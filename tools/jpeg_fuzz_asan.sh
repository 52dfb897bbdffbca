#!/bin/bash
# Host-only: build the entropy decoder with ASan/UBSan and decode seeded
# corruptions of small JPEGs (CPU, no GPU).  Usage: bash tools/jpeg_fuzz_asan.sh [N]
set -euo pipefail
cd "$(dirname "$0")/.."
N=${1:-3000}
D=$(mktemp -d /tmp/hkpj_fuzz.XXXXXX)
trap 'rm -rf "$D"' EXIT
gcc -O1 -g -std=gnu11 -fsanitize=address,undefined -fno-sanitize-recover=all -fno-omit-frame-pointer \
    -Iinclude -o "$D/fuzz" tools/jpeg_fuzz_asan.c hulk-keypoints_amd/csrc/host/jpeg_entropy.c
python - "$D" "$N" <<'PY'
import io, sys
import numpy as np
from PIL import Image
d, n = sys.argv[1], int(sys.argv[2])
rng = np.random.default_rng(31)
def jpeg(h, w, gray=False, **kw):
    img = rng.integers(0, 256, (h, w) if gray else (h, w, 3), dtype=np.uint8)
    b = io.BytesIO(); Image.fromarray(img).save(b, "JPEG", **kw); return b.getvalue()
bases = [jpeg(40, 56, quality=80, subsampling=2), jpeg(33, 47, quality=60, subsampling=0, restart_marker_blocks=2),
         jpeg(24, 24, True, quality=90, optimize=True), jpeg(17, 70, quality=30, subsampling=1, optimize=True)]
for i in range(n):
    b = bytearray(bases[i % len(bases)])
    k = i % 4
    if k == 0:
        for _ in range(int(rng.integers(1, 8))):
            b[int(rng.integers(2, len(b)))] = int(rng.integers(0, 256))
    elif k == 1:
        b = b[:int(rng.integers(2, len(b)))]
    elif k == 2:
        j = int(rng.integers(2, min(len(b), 400)))
        b[j:j + 16] = rng.integers(0, 256, 16).astype(np.uint8).tobytes()
    else:
        b = b[:int(rng.integers(2, len(b)))] + rng.integers(0, 256, int(rng.integers(1, 64))).astype(np.uint8).tobytes()
    open("%s/%05d.jpg" % (d, i), "wb").write(bytes(b))
PY
ls "$D"/*.jpg | xargs "$D/fuzz"
