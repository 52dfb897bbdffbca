"""tools/trcheck.py: the register hazard of untracked asm LDS reads (the compiler
treats an inline-asm ds_read_b64_tr_b16 as complete when issued).  A synthetic
listing pins the checker; the conv_x3 / gram kernels, cross-compiled for gfx950
here, must have no access to a register whose asm read is still in flight."""
import os
import re
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))

import trcheck  # noqa: E402

LISTING = """
_Zk:
\tds_read_b64_tr_b16 v[2:3], v10 offset:0
\tds_read_b64_tr_b16 v[4:5], v10 offset:512
\tv_mov_b32_e32 v6, v2
\ts_cbranch_scc1 .LBB0_2
\tv_mov_b32_e32 v4, 0
.LBB0_2:
\ts_waitcnt lgkmcnt(1)
\tv_add_u32_e32 v7, v2, v8
\tv_add_u32_e32 v9, v4, v8
\ts_waitcnt lgkmcnt(0)
\tv_add_u32_e32 v11, v4, v8
\ts_endpgm
.Lfunc_end0:
"""


def test_checker_finds_each_hazard(tmp_path, capsys):
    f = tmp_path / "k.s"
    f.write_text(LISTING)
    sys.argv = ["trcheck", str(f), "_Zk"]
    trcheck.main()
    out = capsys.readouterr().out
    # v2 read before any wait; v4 overwritten on the branch path while its read
    # is in flight; v4 read after lgkmcnt(1) (only v[2:3] retired); clean after lgkmcnt(0)
    assert "READ  block 0 +2: v_mov_b32_e32 v6, v2" in out
    assert "WRITE block 1 +0: v_mov_b32_e32 v4, 0" in out
    assert "v_add_u32_e32 v9, v4, v8" in out
    assert "v7, v2" not in out and "v11" not in out
    assert out.strip().endswith("hazards: 3")


@pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="hipcc absent")
@pytest.mark.parametrize("src", ["conv_x3.hip", "gram.hip"])
def test_kernels_have_no_inflight_register_access(tmp_path, src, capsys):
    out = tmp_path / "k.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
                    "-ffp-contract=off", "-Wno-unused-function", "-Wno-unused-variable", "--cuda-device-only", "-S",
                    os.path.join(REPO, "hulk-keypoints_amd", "csrc", src), "-o", str(out)],
                   check=True, capture_output=True, timeout=600)
    text = out.read_text()
    kernels = sorted(set(re.findall(r"^(_ZN3hkp\w*kernel\w*):", text, re.M)))
    assert kernels
    bad = {}
    for k in kernels:
        sys.argv = ["trcheck", str(out), k]
        trcheck.main()
        res = capsys.readouterr().out.strip().split("\n")[-1]
        if res != "hazards: 0":
            bad[k] = res
    assert not bad, bad
